#!/bin/bash
# round-4 second pass: GPU suite, smoke, bench, config-5 profile, small-miss A/B,
# 2 MiB placement A/B, UTCL tail counters
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$PWD}
TAG=${1:-r04c}
mkdir -p gpurun_out
(cd /tmp && timeout -s KILL 60 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/counters_avail.txt 2>&1) || echo "counter list failed"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.log 2>&1 && \
bash tools/profile_config5.sh _$TAG
rc=$?
tail -3 gpurun_out/pytest_gpu_$TAG.log; grep -v amdgpu.ids gpurun_out/smoke_$TAG.log; tail -c 600 gpurun_out/bench_$TAG.log
exit $rc
