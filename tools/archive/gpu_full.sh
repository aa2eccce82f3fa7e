#!/bin/bash
# Full GPU pass for a round: tests, smoke, bench, then rocprofv3 kernel trace +
# separate FETCH_SIZE / WRITE_SIZE passes (tools/profile_r01.sh).  Run on the
# GPU box from the repo root:  bash tools/gpu_full.sh <tag>
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$PWD}
TAG=${1:-run}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.log 2>&1 && \
bash tools/profile_r03.sh $TAG
rc=$?
tail -2 gpurun_out/pytest_gpu_$TAG.log; cat gpurun_out/smoke_$TAG.log | grep -v amdgpu.ids; tail -c 1500 gpurun_out/bench_$TAG.log
exit $rc
