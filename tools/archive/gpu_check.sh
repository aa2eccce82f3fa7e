#!/bin/bash
# GPU suite, smoke and one default bench line (no rocprofv3 passes):
#   bash tools/gpu_check.sh <tag>     (on the GPU box, from the repo root)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$PWD}
TAG=${1:-check}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu_$TAG.log; grep -v amdgpu.ids gpurun_out/smoke_$TAG.log; tail -c 600 gpurun_out/bench_$TAG.log
exit $rc
