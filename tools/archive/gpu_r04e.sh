#!/bin/bash
# round-4 final pass: GPU suite, smoke, bench (defaults), bench in the driver's
# shape x6 (fresh processes), rocprofv3 trace + FETCH/WRITE passes (profile_r03.sh)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$PWD}
TAG=${1:-r04final}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.log 2>&1 && \
for k in 1 2 3 4 5 6; do timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_driver_shape_$k.log 2>&1 || exit 1; done && \
bash tools/profile_r03.sh $TAG
rc=$?
tail -2 gpurun_out/pytest_gpu_$TAG.log; grep -v amdgpu.ids gpurun_out/smoke_$TAG.log | tail -2
for f in gpurun_out/bench_$TAG.log gpurun_out/bench_driver_shape_*.log; do python3 -c "import json,sys; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); print('$f', d['per_gpu']['frac_of_hbm_peak'], d['roofline']['frac'])"; done
exit $rc
