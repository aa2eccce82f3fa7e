#!/bin/bash
# round 4, fused combines with the P = 8 and P = 4 LDS caps: the fused-combine /
# loopback / config-size GPU tests, then the two library builds alternated
# (tools/multi_cap_ab.sh; build them first with `bash tools/multi_cap_ab.sh build`)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$PWD}
TAG=${1:-r04g}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_schedule_fused_gpu.py \
    tests/test_coll_loopback_gpu.py tests/test_config_size_gpu.py > gpurun_out/pytest_fused_$TAG.log 2>&1 && \
bash tools/multi_cap_ab.sh > /dev/null
rc=$?
tail -1 gpurun_out/pytest_fused_$TAG.log
cat gpurun_out/multi_cap_ab.log
exit $rc
