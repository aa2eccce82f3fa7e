#!/bin/bash
# round 4, fused 8-operand combine at one workgroup per CU: the fused-combine
# parity tests, config5_combine three times, the config-5 rocprofv3 passes
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$PWD}
TAG=${1:-r04f}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_schedule_fused_gpu.py \
    tests/test_coll_loopback_gpu.py tests/test_config_size_gpu.py > gpurun_out/pytest_fused_$TAG.log 2>&1 && \
for k in 1 2 3; do timeout -k 10 120 python bench.py --only-config5 --steps 20 --warmup 3 > gpurun_out/config5_$TAG.$k.log 2>&1 || exit 1; done && \
bash tools/profile_config5.sh _$TAG
rc=$?
tail -1 gpurun_out/pytest_fused_$TAG.log
for k in 1 2 3; do python3 -c "import json; d=json.loads([l for l in open('gpurun_out/config5_$TAG.$k.log') if l.startswith('{')][-1])['config5_combine']; print(d['two_operand']['frac'], d['chain8']['frac'], d['chain8']['kernel_us'])"; done
exit $rc
