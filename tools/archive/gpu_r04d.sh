#!/bin/bash
# round-4 probes: small-miss padding A/B, 2 MiB placement A/B, UTCL tail counters
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$PWD}
mkdir -p gpurun_out
bash tools/small_miss_ab.sh > /dev/null && \
timeout -k 10 400 python3 tools/align2m_ab.py 3 > gpurun_out/align2m_ab.log 2>&1 && \
bash tools/tail_utcl.sh > /dev/null
rc=$?
tail -30 gpurun_out/small_miss_ab.log; cat gpurun_out/align2m_ab.log; cat gpurun_out/tail_utcl.log
exit $rc
