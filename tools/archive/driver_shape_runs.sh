#!/bin/bash
# N fresh processes of bench.py in the driver's shape (--steps 20 --warmup 5), the
# headline fraction and the live kernel fraction of each:
#   bash tools/driver_shape_runs.sh <tag> [N = 6]
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$PWD}
TAG=${1:-ds}
N=${2:-6}
mkdir -p gpurun_out
for k in $(seq 1 $N); do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_${TAG}_$k.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/bench_${TAG}_$k.log') if l.startswith('{')][-1]); print('run $k', d['per_gpu']['frac_of_hbm_peak'], d['roofline']['frac'])"
done
