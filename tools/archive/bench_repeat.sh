#!/bin/bash
# N default bench lines in separate processes (same box): bash tools/bench_repeat.sh <tag> [N=2]
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$PWD}
mkdir -p gpurun_out
for i in $(seq 1 ${2:-2}); do
  timeout -k 10 300 python bench.py > gpurun_out/bench_$1_$i.log 2>&1 || exit 1
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/bench_$1_$i.log') if l.startswith('{')][-1]); r=d['roofline']
print('run $i value', d['value'], d['per_gpu']['frac_of_hbm_peak'], 'fresh', d['sync_variants']['fresh_args']['frac_of_hbm_peak'], 'roofline mean/median/p10-p90', r['mean_launch_us'], r['median_launch_us'], r['p10_p90_us'], r['frac'])
"
done
