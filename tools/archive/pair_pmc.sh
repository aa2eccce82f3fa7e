#!/bin/bash
# round 5: per-pair duration and UTCL1 translation counters of the headline
# loop, three fresh processes (each draws its own placement); tools/archive/pair_pmc.py
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/pair_pmc
export TMPDIR=/tmp
mkdir -p $OUT
for i in 1 2 3; do
  timeout -s KILL 150 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum --kernel-trace \
      --output-format csv -d $OUT/run$i -o run -- python3 $R/bench.py --no-extras --no-cpu-baseline --no-variants \
      --steps 400 --warmup 8 > $OUT/run$i.log 2>&1 || exit $?
  python3 $R/tools/archive/pair_pmc.py $OUT/run$i > $OUT/summary$i.txt 2>&1 || exit $?
  cat $OUT/summary$i.txt
done
