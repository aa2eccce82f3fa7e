#!/bin/bash
# VERDICT r3 item 2, bounded: address-translation counters on the slow and fast
# launches of the headline loop (tools/slow_kernel_pmc.sh's loop, one --pmc pass
# per counter group, each under its own kill timer), summarised by
# tools/slow_pmc_summary.py.  Pass 1: the three UTCL1 counters of the TCP block
# (<= 4 per pass); then every UTCL2 / translation counter this box lists
# (rocprofv3 -L, gpurun_out/counters_avail.txt), one per pass.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd /tmp
export TMPDIR=/tmp
mkdir -p $R/gpurun_out
AV=$R/gpurun_out/counters_avail.txt
[ -s $AV ] || timeout -s KILL 60 rocprofv3 -L > $AV 2>&1
run() {   # tag, counters...
  local tag=$1; shift
  local out=$R/gpurun_out/slow_pmc_$tag
  mkdir -p $out
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $out -o run -- \
      python3 $R/bench.py --no-cpu-baseline --no-extras --no-variants --steps 300 --warmup 20 > $out/run.log 2>&1 || return 1
  python3 $R/tools/slow_pmc_summary.py $out >> $R/gpurun_out/tail_utcl.log 2>&1
}
: > $R/gpurun_out/tail_utcl.log
run utcl1 TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_PERMISSION_MISS_sum || exit 1
n=0
for c in $(grep -oE '\b[A-Z0-9_]*(UTCL2|TRANSLATION|TLB)[A-Z0-9_]*\b' $AV | grep -v '^TCP_UTCL1' | sort -u); do
  [ $n -ge 4 ] && break
  run x$n $c || exit 1
  n=$((n + 1))
done
cat $R/gpurun_out/tail_utcl.log
