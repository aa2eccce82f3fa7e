#!/bin/bash
# What in the keep-alive costs a back-to-back caller?  bench.py --steps 20
# --warmup 5 --no-extras with the keep-alive off (0), on (40: the first gapped
# call starts the thread, pinned off the caller's core; exit-time counters show
# arms / packets), on with the thread unpinned (40nopin), and with a thread that
# only naps 1 ms, pinned (40empty) and unpinned (40emptynopin).
mkdir -p gpurun_out/dbg3
rm -f gpurun_out/dbg3/b_*
for i in 1 2 3; do
  for v in 0 40 40nopin 40empty 40emptynopin; do
    unset MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_NOTHREAD MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_EMPTY MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_NOPIN
    K=40
    case $v in
      0) K=0 ;;
      40nopin) export MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_NOPIN=1 ;;
      40empty) export MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_EMPTY=1 ;;
      40emptynopin) export MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_EMPTY=1 MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_NOPIN=1 ;;
    esac
    MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_DEBUG=1 MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_US=$K timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > gpurun_out/dbg3/b_${v}_$i.log 2>&1 || exit 1
  done
done
