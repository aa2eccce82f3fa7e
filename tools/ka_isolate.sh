mkdir -p gpurun_out/dbg3
for i in 1 2; do
  for v in 0 40 40nt; do
    if [ $v = 40nt ]; then export MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_NOTHREAD=1; K=40; else unset MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_NOTHREAD; K=$v; fi
    MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_DEBUG=1 MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_US=$K timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > gpurun_out/dbg3/b_${v}_$i.log 2>&1 || exit 1
  done
done
