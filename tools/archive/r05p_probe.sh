# round 5 one-shot: the first timed call after the barrier, with the last
# warm-up step before (BENCH_WARMUP_ORDER=before) or after the barrier (default),
# alternated, in the driver's --steps 20 --warmup 5 shape; BENCH_TEST_PG=1 adds
# the N > 1 timing protocol's RCCL barrier at one rank
set -o pipefail
O=gpurun_out/r05p; mkdir -p $O
bash tools/gpu_round.sh r05p pytest smoke || exit $?
for i in 1 2 3; do
  for o in late before; do
    BENCH_WARMUP_ORDER=$o timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_ds_${o}_$i.log 2>&1 || exit $?
  done
done
for i in 1 2; do
  for o in late before; do
    BENCH_WARMUP_ORDER=$o BENCH_TEST_PG=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-extras > $O/bench_pg_${o}_$i.log 2>&1 || exit $?
  done
done
python - <<'PY'
import json,glob
for f in sorted(glob.glob('gpurun_out/r05p/bench_*.log')):
    d=[json.loads(l) for l in open(f) if l.startswith('{')][-1]
    c=d["call_distribution"]
    print(f.split('/')[-1], d["value"], round(d["value"]*2**30/8e12,4), c["median_us"], c["mean_us"], c.get("first_call_us"), c.get("idle_gap_before_first_us"), c["slow_share"])
PY
