for r in 1 2 3; do
  for w in 5 50; do
    timeout -k 10 120 python3 -u bench.py --no-extras --no-cpu-baseline --warmup $w --steps 50 2>/dev/null | python3 -c "import json,sys; d=json.loads([l for l in sys.stdin if l.startswith('{')][-1]); print('warmup', $w, d['value'], d['ms_per_step'])" || exit 1
  done
done
