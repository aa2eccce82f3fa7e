"""`python3 bench.py --gpus N` with no WORLD_SIZE starts N ranks itself
(torch.distributed.run on 127.0.0.1) before any GPU call, so the driver's
N > 1 run measures N GPUs.  Checked here with --cpu-standin: the same
launch and max-over-ranks plumbing with gloo and a numpy step (no GPU)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, timeout=240):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout          # rank 0 alone prints the line
    return json.loads(lines[0])


def test_bench_spawns_two_ranks():
    out = _run(["--gpus", "2", "--steps", "3", "--warmup", "1", "--cpu-standin"])
    assert out["n_gpus"] == 2 and out["steps"] == 3 and out["warmup"] == 1


def test_bench_single_rank_does_not_spawn():
    out = _run(["--gpus", "1", "--steps", "2", "--warmup", "1", "--cpu-standin"])
    assert out["n_gpus"] == 1
