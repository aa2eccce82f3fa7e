"""bench.py's N > 1 path on a one-GPU box: `--gpus 2` starts two ranks itself
(torch.distributed.run), each runs the real synchronous MPI_Reduce_local loop
through the direct dispatch, and rank 0 reports the max-over-ranks timing as
one JSON line.  BENCH_TEST_SHARE_GPU=1 puts both ranks on the one GPU with a
gloo group (RCCL refuses two ranks on one GPU); the line is marked a rehearsal.
The driver's 8-GPU run takes the same path with RCCL and one GPU per rank."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_two_ranks_share_one_gpu():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["BENCH_TEST_SHARE_GPU"] = "1"
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "4",
                        "--warmup", "2", "--mib", "64", "--no-extras"],
                       env=env, cwd=ROOT, capture_output=True, text=True, timeout=100)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 4 and out["warmup"] == 2
    assert out["data"].startswith("REHEARSAL")
    assert out["value"] > 0 and out["ms_per_step"] > 0
    # each rank's own loop, its direct-dispatch state and share of direct calls
    pr = out["per_rank"]
    assert [r["rank"] for r in pr] == [0, 1], pr
    assert all(r["seconds"] > 0 and r["direct_state"] in (1, 2) and r["direct_share"] == 1.0 for r in pr), pr
    # round 5: each rank's call distribution, and the CPU baseline beside the parked rank
    assert all(r["call_median_us"] > 0 and len(r["call_p10_p90_us"]) == 2 for r in pr), pr
    assert out["call_distribution"]["calls"] == 4
    assert out["cpu_baseline"]["ranks_parked"] == 1 and out["cpu_baseline"]["value"] > 0
