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
    assert [r["rank"] for r in out["per_rank"]] == [0]


def test_bench_eight_ranks_report_per_rank():
    """at N > 1 the line carries every rank's own timed loop
    beside the max-over-ranks value, so a lagging GPU (or a rank off the direct
    path, in the GPU run) is visible.  VERDICT r4 item 3: the N > 1 line also
    carries (a) the collectives' per-rank times and xGMI fractions, (b) the CPU
    baseline from rank 0 with the other ranks parked, (c) the timed calls'
    median and p10 / p90.  8 gloo ranks on the CPU."""
    out = _run(["--gpus", "8", "--steps", "5", "--warmup", "1", "--cpu-standin", "--cpu-iters", "1"], timeout=400)
    assert out["n_gpus"] == 8
    pr = out["per_rank"]
    assert [r["rank"] for r in pr] == list(range(8))
    assert all(r["seconds"] > 0 and r["call_median_us"] > 0 for r in pr)
    # value's time is the slowest rank's
    assert abs(max(r["ms_per_step"] for r in pr) - out["ms_per_step"]) <= 1e-3 * out["ms_per_step"] + 1e-4
    # (a) collectives rows
    for key, kind in (("config4_allreduce_fp32_sum_256MiB", "allreduce"),
                      ("config5_reduce_scatter_block_fp16_sum_1GiB", "reduce_scatter")):
        row = out["collectives"][key]["rccl"]
        assert len(row["per_rank_ms"]) == 8 and row["ms"] == max(row["per_rank_ms"])
        factor = 2 * 7 / 8 if kind == "allreduce" else 7 / 8
        assert abs(row["frac_of_xgmi"] - row["busbw_GBps"] / (7 * 153.0)) < 1e-3
        assert abs(row["frac_of_links_in_use"] - row["busbw_GBps"] / (7 * 153.0)) < 1e-3   # N - 1 = 7 links
        assert row["busbw_GBps"] > 0 and factor > 0
    # (b) the CPU baseline beside 7 parked ranks
    cb = out["cpu_baseline"]
    assert cb["ranks_parked"] == 7 and cb["cores"] >= 1 and cb["value"] > 0 and cb["kind"] == "port"
    # (c) the timed calls one by one
    cd = out["call_distribution"]
    assert cd["calls"] == 5
    assert cd["min_us"] <= cd["p10_us"] <= cd["median_us"] <= cd["p90_us"] <= cd["max_us"]
