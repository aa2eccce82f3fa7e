"""The committed bench line (profiles/r06/bench_r06zc_ds.log, measured on MI355X) against
the driver's contract and against itself: BASELINE.json's metric, the
required keys, value = algorithmic bytes x N / time, roofline.frac =
achieved / peak with achieved = 805,306,368 B / mean launch time, and the
PMC traffic it quotes equal to profiles/pmc_traffic.json, and its live
launch time in agreement with the committed rocprofv3 average."""
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LINE = os.path.join(ROOT, "profiles", "r06", "bench_r06zc_ds.log")
GIB = float(1 << 30)


@pytest.fixture(scope="module")
def line():
    with open(LINE) as f:
        rows = [json.loads(ln) for ln in f if ln.startswith("{")]
    assert rows, "no JSON line in " + LINE
    return rows[-1]


def test_contract_keys(line):
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        base = json.load(f)
    assert line["metric"] == base["metric"]
    for k in ("value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in line, k
    assert line["unit"] == "GiB/s" and line["higher_is_better"] is True and line["scaling"] == "weak"
    assert line["vs_baseline"] is None          # BASELINE.md publishes no number for this metric
    assert line["dtype"] == "f32" and "workload" in line["config"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in line["roofline"], k
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in line["cpu_baseline"], k
    assert line["cpu_baseline"]["kind"] in ("port", "reference")


def test_value_is_bytes_over_time(line):
    alg = line["config"]["algorithmic_bytes_per_call"]
    assert alg == 3 * 256 * (1 << 20)
    v = alg * line["n_gpus"] / (line["ms_per_step"] * 1e-3) / GIB
    assert v == pytest.approx(line["value"], rel=2e-3)


def test_roofline_is_self_consistent(line):
    r = line["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert r["achieved"] == pytest.approx(r["algorithmic_bytes_per_launch"] / (r["mean_launch_us"] * 1e-6) / 1e9,
                                          rel=2e-3)
    assert r["frac"] == pytest.approx(r["achieved"] / r["peak"], rel=1e-3)
    with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as f:
        pmc = json.load(f)
    # the line quotes the summary committed when it ran; a later PMC pass of the
    # same kernel differs by a few KiB of counter noise
    assert r["traffic"] == pytest.approx(pmc["hbm_bytes_per_launch"], rel=1e-4)
    assert 1.0 <= r["traffic"] / r["algorithmic_bytes_per_launch"] < 1.01


def test_live_kernel_time_agrees_with_rocprof(line):
    """bench.py times the kernel the synchronous call runs; rocprofv3's
    --kernel-trace --stats average for that kernel (profiles/r04/r04_kernel_stats.csv,
    summarised in pmc_traffic.json) must agree with it."""
    r = line["roofline"]
    with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as f:
        pmc = json.load(f)
    assert "mpir_tile_SUM_MPIR_HIP_F32" in r["kernel"] and "mpir_tile_SUM_MPIR_HIP_F32" in pmc["kernel"]
    assert r["mean_launch_us"] == pytest.approx(pmc["rocprof_avg_launch_ns"] * 1e-3, rel=0.05)


def test_per_rank_and_config5_blocks(line):
    """Round 4: every rank's own loop beside value (value's time is the slowest
    rank's), and config 5's fp16 combine with its PMC traffic."""
    pr = line["per_rank"]
    assert [r["rank"] for r in pr] == list(range(line["n_gpus"]))
    assert max(r["seconds"] for r in pr) * 1e3 / line["steps"] == pytest.approx(line["ms_per_step"], rel=2e-3)
    assert all(r["direct_state"] in (1, 2) and r["direct_share"] == 1.0 for r in pr)
    c5 = line["config5_combine"]
    for key, alg in (("two_operand", 3 * 256 * (1 << 20)), ("chain8", 9 * 128 * (1 << 20))):
        b = c5[key]
        assert b["frac"] == pytest.approx(alg / (b["kernel_us"] * 1e-6) / 8.0e12, rel=2e-3)
        assert 1.0 <= b["traffic_over_algorithmic"] < 1.01


def test_call_distribution(line):
    """Round 5 (VERDICT r4 #3c): the K timed calls one by one, and the mean call
    split into the kernel's CP-timestamped mean + a fixed remainder."""
    cd = line["call_distribution"]
    assert cd["calls"] == line["steps"]
    assert cd["min_us"] <= cd["p10_us"] <= cd["median_us"] <= cd["p90_us"] <= cd["max_us"]
    # the stamps' mean is the loop's own mean (one clock read per call inside it)
    assert cd["mean_us"] == pytest.approx(line["ms_per_step"] * 1e3, rel=5e-3)
    alg = line["config"]["algorithmic_bytes_per_call"]
    assert cd["frac_of_hbm_peak_at_median"] == pytest.approx(alg / (cd["median_us"] * 1e-6) / 8.0e12, rel=2e-3)
    d = cd["decomposition"]
    assert d["kernel_mean_us"] == pytest.approx(line["roofline"]["mean_launch_us"], abs=0.01)
    assert d["call_mean_us"] == pytest.approx(d["kernel_mean_us"] + d["fixed_us"], abs=0.02)
    assert d["kernel_us_for_call_at_0.80"] == pytest.approx(alg / (0.8 * 8.0e12) * 1e6 - d["fixed_us"], abs=0.02)
    pr = line["per_rank"][0]
    assert pr["call_median_us"] == cd["median_us"] and pr["call_p10_p90_us"] == [cd["p10_us"], cd["p90_us"]]
    # the slow calls (> median + 4 us) and the per-pair medians (4 rotating pairs)
    assert 0.0 <= cd["slow_share"] <= 1.0 and cd["slow_excess_us_per_call"] >= 0.0
    assert len(cd["median_us_by_pair"]) == 4
    assert min(cd["median_us_by_pair"]) <= cd["median_us"] <= max(cd["median_us_by_pair"]) + 1e-6
    # the first timed call and the host gap before it: the last warm-up step runs
    # after the barrier, so the gap is a device sync, not a barrier
    assert cd["min_us"] <= cd["first_call_us"] <= cd["max_us"]
    assert 0.0 < cd["idle_gap_before_first_us"] < 50.0
    assert "after the barrier" in line["value_conditions"]["warmup"]


def test_placement_recorded_and_bound(line):
    """Round 6: every rank's placement -- its CPU and NUMA
    node before and after the timed loop, its GPU's node, the nodes of the
    completion signal and error word -- and the binding the bench applied: the
    calling thread on its GPU's node (value_conditions.placement), with the
    as-launched loop beside it (sync_variants.launch_placement)."""
    for r in line["per_rank"]:
        pl = r["placement"]
        for k in ("cpu_before_loop", "cpu_after_loop", "cpu_node", "gpu_node", "signal_node", "error_word_node",
                  "allowed_cpus"):
            assert k in pl, k
        assert pl["gpu_node"] >= 0 and pl["cpu_node"] == pl["gpu_node"]      # bound near its GPU
        assert pl["ring_in_vram"] == 1          # the library's AQL ring in device memory
    vc = line["value_conditions"]["placement"]
    assert vc["mode"] == "gpu-node" and vc["gpu_node"] == line["per_rank"][0]["placement"]["gpu_node"]
    lp = line["sync_variants"]["launch_placement"]
    assert lp["value"] > 0 and lp["placement"]["gpu_node"] == vc["gpu_node"]
    assert "BENCH_BIND=none" in lp["env"]
    # since r06l the child's AQL rings are the library's (VRAM), like the main loop's:
    # the comparison is the placement's alone (DESIGN.md §(d), "Where the caller runs")
    assert lp["HSA_ALLOCATE_QUEUE_DEV_MEM_seen"] == "1"
    assert line["config"]["runtime"]["HSA_ALLOCATE_QUEUE_DEV_MEM"] == "1"


def test_build_id_in_line(line):
    """Round 6: the line names the sources its binaries came from."""
    bid = dict(kv.split("=", 1) for kv in line["config"]["build_id"].split())
    assert set(bid) == {"src", "tiles", "git"} and len(bid["src"]) == 16 and len(bid["tiles"]) == 16


def test_call_split_in_line(line):
    """Round 6: the profiled calls' split -- entry -> doorbell, the kernel (CP
    clock), doorbell -> completion seen minus the kernel (neither depends on the
    runtime's clock translation) -- and the timed region's cost outside the calls."""
    sp = line["call_distribution"]["decomposition"]["split_medians"]
    assert sp["calls"] == line["steps"]
    assert 0 < sp["host_to_doorbell_us"] < 5 and 0 < sp["doorbell_to_seen_minus_kernel_us"] < 20
    assert sp["kernel_us"] == pytest.approx(line["roofline"]["median_launch_us"], rel=0.03)
    assert 0 < line["call_distribution"]["timed_region_outside_calls_us"] < 100
