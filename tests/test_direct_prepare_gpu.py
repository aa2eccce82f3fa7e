"""MPIR_Hip_direct_prepare: the direct path's initialisation (HSA queue, the
device-only code object, kernarg slots, dispatch-id probe) done ahead of the
first call, as MPI_Init would.  Each case is a fresh child
process, since the path initialises once per process: with prepare, the first
synchronous call is an ordinary direct call; without, it carries the
initialisation.  Both bit-exact."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = os.path.join(ROOT, "tests", "progs", "direct_prepare_child.py")


def _run(flag, child=CHILD):
    r = subprocess.run([sys.executable, "-u", child, flag], capture_output=True, text=True, timeout=100)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0 and lines, (r.returncode, r.stdout[-2000:], r.stderr[-3000:])
    return json.loads(lines[-1])


@pytest.mark.gpu
def test_direct_prepare_moves_init_out_of_the_first_call(cuda):
    lazy, eager = _run("0"), _run("1")
    if lazy["state"] not in (1, 2):
        pytest.skip(f"direct dispatch unavailable (state {lazy['state']})")
    assert lazy["ok"] and eager["ok"], (lazy, eager)
    assert eager["prepare_state"] == eager["state"] and eager["state"] in (1, 2), eager
    assert lazy["direct"] == 1 and eager["direct"] == 1, (lazy, eager)
    # the initialisation left the first call: it now costs what any call of
    # this size does (16 MiB operands: tens of us), far below the lazy one
    assert eager["first_call_ms"] < 1.0, eager
    assert eager["first_call_ms"] < lazy["first_call_ms"], (lazy, eager)


@pytest.mark.gpu
def test_first_profiled_call_after_failed_probe(cuda):
    """the twin queue's probe fails inside the first
    profiled call (test hook).  That call reads the read-back flag after the
    probe, so it already follows the read-back protocol: every call completes
    bit-exact through the direct path, profiled or not, and the state reports
    2 (flushes read back)."""
    out = _run("-", os.path.join(ROOT, "tests", "progs", "probe_fail_child.py"))
    if out["state_before"] not in (1, 2):
        pytest.skip(f"direct dispatch unavailable (state {out['state_before']})")
    assert out["ok"], out["calls"]
    assert out["direct"] == len(out["calls"]), out
    assert out["state_after"] == 2, out
    assert all(c[4] > 0 for c in out["calls"] if c[0]), out["calls"]      # the twin queue's timestamps
