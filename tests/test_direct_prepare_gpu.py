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


def _run(flag):
    r = subprocess.run([sys.executable, "-u", CHILD, flag], capture_output=True, text=True, timeout=100)
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
