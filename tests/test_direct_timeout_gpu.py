"""A kernarg slot that never lands: the failure mode the checked kernels guard
against (direct_tiles.hip checked_args).  Run in a child process,
since a timed-out dispatch closes the direct path for the rest of the process:
the test hook MPIR_Hip_direct_test_write_delay_us moves the write behind the
doorbell and holds it back 2.2 s, past the checked kernel's 2 s wait.  The call must fail with MPI_ERR_OTHER and
leave inoutbuf untouched -- the second resident round of workgroups, started
after the first gave up, must not combine the arguments that arrive 0.2 s
later -- and the next call must take the HIP path, bit-exact."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = os.path.join(ROOT, "tests", "progs", "direct_timeout_child.py")


@pytest.mark.gpu
def test_direct_dispatch_slot_never_lands(cuda, mpi):
    r = subprocess.run([sys.executable, "-u", CHILD], capture_output=True, text=True, timeout=100)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0 and lines, (r.returncode, r.stdout[-2000:], r.stderr[-3000:])
    out = json.loads(lines[-1])
    if out["state"] != 1:
        pytest.skip(f"direct dispatch not in nonce mode (state {out['state']})")
    assert out["warm_ok"], out
    assert out["failed_rc_class"] == mpi.MPI_ERR_OTHER, out
    assert out["untouched"], out                        # no workgroup combined anything
    assert out["failed_direct"] == 0, out
    assert out["after_ok"] and out["after_direct"] == 0, out
    assert out["failed_call_s"] < 10.0, out             # two resident rounds did not each wait 2 s+
