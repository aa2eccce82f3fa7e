"""The direct AQL dispatch under a tool that intercepts its queue.

rocprofv3 --kernel-trace re-submits the library's packets to a hardware queue
of its own, so the dispatch id the CP hands each kernel is not the index the
host wrote the packet at, and the checked kernels' nonce (the index + 1,
direct_tiles.hip checked_args) never matches: before the queue probe, every
kernarg-cache miss under the profiler waited out the 10 ms net and failed the
call ("direct dispatch: queue error").  direct_dispatch.hip probe_ids now
detects the mismatch when the queue is created and switches the device to
read-back flushes with unchecked kernels (MPIR_Hip_direct_state 2).  Run as a
child under rocprofv3: fresh arguments on every call and repeated ones, each
result bit-exact against torch's fp32 add, every call on the direct path."""
import json
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = os.path.join(ROOT, "tests", "progs", "direct_intercept_child.py")


@pytest.mark.gpu
def test_direct_dispatch_under_rocprofv3(tmp_path, cuda):
    rocprof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(rocprof):
        pytest.skip("rocprofv3 not installed")
    env = dict(os.environ, TMPDIR="/tmp")
    cmd = [rocprof, "--kernel-trace", "--output-format", "csv", "-d", str(tmp_path / "trace"), "-o", "run",
           "--", sys.executable, "-u", CHILD]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=env, cwd="/tmp")
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0 and lines, (r.returncode, r.stdout[-2000:], r.stderr[-3000:])
    out = json.loads(lines[-1])
    assert out["bad"] == 0, out
    assert out["direct"] == out["calls"], out          # none fell back to the HIP path
    # the probe saw the interception (state 1 would mean the ids matched the
    # indices, and the nonce protocol then stays correct as well)
    assert out["state"] == 2, out
