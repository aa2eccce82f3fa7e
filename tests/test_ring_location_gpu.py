"""Where the direct path's AQL ring lives (MPIR_Hip_direct_ring_location):
device memory under the library's default, also in an interpreter that
imported numpy and torch before loading it (the package's load() applies the
default there, DESIGN.md §(d) "Where the caller runs"); host memory when the
job sets HSA_ALLOCATE_QUEUE_DEV_MEM=0."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, os, sys
import numpy                      # pool threads before the library, as most scripts have
import torch
sys.path.insert(0, os.path.join({root!r}, "mpich-pip_amd"))
import mpich_pip_amd as m
lib = m.load()
lib.MPIX_Reduce_local_set_errhandler(m.MPI_ERRORS_RETURN)
torch.cuda.set_device(0)
before = lib.MPIR_Hip_direct_ring_location(0)
a = torch.ones(1 << 16, device="cuda")
b = torch.ones(1 << 16, device="cuda")
torch.cuda.synchronize()
rc = m.reduce_local(a.data_ptr(), b.data_ptr(), 1 << 16, m.MPI_FLOAT, m.MPI_SUM)
ok = bool(torch.all(b == 2).item())
print(json.dumps({"rc": rc, "ok": ok, "before": before, "after": lib.MPIR_Hip_direct_ring_location(0),
                  "direct": lib.MPIR_Hip_direct_dispatches(), "rings_default": m.RINGS_DEFAULT}))
"""


def run(env_value=None):
    env = {k: v for k, v in os.environ.items() if k != "HSA_ALLOCATE_QUEUE_DEV_MEM"}
    if env_value is not None:
        env["HSA_ALLOCATE_QUEUE_DEV_MEM"] = env_value
    p = subprocess.run([sys.executable, "-c", CHILD.replace("{root!r}", repr(ROOT))], capture_output=True, text=True, timeout=180,
                       env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    return json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])


def test_ring_in_vram_after_numpy_and_torch():
    d = run()
    assert d["rc"] == 0 and d["ok"] and d["direct"] >= 1
    assert d["rings_default"] == 1
    assert d["before"] == -1            # no queue before the first direct call
    assert d["after"] == 1


def test_job_value_zero_keeps_host_ring():
    d = run("0")
    assert d["rc"] == 0 and d["ok"] and d["direct"] >= 1
    assert d["rings_default"] == 0
    assert d["after"] == 0
