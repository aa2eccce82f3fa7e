"""MPIR_CVAR_REDUCE_LOCAL_BIND=gpu-node (opt-in): the calling thread binds
itself to its GPU's NUMA node at its first synchronous device call, within the
CPUs it could already use; unset, the library leaves the caller's affinity
alone (DESIGN.md §(d), "Where the caller runs")."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = os.path.join(ROOT, "tests", "progs", "bind_child.py")


def node_cpus(node):
    out = set()
    for part in open(f"/sys/devices/system/node/node{node}/cpulist").read().strip().split(","):
        a, _, b = part.partition("-")
        out.update(range(int(a), int(b or a) + 1))
    return out


def run(env_extra):
    env = dict(os.environ)
    env.pop("MPIR_CVAR_REDUCE_LOCAL_BIND", None)
    env.pop("MPIR_CVAR_REDUCE_LOCAL_SIGNAL_NODE", None)
    env.update(env_extra)
    p = subprocess.run([sys.executable, CHILD], capture_output=True, text=True, timeout=180, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    return json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])


def test_bind_gpu_node():
    d = run({"MPIR_CVAR_REDUCE_LOCAL_BIND": "gpu-node"})
    assert d["rc"] == 0 and d["ok"] and d["direct"] >= 1
    g = d["placement"]["gpu_node"]
    if g < 0:
        pytest.skip("the GPU reports no NUMA node")
    want = node_cpus(g) & set(d["before"])
    if not want:
        assert d["after"] == d["before"]            # nothing allowed there: left alone
    else:
        assert set(d["after"]) == want
        assert d["placement"]["cpu_node"] == g


def test_unset_leaves_affinity_alone():
    d = run({})
    assert d["rc"] == 0 and d["ok"]
    assert d["after"] == d["before"]


def test_signal_node_knob():
    """MPIR_CVAR_REDUCE_LOCAL_SIGNAL_NODE=0 (the placement A/B's knob): the
    unprofiled calls complete on a signal the library allocated on node 0,
    and results are unchanged."""
    d = run({"MPIR_CVAR_REDUCE_LOCAL_SIGNAL_NODE": "0", "BIND_CHILD_CALLS": "50"})
    assert d["rc"] == 0 and d["ok"] and d["direct"] >= 50
    assert d["placement"]["signal_node"] in (0, -1)     # -1: the page's node not reported


def test_signal_node_knob_missing_node_falls_back():
    d = run({"MPIR_CVAR_REDUCE_LOCAL_SIGNAL_NODE": "99", "BIND_CHILD_CALLS": "20"})
    assert d["rc"] == 0 and d["ok"] and d["direct"] >= 20
