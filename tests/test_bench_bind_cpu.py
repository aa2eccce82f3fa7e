"""bench.py's placement helpers without a GPU (round 6): the calling thread is
bound to the CPUs of its GPU's NUMA node within the allowed set, left alone
when that set is empty, the GPU has no node, or BENCH_BIND=none; unbind()
restores the launch affinity (the CPU baseline deals threads over every socket)."""
import os
import sys
import threading

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


class FakeM:
    def __init__(self, node):
        self.node = node

    def placement(self, dev):
        return {"cpu": 0, "cpu_node": 0, "gpu_node": self.node, "signal_node": -1, "error_word_node": -1}


def in_thread(fn):
    """run fn on a fresh thread (affinity changes stay off the test runner's thread)"""
    out = {}

    def body():
        out["before"] = os.sched_getaffinity(0)
        out["ret"] = fn()
        out["after"] = os.sched_getaffinity(0)
        bench.unbind()
        out["restored"] = os.sched_getaffinity(0)
    t = threading.Thread(target=body)
    t.start()
    t.join()
    return out


def test_node_cpus_parses_sysfs():
    cpus = bench.node_cpus(0)
    if not os.path.exists("/sys/devices/system/node/node0/cpulist"):
        pytest.skip("no NUMA sysfs")
    assert cpus and all(isinstance(c, int) for c in cpus)
    assert bench.node_cpus(10 ** 6) == set()


def test_bind_to_gpu_node(monkeypatch):
    monkeypatch.delenv("BENCH_BIND", raising=False)
    if not bench.node_cpus(0):
        pytest.skip("no NUMA sysfs")
    out = in_thread(lambda: bench.bind_near_gpu(FakeM(0), 0))
    want = bench.node_cpus(0) & out["before"]
    assert out["ret"]["mode"] == "gpu-node" and out["ret"]["cpus"] == len(want)
    assert out["after"] == want
    assert out["restored"] == out["before"]


@pytest.mark.parametrize("node,env,mode", [(-1, None, "unbound"), (10 ** 6, None, "unbound"),
                                           (0, "none", "none (as launched)")])
def test_left_alone(monkeypatch, node, env, mode):
    if env is None:
        monkeypatch.delenv("BENCH_BIND", raising=False)
    else:
        monkeypatch.setenv("BENCH_BIND", env)
    out = in_thread(lambda: bench.bind_near_gpu(FakeM(node), 0))
    assert out["ret"]["mode"] == mode
    assert out["after"] == out["before"]
