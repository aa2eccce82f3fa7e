"""The N > 1 plumbing of bench.py over RCCL, rehearsed at WORLD_SIZE 1 on one
GPU (BENCH_TEST_PG=1): launched as the driver launches it
(`torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1`),
the RCCL process group, its barriers and the max over ranks around the timed
loop, and the collectives child (bench_coll.py, configs 4-5 over RCCL at N = 1)
-- everything the 8-GPU scaling run goes through except the second rank."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_under_torchrun_with_rccl_group():
    env = dict(os.environ, BENCH_TEST_PG="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--steps", "5", "--warmup", "2", "--mib", "64", "--no-extras", "--no-variants",
           "--no-cpu-baseline", "--collectives", "on"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and d["steps"] == 5 and d["value"] > 0
    assert d["per_rank"][0]["direct_state"] in (1, 2) and d["per_rank"][0]["direct_share"] == 1.0
    assert d["per_rank"][0]["placement"]["ring_in_vram"] == 1
    coll = d.get("collectives")
    assert coll is not None and "error" not in coll, coll
