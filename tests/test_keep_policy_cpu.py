"""The result store policy's window (hip_reduce.hip keep_for): results above
MPIR_CVAR_REDUCE_LOCAL_KEEP_MIN_MB (default 16 MiB) and at most
MPIR_CVAR_REDUCE_LOCAL_KEEP_MB (default 64 MiB) are stored sc1, the rest nt
("Store policy by result size").  The setters need no GPU."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys
sys.path.insert(0, sys.argv[1])
import mpich_pip_amd as m
lib = m.load()
lo = lib.MPIR_Hip_set_keep_min_bytes(5 << 20)
hi = lib.MPIR_Hip_set_keep_bytes(7 << 20)
print(lo, hi, lib.MPIR_Hip_set_keep_min_bytes(lo), lib.MPIR_Hip_set_keep_bytes(hi))
"""


def run(env_extra):
    env = {k: v for k, v in os.environ.items() if not k.startswith("MPIR_CVAR_REDUCE_LOCAL_KEEP")}
    env.update(env_extra)
    p = subprocess.run([sys.executable, "-c", CHILD, os.path.join(ROOT, "mpich-pip_amd")], capture_output=True,
                       text=True, timeout=60, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    return [int(x) for x in p.stdout.split()]


def test_defaults_and_setters():
    assert run({}) == [16 << 20, 64 << 20, 5 << 20, 7 << 20]


def test_environment():
    assert run({"MPIR_CVAR_REDUCE_LOCAL_KEEP_MIN_MB": "0", "MPIR_CVAR_REDUCE_LOCAL_KEEP_MB": "32"})[:2] == [0, 32 << 20]
