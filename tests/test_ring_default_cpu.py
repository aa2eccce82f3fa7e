"""The library's load-time default HSA_ALLOCATE_QUEUE_DEV_MEM=1 (AQL rings in
VRAM; direct_dispatch.hip default_rings_in_vram) is applied only where it is
safe and can still act: in a single-threaded
process whose HSA runtime has not started and whose environment has no
value.  A process that already runs a second thread keeps ROCm's placement
when it loads the library by itself (setenv could move the environment under
another thread's getenv); the Python package's load() applies the default with
threads allowed (round 6: numpy / torch pools are parked threads).  A job's own
value is never overridden.  Each case is a fresh child process
(no numpy, so the interpreter is single-threaded until the case starts a
thread)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import ctypes, os, sys, threading, time
sys.path.insert(0, os.path.join({root!r}, "mpich-pip_amd"))
if sys.argv[1] == "thread":
    ev = threading.Event()
    threading.Thread(target=ev.wait, daemon=True).start()
import mpich_pip_amd as m
if sys.argv[1] == "thread_raw":       # the library alone: its constructor's rule
    threading.Thread(target=threading.Event().wait, daemon=True).start()
    ctypes.CDLL(m.LIB_PATH, mode=ctypes.RTLD_GLOBAL)
elif sys.argv[1] == "numpy_first":
    import numpy                       # OpenBLAS starts its pool threads
    m.load()
else:
    m.load()
libc = ctypes.CDLL(None)
libc.getenv.restype = ctypes.c_char_p
v = libc.getenv(b"HSA_ALLOCATE_QUEUE_DEV_MEM")
print(v.decode() if v is not None else "unset")
"""


def _run(mode, env_value=None):
    env = {k: v for k, v in os.environ.items() if k != "HSA_ALLOCATE_QUEUE_DEV_MEM"}
    if env_value is not None:
        env["HSA_ALLOCATE_QUEUE_DEV_MEM"] = env_value
    p = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT), mode], capture_output=True, text=True,
                       timeout=60, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    return p.stdout.split()[-1]


def test_single_threaded_load_defaults_rings_to_vram():
    assert _run("plain") == "1"


def test_threaded_process_is_left_alone_by_the_constructor():
    assert _run("thread_raw") == "unset"


def test_python_load_applies_it_in_a_threaded_interpreter():
    """load() asks for the default with threads allowed: an interpreter that
    imported numpy (or torch) first runs pool threads, and its queues would
    otherwise keep ROCm's host-memory rings."""
    assert _run("thread") == "1"
    assert _run("numpy_first") == "1"
    assert _run("numpy_first", "0") == "0"


def test_job_value_is_kept():
    assert _run("plain", "0") == "0"
