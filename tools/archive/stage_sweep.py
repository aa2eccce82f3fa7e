#!/usr/bin/env python3
"""Host-operand staging sweep: MPI_Reduce_local fp32 SUM, 256 MiB operands in
host memory (pinned and pageable), per (chunk MiB, slots) setting of the
up / comp / down pipeline (hip_reduce.hip, stage_chunk()).  Each setting runs
in its own child process (the knobs are read once per process).

    python tools/stage_sweep.py            # on the GPU box
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    sys.path.insert(0, os.path.join(ROOT, "mpich-pip_amd"))
    import numpy as np
    import torch
    import mpich_pip_amd as m
    lib = m.load()
    lib.MPIX_Reduce_local_set_errhandler(m.MPI_ERRORS_RETURN)
    n = 64 << 20
    out = {}
    for kind in ("pinned", "pageable"):
        if kind == "pinned":
            a = torch.rand(n).pin_memory()
            b = torch.rand(n).pin_memory()
            pa, pb = a.data_ptr(), b.data_ptr()
            ref = (a + b).numpy()
        else:
            a = np.random.default_rng(1).random(n, dtype=np.float32)
            b = np.random.default_rng(2).random(n, dtype=np.float32)
            pa, pb = a.ctypes.data, b.ctypes.data
            ref = a + b
        assert lib.MPI_Reduce_local(pb, pa, n, m.MPI_FLOAT, m.MPI_SUM) == 0
        got = a.numpy() if kind == "pinned" else a
        ok = bool(np.array_equal(got, ref))
        k = 5
        t0 = time.perf_counter()
        for _ in range(k):
            assert lib.MPI_Reduce_local(pb, pa, n, m.MPI_FLOAT, m.MPI_SUM) == 0
        dt = (time.perf_counter() - t0) / k
        out[kind] = {"ms": round(dt * 1e3, 2), "GiBps_alg": round(3 * n * 4 / dt / 2 ** 30, 1), "exact": ok}
    print(json.dumps(out), flush=True)


def main():
    rows = []
    for chunk in (16, 32, 64):
        for slots in (2, 3, 4):
            env = dict(os.environ, MPIR_CVAR_REDUCE_LOCAL_STAGE_CHUNK_MB=str(chunk),
                       MPIR_CVAR_REDUCE_LOCAL_STAGE_SLOTS=str(slots))
            r = subprocess.run([sys.executable, __file__, "--child"], env=env, capture_output=True, text=True,
                               timeout=300)
            line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
            res = json.loads(line[-1]) if line else {"error": r.stderr[-300:]}
            rows.append({"chunk_MiB": chunk, "slots": slots, **res})
            print(json.dumps(rows[-1]), flush=True)


if __name__ == "__main__":
    child() if "--child" in sys.argv else main()
