#!/usr/bin/env python3
"""Config 5's reference-order MPI_Reduce_scatter_block on one GPU through the
loopback communicator (8 virtual ranks, one thread each, device-copy
transport), with the exchange pipelined against the fold
(MPIR_CVAR_DEVICE_COLL_PIPELINE_KB = 32768, the default) and unpipelined (0),
alternated; wall time per collective call (all ranks), median over reps.  The
results of the two are compared byte for byte.

    python3 tools/archive/pipeline_ab.py [reps = 7]
"""
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "mpich-pip_amd"))


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    import mpich_pip_amd as m
    lib = m.load()
    import torch
    lib.MPIX_Reduce_local_set_errhandler(m.MPI_ERRORS_RETURN)
    torch.cuda.set_device(0)
    p = 8
    rc_ = (1 << 29) // p                         # 1 GiB of fp16 per rank
    comms = m.comm_create_loopback(p)
    send = [(torch.rand(rc_ * p, device="cuda") - 0.5).half() for _ in range(p)]
    recv = [torch.empty(rc_, dtype=torch.float16, device="cuda") for _ in range(p)]
    torch.cuda.synchronize()

    def call():
        errs = []

        def rank(r):
            rc = m.reduce_scatter_block(send[r].data_ptr(), recv[r].data_ptr(), rc_, m.MPIX_C_FLOAT16, m.MPI_SUM,
                                        comms[r], m.MPIX_HIP_ALG_REFERENCE_ORDER)
            if rc:
                errs.append(m.error_string(rc))
        ths = [threading.Thread(target=rank, args=(r,)) for r in range(p)]
        t0 = time.perf_counter()
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        dt = time.perf_counter() - t0
        assert not errs, errs
        return dt

    res = {"0": [], "32768": []}
    outs = {}
    for r in range(reps + 1):
        for kb in (["0", "32768"] if r % 2 == 0 else ["32768", "0"]):
            os.environ["MPIR_CVAR_DEVICE_COLL_PIPELINE_KB"] = kb
            dt = call()
            if r:
                res[kb].append(dt)
            if r == 0:
                outs[kb] = [x.clone() for x in recv]
    same = all(torch.equal(a.view(torch.int16), b.view(torch.int16)) for a, b in zip(outs["0"], outs["32768"]))
    for kb, v in res.items():
        v.sort()
        print(f"PIPELINE_KB={kb:>5}: median {v[len(v) // 2] * 1e3:8.3f} ms per call (min {v[0] * 1e3:.3f}, "
              f"max {v[-1] * 1e3:.3f}) over {len(v)}")
    print("outputs pipelined vs unpipelined:", "identical" if same else "DIFFER")
    for c in comms:
        m.comm_free(c)


if __name__ == "__main__":
    main()
