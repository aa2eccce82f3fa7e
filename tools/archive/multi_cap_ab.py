#!/usr/bin/env python3
"""The fused 8- and 4-operand combines through the library's own entry point
(MPIX_Reduce_local_multi), one library build per process: the product (an LDS
reservation capping the workgroups per CU, reduce_kernels.hpp multi_lds_cap)
against a build with -DMPIR_MULTI_CAP_LDS=0 (no cap, as before round 4).  Alternate the two
builds with tools/multi_cap_ab.sh.

    python3 tools/multi_cap_ab.py <dir holding libmpich_reduce_local.so> [--rounds 6]

Cases: config 4's TREE8 fp32 SUM over 8 x 32 MiB blocks and config 5's CHAIN8
fp16 SUM over 8 x 128 MiB (8 ranks), TREE4 over 4 x 64 MiB and CHAIN4 over
4 x 256 MiB (4 ranks), blocks at the collective's staging stride (+4352 B),
operand sets rotated past the Infinity Cache; HIP events around batches of 20
back-to-back launches on one stream; median us per launch and fraction of
8 TB/s per round.  The first launch's output is hashed so the two builds can be
compared for identical results.
"""
import argparse
import hashlib
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpich-pip_amd"))
MIB = 1 << 20


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libdir")
    ap.add_argument("--rounds", type=int, default=6)
    args = ap.parse_args()
    import mpich_pip_amd as m
    m.load(os.path.join(os.path.abspath(args.libdir), "libmpich_reduce_local.so"))
    import torch
    torch.cuda.set_device(0)
    tag = os.path.basename(os.path.abspath(args.libdir))
    st = torch.cuda.Stream()
    g = torch.Generator(device="cuda").manual_seed(0xCA9)
    for name, p, blk_bytes, dt, tdt, order in (
            ("TREE8 fp32 8 x 32 MiB", 8, 32 * MIB, m.MPI_FLOAT, torch.float32, m.MPIX_ORDER_TREE),
            ("CHAIN8 fp16 8 x 128 MiB", 8, 128 * MIB, m.MPIX_C_FLOAT16, torch.float16, m.MPIX_ORDER_CHAIN),
            ("TREE4 fp32 4 x 64 MiB", 4, 64 * MIB, m.MPI_FLOAT, torch.float32, m.MPIX_ORDER_TREE),
            ("CHAIN4 fp16 4 x 256 MiB", 4, 256 * MIB, m.MPIX_C_FLOAT16, torch.float16, m.MPIX_ORDER_CHAIN)):
        esz = torch.tensor([], dtype=tdt).element_size()
        n = blk_bytes // esz
        stride = (blk_bytes + 4352) // esz
        nsets = max(3, (3 << 30) // ((p + 1) * blk_bytes) + 1)
        sets = [torch.empty(p * stride, device="cuda", dtype=tdt).uniform_(-1, 1, generator=g) for _ in range(nsets)]
        outs = [torch.empty(n, device="cuda", dtype=tdt) for _ in range(nsets)]
        ops = [[s.data_ptr() + j * stride * esz for j in range(p)] for s in sets]
        torch.cuda.synchronize()

        def launch(i):
            rc = m.reduce_local_multi(ops[i % nsets], outs[i % nsets].data_ptr(), n, dt, m.MPI_SUM, order,
                                      st.cuda_stream)
            assert rc == 0, m.error_string(rc)
        launch(0)
        torch.cuda.synchronize()
        digest = hashlib.sha256(outs[0].cpu().numpy().tobytes()).hexdigest()[:16]
        k, per = 1, []
        for r in range(args.rounds):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(st):
                launch(k)
                k += 1
                e0.record(st)
                for _ in range(20):
                    launch(k)
                    k += 1
                e1.record(st)
            e1.synchronize()
            per.append(e0.elapsed_time(e1) * 1e3 / 20)
        med = statistics.median(per)
        print(f"{tag} {name}: median {med:.2f} us = {(p + 1) * blk_bytes / (med * 1e-6) / 8e12:.4f} of 8 TB/s "
              f"(rounds {', '.join(f'{x:.1f}' for x in per)}) output sha256 {digest}", flush=True)
        del sets, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
