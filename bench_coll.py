#!/usr/bin/env python3
"""Config 4 / 5 collectives on N GPUs, one process per GPU.

    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench_coll.py [--steps K]

(bench.py runs this automatically, as isolated child processes, when it is
launched with WORLD_SIZE > 1; its results land in bench.py's JSON line under
"collectives".)

Per rank: builds an RCCL communicator through the C ABI (MPIX_Hip_comm_create;
unique id exchanged over a TCPStore on 127.0.0.1), then
  1. a self-check on the real xGMI transport: reference-order
     MPIX_Allreduce_hip, MPIX_Reduce_hip, MPIX_Scan_hip, MPIX_Exscan_hip (fp32 SUM)
     and MPIX_Reduce_scatter_block_hip (fp16 SUM) on deterministic finite per-rank inputs, compared bit for bit with numpy
     evaluating the same association (recursive-halving tree per block /
     pairwise chain -- see expect_* below; numpy's fp32/fp16 adds round like
     the reference's).  The full parity suite against the oracle lives in
     tests/ (test_coll_*); this bench imports nothing from oracle/;
  2. timing, config 4: MPI_Allreduce fp32 SUM, 256 MiB (67,108,864 floats);
     config 5: MPI_Reduce_scatter_block fp16 SUM, 1 GiB sendbuf per rank
     (recvcount 2^29 / N).  Both algorithms (RCCL, reference order); K timed
     calls between a barrier and a device sync, max over ranks.
Reports bus bandwidth the RCCL-tests way: allreduce 2(N-1)/N * bytes / t,
reduce-scatter (N-1)/N * sendbytes / t, every rank's own time beside the
max-over-ranks one, and the bus bandwidth as a fraction of the xGMI roofline
(coll_row below): 7 links x 153 GB/s per GPU on a fully connected 8-GPU node
(SURVEY.md:254 and :399), and of the N - 1 links an N-rank collective can use.
"""
from __future__ import annotations

import argparse
import ctypes
import datetime
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mpich-pip_amd"))
sys.path.insert(0, ROOT)


XGMI_LINK_GBPS = 153.0        # one xGMI link, GB/s per direction (SURVEY.md:254)
XGMI_LINKS = 7                # per GPU, fully connected 8-GPU node


def coll_row(per_rank_s: list, world: int, nbytes: int, kind: str) -> dict:
    """One timed collective: per-rank seconds per call -> its report row.
    kind "allreduce": busbw = 2(N-1)/N * bytes / t; "reduce_scatter": (N-1)/N
    * sendbytes / t (RCCL-tests).  t is the slowest rank's.  frac_of_xgmi =
    busbw / (7 x 153 GB/s), the per-GPU xGMI peak of the 8-GPU node;
    frac_of_links_in_use = busbw / ((N-1) x 153 GB/s), the links an N-rank
    collective can drive (one to each peer)."""
    t = max(per_rank_s)
    factor = 2 * (world - 1) / world if kind == "allreduce" else (world - 1) / world
    bus = factor * nbytes / t / 1e9
    row = {"ms": round(t * 1e3, 3), "per_rank_ms": [round(x * 1e3, 3) for x in per_rank_s],
           "busbw_GBps": round(bus, 1),
           "frac_of_xgmi": round(bus / (XGMI_LINKS * XGMI_LINK_GBPS), 4),
           "frac_of_links_in_use": round(bus / (max(1, world - 1) * XGMI_LINK_GBPS), 4) if world > 1 else None,
           "xgmi_peak": f"{XGMI_LINKS} links x {XGMI_LINK_GBPS:g} GB/s per GPU (SURVEY.md:254)"}
    if kind == "allreduce":
        row["algbw_GBps"] = round(nbytes / t / 1e9, 1)
    return row


def _bitrev(n: int, bits: int) -> int:
    return int(format(n, f"0{bits}b")[::-1], 2) if bits else 0


def expect_allreduce(xs):
    """Reference-order allreduce for a power-of-two rank count: block b, owned
    by newrank n = bitrev(b), is ((y0+y1)+(y2+y3))+... with y_j = x_{n^j}
    (reduce_intra_reduce_scatter_gather.c:186-249)."""
    import numpy as np
    p, count = len(xs), len(xs[0])
    bits = p.bit_length() - 1
    cnts = [count // p + (1 if i < count % p else 0) for i in range(p)]
    disps = [sum(cnts[:i]) for i in range(p)]
    out = np.empty_like(xs[0])
    for n in range(p):
        b = _bitrev(n, bits)
        sl = slice(disps[b], disps[b] + cnts[b])
        v = [xs[n ^ j][sl].copy() for j in range(p)]
        step = 1
        while step < p:
            for j in range(0, p, 2 * step):
                v[j] = v[j] + v[j + step]
            step *= 2
        out[sl] = v[0]
    return out


def expect_reduce_scatter_block(xs, rank: int, rcount: int):
    """Pairwise chain ((x_r + x_{r-1}) + x_{r-2}) + ... on block r
    (reduce_scatter_block_intra_pairwise.c:97-134)."""
    p = len(xs)
    sl = slice(rank * rcount, (rank + 1) * rcount)
    acc = xs[rank][sl].copy()
    for i in range(1, p):
        acc = acc + xs[(rank - i) % p][sl]
    return acc


def _tree(vs):
    """((v0+v1)+(v2+v3))+... (left operand first; len(vs) a power of two)."""
    v = [x.copy() for x in vs]
    step = 1
    while step < len(v):
        for j in range(0, len(v), 2 * step):
            v[j] = v[j] + v[j + step]
        step *= 2
    return v[0]


def expect_scan(xs, rank: int, exclusive: bool = False):
    """Recursive-doubling scan order (scan_intra_recursive_doubling.c:94-147,
    exscan_intra_recursive_doubling.c:105-170): rank r's result is the chain
    x_r + T(r^m_1) + T(r^m_2) + ... over the set bits m of r (increasing),
    T(d) the tree over x_{d^j}, j < m (exscan: without x_r; None at rank 0)."""
    parts, m = [], 1
    while m <= rank:
        if rank & m:
            d = rank ^ m
            parts.append(_tree([xs[d ^ j] for j in range(m)]))
        m <<= 1
    chain = parts if exclusive else [xs[rank]] + parts
    if not chain:
        return None
    acc = chain[0].copy()
    for x in chain[1:]:
        acc = acc + x
    return acc


# the self-check's sizes (main, part 1)
SELF_N = (1 << 16) + 3          # fp32 allreduce / reduce / scan / exscan
SELF_RCOUNT = (1 << 17) + 3     # fp16 reduce_scatter_block recvcount: pairwise at every N >= 2
INT_N = 4099                    # int32 allreduce over RCCL


def call_plan(world: int, ar_mib: int = 256, rs_mib: int = 1024, warmup: int = 3, steps: int = 10) -> list:
    """Every collective main() issues on each rank, in its order, as
    (call, count, type, op, algorithm[, root]) -- what a rank of this bench
    asks of RCCL through the C ABI.  tests/test_rccl_sequence_cpu.py replays it
    against a recording librccl stand-in at N = 2..8 and checks that the ranks'
    RCCL call sequences match one another (no GPU)."""
    plan = [("allreduce", SELF_N, "f32", "sum", "ref"),
            ("reduce_scatter_block", SELF_RCOUNT, "f16", "sum", "ref"),
            ("reduce", SELF_N, "f32", "sum", "ref", world - 1),
            ("scan", SELF_N, "f32", "sum", "ref"), ("exscan", SELF_N, "f32", "sum", "ref"),
            ("allreduce", SELF_N, "f32", "sum", "rccl"),
            ("reduce_scatter_block", SELF_RCOUNT, "f16", "sum", "rccl"),
            ("allreduce", INT_N, "i32", "sum", "rccl"),
            ("allreduce", 8, "f64", "min", "rccl")]             # the flags
    barrier = ("allreduce", 1, "f64", "sum", "rccl")
    per_rank = ("allreduce", world, "f64", "sum", "rccl")
    count = ar_mib * (1 << 20) // 4
    rc_ = rs_mib * (1 << 20) // 2 // world
    for call, n, ty in (("allreduce", count, "f32"), ("reduce_scatter_block", rc_, "f16")):
        for alg in ("rccl", "ref"):
            plan += [(call, n, ty, "sum", alg)] * warmup + [barrier] + [(call, n, ty, "sum", alg)] * steps + [per_rank]
    return plan


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--ar-mib", type=int, default=256)
    ap.add_argument("--rs-mib", type=int, default=1024)
    ap.add_argument("--store-port", type=int, default=int(os.environ.get("COLL_STORE_PORT", "29611")))
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist
    import mpich_pip_amd as m

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # local % count: bench.py's one-GPU rehearsal (BENCH_TEST_SHARE_GPU) puts
    # every rank on the one card, where RCCL refuses the communicator and the
    # error is what bench.py reports
    torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
    lib = m.load()
    lib.MPIX_Reduce_local_set_errhandler(m.MPI_ERRORS_RETURN)

    store = dist.TCPStore("127.0.0.1", args.store_port, world, rank == 0,
                          timeout=datetime.timedelta(seconds=120))
    if rank == 0:
        uid = ctypes.create_string_buffer(128)
        assert lib.MPIX_Hip_comm_get_unique_id(uid) == 0
        store.set("mpix_uid", uid.raw)
    raw = store.get("mpix_uid")
    comm = ctypes.c_void_p()
    rc = lib.MPIX_Hip_comm_create(ctypes.c_char_p(raw), world, rank, ctypes.byref(comm))
    if rc:
        raise RuntimeError(m.error_string(rc))
    C = comm.value
    F32, F16, SUM, MAX = m.MPI_FLOAT, m.MPIX_C_FLOAT16, m.MPI_SUM, m.MPI_MAX
    REF, RCCL = m.MPIX_HIP_ALG_REFERENCE_ORDER, m.MPIX_HIP_ALG_RCCL

    scratch = torch.zeros(1, dtype=torch.float64, device="cuda")

    def barrier():
        torch.cuda.synchronize()
        assert m.allreduce(m.MPI_IN_PLACE, scratch.data_ptr(), 1, m.MPI_DOUBLE, SUM, C, RCCL) == 0

    def per_rank(x):
        """every rank's x, in rank order (a SUM of one-hot rows)"""
        t = torch.zeros(world, dtype=torch.float64, device="cuda")
        t[rank] = x
        assert m.allreduce(m.MPI_IN_PLACE, t.data_ptr(), world, m.MPI_DOUBLE, SUM, C, RCCL) == 0
        return t.cpu().tolist()

    out = {"n_ranks": world}

    # ---- 1. self-check over the real transport (small, deterministic, finite inputs)
    pof2 = world & (world - 1) == 0
    n = SELF_N
    xs = [np.random.default_rng(77 + r).uniform(-1, 1, n).astype(np.float32) for r in range(world)]
    send = torch.from_numpy(xs[rank].copy()).cuda()
    recv = torch.zeros_like(send)
    torch.cuda.synchronize()
    assert m.allreduce(send.data_ptr(), recv.data_ptr(), n, F32, SUM, C, REF) == 0
    ok_ar = bool(np.array_equal(recv.cpu().numpy().view(np.uint32), expect_allreduce(xs).view(np.uint32))) \
        if pof2 else True
    # large enough that MPICH takes the pairwise algorithm at every N >= 2
    # (p * recvcount * 2 B >= 524288, reduce_scatter_block.c:136-141)
    rcount = SELF_RCOUNT
    hs = [np.random.default_rng(91 + r).uniform(-4, 4, rcount * world).astype(np.float16) for r in range(world)]
    hsend = torch.from_numpy(hs[rank].copy()).cuda()
    hrecv = torch.zeros(rcount, dtype=torch.float16, device="cuda")
    torch.cuda.synchronize()
    assert m.reduce_scatter_block(hsend.data_ptr(), hrecv.data_ptr(), rcount, F16, SUM, C, REF) == 0
    ok_rs = bool(np.array_equal(hrecv.cpu().numpy().view(np.uint16),
                                expect_reduce_scatter_block(hs, rank, rcount).view(np.uint16)))
    # MPI_Reduce to the last rank: the long path's block values are the allreduce's
    root = world - 1
    rrecv = torch.zeros_like(send)
    torch.cuda.synchronize()
    assert m.reduce(send.data_ptr(), rrecv.data_ptr() if rank == root else 0, n, F32, SUM, root, C, REF) == 0
    ok_rd = bool(np.array_equal(rrecv.cpu().numpy().view(np.uint32), expect_allreduce(xs).view(np.uint32))) \
        if (pof2 and rank == root) else True
    # MPI_Scan / MPI_Exscan (recursive-doubling order)
    srecv = torch.zeros_like(send)
    erecv = torch.zeros_like(send)
    torch.cuda.synchronize()
    assert m.scan(send.data_ptr(), srecv.data_ptr(), n, F32, SUM, C, REF) == 0
    assert m.exscan(send.data_ptr(), erecv.data_ptr(), n, F32, SUM, C, REF) == 0
    ok_sc = bool(np.array_equal(srecv.cpu().numpy().view(np.uint32), expect_scan(xs, rank).view(np.uint32)))
    ex = expect_scan(xs, rank, exclusive=True)
    ok_ex = True if ex is None else bool(np.array_equal(erecv.cpu().numpy().view(np.uint32), ex.view(np.uint32)))
    # RCCL mode (tests/test_coll_rccl_gpu.py's checks at this world size): RCCL
    # reorders the sum, so fp32/fp16 against the reference association within
    # |got - ref| <= gamma_{p-1} * sum|x_i|; int32 exact
    rrecv = torch.zeros_like(send)
    torch.cuda.synchronize()
    assert m.allreduce(send.data_ptr(), rrecv.data_ptr(), n, F32, SUM, C, RCCL) == 0
    ref64 = expect_allreduce(xs).astype(np.float64) if pof2 else np.sum([x.astype(np.float64) for x in xs], axis=0)
    mag = np.sum([np.abs(x.astype(np.float64)) for x in xs], axis=0)
    g32 = (world - 1) * 2.0 ** -24 / (1 - (world - 1) * 2.0 ** -24)
    ok_rccl_ar = bool(np.all(np.abs(rrecv.cpu().numpy().astype(np.float64) - ref64) <= g32 * mag + 1e-45))
    hr2 = torch.zeros(rcount, dtype=torch.float16, device="cuda")
    torch.cuda.synchronize()
    assert m.reduce_scatter_block(hsend.data_ptr(), hr2.data_ptr(), rcount, F16, SUM, C, RCCL) == 0
    sl = slice(rank * rcount, (rank + 1) * rcount)
    href = expect_reduce_scatter_block(hs, rank, rcount).astype(np.float64)
    hmag = np.sum([np.abs(h[sl].astype(np.float64)) for h in hs], axis=0)
    g16 = (world - 1) * 2.0 ** -11 / (1 - (world - 1) * 2.0 ** -11)
    # the reference chain rounds to fp16 at every step too: allow both chains' error
    ok_rccl_rs = bool(np.all(np.abs(hr2.cpu().numpy().astype(np.float64) - href) <= 2 * g16 * hmag + 2.0 ** -24))
    ints = [np.random.default_rng(300 + r).integers(-2 ** 31, 2 ** 31, INT_N, dtype=np.int64).astype(np.int32)
            for r in range(world)]
    isend = torch.from_numpy(ints[rank].copy()).cuda()
    irecv = torch.zeros_like(isend)
    torch.cuda.synchronize()
    assert m.allreduce(isend.data_ptr(), irecv.data_ptr(), INT_N, m.MPI_INT, SUM, C, RCCL) == 0
    iwant = np.sum([x.astype(np.int64) for x in ints], axis=0).astype(np.uint32).view(np.int32)
    ok_rccl_int = bool(np.array_equal(irecv.cpu().numpy(), iwant))
    flags = torch.tensor([float(ok_ar), float(ok_rs), float(ok_rd), float(ok_sc), float(ok_ex), float(ok_rccl_ar),
                          float(ok_rccl_rs), float(ok_rccl_int)], dtype=torch.float64, device="cuda")
    assert m.allreduce(m.MPI_IN_PLACE, flags.data_ptr(), 8, m.MPI_DOUBLE, m.MPI_MIN, C, RCCL) == 0
    out["parity_reference_order"] = {
        "allreduce_fp32_sum_bitexact": bool(flags[0].item() == 1.0) if pof2 else "not checked (non-pof2 N)",
        "reduce_scatter_block_fp16_sum_bitexact": bool(flags[1].item() == 1.0),
        "reduce_fp32_sum_bitexact": bool(flags[2].item() == 1.0) if pof2 else "not checked (non-pof2 N)",
        "scan_fp32_sum_bitexact": bool(flags[3].item() == 1.0),
        "exscan_fp32_sum_bitexact": bool(flags[4].item() == 1.0),
        "checker": "numpy, same association (full oracle parity: tests/test_coll_*)"}
    out["parity_rccl"] = {
        "allreduce_fp32_sum_within_gamma": bool(flags[5].item() == 1.0),
        "reduce_scatter_block_fp16_sum_within_gamma": bool(flags[6].item() == 1.0),
        "allreduce_int32_sum_exact": bool(flags[7].item() == 1.0),
        "tolerance": "|got - ref| <= gamma_{p-1} * sum|x_i|, gamma_k = k u / (1 - k u) (SURVEY.md §8c)"}

    # ---- 2. timing
    def timed(fn):
        for _ in range(args.warmup):
            fn()
        barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            fn()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        return [x / args.steps for x in per_rank(dt)]

    count = args.ar_mib * (1 << 20) // 4
    a = torch.rand(count, device="cuda") * 2 - 1
    b = torch.empty_like(a)
    def ar(alg):
        rc = m.allreduce(a.data_ptr(), b.data_ptr(), count, F32, SUM, C, alg, 0)
        if rc:
            raise RuntimeError(m.error_string(rc))

    def rs(alg):
        rc = m.reduce_scatter_block(hs_.data_ptr(), hr_.data_ptr(), rc_, F16, SUM, C, alg, 0)
        if rc:
            raise RuntimeError(m.error_string(rc))

    res = {}
    for name, alg in (("rccl", RCCL), ("reference_order", REF)):
        res[name] = coll_row(timed(lambda: ar(alg)), world, count * 4, "allreduce")
    out["config4_allreduce_fp32_sum_256MiB"] = res
    del a, b
    torch.cuda.empty_cache()

    total = args.rs_mib * (1 << 20) // 2
    rc_ = total // world
    hs_ = (torch.rand(rc_ * world, device="cuda") - 0.5).half()
    hr_ = torch.empty(rc_, dtype=torch.float16, device="cuda")
    res = {}
    for name, alg in (("rccl", RCCL), ("reference_order", REF)):
        res[name] = coll_row(timed(lambda: rs(alg)), world, rc_ * world * 2, "reduce_scatter")
    out["config5_reduce_scatter_block_fp16_sum_1GiB"] = res
    m.comm_free(C)
    if rank == 0:
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
