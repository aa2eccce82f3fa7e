"""CHAIN folds of 3, 5, 6 and 7 operands: one fused pass against the greedy
4 / 2 chunks the library ran before round 5 (each chunk's first operand the
running output).  Reduce_scatter_block's pairwise schedule at p ranks folds p
blocks of 1 GiB / p (fp16, config 5's sendbuf) in this order
(reduce_scatter_block_intra_pairwise.c:97-134).

    python tools/archive/chain_np2.py [rounds = 9]

Both forms through MPIX_Reduce_local_multi on one stream (the chunks are the
library's own P = 4 / P = 2 fused kernels, exactly the calls the old loop
made), HIP events over batches of 10, two operand sets alternated, forms
interleaved per round; outputs compared bit for bit.  Fraction of 8 TB/s on
the fused pass's algorithmic bytes ((p + 1) blocks) for both, so the ratio is
the time ratio.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mpich-pip_amd")]

import torch  # noqa: E402
import mpich_pip_amd as m  # noqa: E402


def greedy_chunks(n):
    """the pre-round-5 loop: chunks of P = 8 / 4 / 2 operands"""
    out, i = [], 1
    while i < n:
        left = n - i
        P = 8 if left >= 7 else (4 if left >= 3 else 2)
        out.append((i, P))
        i += P - 1
    return out


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 9
    lib = m.load()
    lib.MPIX_Reduce_local_set_errhandler(m.MPI_ERRORS_RETURN)
    torch.cuda.set_device(0)
    s = torch.cuda.Stream()
    F16, SUM, CHAIN = m.MPIX_C_FLOAT16, m.MPI_SUM, m.MPIX_ORDER_CHAIN
    g = torch.Generator(device="cuda").manual_seed(3)
    for p in (3, 5, 6, 7):
        count = ((1 << 29) // p) // 8192 * 8192          # fp16 elements per block, 1 GiB / p
        sets = [[(torch.rand(count, device="cuda", generator=g) * 2 - 1).half() for _ in range(p)] for _ in range(2)]
        outs = [torch.empty(count, device="cuda", dtype=torch.float16) for _ in range(2)]
        torch.cuda.synchronize()

        def fused(k):
            ys = [t.data_ptr() for t in sets[k % 2]]
            assert m.reduce_local_multi(ys, outs[k % 2].data_ptr(), count, F16, SUM, CHAIN, s.cuda_stream) == 0

        def greedy(k):
            ys = [t.data_ptr() for t in sets[k % 2]]
            out = outs[k % 2].data_ptr()
            acc = ys[0]
            for i, P in greedy_chunks(p):
                ops = [acc] + ys[i:i + P - 1]
                assert m.reduce_local_multi(ops, out, count, F16, SUM, CHAIN, s.cuda_stream) == 0
                acc = out

        # outputs
        with torch.cuda.stream(s):
            fused(0)
        s.synchronize()
        a = outs[0].clone()
        with torch.cuda.stream(s):
            greedy(0)
        s.synchronize()
        same = bool(torch.equal(a.view(torch.int16), outs[0].view(torch.int16)))
        times = {"fused": [], "greedy": []}
        batch = 10
        for r in range(rounds):
            for name, fn in (("fused", fused), ("greedy", greedy)) if r % 2 == 0 else (("greedy", greedy), ("fused", fused)):
                with torch.cuda.stream(s):
                    fn(0)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(s)
                    for b in range(batch):
                        fn(b + 1)
                    e1.record(s)
                s.synchronize()
                if r:
                    times[name].append(e0.elapsed_time(e1) * 1e3 / batch)
        alg = (p + 1) * count * 2
        med = {k: float(np.median(v)) for k, v in times.items()}
        chunks = " + ".join(str(P) for _, P in greedy_chunks(p))
        print(f"CHAIN{p} fp16, {p} x {count * 2 / 2**20:.1f} MiB: fused {med['fused']:.1f} us "
              f"({alg / (med['fused'] * 1e-6) / 8e12:.4f} of 8 TB/s), greedy {chunks} {med['greedy']:.1f} us "
              f"({alg / (med['greedy'] * 1e-6) / 8e12:.4f}); fused/greedy time {med['fused'] / med['greedy']:.3f}; "
              f"outputs {'identical' if same else 'DIFFER'}", flush=True)
        del sets, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
