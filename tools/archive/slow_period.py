"""Are the headline loop's slow calls periodic in time?  (round 5)

    python tools/archive/slow_period.py [calls = 8000] [reps = 3]

The bench's synchronous 256 MiB fp32 SUM call, four resident pairs rotated, K
calls back to back from C with a CLOCK_MONOTONIC stamp after each
(fastcall.c reduce_local_loop).  A call is slow when it takes more than the
median + 4 us (bench.py call_stats).  Per rep: the slow share, the intervals
between the starts of consecutive slow calls (median, and the share within
+-5 % of their median), and the strongest period of the slow-call indicator
over 0.5-50 ms (a periodogram of the 0/1 series sampled per call).  A firmware
or power-management event on a fixed clock would show as one sharp period.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mpich-pip_amd")]

import torch  # noqa: E402
import mpich_pip_amd as m  # noqa: E402


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 8000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    lib = m.load()
    lib.MPIX_Reduce_local_set_errhandler(m.MPI_ERRORS_RETURN)
    torch.cuda.set_device(0)
    lib.MPIR_Hip_direct_prepare(0)
    count = 64 << 20
    g = torch.Generator(device="cuda").manual_seed(0x5EED)
    pairs = []
    for _ in range(4):
        a = torch.empty(count, device="cuda").uniform_(-1, 1, generator=g)
        b = torch.empty(count, device="cuda").uniform_(-1, 1, generator=g)
        pairs.append((b.data_ptr(), a.data_ptr(), count, m.MPI_FLOAT, m.MPI_SUM, a, b))
    torch.cuda.synchronize()
    sets = tuple(p[:5] for p in pairs)
    loop = m.fast_reduce_local_loop()
    assert loop(sets, 0, 50) == 0
    for r in range(reps):
        st = np.zeros(calls + 1, np.int64)
        assert loop(sets, 0, calls, st) == 0
        d = np.diff(st) * 1e-3                                  # us per call
        t = (st[:-1] - st[0]) * 1e-6                            # ms, start of each call
        med = float(np.median(d))
        slow = d > med + 4.0
        idx = np.nonzero(slow)[0]
        print(f"rep {r}: {calls} calls over {t[-1] + d[-1] * 1e-3:.1f} ms, median {med:.2f} us, mean {d.mean():.2f}, "
              f"slow {slow.mean():.3f} ({idx.size}), slow excess {np.sum(d[slow] - med) / calls:.3f} us/call")
        if idx.size < 3:
            continue
        gaps = np.diff(t[idx])
        # consecutive slow calls (a stretch spanning two launches) count once
        runs = gaps[gaps > 2 * med * 1e-3]
        gm = float(np.median(runs)) if runs.size else float("nan")
        near = float(np.mean(np.abs(runs - gm) <= 0.05 * gm)) if runs.size else float("nan")
        print(f"  slow-call starts: {idx.size}, separate events {runs.size + 1}, interval median {gm:.3f} ms "
              f"(p10 {np.percentile(runs, 10):.3f}, p90 {np.percentile(runs, 90):.3f}), within 5 % of it {near:.2f}")
        # periodogram of the slow indicator on the call-time grid
        x = slow.astype(float) - slow.mean()
        periods = np.linspace(0.5, 50.0, 2000)                 # ms
        pw = np.array([abs(np.sum(x * np.exp(-2j * np.pi * t / p))) ** 2 for p in periods]) / max(1, idx.size)
        top = np.argsort(pw)[::-1][:5]
        print("  strongest periods (ms, power / mean power): " +
              ", ".join(f"{periods[i]:.2f} ({pw[i] / pw.mean():.1f})" for i in top))
        # slow calls by position in the run of four pairs and by run length
        longest = cur = 0
        for s_ in slow:
            cur = cur + 1 if s_ else 0
            longest = max(longest, cur)
        print(f"  slow by pair: {[int(np.sum(slow[p::4])) for p in range(4)]}; longest run of slow calls {longest}")


if __name__ == "__main__":
    main()
