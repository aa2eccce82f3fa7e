"""8 ranks of one node doing a 64 MiB fp32 SUM host combine at the same moment
(tests/_local_ranks.py), with the host pool sized by the node's rank count
(MPI_LOCALNRANKS=8, the library's default since round 5) against round 4's
sizing (every rank min(16, usable CPUs): MPIR_CVAR_REDUCE_LOCAL_STAGE_THREADS),
next to 8 x one rank's single-thread loop (the reference's shape, opsum.c:21-76).
Cases alternate; medians of `rounds` runs.  Aggregate GiB/s counts 3 x operand
bytes per call over the span from the first start to the last end.  Two
lengths: a burst of 3 calls per rank (shorter than a CFS quota period, so a
cgroup quota does not bind yet) and a sustained run of `sustained` calls per
rank (several 100 ms periods: a quota binds).

    python tools/local_ranks_ab.py [rounds = 5] [ranks = 8] [sustained = 40]
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import _local_ranks as L  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    ranks = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    sustained = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    usable = L.usable_cpus()
    old = min(16, usable)
    cases = {
        f"{ranks} ranks, MPI_LOCALNRANKS={ranks} (round 5)": dict(nranks=ranks, localnranks=ranks),
        f"{ranks} ranks, {old} threads each (round 4 sizing)": dict(nranks=ranks, stage_threads=old),
        f"{ranks} ranks, 1 thread each (reference shape)": dict(nranks=ranks, stage_threads=1),
        "1 rank, 1 thread": dict(nranks=1, stage_threads=1),
    }
    print(f"usable CPUs {usable} (affinity {len(os.sched_getaffinity(0))}, os.cpu_count {os.cpu_count()}), "
          f"{rounds} rounds, 64 MiB fp32 SUM per call, all results bit-exact vs oracle")
    for reps in (3, sustained):
        res = {k: [] for k in cases}
        thr = {}
        for _ in range(rounds):
            for k, kw in cases.items():
                r = L.run(reps=reps, **kw)
                assert r["exact"], r
                res[k].append(r["gib_s"])
                thr[k] = r["threads"]
        print(f" {reps} calls per rank:")
        for k, v in res.items():
            print(f"  {k:46s} threads {thr[k]:4d}  aggregate GiB/s median {statistics.median(v):8.2f}  "
                  f"min {min(v):8.2f}  max {max(v):8.2f}")
        one = statistics.median(res["1 rank, 1 thread"])
        print(f"  {ranks} x the single-thread loop alone: {ranks * one:8.2f} GiB/s")


if __name__ == "__main__":
    main()
