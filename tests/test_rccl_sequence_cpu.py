"""The device collectives' RCCL call sequences at N = 2..8 ranks, without a GPU
(VERDICT r5 item 3).

csrc/host/coll_hip.c -- the product source, compiled unchanged -- runs one
process per rank against a recording librccl stand-in (tests/progs/rccl_stub.c,
loaded through MPIR_TEST_RCCL_LIBRARY) with its HIP calls and kernels replaced
by stand-ins that move no data (tests/progs/coll_trace.c), so configs 4 and 5
run at their full counts in no memory.  Checked, per plan and rank count:
  * every rank's grouped ncclSend / ncclRecv sit inside balanced
    ncclGroupStart / ncclGroupEnd brackets;
  * for every ordered pair of ranks (a, b), the k-th send a -> b and the k-th
    recv at b from a carry equal bytes and type and fall in the same group epoch
    (the i-th group on each rank): no rank waits on a transfer its peer posts in
    a later group;
  * ncclAllReduce / ncclReduceScatter / ncclReduce are issued by every rank in
    the same order, with the same count, type, op and root, after the same number
    of groups;
  * config 4 (MPI_Allreduce fp32 SUM, 256 MiB): ncclAllReduce count 67,108,864;
    config 5 (MPI_Reduce_scatter_block fp16 SUM, 1 GiB per rank): ncclReduceScatter
    recvcount 2^29 / N (67,108,864 at N = 8); the reference-order schedules move
    the bytes their reference schedules move;
  * bench_coll.py's own sequence of calls (bench_coll.call_plan) at N = 2 and 8.
A checker that missed a changed sequence would be worthless: the last test
alters one rank's log in several ways and expects each to be caught.

Reference schedules: reduce_scatter_block_intra_pairwise.c:97-134,
allreduce_intra_reduce_scatter_allgather.c:170-260 / reduce_intra_reduce_scatter_gather.c
(coll_hip.c's reference order); RCCL mode: MPIR_Allreduce -> ncclAllReduce.
"""
import collections
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "mpich-pip_amd", "csrc", "host")
ROCM_INC = "/opt/rocm/include"
NCCL_F16, NCCL_F32, NCCL_SUM = 6, 7, 0       # rccl.h ncclDataType_t / ncclRedOp_t

CONFIG4 = [("allreduce", 67108864, "f32", "sum", "rccl"), ("allreduce", 67108864, "f32", "sum", "ref")]


def config5(n):
    rc = (1 << 29) // n          # 1 GiB of fp16 per rank
    return [("reduce_scatter_block", rc, "f16", "sum", "rccl"), ("reduce_scatter_block", rc, "f16", "sum", "ref")]


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    if not os.path.exists(os.path.join(ROCM_INC, "rccl", "rccl.h")):
        pytest.skip("needs the ROCm headers (rccl.h, hip_runtime_api.h) to compile against")
    d = tmp_path_factory.mktemp("rccl_trace")
    stub = str(d / "librccl_stub.so")
    exe = str(d / "coll_trace")
    subprocess.run(["gcc", "-shared", "-fPIC", "-O1", "-Wall", "-I" + ROCM_INC, "-D__HIP_PLATFORM_AMD__", "-o", stub,
                    os.path.join(ROOT, "tests", "progs", "rccl_stub.c")], check=True)
    subprocess.run(["gcc", "-O1", "-std=gnu99", "-Wall", "-I" + os.path.join(ROOT, "include"), "-I" + HOST,
                    "-I" + ROCM_INC, "-D__HIP_PLATFORM_AMD__", "-o", exe,
                    os.path.join(ROOT, "tests", "progs", "coll_trace.c")] +
                   [os.path.join(HOST, f) for f in ("coll_hip.c", "op_kernels.c", "errutil.c", "reduce_local.c",
                                                   "op_objects.c")] + ["-ldl", "-lpthread"], check=True)
    return d, stub, exe


def run_plan(harness, n, plan, tag):
    d, stub, exe = harness
    text = "".join(" ".join(str(x) for x in step) + "\n" for step in plan)
    log = str(d / f"{tag}_n{n}")
    env = dict(os.environ, MPIR_TEST_RCCL_LIBRARY=stub, RCCL_STUB_LOG=log)
    procs = [subprocess.Popen([exe, str(r), str(n)], stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True, env=env) for r in range(n)]
    for r, p in enumerate(procs):
        out, err = p.communicate(text, timeout=120)
        assert p.returncode == 0, f"rank {r}: exit {p.returncode}: {err}"
    logs = []
    for r in range(n):
        with open(f"{log}.{r}") as f:
            logs.append([ln.split() for ln in f.read().splitlines()])
    return logs


class Mismatch(AssertionError):
    pass


def check(logs):
    """The cross-rank rules of the module docstring; returns, per rank, the
    collectives issued and the bytes received per call of the plan."""
    n = len(logs)
    per_rank = []
    for r, log in enumerate(logs):
        if log[0] != ["init", str(r), str(n)] or log[-1] != ["destroy"]:
            raise Mismatch(f"rank {r}: log not framed by init / destroy")
        depth, groups, call = 0, 0, -1
        sends, recvs, colls = collections.defaultdict(list), collections.defaultdict(list), []
        recv_bytes = collections.Counter()
        for ev in log[1:-1]:
            kind = ev[0]
            if kind == "group_start":
                if depth:
                    raise Mismatch(f"rank {r}: nested group")
                depth = 1
            elif kind == "group_end":
                if not depth:
                    raise Mismatch(f"rank {r}: group_end without group_start")
                depth = 0
                groups += 1
            elif kind in ("send", "recv"):
                if not depth:
                    raise Mismatch(f"rank {r}: {kind} outside a group")
                nbytes, ty, peer = int(ev[1]), int(ev[2]), int(ev[3])
                (sends if kind == "send" else recvs)[peer].append((nbytes, ty, groups))
                if kind == "recv":
                    recv_bytes[call] += nbytes
            elif kind in ("allreduce", "reduce_scatter", "reduce"):
                if depth:
                    raise Mismatch(f"rank {r}: collective inside a group")
                colls.append((kind, tuple(ev[1:]), groups))
            elif kind == "note" and ev[1] == "call":
                call = int(ev[2])
        if depth:
            raise Mismatch(f"rank {r}: unterminated group")
        per_rank.append({"groups": groups, "sends": sends, "recvs": recvs, "colls": colls, "recv_bytes": recv_bytes})
    # the same number of groups and the same collectives, at the same places
    for r in range(1, n):
        if per_rank[r]["groups"] != per_rank[0]["groups"]:
            raise Mismatch(f"rank {r}: {per_rank[r]['groups']} groups against {per_rank[0]['groups']} on rank 0")
        if per_rank[r]["colls"] != per_rank[0]["colls"]:
            raise Mismatch(f"rank {r}: collectives differ from rank 0's")
    # every send matched by its peer's recv: bytes, type, group epoch
    for a in range(n):
        for b in range(n):
            s, v = per_rank[a]["sends"].get(b, []), per_rank[b]["recvs"].get(a, [])
            if s != v:
                raise Mismatch(f"sends {a}->{b} {s[:4]}... against recvs at {b} from {a} {v[:4]}...")
    return per_rank


@pytest.mark.parametrize("n", [2, 3, 4, 5, 6, 7, 8])
def test_config4_allreduce_sequences(harness, n):
    res = check(run_plan(harness, n, CONFIG4, "c4"))
    # RCCL mode: one ncclAllReduce of the whole vector
    kind, args, _ = res[0]["colls"][0]
    assert kind == "allreduce" and args == ("67108864", str(NCCL_F32), str(NCCL_SUM))
    assert len(res[0]["colls"]) == 1          # the reference order uses send / recv only
    # reference order: the reduce-scatter moves the pof2 blocks, the allgather brings
    # back the rest -- every rank ends holding the whole 256 MiB
    pof2 = 1 << (n.bit_length() - 1)
    for r, pr in enumerate(res):
        got = pr["recv_bytes"][1]
        assert got > 0
        if n == pof2:
            # (p - 1) blocks in the reduce-scatter + (p - 1) in the allgather
            assert got == 2 * (n - 1) * (256 << 20) // n, (r, got)


@pytest.mark.parametrize("n", [2, 3, 4, 5, 6, 7, 8])
def test_config5_reduce_scatter_block_sequences(harness, n):
    res = check(run_plan(harness, n, config5(n), "c5"))
    kind, args, _ = res[0]["colls"][0]
    assert kind == "reduce_scatter" and args == (str((1 << 29) // n), str(NCCL_F16), str(NCCL_SUM))
    if n == 8:
        assert args[0] == "67108864"
    # the pairwise schedule: block r from every other rank, one exchange
    for r, pr in enumerate(res):
        assert pr["recv_bytes"][1] == (n - 1) * ((1 << 29) // n) * 2, r
        assert sorted(pr["recvs"]) == sorted(set(range(n)) - {r})


@pytest.mark.parametrize("n", [2, 8])
def test_bench_coll_plan_sequences(harness, n):
    sys.path.insert(0, ROOT)
    import bench_coll
    plan = bench_coll.call_plan(n, warmup=1, steps=2)
    res = check(run_plan(harness, n, plan, "bench"))
    # its RCCL collectives: the self-check's three (+ the flags), then per
    # algorithm pair of each config a barrier and a per-rank gather around the
    # timed calls (3 RCCL calls per RCCL-mode config, 2 per reference-order one)
    kinds = [c[0] for c in res[0]["colls"]]
    assert kinds.count("reduce_scatter") == 1 + 3     # self-check + config 5 rccl x (1 warm-up + 2 timed)
    counts = {c[1][0] for c in res[0]["colls"] if c[0] == "allreduce"}
    assert "67108864" in counts and str(bench_coll.INT_N) in counts


def test_checker_catches_changed_sequences(harness):
    n = 4
    good = run_plan(harness, n, CONFIG4 + config5(n), "mut")
    check(good)

    def mutated(fn):
        logs = [list(map(list, log)) for log in good]
        fn(logs)
        with pytest.raises(Mismatch):
            check(logs)
    # one recv's byte count
    def bytes_(logs):
        i = next(i for i, ev in enumerate(logs[2]) if ev[0] == "recv")
        logs[2][i][1] = str(int(logs[2][i][1]) + 2)
    mutated(bytes_)
    # a send dropped
    def drop(logs):
        i = next(i for i, ev in enumerate(logs[1]) if ev[0] == "send")
        del logs[1][i]
    mutated(drop)
    # a send moved into the next group
    def move(logs):
        i = next(i for i, ev in enumerate(logs[3]) if ev[0] == "send")
        ev = logs[3].pop(i)
        j = next(j for j in range(i, len(logs[3])) if logs[3][j][0] == "group_start")
        logs[3].insert(j + 1, ev)
    mutated(move)
    # a collective's count
    def count(logs):
        i = next(i for i, ev in enumerate(logs[0]) if ev[0] == "reduce_scatter")
        logs[0][i][1] = "1"
    mutated(count)
    # a collective issued inside a group
    def inside(logs):
        i = next(i for i, ev in enumerate(logs[1]) if ev[0] == "allreduce")
        ev = logs[1].pop(i)
        j = next(j for j, e in enumerate(logs[1]) if e[0] == "group_start")
        logs[1].insert(j + 1, ev)
    mutated(inside)


@pytest.mark.parametrize("kb,chunks", [(0, 1), (32768, 4), (65536, 2)])
def test_pipelined_reference_order_chunks(harness, kb, chunks, monkeypatch):
    """Config 5's reference order at N = 8 (8 x 128 MiB blocks): with
    MPIR_CVAR_DEVICE_COLL_PIPELINE_KB = chunk, the exchange runs in
    128 MiB / chunk groups and the CHAIN8 fold in as many chunk folds, each
    chunk's fold after its group (coll_hip.c exchange_fold_pipelined); 0 turns
    the pipeline off.  The cross-rank rules hold either way."""
    monkeypatch.setenv("MPIR_CVAR_DEVICE_COLL_PIPELINE_KB", str(kb))
    n = 8
    logs = run_plan(harness, n, [config5(n)[1]], f"pipe{kb}")
    res = check(logs)
    for r, log in enumerate(logs):
        assert res[r]["groups"] == chunks
        folds = [ev for ev in log if ev[:2] == ["note", "combine"]]
        assert len(folds) == chunks
        assert sum(int(ev[3]) for ev in folds) == (1 << 29) // n          # every element folded once
        assert all(ev[2] == "8" and ev[-1] == "chain" for ev in folds)
        # each fold follows its chunk's group
        pos = [i for i, ev in enumerate(log) if ev[0] == "group_end"]
        fpos = [i for i, ev in enumerate(log) if ev[:2] == ["note", "combine"]]
        assert all(f > g for f, g in zip(fpos, pos))


@pytest.mark.parametrize("n", [3, 5, 6, 7])
def test_pipelined_allreduce_non_pof2(harness, n):
    """Config 4's reference order at rank counts with a pre-fold (excluded
    ranks take part in every chunk's group with no transfers): the blocks of
    256 MiB / pof2 are pipelined, and the sequences still match."""
    logs = run_plan(harness, n, [CONFIG4[1]], "arnp")
    res = check(logs)
    pof2 = 1 << (n.bit_length() - 1)
    block = (256 << 20) // pof2
    chunks = -(-block // (32 << 20))
    # pre-fold group + reduce-scatter chunks + allgather chunks
    assert all(pr["groups"] == 1 + 2 * chunks for pr in res), [pr["groups"] for pr in res]
