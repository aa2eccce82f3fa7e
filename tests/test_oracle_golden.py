"""Pin the CPU oracle before trusting it (CPU only).

* every known-answer case the reference's own tests hold (tests/golden/,
  generated from test/mpi/coll/allred.c, opsum.c, opmax.c, opmin.c,
  opprod.c closed forms) folds to the closed-form solution, bit for bit;
* every reference output recorded in SURVEY.md §7/§8c is reproduced;
* the oracle's _Float16 lowering agrees with numpy's IEEE half conversion;
* the oracle's validation reproduces MPI_Reduce_local's error classes.
"""
import json
import os

import numpy as np
import pytest

import _types as T

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_kat():
    man = json.load(open(os.path.join(GOLD, "kat_reference.json")))
    data = np.load(os.path.join(GOLD, "kat_reference.npz"))
    return man["cases"], data


def test_golden_files_match_manifest():
    import hashlib
    man = json.load(open(os.path.join(GOLD, "kat_reference.json")))
    digest = hashlib.sha256(open(os.path.join(GOLD, "kat_reference.npz"), "rb").read()).hexdigest()
    assert digest == man["sha256_npz"]
    assert len(man["cases"]) > 2000


def test_oracle_folds_reference_kats(orc):
    cases, data = load_kat()
    bad = []
    for c in cases:
        ranks = data[c["key"] + "_ranks"]
        sol = data[c["key"] + "_sol"]
        acc = ranks[0].copy()
        for r in range(1, c["p"]):
            src = ranks[r].copy()
            rc = orc.reduce_local(src, acc, c["count"], c["handle"], c["op_handle"])
            assert rc == 0, c["id"]
        if not np.array_equal(acc, sol):
            bad.append(c["id"])
    assert not bad, f"{len(bad)} KAT mismatches, e.g. {bad[:5]}"


def probe_cases():
    return json.load(open(os.path.join(GOLD, "probe_survey.json")))["cases"]


@pytest.mark.parametrize("case", probe_cases(), ids=lambda c: c["id"])
def test_oracle_reproduces_survey_probes(orc, case):
    import mpich_pip_amd as m
    w = case["width"]
    dt = {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[w]
    io = np.array(case["inout"], dtype=dt)
    src = np.array(case["in"], dtype=dt)
    rc = orc.reduce_local(src, io, len(io), m.DATATYPES[case["datatype"]], m.OPS[case["op"]])
    assert rc == case.get("expect_rc", 0)
    assert [int(x) for x in io] == case["expect"]


def test_oracle_half_conversion_matches_numpy(orc):
    lib = orc.load()
    # every half -> float (numpy widens exactly; NaNs compared as NaN class + payload)
    h = np.arange(65536, dtype=np.uint32).astype(np.uint16)
    ref = h.view(np.float16).astype(np.float32)
    got = np.array([lib.oracle_h2f(int(x)) for x in h[::7]], dtype=np.float32)
    r = ref[::7]
    nan = np.isnan(r)
    assert np.array_equal(np.isnan(got), nan)
    assert np.array_equal(got[~nan].view(np.uint32), r[~nan].view(np.uint32))
    # float -> half rounding on random finite floats incl. subnormal / overflow ranges
    rng = np.random.default_rng(7)
    f = np.concatenate([rng.uniform(-70000, 70000, 4000), rng.uniform(-1e-4, 1e-4, 4000),
                        rng.uniform(-6.2e-8, 6.2e-8, 2000)]).astype(np.float32)
    got = np.array([lib.oracle_f2h(float(x)) for x in f], dtype=np.uint16)
    assert np.array_equal(got, f.astype(np.float16).view(np.uint16))


def test_oracle_validation_error_classes(orc):
    import mpich_pip_amd as m
    a = np.ones(4, dtype=np.float32)
    b = np.ones(4, dtype=np.float32)
    F = m.MPI_FLOAT
    assert orc.reduce_local(a, b, 4, F, m.MPI_OP_NULL) == m.MPI_ERR_OP
    assert orc.reduce_local(a, b, 4, F, m.MPI_REPLACE) == m.MPI_ERR_OP
    assert orc.reduce_local(a, b, 4, F, m.MPI_NO_OP) == m.MPI_ERR_OP
    assert orc.reduce_local(a, b, 4, F, m.MPI_BAND) == m.MPI_ERR_OP          # check_dtype
    assert orc.reduce_local(a, a, 4, F, m.MPI_SUM) == m.MPI_ERR_BUFFER       # alias
    assert orc.reduce_local(a, a, 0, F, m.MPI_SUM) == 0                      # count 0 skips alias
    assert orc.reduce_local(a, b, 4, F, m.MPI_LAND) == m.MPI_ERR_OP          # op_errno quirk
    assert orc.reduce_local(a, b, -3, F, m.MPI_SUM) == 0                     # count < 0 unvalidated


def test_oracle_matrix_self_consistency(orc):
    """check_dtype vs compute switch: only LAND/LOR on floats differ."""
    import mpich_pip_amd as m
    for op in T.OPS:
        for t in T.ALL_TYPES:
            chk = orc.check_dtype(m.OPS[op], m.DATATYPES[t])
            assert (chk == 0) == T.check_ok(op, t), (op, t)
            x = np.zeros(32 * 4, dtype=np.uint8)
            y = np.zeros(32 * 4, dtype=np.uint8)
            rc = orc.reduce_local(x, y, 4, m.DATATYPES[t], m.OPS[op], check=False)
            assert (rc == 0) == T.compute_ok(op, t), (op, t, rc)
