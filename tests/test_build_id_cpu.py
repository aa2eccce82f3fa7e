"""The build id embedded in libmpir_hip.so and the direct path's code object
(Makefile BUILD_ID): both hashes recomputed here from the
tree, so the suite fails when the binaries that would ship to the GPU box were
built from other sources than the ones checked in."""
import hashlib
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mpich-pip_amd")
SUFFIXES = (".c", ".h", ".hip", ".hpp")


def _hash(paths):
    h = hashlib.sha256()
    for p in paths:
        with open(os.path.join(PKG, p), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def src_hash():
    # the Makefile's SRC_FILES: `find csrc ../include -type f ... | LC_ALL=C sort`
    rel = []
    for top in ("csrc", "../include"):
        for dp, _, fs in os.walk(os.path.join(PKG, top)):
            for f in fs:
                if f.endswith(SUFFIXES):
                    rel.append(os.path.relpath(os.path.join(dp, f), PKG) if top == "csrc"
                               else "../include/" + os.path.relpath(os.path.join(dp, f), os.path.join(PKG, top)))
    return _hash(sorted(rel))


def tiles_hash():
    # the Makefile's TILES_SRC: direct_tiles.hip, then HDRS in their order
    mk = open(os.path.join(PKG, "Makefile")).read()
    m = re.search(r"^HDRS\s*:=\s*((?:.*\\\n)*.*)$", mk, re.M)
    hdrs = m.group(1).replace("\\\n", " ").split()
    return _hash(["csrc/hip/direct_tiles.hip"] + hdrs)


def fields(bid: str) -> dict:
    return dict(kv.split("=", 1) for kv in bid.split())


def test_library_build_id_matches_sources(mpi):
    bid = fields(mpi.build_id())
    assert set(bid) == {"src", "tiles", "git"}
    assert bid["src"] == src_hash(), "libmpir_hip.so was built from other sources: rebuild (make -C mpich-pip_amd)"
    assert bid["tiles"] == tiles_hash()


def test_code_object_carries_the_library_tiles_hash(mpi):
    co = os.path.join(PKG, "lib", "libmpir_hip_tiles.hsaco")
    if not os.path.exists(co):
        pytest.fail("code object not built")
    data = open(co, "rb").read()
    want = ("mpir-tiles-build:" + fields(mpi.build_id())["tiles"]).encode()
    assert want in data, "the .hsaco and libmpir_hip.so come from different builds"
