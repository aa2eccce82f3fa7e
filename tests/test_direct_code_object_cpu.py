"""The direct AQL dispatch's code object (lib/libmpir_hip_tiles.hsaco, built
from csrc/hip/direct_tiles.hip) against what direct_dispatch.hip loads from
it: for every (op, element class) whose launcher is launch_reduce, the five
kernels of plan_reduce's launch plan in their unchecked and checked forms, each
taking one 128-byte kernarg slot, and no hidden arguments (a bare AQL packet launches them, so a kernel
that read gridDim or any other implicit argument would read garbage).  A
kernel missing or mis-sized here would silently send its calls to the HIP
launch path (the host skips it), so this pins the contract at build time.
Runs on CPU: it reads the ELF notes with llvm-readelf."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HSACO = os.path.join(ROOT, "mpich-pip_amd", "lib", "libmpir_hip_tiles.hsaco")
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"

# the (op, class) matrix of the reg_*.hip units whose launcher is launch_reduce
INTS = ["I8", "U8", "I16", "U16", "I32", "U32", "I64", "U64"]
REALS = ["F16", "F32", "F64"]
CPLX = ["CF32", "CF64"]
PAIRS = ["P2INT", "PFLOATINT", "PLONGINT", "PSHORTINT", "PDOUBLEINT"]
MATRIX = {
    "SUM": INTS + REALS + CPLX + ["F80"], "PROD": INTS + REALS + CPLX + ["F80"],
    "MAX": INTS + REALS + ["F80"], "MIN": INTS + REALS + ["F80"],
    "LAND": INTS, "LOR": INTS, "BAND": INTS, "BOR": INTS, "BXOR": INTS,
    "LXOR": INTS + REALS + ["F80"], "MAXLOC": PAIRS, "MINLOC": PAIRS,
}
# plan kind -> kernarg bytes: every kernel takes one 128-byte KargSlot (reduce_kernels.hpp)
# each plan kind unchecked (mpir_<kind>_) and checked (mpir_c<kind>_)
KINDS = {f"mpir_{c}{k}_": 128 for c in ("", "c") for k in ("tile", "tilex", "tiles", "elems", "elemsu")}


def kernels():
    if not os.path.exists(HSACO) or not shutil.which(READELF):
        pytest.skip("code object or llvm-readelf missing (run __graft_entry__.build())")
    notes = subprocess.run([READELF, "--notes", HSACO], capture_output=True, text=True, check=True).stdout
    out = {}
    # one metadata block per kernel: its .name, .kernarg_segment_size and .args
    for block in re.split(r"\n\s+- \.agpr_count", notes)[1:]:
        name = re.search(r"\.name:\s+(\S+)", block)
        size = re.search(r"\.kernarg_segment_size:\s+(\d+)", block)
        if name and size:
            seg = [int(m) for m in re.findall(r"\.(?:group|private)_segment_fixed_size:\s+(\d+)", block)]
            out[name.group(1)] = (int(size.group(1)), "hidden_" in block,
                                  any(seg) or "uses_dynamic_stack: true" in block)
    return out


def test_every_plan_kernel_present_with_its_argument_size():
    ks = kernels()
    want = {f"{p}{op}_MPIR_HIP_{e}": size for op, es in MATRIX.items() for e in es for p, size in KINDS.items()}
    assert len(want) == 114 * 10
    missing = sorted(set(want) - set(ks))
    assert not missing, missing[:10]
    wrong = {k: ks[k][0] for k in want if ks[k][0] != want[k]}
    assert not wrong, list(wrong.items())[:10]


def test_dispatch_id_probe_present():
    """mpir_probe_dispatch_id: the queue check (direct_dispatch.hip probe_ids)
    that picks the nonce protocol or read-back flushes; without it the host
    always takes read-back flushes."""
    ks = kernels()
    assert ks.get("mpir_probe_dispatch_id", (0,))[0] == 128


def test_no_kernel_reads_a_hidden_argument():
    ks = kernels()
    hidden = sorted(k for k, (_, h, _) in ks.items() if h)
    assert not hidden, hidden[:10]


def test_no_kernel_needs_lds_or_scratch():
    """The packets carry group / private segment sizes of 0 (direct_dispatch.hip
    also skips, at load time, any kernel whose symbol asks for more)."""
    ks = kernels()
    seg = sorted(k for k, (_, _, s) in ks.items() if s)
    assert not seg, seg[:10]
