"""Every environment variable the product reads is in INTEGRATION.md's runtime
table (no undocumented switches in mpich-pip_amd/)."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mpich-pip_amd")
# set by our own mpiexec for its ranks (csrc/runtime/mpiexec.c), not user-facing
LAUNCHER_INTERNAL = {"MPIR_PIP_RANK", "MPIR_PIP_SIZE", "MPIR_PIP_SHM"}


def read_names():
    pat = re.compile(r'\b(?:getenv|cvar_long|os\.environ\.get)\(\s*"([A-Za-z0-9_]+)"')
    names = set()
    for base, _, files in os.walk(PKG):
        if os.sep + "build" in base:
            continue
        for f in files:
            if f.endswith((".c", ".h", ".hip", ".hpp", ".cpp", ".py")):
                with open(os.path.join(base, f), encoding="utf-8", errors="replace") as fh:
                    names.update(pat.findall(fh.read()))
    return names


def test_every_variable_is_documented():
    names = read_names()
    assert "MPIR_CVAR_REDUCE_LOCAL_DISPATCH" in names     # the scan sees the sources
    with open(os.path.join(ROOT, "INTEGRATION.md"), encoding="utf-8") as fh:
        doc = fh.read()
    missing = []
    for n in sorted(names - LAUNCHER_INTERNAL):
        # the table abbreviates a run of MPIR_CVAR_ names after the first: `_SUFFIX`
        short = "`_" + n[len("MPIR_CVAR_"):] if n.startswith("MPIR_CVAR_") else None
        if n not in doc and not (short and short in doc):
            missing.append(n)
    assert not missing, f"read by the library but not in INTEGRATION.md: {missing}"


def test_local_rank_variables_documented():
    """The launchers' node-local rank counts the host pool reads (round 5;
    hip_reduce.hip local_ranks reads them in a loop the scan above cannot see)."""
    with open(os.path.join(ROOT, "mpich-pip_amd", "csrc", "hip", "hip_reduce.hip"), encoding="utf-8") as fh:
        src = fh.read()
    with open(os.path.join(ROOT, "INTEGRATION.md"), encoding="utf-8") as fh:
        doc = fh.read()
    for name in ("MPI_LOCALNRANKS", "MPIR_PIP_SIZE", "LOCAL_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_SIZE"):
        assert f'"{name}"' in src, name
        assert name in doc, name
