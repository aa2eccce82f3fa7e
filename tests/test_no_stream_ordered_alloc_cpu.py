"""The product takes no stream-ordered allocations (hipMallocAsync /
hipFreeAsync / memory pools).  Round 1's TREE combine fallback did, one
library stream per host thread, and concurrent MINLOC folds came out
corrupted (commit e7b5d60): the default pool hands a block freed on one
stream to another stream while the first stream's kernels still read it
(tools/mempool_race.hip, profiles/archive/r02/mempool_race.log).  The GPU side of the
regression is test_schedule_fused_gpu.py::test_concurrent_threads_minloc_tree16_regression."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "mpich-pip_amd", "csrc")
BANNED = re.compile(r"\b(hipMallocAsync|hipFreeAsync|hipMallocFromPoolAsync|hipMemPool\w*|hipDeviceGetDefaultMemPool)\b")


def test_no_stream_ordered_allocation_in_product_sources():
    hits = []
    for d, _, files in os.walk(CSRC):
        for f in files:
            if f.endswith((".c", ".h", ".hip", ".hpp", ".cpp")):
                p = os.path.join(d, f)
                with open(p, errors="replace") as fh:
                    for i, line in enumerate(fh, 1):
                        if BANNED.search(line):
                            hits.append(f"{os.path.relpath(p, ROOT)}:{i}: {line.strip()}")
    assert not hits, "\n".join(hits)
