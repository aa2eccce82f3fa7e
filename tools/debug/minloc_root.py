# debug: MPIX_Reduce_hip MINLOC DOUBLE_INT p=8 count=3 root=4 mismatch
import sys, os
ROOT = os.getcwd()
for d in (ROOT, ROOT + "/mpich-pip_amd", ROOT + "/tests"):
    sys.path.insert(0, d)
import numpy as np, torch, threading
import _types as T, mpich_pip_amd as mpi, oracle
from oracle import schedules as S
lib = mpi.load(); lib.MPIX_Reduce_local_set_errhandler(mpi.MPI_ERRORS_RETURN)
t, op = "MPI_DOUBLE_INT", "MPI_MINLOC"
p, count = 8, 3
esz = T.elem_size(t); dt, o = mpi.DATATYPES[t], mpi.OPS[op]
rng = np.random.default_rng(7 * p)
xs = [T.to_bytes(T.gen(t, count, rng, op)) for _ in range(p)]
PT = T.PAIRS[t]
for root in range(p):
    want = S.reduce_auto(xs, count, esz, dt, o, root)
    # 1) fused tree on relrank-ordered device slots
    slots = [torch.from_numpy(xs[(r + root) % p].copy()).cuda() for r in range(p)]
    out = torch.zeros(count * esz, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    rc = mpi.reduce_local_multi([s.data_ptr() for s in slots], out.data_ptr(), count, dt, o, mpi.MPIX_ORDER_TREE)
    torch.cuda.synchronize()
    g1 = out.cpu().numpy()
    # 2) step by step with MPI_Reduce_local on device
    acc = [s.clone() for s in slots]
    mask = 1
    while mask < p:
        for r in range(0, p, 2 * mask):
            if r + mask < p:
                assert mpi.reduce_local(acc[r + mask].data_ptr(), acc[r].data_ptr(), count, dt, o) == 0
        mask <<= 1
    torch.cuda.synchronize()
    g2 = acc[0].cpu().numpy()
    print(root, "fused", rc, np.array_equal(g1, want), "steps", np.array_equal(g2, want))
    if not np.array_equal(g1, want) or not np.array_equal(g2, want):
        print("  want ", want.view(PT)); print("  fused", g1.view(PT)); print("  steps", g2.view(PT))
