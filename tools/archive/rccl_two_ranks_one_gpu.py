# probe: can RCCL put 2 ranks on one GPU?  (expect ncclInvalidUsage)
import sys, os, ctypes, multiprocessing as mp
ROOT=os.getcwd(); sys.path.insert(0, ROOT+'/mpich-pip_amd')
def main(rank, uid, q):
    import torch, mpich_pip_amd as m
    lib=m.load(); lib.MPIX_Reduce_local_set_errhandler(m.MPI_ERRORS_RETURN)
    torch.cuda.set_device(0)
    c=ctypes.c_void_p()
    rc=lib.MPIX_Hip_comm_create(ctypes.c_char_p(uid), 2, rank, ctypes.byref(c))
    q.put((rank, rc, m.error_string(rc) if rc else "ok"))
if __name__=='__main__':
    import mpich_pip_amd as m
    uid=ctypes.create_string_buffer(128); print("uid rc", m.load().MPIX_Hip_comm_get_unique_id(uid))
    ctx=mp.get_context("spawn"); q=ctx.Queue()
    ps=[ctx.Process(target=main,args=(r,uid.raw,q)) for r in range(2)]
    [p.start() for p in ps]
    for _ in range(2): print(q.get(timeout=100))
    [p.join(30) for p in ps]
