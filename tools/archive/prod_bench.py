# why does bench.py's config-3 PROD read 0.77 with 4 rotating all-ones buffers?
import os, sys
ROOT = os.getcwd()
sys.path[:0] = [ROOT, ROOT + "/mpich-pip_amd"]
import torch, mpich_pip_amd as m
lib = m.load()
MIB = 1 << 20
count = 64 * MIB
g = torch.Generator(device="cuda").manual_seed(1)
pairs = [((torch.rand(count, device="cuda", generator=g) * 2 - 1), (torch.rand(count, device="cuda", generator=g) * 2 - 1)) for _ in range(4)]
s = torch.cuda.Stream()

def run(name, ins, ios, op, k=15, w=5):
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(k)]
    with torch.cuda.stream(s):
        for i in range(w + k):
            if i >= w:
                evs[i - w][0].record(s)
            assert lib.MPIX_Reduce_local_stream(ins[i % len(ins)].data_ptr(), ios[i % len(ios)].data_ptr(), count,
                                                m.MPI_FLOAT, op, s.cuda_stream) == 0
            if i >= w:
                evs[i - w][1].record(s)
    s.synchronize()
    ms = sorted(a.elapsed_time(b) for a, b in evs)
    print(f"{name:45s} median {ms[k // 2] * 1e3:8.2f} us  frac {3 * 4 * count / (ms[k // 2] * 1e-3) / 8e12:.3f}", flush=True)

a = [p[0] for p in pairs]
b = [p[1] for p in pairs]
ones4 = [torch.ones(count, device="cuda") for _ in range(4)]
ones2 = ones4[:2]
for rep in range(2):
    run("SUM  in = pair b", b, a, m.MPI_SUM)
    run("PROD in = 4 separate ones", ones4, a, m.MPI_PROD)
    run("PROD in = 2 separate ones", ones2, a, m.MPI_PROD)
    run("SUM  in = 4 separate ones", ones4, a, m.MPI_SUM)
    near1 = [(x * 1e-6 + 1.0) for x in b]
    run("PROD in = 4 separate random~1", near1, a, m.MPI_PROD)
    del near1
    for x in b:
        x.fill_(1.0)
    run("PROD in = pair b filled with 1.0", b, a, m.MPI_PROD)
    for x in b:
        x.uniform_(-1, 1)
