#!/usr/bin/env python3
"""Does HSA_ALLOCATE_QUEUE_DEV_MEM=1 (AQL rings in VRAM, which libmpir_hip.so
defaults at load) hurt the other HSA clients of the process?  VERDICT r3 item 5.

Alternated fresh child processes with the variable 0 and 1 -- the library is
never loaded, so only ROCm's own queues are measured:
  * HIP launch + sync: one tiny torch kernel then torch.cuda.synchronize(),
    median us over 3000;
  * RCCL through torch.distributed (backend nccl), one rank: all_reduce of
    256 MiB fp32 (GB/s of the buffer per call, median of 20) and of 8 bytes
    (us per call, median of 500).

    python3 tools/ring_placement_ab.py [rounds]     (on the GPU box)
"""
import json
import os
import socket
import subprocess
import sys
import time


def child():
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    x = torch.zeros(1, device="cuda")
    for _ in range(200):
        x.add_(1)
        torch.cuda.synchronize()
    ts = []
    for _ in range(3000):
        t0 = time.perf_counter()
        x.add_(1)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    out = {"hip_launch_sync_us": round(ts[len(ts) // 2] * 1e6, 2)}
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{os.environ['AB_PORT']}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    big = torch.rand(64 << 20, device="cuda")
    small = torch.zeros(2, device="cuda")
    for _ in range(5):
        dist.all_reduce(big)
        dist.all_reduce(small)
    torch.cuda.synchronize()
    tb = []
    for _ in range(20):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dist.all_reduce(big)
        torch.cuda.synchronize()
        tb.append(time.perf_counter() - t0)
    tb.sort()
    tsml = []
    for _ in range(500):
        t0 = time.perf_counter()
        dist.all_reduce(small)
        torch.cuda.synchronize()
        tsml.append(time.perf_counter() - t0)
    tsml.sort()
    out["rccl_allreduce_256MiB_GBps"] = round((256 << 20) / tb[len(tb) // 2] / 1e9, 1)
    out["rccl_allreduce_8B_us"] = round(tsml[len(tsml) // 2] * 1e6, 2)
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    res = {"0": [], "1": []}
    for r in range(rounds):
        for v in (("0", "1") if r % 2 == 0 else ("1", "0")):
            with socket.socket() as s:
                s.bind(("127.0.0.1", 0))
                port = s.getsockname()[1]
            env = dict(os.environ, HSA_ALLOCATE_QUEUE_DEV_MEM=v, AB_PORT=str(port))
            p = subprocess.run([sys.executable, os.path.abspath(__file__), "--child"], env=env, capture_output=True,
                               text=True, timeout=240)
            lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
            if p.returncode != 0 or not lines:
                print(f"child {v} failed: {p.stderr[-1500:]}", flush=True)
                sys.exit(1)
            d = json.loads(lines[-1])
            res[v].append(d)
            print(f"round {r} HSA_ALLOCATE_QUEUE_DEV_MEM={v}: {d}", flush=True)
    for v, ds in res.items():
        med = {k: sorted(d[k] for d in ds)[len(ds) // 2] for k in ds[0]}
        print(f"median HSA_ALLOCATE_QUEUE_DEV_MEM={v}: {json.dumps(med)}", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child()
    else:
        main()
