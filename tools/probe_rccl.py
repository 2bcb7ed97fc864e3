"""Host time of the collectives bench.py's multi-GPU path issues, on one rank
of an RCCL ("nccl") group (diagnostic: where the timed region's host time goes)."""
import os
import time

import torch
import torch.distributed as dist

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
x = torch.zeros(3, dtype=torch.float64, device=dev)
p = torch.zeros(1, dtype=torch.int64, device=dev)


def us(t):
    return f"{(time.perf_counter() - t) * 1e6:9.1f}"


for i in range(4):
    t = time.perf_counter()
    dist.barrier()
    print(i, "barrier", us(t), flush=True)
    t = time.perf_counter()
    dist.all_reduce(p, op=dist.ReduceOp.MAX)
    torch.cuda.synchronize()
    print(i, "allreduce i64 MAX + sync", us(t), flush=True)
    t = time.perf_counter()
    w = dist.all_reduce(x, op=dist.ReduceOp.SUM, async_op=True)
    print(i, "allreduce f64 async enqueue", us(t), flush=True)
    t = time.perf_counter()
    w.wait()
    print(i, "wait", us(t), flush=True)
    t = time.perf_counter()
    torch.cuda.synchronize()
    print(i, "sync", us(t), flush=True)
    g = [torch.zeros_like(x[:1])]
    t = time.perf_counter()
    dist.all_gather(g, x[:1].clone())
    torch.cuda.synchronize()
    print(i, "all_gather + sync", us(t), flush=True)
dist.destroy_process_group()

# enqueue cost while the device is busy (a spin kernel on the current stream)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
side = torch.cuda.Stream(device=dev)
for mode in ("current", "side", "current", "side"):
    dist.all_reduce(x, op=dist.ReduceOp.SUM)
    torch.cuda.synchronize()
    torch.cuda._sleep(2_000_000)   # ~1 ms of spinning on the current stream
    t = time.perf_counter()
    if mode == "side":
        with torch.cuda.stream(side):
            w = dist.all_reduce(x, op=dist.ReduceOp.SUM, async_op=True)
    else:
        w = dist.all_reduce(x, op=dist.ReduceOp.SUM, async_op=True)
    print("busy device:", mode, "async enqueue", us(t), flush=True)
    t = time.perf_counter()
    w.wait()
    torch.cuda.synchronize()
    print("busy device:", mode, "wait + sync", us(t), flush=True)
    t = time.perf_counter()
    torch.cuda._sleep(2_000_000)
    dist.barrier()
    print("busy device: barrier after a 1 ms kernel", us(t), flush=True)
dist.destroy_process_group()
