#!/usr/bin/env python3
"""gloo_cuda_probe.py -- which torch.distributed gloo operations accept HIP
(device) tensors on this build: two processes on GPU 0, each op tried once.
Run on the GPU box: python tools/gloo_cuda_probe.py"""
import json
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    res = {}

    def tryop(name, fn):
        try:
            fn()
            torch.cuda.synchronize()
            res[name] = "ok"
        except Exception as e:  # noqa: BLE001
            res[name] = f"{type(e).__name__}: {str(e)[:160]}"

    t = torch.full((8,), rank + 1, dtype=torch.uint8, device=dev)
    tryop("broadcast", lambda: dist.broadcast(t, src=0))
    a = torch.full((4,), rank + 1, dtype=torch.int64, device=dev)
    tryop("all_reduce", lambda: dist.all_reduce(a))
    def sr():
        x = torch.full((16,), rank, dtype=torch.uint8, device=dev)
        y = torch.empty_like(x)
        ops = [dist.P2POp(dist.isend, x, (rank + 1) % world), dist.P2POp(dist.irecv, y, (rank - 1) % world)]
        for r in dist.batch_isend_irecv(ops):
            r.wait()
        assert int(y[0]) == (rank - 1) % world
    tryop("batch_isend_irecv", sr)
    def ga():
        x = torch.full((3, 4), rank, dtype=torch.int64, device=dev)
        out = [torch.empty_like(x) for _ in range(world)] if rank == 0 else None
        dist.gather(x, out, dst=0)
    tryop("gather", ga)
    def ag():
        x = torch.full((3, 4), rank, dtype=torch.int64, device=dev)
        out = [torch.empty_like(x) for _ in range(world)]
        dist.all_gather(out, x)
    tryop("all_gather", ag)
    tryop("all_gather_object", lambda: dist.all_gather_object([None] * world, {"r": rank}))
    q.put((rank, res))
    dist.destroy_process_group()


def main():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = sorted(q.get(timeout=180) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    print(json.dumps({"torch": torch.__version__, "results": dict(out)}, indent=1))
    sys.exit(0 if all(p.exitcode == 0 for p in ps) else 1)


if __name__ == "__main__":
    main()
