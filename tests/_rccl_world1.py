"""Child process of tests/test_gpu_rccl_world1.py: RCCL (torch.distributed
"nccl") at world size 1 on cuda:0, through every collective the N > 1
bench path uses (dips_amd/shard.py, bench.py), on the dtypes it uses --
the one hardware check of the RCCL calls this pool allows (RCCL refuses
two ranks on one GPU).  Prints one JSON line."""
import json
import os
from datetime import timedelta

import torch
import torch.distributed as dist


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev, timeout=timedelta(seconds=60))
    assert dist.get_world_size() == 1 and dist.get_backend() == "nccl"
    out = {"rccl_version": ".".join(map(str, torch.cuda.nccl.version()))}
    g = torch.Generator(device="cpu").manual_seed(5)
    # 'overall': broadcast of the reference frame (uint8, shard.broadcast_reference)
    frame = torch.randint(0, 256, (216, 384, 3), generator=g, dtype=torch.uint8).to(dev)
    ref = frame.clone()
    dist.broadcast(ref, src=0)
    out["broadcast_u8"] = bool(torch.equal(ref, frame))
    # 'per-frame': the halo frame by send / recv (shard.per_frame_overlapped),
    # here rank 0 to itself
    halo = torch.empty_like(frame)
    works = dist.batch_isend_irecv([dist.P2POp(dist.isend, frame, 0), dist.P2POp(dist.irecv, halo, 0)])
    for w in works:
        w.wait()
    out["sendrecv_self_u8"] = bool(torch.equal(halo, frame))
    # the series gather (int64 [n, 4], shard.SeriesGather)
    series = torch.randint(-2**62, 2**62, (1000, 4), generator=g, dtype=torch.int64).to(dev)
    recv = [torch.zeros_like(series)]
    dist.gather(series, recv, dst=0)
    out["gather_i64"] = bool(torch.equal(recv[0], series))
    parts = [torch.zeros_like(series)]
    dist.all_gather(parts, series)
    out["all_gather_i64"] = bool(torch.equal(parts[0], series))
    # the max-over-ranks time (bench.py) and the self-check flag (shard.py)
    t = torch.tensor([21.5], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    flag = torch.ones(1, dtype=torch.int32, device=dev)
    dist.all_reduce(flag)
    out["all_reduce"] = bool(t.item() == 21.5 and flag.item() == 1)
    objs = [None]
    dist.all_gather_object(objs, {"rank": 0, "ms": 21.5})
    out["all_gather_object"] = objs == [{"rank": 0, "ms": 21.5}]
    dist.barrier()
    torch.cuda.synchronize()
    dist.destroy_process_group()
    out["ok"] = all(v for k, v in out.items() if k != "rccl_version")
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
