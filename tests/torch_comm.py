"""libycrdt's host exchange over a torch.distributed process group (gloo, CPU tensors) — TEST
INFRASTRUCTURE ONLY: the package ships its own torch-free transport (crdt_amd/hosthub.py); this
one checks the same library code over a second, independent transport."""
import numpy as np


def comm_over_torch(crdt_amd, engine, group=None):
    import torch
    import torch.distributed as dist

    world, rank = dist.get_world_size(group), dist.get_rank(group)

    def allreduce(a, op):
        t = torch.from_numpy(a.astype(np.int64))
        dist.all_reduce(t, op=dist.ReduceOp.MAX if op else dist.ReduceOp.SUM, group=group)
        a[:] = (t.numpy() & 0xFFFFFFFF).astype(np.uint32)

    def allgather(b):
        t = torch.frombuffer(bytearray(b), dtype=torch.uint8) if b else torch.zeros(0, dtype=torch.uint8)
        outs = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(outs, t, group=group)
        return b"".join(o.numpy().tobytes() for o in outs)

    return crdt_amd.Comm.over(engine, world, rank, allreduce, allgather)
