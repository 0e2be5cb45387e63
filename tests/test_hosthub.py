"""crdt_amd/hosthub.py — the torch-free host exchange the ranks bootstrap with (RCCL unique id) and
that carries libycrdt's collectives when ranks share a device — at world sizes 2 and 3 on the CPU:
all-gather of unequal payloads, broadcast, all-reduce sum (mod 2^32) / max of u32 words."""
import multiprocessing as mp
import os
import socket
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(world, rank, port, q):
    sys.path.insert(0, os.path.dirname(HERE))
    from crdt_amd.hosthub import HostHub

    hub = HostHub(world, rank, "127.0.0.1", port, timeout=60)
    out = {"rank": rank}
    out["gather"] = hub.allgather(bytes([rank]) * (rank * 1000 + 1))
    out["bcast"] = hub.bcast(b"unique-id-from-rank-0" if rank == 0 else None)
    a = np.array([rank, 0xFFFFFFFF, 7 * rank + 1], dtype=np.uint32)
    b = a.copy()
    hub.allreduce_u32(a, 0)
    hub.allreduce_u32(b, 1)
    out["sum"], out["max"] = a.tolist(), b.tolist()
    hub.barrier()
    out["torch"] = "torch" in sys.modules
    hub.close()
    q.put(out)


@pytest.mark.parametrize("world", [2, 3])
def test_hosthub(world):
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(world, r, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
    assert [p.exitcode for p in ps] == [0] * world
    res = sorted([q.get() for _ in range(world)], key=lambda r: r["rank"])
    for r in res:
        assert r["gather"] == [bytes([k]) * (k * 1000 + 1) for k in range(world)]
        assert r["bcast"] == b"unique-id-from-rank-0"
        assert r["sum"] == [sum(range(world)), (0xFFFFFFFF * world) & 0xFFFFFFFF, sum(7 * k + 1 for k in range(world))]
        assert r["max"] == [world - 1, 0xFFFFFFFF, 7 * (world - 1) + 1]
        assert not r["torch"]
