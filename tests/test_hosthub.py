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


def _rogue(port, kind):
    """A connection that is no rank of the job: a wrong token, or a length header past the cap."""
    import struct
    import time

    for _ in range(200):
        try:
            s = socket.create_connection(("127.0.0.1", port), timeout=10)
            break
        except OSError:
            time.sleep(0.05)
    if kind == "token":
        s.sendall(struct.pack("<I", 1) + b"\0" * 32)
    else:
        s.sendall(b"\xff" * 64)
    time.sleep(0.5)
    s.close()


def test_hosthub_drops_connections_without_the_job_token():
    """Rank 0 drops a connection whose handshake carries a wrong token (the hub
    accepted any peer that sent a rank number) and still forms the job with the real ranks."""
    import threading

    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    p0 = ctx.Process(target=_worker, args=(2, 0, port, q))
    p0.start()
    for kind in ("token", "junk"):
        t = threading.Thread(target=_rogue, args=(port, kind))
        t.start()
        t.join(30)
    p1 = ctx.Process(target=_worker, args=(2, 1, port, q))
    p1.start()
    p0.join(120)
    p1.join(120)
    assert [p0.exitcode, p1.exitcode] == [0, 0]
    res = sorted([q.get() for _ in range(2)], key=lambda r: r["rank"])
    assert res[1]["bcast"] == b"unique-id-from-rank-0"


def test_hosthub_frame_cap():
    import struct

    from crdt_amd import hosthub

    a, b = socket.socketpair()
    try:
        a.sendall(struct.pack("<Q", hosthub._MAX_FRAME + 1))
        with pytest.raises(ConnectionError):
            hosthub._recv(b)
    finally:
        a.close()
        b.close()
