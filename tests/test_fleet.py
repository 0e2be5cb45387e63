"""The N>1 path on CPU: doc routing and the two cross-rank exchange steps of crdt_amd/fleet.py,
run as world_size-2 gloo process groups (the GPU box runs the same code over RCCL).

* sv_allreduce_max: every doc's updates are split over the ranks (ingest not routed); the
  all-reduced state vectors must equal the oracle's encodeStateVector of a doc that applied ALL
  of that doc's updates (Yjs getStateVector Y@28925).
* ds_allgather: every rank holds some delete sets; the union must equal the oracle's
  mergeDeleteSets / sortAndMergeDeleteSet (oracle/ymerge.py, Y@10486 / Y@10246).
"""
import os
import random
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from crdt_amd import fleet


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _docs():
    """6 docs; doc d gets 1 + d replica updates (independent clients, map sets + deletes)."""
    from oracle.yref import Doc as ODoc

    rng = random.Random(7)
    docs = {}
    for d in range(6):
        ups = []
        for r in range(1 + d):
            client = rng.choice([1 + r, 1000 + rng.randrange(1 << 20), rng.randrange(1, 1 << 32)])
            x = ODoc(client)
            for _ in range(rng.randrange(1, 12)):
                k = f"k{rng.randrange(5)}"
                if rng.random() < 0.8:
                    x.map_set("users", k, bytes([125, rng.randrange(64)]))
                else:
                    x.map_delete("users", k)
            ups.append(x.encode_state_as_update())
        docs[d] = ups
    return docs


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle.yref import Doc as ODoc

        docs = _docs()
        # --- SV all-reduce: updates of each doc split round-robin over the ranks
        svs = {}
        for d, ups in docs.items():
            mine = [u for i, u in enumerate(ups) if (i + d) % world == rank]
            if mine:
                x = ODoc(0x7FFFFFF0)
                for u in mine:
                    x.apply_update(u)
                svs[d] = x.encode_state_vector()
        got = fleet.sv_allreduce_max(svs)
        for d, ups in docs.items():
            x = ODoc(0x7FFFFFF0)
            for u in ups:
                x.apply_update(u)
            want = x.encode_state_vector()
            assert fleet.decode_sv(got[d]) == fleet.decode_sv(want), d
            assert got[d] == want, d  # 13.6 canonical order, as the engine writes
        # --- DS all-gather: random ranges, overlapping / adjacent / nested across ranks
        rng = random.Random(100 + rank)
        clients = [1, 7, 2 ** 31 + 5, 2 ** 32 - 1]
        mine = [(rng.choice(clients), rng.randrange(200), rng.randrange(1, 20)) for _ in range(40)]
        union = fleet.ds_allgather(torch.tensor(mine, dtype=torch.int64))
        everyone = [None] * world
        dist.all_gather_object(everyone, mine)
        q.put((rank, union.tolist(), everyone))
    finally:
        dist.destroy_process_group()


def test_route_is_stable_and_total():
    items = [(f"topic{i}", b"u") for i in range(1000)]
    parts = fleet.route(items, 8)
    assert sum(len(p) for p in parts) == 1000
    assert all(60 < len(p) < 190 for p in parts)  # roughly balanced
    assert fleet.shard_of("topic17", 8) == fleet.shard_of(b"topic17", 8)
    assert [fleet.shard_of(f"topic{i}", 8) for i in range(50)] == [fleet.shard_of(f"topic{i}", 8) for i in range(50)]


def test_sv_codec_roundtrip():
    d = {1: 5, 2 ** 32 - 1: 300, 77: 0}
    b = fleet.encode_sv(d)
    assert fleet.decode_sv(b) == d
    assert list(fleet.decode_sv(b)) == sorted(d, reverse=True)


def test_merge_ranges_matches_yjs_rule():
    from oracle.ymerge import merge_delete_sets

    rng = random.Random(3)
    for _ in range(50):
        rs = [(rng.choice([3, 9, 2 ** 32 - 2]), rng.randrange(100), rng.randrange(0, 9)) for _ in range(rng.randrange(0, 30))]
        got = fleet.merge_ranges(torch.tensor(rs, dtype=torch.int64).reshape(-1, 3)).tolist()
        ds = {}
        for c, k, n in rs:
            if n:
                ds.setdefault(c, []).append([k, n])
        want = merge_delete_sets([ds])
        assert got == [[c, k, n] for c in sorted(want) for k, n in want[c]]


def test_read_delete_set_section():
    from oracle.ymerge import wvu

    out = bytearray()
    for v in (2, 9, 2, 0, 3, 10, 1, 2 ** 32 - 1, 1, 5, 6):
        wvu(out, v)
    assert fleet.read_delete_set(bytes(out)).tolist() == [[9, 0, 3], [9, 10, 1], [2 ** 32 - 1, 5, 6]]


@pytest.mark.timeout(180)
def test_exchange_world2_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(150)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = [q.get() for _ in range(world)]
    from oracle.ymerge import merge_delete_sets

    for rank, union, everyone in res:
        ds = {}
        for part in everyone:
            for c, k, n in part:
                ds.setdefault(c, []).append([k, n])
        want = merge_delete_sets([ds])
        assert union == [[c, k, n] for c in sorted(want) for k, n in want[c]], rank
    assert res[0][1] == res[1][1]


@pytest.mark.gpu
def test_exchange_rccl_world1_on_gpu():
    """The same exchange on cuda tensors over RCCL (backend "nccl"), world 1 on the one-GPU box."""
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, init_method=f"tcp://127.0.0.1:{_free_port()}")
    try:
        svs = {0: fleet.encode_sv({5: 3, 2 ** 32 - 1: 9}), 3: fleet.encode_sv({1: 1})}
        got = fleet.sv_allreduce_max(svs)
        assert got == svs
        r = torch.tensor([[9, 0, 3], [9, 3, 2], [9, 10, 1], [2 ** 32 - 1, 5, 6]], dtype=torch.int64)
        u = fleet.ds_allgather(r)
        assert u.device.type == "cuda"
        assert u.tolist() == [[9, 0, 5], [9, 10, 1], [2 ** 32 - 1, 5, 6]]
    finally:
        dist.destroy_process_group()
