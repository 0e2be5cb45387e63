"""The N>1 path on CPU: doc routing (the library's ycrdt_route, host-only) and the two cross-rank
exchange rules, restated in torch (tests/fleet_ref.py), run as world_size-2 gloo process groups;
tests/test_gpu_exchange.py runs libycrdt's native exchanges over the same kind of group.

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

from tests import fleet_ref as fleet


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
    """libycrdt's ycrdt_route (host-only, no GPU): in range, balanced, stable, str == bytes."""
    import crdt_amd

    for world in (1, 2, 3, 8):
        ranks = [crdt_amd.route(f"topic{i}", world) for i in range(4000)]
        assert all(0 <= r < world for r in ranks)
        counts = [ranks.count(r) for r in range(world)]
        assert min(counts) > 0.8 * 4000 / world and max(counts) < 1.2 * 4000 / world, counts
    assert crdt_amd.route("topic17", 8) == crdt_amd.route(b"topic17", 8)
    # pinned values: the routing of a topic must not change between releases (a fleet's doc owners)
    assert [crdt_amd.route(f"topic{i}", 8) for i in range(12)] == ROUTE_PINNED


ROUTE_PINNED = [6, 0, 5, 1, 4, 0, 5, 7, 1, 6, 4, 7]  # FNV-1a 64 + fmix64, mod 8


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
