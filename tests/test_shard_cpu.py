"""World-size-2 CPU check of the C4 key-hash partition and its exchange (gloo), restating the device
rule of yc_merge.hip (k_key_shard / k_seg_shard / k_shard_export) on the items of Yjs-generated C4
and nested fixtures:
  * every item's list is resolved as Item.getMissing does (explicit parent, else the origin's /
    right origin's list); a nested list's top-level list is the list holding its parent item;
  * shard = mix64(FNV-1a(root name varString, 0x5A, parentSub varString)) % world, the same hash
    the device's key table holds for a top-level list;
  * partition property: an item's origin, right origin and parent item (when present in the doc)
    live on the same shard, so winners, YATA, dead types and merge adjacency are shard-local;
  * exchange: each rank exports a payload for the items it owns, a gloo all_reduce(SUM) of the
    vectors reconstructs every item's payload exactly once on both ranks."""
import json
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
M64 = (1 << 64) - 1


def _fnv_bytes(h, b):
    for x in b:
        h = ((h ^ x) * 1099511628211) & M64
    return h


def list_hash(root: bytes, psub):
    h = _fnv_bytes(1469598103934665603, root)
    if psub is not None:
        h = _fnv_bytes(h, bytes([0x5A, 0, 0, 0]))
        h = _fnv_bytes(h, psub)
    return h or 1


def shard_of_hash(h, n):
    h ^= h >> 33
    h = (h * 0xFF51AFD7ED558CCD) & M64
    h ^= h >> 33
    return h % n


def items_and_shards(updates, world):
    """{unit id: (origin, right origin, parent item | None, shard)} for every item unit."""
    from oracle.ymerge import ITEM, Dec, lazy_structs

    units, lst = {}, {}
    for u in updates:
        for s in lazy_structs(Dec(u)):
            if s.kind != ITEM:
                continue
            for i in range(s.length):
                uid = (s.client, s.clock + i)
                if uid in units:
                    continue
                o = s.origin if i == 0 else (s.client, s.clock + i - 1)
                units[uid] = (o, s.right_origin)
                if o is None and s.right_origin is None:
                    lst[uid] = (s.parent, s.parent_sub)  # root name varString | parent item id
    pending = [u for u in units if u not in lst]
    while pending:
        nxt = []
        for u in pending:
            o, r = units[u]
            src = o if o is not None else r
            if src in lst:
                lst[u] = lst[src]
            elif src in units:
                nxt.append(u)
        if len(nxt) == len(pending):
            break
        pending = nxt

    def top(L, depth=0):
        parent, psub = L
        if isinstance(parent, bytes) or depth > 64:
            return L
        return top(lst[parent], depth + 1) if parent in lst else L

    out = {}
    for u, (o, r) in units.items():
        if u not in lst:
            continue
        parent, psub = lst[u]
        t = top(lst[u])
        h = list_hash(t[0], t[1]) if isinstance(t[0], bytes) else 0
        out[u] = (o, r, parent if not isinstance(parent, bytes) else None, shard_of_hash(h, world))
    return out


def _cases():
    with open(os.path.join(ROOT, "tests", "golden", "configs.json")) as f:
        cases = [c for c in json.load(f)["cases"] if c["name"].startswith(("c4_", "c3_"))]
    with open(os.path.join(ROOT, "tests", "golden", "nested.json")) as f:
        cases += json.load(f)["cases"][:40]
    return cases


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        report = []
        for c in _cases():
            items = items_and_shards([bytes.fromhex(u) for u in c["updates"]], world)
            order = sorted(items)
            # partition property: references stay on the item's shard
            for u in order:
                o, r, p, sh = items[u]
                for ref in (o, r, p):
                    if ref is not None and ref in items:
                        assert items[ref][3] == sh, (c["name"], u, ref)
            # exchange: owner-exported payloads summed over the ranks
            vec = torch.zeros(len(order), dtype=torch.int64)
            for i, u in enumerate(order):
                if items[u][3] == rank:
                    vec[i] = 1 + (u[0] % 1000003) * 7 + u[1]
            dist.all_reduce(vec)
            want = torch.tensor([1 + (u[0] % 1000003) * 7 + u[1] for u in order], dtype=torch.int64)
            assert torch.equal(vec, want), c["name"]
            report.append((c["name"], len(order), sum(1 for u in order if items[u][3] == rank)))
        q.put((rank, report))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(240)
def test_shard_partition_and_exchange_world2_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(200)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = dict(q.get() for _ in range(world))
    for (name, n, a), (_, _, b) in zip(res[0], res[1]):
        assert a + b == n, name  # every item owned exactly once
    # the C4 cases really are split (both ranks own items)
    c4 = [(a, b) for (name, _, a), (_, _, b) in zip(res[0], res[1]) if name.startswith("c4_")]
    assert c4 and all(a > 0 and b > 0 for a, b in c4)
