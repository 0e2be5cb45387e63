"""TEST REFERENCE (not product code): a torch restatement of the fleet exchanges that libycrdt
implements natively (crdt_amd/csrc/yc_comm.hip: ycrdt_comm_fleet_sv_allreduce_max,
ycrdt_comm_ds_allgather, ycrdt_route). tests/test_fleet.py runs it as world-size-2 gloo groups on
CPU to pin the exchange rules against the oracle; tests/test_gpu_exchange.py runs the library's own
exchanges the same way (host exchange over gloo) and compares.

Doc-fleet sharding and the cross-rank exchange steps.

One process per GPU. Documents (crdt.js topics) are independent, so the merge itself needs no
collective: `shard_of` routes every update of a doc to one rank, which merges its docs on its own
GPU (bench.py, "scaling": "weak"). Two exchange steps exist, and only these use a collective:

* `sv_allreduce_max` — the fleet's state vectors when ingest is NOT routed by doc (any rank may
  have received any update): per (doc, client) the max clock over ranks, i.e. the state vector of
  the union of what the ranks hold (Yjs getStateVector Y@28925 is per-client max of clock+len).
  The (doc, client) key space comes from an all-gather of distinct keys, sort-unique
  (SURVEY.md §8(e)); the clocks are then one dense all-reduce(MAX) over that key space.
* `ds_allgather` — delete-set ranges (client, clock, len) all-gathered and unioned with Yjs's
  sortAndMergeDeleteSet rule (Y@10246: sort by clock, merge while a.clock + a.len >= b.clock).

Both run on torch tensors of the group's device: `cuda` tensors over RCCL (backend "nccl") on the
GPU box, CPU tensors over gloo in the multi-process tests. The sort / unique / segmented-merge
steps are torch ops on the same device. State vectors travel in and out as Yjs v1 bytes
(`decode_sv` / `encode_sv`, readStateVector Y@22536 / writeStateVector Y@22723), in the 13.6
canonical order (clients descending) the engine writes.
"""
import hashlib

import torch
import torch.distributed as dist


# ---- routing --------------------------------------------------------------------------------
def shard_of(doc_id, world: int) -> int:
    """Stable rank for a doc / topic name: the same on every rank and every run (no Python hash())."""
    b = doc_id.encode() if isinstance(doc_id, str) else bytes(doc_id)
    return int.from_bytes(hashlib.blake2b(b, digest_size=8).digest(), "little") % world


def route(items, world: int):
    """[(doc_id, update), ...] → per-rank lists, every update of a doc on the same rank."""
    out = [[] for _ in range(world)]
    for doc_id, u in items:
        out[shard_of(doc_id, world)].append((doc_id, u))
    return out


# ---- state vector bytes (lib0 varuint, Yjs v1) ----------------------------------------------
def _rvu(b, p):
    v, s = 0, 0
    while True:
        if p >= len(b):
            raise ValueError("Integer out of range!")
        r = b[p]
        p += 1
        v |= (r & 0x7F) << s
        s += 7
        if r < 0x80:
            return v, p


def _wvu(out, v):
    while v > 0x7F:
        out.append(0x80 | (v & 0x7F))
        v >>= 7
    out.append(v)


def decode_sv(sv: bytes) -> dict:
    """Yjs readStateVector (Y@22536): varuint n, then (client, clock) × n."""
    n, p = _rvu(sv, 0)
    d = {}
    for _ in range(n):
        c, p = _rvu(sv, p)
        k, p = _rvu(sv, p)
        d[c] = k
    return d


def encode_sv(d: dict) -> bytes:
    """Yjs writeStateVector (Y@22723) in 13.6 canonical order (clients descending)."""
    out = bytearray()
    _wvu(out, len(d))
    for c in sorted(d, reverse=True):
        _wvu(out, c)
        _wvu(out, d[c])
    return bytes(out)


# ---- collectives ----------------------------------------------------------------------------
def _device(group=None):
    return torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else torch.device("cpu")


def _allgather_var(t: torch.Tensor, group=None) -> torch.Tensor:
    """All-gather of a 1-D/2-D tensor whose first dimension differs per rank (padded exchange)."""
    world = dist.get_world_size(group)
    n = torch.tensor([t.shape[0]], dtype=torch.int64, device=t.device)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n, group=group)
    ns = [int(x.item()) for x in ns]
    m = max(ns) if ns else 0
    pad = torch.zeros((m,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    pad[: t.shape[0]] = t
    outs = [torch.zeros_like(pad) for _ in range(world)]
    dist.all_gather(outs, pad, group=group)
    return torch.cat([o[:k] for o, k in zip(outs, ns)])


def sv_allreduce_max(svs, group=None):
    """svs: {doc_index: state vector bytes} held by this rank (any subset of the fleet's docs).

    Returns {doc_index: state vector bytes} for EVERY doc known to any rank: per client the max
    clock over ranks. Collectives: one all-gather of the distinct (doc, client) keys, one
    all-reduce(MAX) of a dense u32 clock vector over the sorted key space.
    """
    dev = _device(group)
    keys, clocks = [], []
    for doc, sv in svs.items():
        for c, k in decode_sv(sv).items():
            keys.append((int(doc) << 32) | c)
            clocks.append(k)
    kt = torch.tensor(keys, dtype=torch.int64, device=dev)
    space = torch.unique(_allgather_var(kt, group))  # sorted, identical on every rank
    dense = torch.zeros(space.shape[0], dtype=torch.int64, device=dev)
    if kt.numel():
        idx = torch.searchsorted(space, kt)
        dense.scatter_reduce_(0, idx, torch.tensor(clocks, dtype=torch.int64, device=dev), reduce="amax")
    dist.all_reduce(dense, op=dist.ReduceOp.MAX, group=group)
    out = {}
    sp, dn = space.cpu().tolist(), dense.cpu().tolist()
    for key, k in zip(sp, dn):
        out.setdefault(key >> 32, {})[key & 0xFFFFFFFF] = k
    return {doc: encode_sv(d) for doc, d in out.items()}


def merge_ranges(r: torch.Tensor) -> torch.Tensor:
    """Union of delete-set ranges r = [n, 3] int64 (client, clock, len), Yjs sortAndMergeDeleteSet
    (Y@10246): per client sorted by clock, a range is merged into the previous one while
    prev.clock + prev.len >= clock. Returns [m, 3] sorted by (client, clock)."""
    if r.numel() == 0:
        return r.reshape(0, 3)
    r = r[r[:, 2] > 0]
    if r.numel() == 0:
        return r.reshape(0, 3)
    # clients as dense ranks (client ids use all 32 bits; rank << 34 must not overflow int64)
    _, ci = torch.unique(r[:, 0], return_inverse=True)
    order = torch.argsort((ci << 33) | r[:, 1], stable=True)
    c, s, e, ci = r[order, 0], r[order, 1], r[order, 1] + r[order, 2], ci[order]
    # running max of the end within a client: client ranks ascend, so offsetting every end by
    # rank << 34 lets one global cummax stay inside each client's segment (ends < 2^34)
    off = ci << 34
    run_end = torch.cummax(e + off, 0).values - off
    prev_end = torch.cat([torch.full((1,), -1, dtype=torch.int64, device=r.device), run_end[:-1]])
    prev_c = torch.cat([torch.full((1,), -1, dtype=torch.int64, device=r.device), c[:-1]])
    new = (c != prev_c) | (s > prev_end)
    rid = torch.cumsum(new.to(torch.int64), 0) - 1
    m = int(rid[-1].item()) + 1
    rc = torch.zeros(m, dtype=torch.int64, device=r.device).scatter_(0, rid[new], c[new])
    rs = torch.zeros(m, dtype=torch.int64, device=r.device).scatter_(0, rid[new], s[new])
    re = torch.zeros(m, dtype=torch.int64, device=r.device).scatter_reduce_(0, rid, e, reduce="amax", include_self=False)
    return torch.stack([rc, rs, re - rs], 1)


def ds_allgather(ranges: torch.Tensor, group=None) -> torch.Tensor:
    """All-gather of every rank's delete-set ranges [n, 3] (client, clock, len), unioned."""
    dev = _device(group)
    return merge_ranges(_allgather_var(ranges.to(dev, torch.int64), group))


def read_delete_set(ds_section: bytes):
    """A Yjs v1 delete-set section (readDeleteSet Y@11619 wire: varuint nClients, then per client:
    client, n, (clock, len) × n) as [n, 3] int64 (client, clock, len)."""
    update = ds_section
    p = 0
    n, p = _rvu(update, p)
    out = []
    for _ in range(n):
        c, p = _rvu(update, p)
        m, p = _rvu(update, p)
        for _ in range(m):
            k, p = _rvu(update, p)
            ln, p = _rvu(update, p)
            out.append((c, k, ln))
    return torch.tensor(out, dtype=torch.int64).reshape(-1, 3)
