"""Key-hash sharding of ONE document (config C4): the integrate phases run per shard
(lists owned by hash(top-level entry) % shards, other shards' segments masked), the per-segment
flag words are combined, and the encode runs on the combined flags. Every shard count must give
the unsharded bytes — on the Yjs fixtures (golden sets, the C3 / C4 config cases) and on a C4-shaped
history generated here (nested YArrays under YMap keys, overwrites that GC whole arrays, concurrent
pushes / inserts / deletes). The RCCL path runs at world size 1 on the one-GPU box (the identity
all-reduce); world-size-2 partition / exchange logic is covered on CPU by tests/test_shard_cpu.py."""
import json
import os
import random

import pytest

crdt_amd = pytest.importorskip("crdt_amd")

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _merge(ups, nshards=None, comm=None):
    b = crdt_amd.Batch(ups)
    if nshards is None:
        b.merge()
    else:
        b.merge_sharded(nshards, comm)
    return b.result()


def test_shards_golden_and_configs(golden):
    with open(os.path.join(ROOT, "tests", "golden", "configs.json")) as f:
        cfg = [c for c in json.load(f)["cases"] if not c["name"].startswith("c5_")]
    cases = [c for s in ("kat", "map", "array", "nested") for c in golden[s]] + cfg
    for c in cases:
        ups = [bytes.fromhex(u) for u in c["updates"]]
        for n in (1, 2, 3, 8):
            st, sv = _merge(ups, n)
            assert st.hex() == c["state"], (c["name"], n)
            assert sv.hex() == c["sv"], (c["name"], n)


def _any_int(v):
    return bytes([125, v & 0x3F]) if 0 <= v < 64 else bytes([119, 1, 0x61 + v % 26])


def c4_history(seed, n_rep=8, n_keys=24, rounds=4, ops=25):
    """C4-shaped: replicas on YMap 'docs' whose keys hold nested YArrays; local ops through the
    engine (byte-identical Yjs structs), deltas gossiped after every round."""
    rng = random.Random(seed)
    reps = [crdt_amd.Doc(client_id=1000 + 7 * i) for i in range(n_rep)]
    for d in reps:
        d.track_local(True)
    log = []
    for _ in range(rounds):
        for d in reps:
            for _ in range(ops):
                key = "d%d" % rng.randrange(n_keys)
                if d.map_type_at("docs", key) != 0 or rng.random() < 0.08:
                    d.map_set_type("docs", key, 0)  # new (or overwriting) nested array
                n = d.array_length("docs", parent_key=key)
                x = rng.random()
                if x < 0.6 or n == 0:
                    d.array_insert("docs", rng.randrange(n + 1), [_any_int(rng.randrange(100)) for _ in range(1 + rng.randrange(3))], parent_key=key)
                elif x < 0.85:
                    d.array_insert("docs", n, [_any_int(rng.randrange(100))], parent_key=key)
                else:
                    i = rng.randrange(n)
                    d.array_delete("docs", i, min(n - i, 1 + rng.randrange(2)), parent_key=key)
        deltas = [d.take_local_update() for d in reps]
        log += [u for u in deltas if u]
        for i, d in enumerate(reps):
            for j, u in enumerate(deltas):
                if i != j and u and rng.random() < 0.7:
                    d.apply_update(u)
    return log


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_shards_generated_c4(seed):
    ups = c4_history(seed, n_rep=6 + 2 * seed, n_keys=16 * seed)
    want = _merge(ups)
    for n in (2, 5, 16):
        assert _merge(ups, n) == want, n
    random.Random(seed).shuffle(ups)
    assert _merge(ups, 3) == want


def test_shards_c2_generated():
    from crdt_amd.workload import C2, gen_map

    cfg = dict(C2)
    cfg.update(n_keys=3000, n_replicas=60, ops_per_replica=200)
    ups, _ = gen_map(**cfg)
    want = _merge(ups)
    assert _merge(ups, 4) == want


def test_rccl_world1_exchanges(golden):
    """The native RCCL path at world size 1: the sharded merge, the SV all-reduce and the DS
    all-gather through libycrdt's communicator."""
    eng = crdt_amd.default_engine()
    comm = crdt_amd.Comm(eng, 1, 0, crdt_amd.Comm.unique_id())
    try:
        for c in golden["nested"][:20] + golden["array"][:10]:
            ups = [bytes.fromhex(u) for u in c["updates"]]
            assert _merge(ups, 1, comm) == (bytes.fromhex(c["state"]), bytes.fromhex(c["sv"])), c["name"]
            assert comm.sv_allreduce_max(bytes.fromhex(c["sv_raw"])).hex() == c["sv"], c["name"]
            st = bytes.fromhex(c["state"])
            assert comm.ds_allgather(st) == st, c["name"]
    finally:
        comm.close()


def test_c4_generated_vs_oracle_and_shards():
    """The C4 generator (crdt_amd/workload/ycw_nested.cpp) at reduced scale: GPU merge equals the
    oracle's state, and 8 key-hash shards equal the unsharded merge."""
    from crdt_amd.workload import gen_nested
    from oracle.yref import Doc as ODoc

    ups, st = gen_nested(60, 2000, 300, seed=11)
    o = ODoc(0x7FFFFFF0)
    for u in ups:
        o.apply_update(u)
    want = (o.encode_state_as_update(), o.encode_state_vector())
    assert _merge(ups) == want
    assert _merge(ups, 8) == want
    d = crdt_amd.Doc(client_id=0x7FFFFFF0)
    d.apply_updates(ups)
    assert json.loads(d.root_json("docs", "map")) == json.loads(o.root_json("docs", "map"))


def test_c4_full_size_shards_properties():
    """The generator's C4 (≈47 M items, 2 000 replicas, 100 k nested arrays): 4 key-hash shards give
    the unsharded bytes; the merge is order-independent and idempotent. (BASELINE's C4 scale,
    C4_FULL at 102 M items, runs in bench.py's c4 / c4_sharded legs through the same properties.)"""
    from crdt_amd.workload import C4, gen_nested

    ups, st = gen_nested(**C4)
    b = crdt_amd.Batch(ups)
    s1 = b.merge()
    full = b.result()
    assert s1.items > 40_000_000
    b.merge_sharded(4)
    assert b.result() == full
    r = crdt_amd.Batch(list(reversed(ups)))
    r.merge()
    assert r.result() == full
    i = crdt_amd.Batch([full[0]] + ups[:100])
    i.merge()
    assert i.result() == full
