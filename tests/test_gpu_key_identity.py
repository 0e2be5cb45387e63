"""List identity on the device is exact, not a hash.

A list — a root type, a nested type, a YMap entry — is (document, root name | parent item,
parentSub) (Item.integrate after Item.getMissing, Y@76507; map keys come from users and peers,
crdt.js:434, 294). The engine's key table hashes that identity to find a slot, but a slot is shared
only after the two lists' names compare equal (yc_merge.hip key_insert / same_list). The test hook
YCRDT_KEY_HASH_BITS=8 keeps 8 bits of every list hash, so thousands of distinct lists collide in
at most 256 hash values: results must still be the Yjs / oracle bytes.
"""
import json
import random

import pytest

crdt_amd = pytest.importorskip("crdt_amd")

pytestmark = pytest.mark.gpu


@pytest.fixture
def collide(monkeypatch):
    monkeypatch.setenv("YCRDT_KEY_HASH_BITS", "8")  # read by every merge (yc_engine.hip run_merge)
    yield


def _any_int(v):  # lib0 `any` of a small integer (tag 125, signed varint)
    assert 0 <= v < 64
    return bytes([125, v])


def _oracle_replicas(n_rep, n_keys, ops, seed, roots=("users", "posts")):
    from oracle.yref import Doc as ODoc

    rng = random.Random(seed)
    ups = []
    base = ODoc(1)
    for k in range(n_keys):
        base.map_set(roots[k % len(roots)], f"key{k}", _any_int(k % 64))
    b = base.encode_state_as_update()
    ups.append(b)
    for r in range(n_rep):
        d = ODoc(100 + r)
        d.apply_update(b)
        for _ in range(ops):
            k = rng.randrange(n_keys + 200)  # some keys only replicas write
            root = roots[k % len(roots)]
            if rng.random() < 0.2:
                d.map_delete(root, f"key{k}")
            else:
                d.map_set(root, f"key{k}", _any_int(rng.randrange(64)))
        ups.append(d.encode_state_as_update())
    ref = ODoc(0x7FFFFFF0)
    for u in ups:
        ref.apply_update(u)
    return ups, ref


def test_colliding_map_keys_vs_oracle(collide):
    """2 400 keys of two root maps in <= 256 hash values, 6 replicas of concurrent set / delete."""
    ups, ref = _oracle_replicas(6, 2400, 800, 7)
    d = crdt_amd.Doc(client_id=0x7FFFFFF0)
    d.apply_updates(ups)
    assert d.encode_state_as_update() == ref.encode_state_as_update()
    assert d.encode_state_vector() == ref.encode_state_vector()
    for root in ("users", "posts"):
        got = json.loads(d.root_json(root, "map"))
        assert got == json.loads(ref.root_json(root, "map"))
        assert len(got) > 1000
    # the batch path and per-key reads (the view's key table) agree
    b = crdt_amd.Batch(ups)
    b.merge()
    assert b.result()[0] == ref.encode_state_as_update()
    want = json.loads(ref.root_json("users", "map"))
    for k in ("key0", "key2", "key1998", "key2598", "key2599"):
        st, val = d.map_get("users", k)
        assert st == (1 if k in want else 0), k
        if st == 1:
            assert json.loads(val) == want[k], k


def test_colliding_keys_multidoc(collide):
    """The same key names in many documents of one batch: per-document lists never merge."""
    docs = []
    refs = []
    for i in range(8):
        ups, ref = _oracle_replicas(3, 300, 200, 100 + i)
        docs.append(ups)
        refs.append(ref.encode_state_as_update())
    b = crdt_amd.Batch(docs=docs)
    b.merge()
    assert [u for u, _ in b.result_docs()] == refs


@pytest.mark.parametrize("setname", ["kat", "map", "array", "nested"])
def test_golden_under_collisions(golden, setname, collide):
    """Every Yjs golden case (states, state vectors, deltas, toJSON) with colliding list hashes."""
    from tests.test_gpu_parity import test_gpu_golden
    from tests.test_gpu_view import test_gpu_json_golden

    test_gpu_golden(golden, setname)
    test_gpu_json_golden(golden, setname)


@pytest.mark.parametrize("prefix", ["c3_", "c4_", "c5_"])
def test_configs_under_collisions(prefix, collide):
    from tests.test_gpu_configs import test_gpu_config_batch

    test_gpu_config_batch(prefix)


@pytest.mark.parametrize("part", range(3))
def test_pending_under_collisions(part, collide):
    from tests.test_gpu_pending import test_pending_every_step

    test_pending_every_step(part)


def test_compat135_under_collisions(golden, collide):
    import os

    from tests.test_gpu_compat135 import SETS, test_135_state_and_sv_raw

    e = crdt_amd.Engine(int(os.environ.get("YCRDT_DEVICE", "0")), compat=135)
    try:
        for s in SETS:
            test_135_state_and_sv_raw(golden, s, e)
    finally:
        e.close()


def test_sharded_under_collisions(collide):
    """Key-hash shards take the list's low hash half: colliding lists may share a shard, results stay exact."""
    from tests.test_gpu_configs import _cases

    for c in _cases("c4_")[:10]:
        ups = [bytes.fromhex(u) for u in c["updates"]]
        b = crdt_amd.Batch(ups)
        b.merge()
        full = b.result()
        for n in (2, 5):
            b.merge_sharded(n)
            assert b.result() == full, (c["name"], n)
        assert full[0].hex() == c["state"]
