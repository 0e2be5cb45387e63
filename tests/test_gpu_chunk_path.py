"""The chunk path for large updates (yc_decode.hip k_spec / k_walk), against the CPU oracle.

A large update is cut into 1 KiB chunks; one lane per chunk follows the all-struct chain from the
chunk's first byte, and one wavefront per update follows the true struct sequence through the
section headers, trusting a chunk's chain only once the true sequence has met it. These cases aim
at the places where that can go wrong: many sections ending mid-chunk, structs spanning many
chunks, string contents that are themselves valid struct encodings (chains that run beside the
true sequence), sections of a single struct, and truncated / corrupted large updates (refused
atomically, as Y.applyUpdate throws). Reference semantics: readClientsStructRefs (Y@19286).
"""
import random

import pytest

crdt_amd = pytest.importorskip("crdt_amd")
from oracle.yref import Doc as ODoc  # noqa: E402
from tests.histories import any_int  # noqa: E402
from tests.test_gpu_edges import _merge_both, _same, any_str  # noqa: E402

pytestmark = pytest.mark.gpu


def _snapshot(n_clients, per_client, seed, value=None):
    """One oracle doc written by many clients: its state is a large update of n_clients sections."""
    rng = random.Random(seed)
    full = ODoc(1)
    for c in range(n_clients):
        d = ODoc(100 + 13 * c)
        if c % 50 == 0:  # now and then a client that has seen the others (origins across clients)
            d.apply_update(full.encode_state_as_update())
        for i in range(per_client):
            k = rng.randrange(3 * per_client)
            v = value(rng) if value else any_int(rng.randrange(1000))
            if rng.random() < 0.7:
                d.map_set("users", f"k{k}", v)
            else:
                d.array_insert("messages", 0, [v])
        full.apply_update(d.encode_state_as_update())
    return full.encode_state_as_update()


@pytest.mark.parametrize("mode", ["chunks", "direct"])
@pytest.mark.parametrize("n_clients,per_client", [(900, 3), (60, 40), (2000, 1)])
def test_many_sections(mode, n_clients, per_client, monkeypatch):
    monkeypatch.setenv("YCRDT_DECODE", mode)
    snap = _snapshot(n_clients, per_client, n_clients)
    assert len(snap) > 16384
    extra = ODoc(9)
    extra.map_set("users", "k1", any_int(5))
    d, ref = _merge_both([snap, extra.encode_state_as_update()])
    _same(d, ref)


def test_struct_encodings_inside_strings():
    """String values that are valid struct encodings: chunk chains starting inside them parse real
    looking structs and only meet the true sequence where the strings end."""
    inner = _snapshot(3, 20, 5)[4:]  # struct bytes of a small update, repeated inside the values
    vals = [inner * k for k in (1, 3, 9, 40)]
    snap = _snapshot(30, 8, 6, value=lambda rng: any_str(vals[rng.randrange(4)].decode("latin-1")))
    assert len(snap) > 100_000
    d, ref = _merge_both([snap])
    _same(d, ref)


def test_long_structs_span_chunks():
    snap = _snapshot(40, 4, 7, value=lambda rng2: any_str("x" * rng2.choice([1, 900, 1023, 1025, 5000, 70_000])))
    d, ref = _merge_both([snap])
    _same(d, ref)


def test_truncated_and_corrupted_large_updates():
    snap = _snapshot(600, 5, 8)
    base = ODoc(3)
    base.map_set("users", "a", any_int(1))
    for cut in (len(snap) // 3, len(snap) - 3, 20_000):
        # cut inside the structs: nothing applied; inside the delete set: Yjs has integrated the
        # structs before readDeleteSet throws (Y@11105), and so does the engine
        ref = ODoc(5)
        ref.apply_update(base.encode_state_as_update())
        with pytest.raises(Exception):
            ref.apply_update(snap[:cut])
        d = crdt_amd.Doc(client_id=5)
        d.apply_update(base.encode_state_as_update())
        with pytest.raises(crdt_amd.YcrdtError):
            d.apply_update(snap[:cut])
        _same(d, ref)
    for at in (len(snap) // 2, len(snap) // 5, 17_000):
        bad = bytearray(snap)
        bad[at] = 0x1F  # an info byte with content ref 31 (no such struct), or a broken field
        ref = ODoc(5)
        try:
            ref.apply_update(bytes(bad))
            want = ref.encode_state_as_update()
        except Exception:
            want = None
        d = crdt_amd.Doc(client_id=5)
        if want is None:
            with pytest.raises(crdt_amd.YcrdtError):
                d.apply_update(bytes(bad))
            assert d.encode_state_as_update() == b"\x00\x00"
        else:
            d.apply_update(bytes(bad))
            assert d.encode_state_as_update() == want


def test_batch_of_large_and_small():
    """Large snapshots (chunk path) and many small deltas (direct path) in one batch."""
    snaps = [_snapshot(50, 6, s) for s in (11, 12, 13)]
    small = []
    for i in range(1500):
        o = ODoc(5000 + i)
        o.map_set("users", f"k{i % 37}", any_int(i))
        small.append(o.encode_state_as_update())
    d, ref = _merge_both(snaps + small)
    _same(d, ref)


def _periodic_snapshot(n, seed):
    """One client writing n map entries of identical encoded size (one section): the struct stream
    is periodic, so chunk chains can settle into a phase that never meets the true one."""
    d = ODoc(7)
    for k in range(n):
        d.map_set("users", f"k{k:06d}", any_int(1000 + (k * 7919 + seed) % 9000))
    return d.encode_state_as_update()


@pytest.mark.parametrize("mode", ["auto", "xtab"])
def test_periodic_struct_streams(mode, monkeypatch):
    """Periodic snapshots (the C4 base: identical type items, then identical elements) hand the
    walk over to the exit tables (k_xtab): byte-exact either way, and with every large update of
    the other chunk-path cases forced through the tables."""
    if mode == "xtab":
        monkeypatch.setenv("YCRDT_DECODE", "xtab")
    from crdt_amd.workload import gen_nested

    ups, _ = gen_nested(40, 3000, 60, seed=9)
    assert len(ups[0]) > 64 * 1024
    for batch in ([ups[0]], ups, [_periodic_snapshot(20000, 3)]):
        d, ref = _merge_both(batch)
        _same(d, ref)
    if mode == "xtab":
        for n_clients, per_client in ((900, 3), (60, 40)):
            d, ref = _merge_both([_snapshot(n_clients, per_client, n_clients)])
            _same(d, ref)
        snap = _snapshot(40, 4, 7, value=lambda rng2: any_str("x" * rng2.choice([1, 900, 1023, 1025, 5000, 70_000])))
        d, ref = _merge_both([snap])
        _same(d, ref)
