"""GPU edge cases of the merge path, each checked against the CPU oracle (oracle/yref.c).

Empty and ragged batches, malformed input (atomic refusal, doc unchanged), pending input, structs
longer than the sizer's 15-bit tables and longer than a 16 KiB decode group, client ids at the
ends of the u32 range, unicode keys / values, delete-set-only updates, duplicates and many tiny
updates. Reference semantics: Y.applyUpdate / Y.encodeStateAsUpdate (crdt.js:35,56,294 / 347).
"""
import json
import random

import pytest

crdt_amd = pytest.importorskip("crdt_amd")
from oracle.yref import Doc as ODoc  # noqa: E402
from tests.histories import any_int  # noqa: E402

pytestmark = pytest.mark.gpu


def any_str(s: str) -> bytes:
    """lib0 writeAny of a string of any length: tag 119 + varString."""
    b = s.encode()
    out = bytearray([119])
    n = len(b)
    while n > 0x7F:
        out.append(0x80 | (n & 0x7F))
        n >>= 7
    out.append(n)
    return bytes(out) + b


def _merge_both(updates, client=0x7FFFFFF0):
    ref = ODoc(client)
    for u in updates:
        ref.apply_update(u)
    d = crdt_amd.Doc(client_id=client)
    d.apply_updates(updates)
    return d, ref


def _same(d, ref):
    assert d.encode_state_as_update() == ref.encode_state_as_update()
    assert d.encode_state_vector() == ref.encode_state_vector()


def test_empty_batch_and_empty_update():
    d = crdt_amd.Doc(client_id=1)
    d.apply_updates([])
    assert d.encode_state_as_update() == b"\x00\x00"
    assert d.encode_state_vector() == b"\x00"
    d.apply_update(b"\x00\x00")
    assert d.encode_state_as_update() == b"\x00\x00"
    b = crdt_amd.Batch([b"\x00\x00", b"\x00\x00"])
    b.merge()
    assert b.result() == (b"\x00\x00", b"\x00")


def test_malformed_is_refused_atomically():
    a = ODoc(7)
    a.map_set("users", "k", any_int(5))
    good = a.encode_state_as_update()
    d = crdt_amd.Doc(client_id=1)
    d.apply_update(good)
    before = d.encode_state_as_update()
    for bad in (b"\xff\xff", good[:-3], good[:5], b"\x01\x01\x07\x00\x28\x01"):
        with pytest.raises(crdt_amd.YcrdtError) as ei:
            d.apply_update(bad)
        assert ei.value.kind == "DECODE"
        assert d.encode_state_as_update() == before  # the doc is unchanged


def test_malformed_delete_set_keeps_structs():
    """Yjs decodes and integrates the struct section before it reads the delete set (Y@21330): an
    update whose delete set is cut off throws, but its structs stay in the doc."""
    a = ODoc(7)
    a.map_set("users", "k", any_int(5))
    good = a.encode_state_as_update()
    d = crdt_amd.Doc(client_id=1)
    with pytest.raises(crdt_amd.YcrdtError) as ei:
        d.apply_update(good[:-1])
    assert ei.value.kind == "DECODE"
    assert d.encode_state_as_update() == good


def test_missing_dependencies_are_pending_not_refused():
    """Y.applyUpdate of an update whose predecessor is missing parks it (Yjs pendingStructs); the
    predecessor then integrates both (the exact bytes while pending: test_gpu_pending.py)."""
    a = ODoc(9)
    a.map_set("users", "x", any_int(1))
    u1 = a.encode_state_as_update()
    sv1 = a.encode_state_vector()
    a.map_set("users", "x", any_int(2))
    u2 = a.encode_state_as_update(sv1)  # depends on u1
    d = crdt_amd.Doc(client_id=1)
    d.apply_update(u2)
    # the delta carries the full delete set: x=1 (clock 0), not integrated yet, is a pending range
    assert d.pending() == (True, True)
    assert d.encode_state_vector() == b"\x00"
    d.apply_update(u1)
    assert d.pending() == (False, False)
    ref = ODoc(1)
    ref.apply_update(u1)
    ref.apply_update(u2)
    _same(d, ref)


@pytest.mark.parametrize("size", [100, 16_000, 16_384 + 7, 70_000, 200_000])
def test_long_values_across_groups(size):
    """One struct longer than a decode group / the 15-bit sizer tables, between ordinary ones."""
    rng = random.Random(size)
    a = ODoc(11)
    for i in range(40):
        a.map_set("users", f"k{i}", any_int(i))
    a.map_set("users", "big", any_str("é" * (size // 2) + "x" * (size % 2)))
    a.array_insert("messages", 0, [any_str("m" * size), any_int(3)])
    for i in range(40):
        a.map_set("users", f"k{rng.randrange(50)}", any_str("v" * rng.randrange(1, 300)))
    b = ODoc(12)
    b.map_set("users", "big", any_int(1))
    d, ref = _merge_both([a.encode_state_as_update(), b.encode_state_as_update()])
    _same(d, ref)


def test_extreme_client_ids_and_unicode():
    ups = []
    for c in (0, 1, 127, 128, 2**31 - 1, 2**31, 2**32 - 2, 2**32 - 1):
        x = ODoc(c)
        x.map_set("users", "ключ🔑", any_str("значение 😀 " + str(c)))
        x.map_set("users", f"k{c % 3}", any_int(c % 1000))
        x.array_insert("messages", 0, [any_str("日本語"), any_int(-c % 100)])
        ups.append(x.encode_state_as_update())
    d, ref = _merge_both(ups)
    _same(d, ref)
    # deep-equal, as crdt.js's cache is compared: key order follows each doc's insertion history
    assert json.loads(d.root_json("users", "map")) == json.loads(ref.root_json("users", "map"))
    assert d.root_json("messages", "array") == ref.root_json("messages", "array")


def test_delete_set_only_duplicates_and_tiny_updates():
    a = ODoc(21)
    ups = []
    for i in range(300):  # many tiny incremental updates (ragged batch)
        sv = a.encode_state_vector()
        if i % 5 == 4:
            a.map_delete("users", f"k{i % 7}")
        else:
            a.map_set("users", f"k{i % 7}", any_int(i))
        ups.append(a.encode_state_as_update(sv))
    batch = ups + ups[::7] + [ups[0]] * 5  # duplicates are absorbed
    random.Random(3).shuffle(batch)
    ref2 = ODoc(0x7FFFFFF0)
    for u in ups:
        ref2.apply_update(u)
    d2 = crdt_amd.Doc(client_id=0x7FFFFFF0)
    d2.apply_updates(batch)
    _same(d2, ref2)
    # an update that carries only a delete set: the diff of a deletion-only step
    sv = a.encode_state_vector()
    a.map_delete("users", "k1")
    ds_only = a.encode_state_as_update(sv)
    d2.apply_update(ds_only)
    ref2.apply_update(ds_only)
    _same(d2, ref2)


def test_extreme_clients_merge_updates_and_diff():
    from oracle.ymerge import diff_update, merge_updates
    from tests.v1util import canonical_update

    ups = []
    for c in (0, 2**31, 2**32 - 1):
        x = ODoc(c)
        x.map_set("users", "k", any_int(c % 7))
        x.array_insert("messages", 0, [any_int(1), any_str("x")])
        x.array_delete("messages", 0, 1)
        ups.append(x.encode_state_as_update())
    # the engine writes delete sets in 13.6 canonical client order (DESIGN.md §3 Compat)
    got, want = crdt_amd.merge_updates(ups), canonical_update(merge_updates(ups))
    assert got == want, (got.hex(), want.hex())
    sv = b"\x01\xff\xff\xff\xff\x0f\x01"  # client 2^32-1 at clock 1
    m = merge_updates(ups)
    assert canonical_update(crdt_amd.diff_update(m, sv)) == canonical_update(diff_update(m, sv))


def test_local_ops_by_max_client_id():
    """Local ops whose origins / right origins belong to client 0xFFFFFFFF (the view must not take
    it for "no item"), and a doc whose own client id is 0xFFFFFFFF."""
    other = ODoc(2**32 - 1)
    other.map_set("users", "a", any_int(1))
    other.array_insert("messages", 0, [any_int(1), any_int(2)])
    u = other.encode_state_as_update()
    for me in (5, 2**32 - 1):
        if me == 2**32 - 1:
            u_in = b"\x00\x00"
        else:
            u_in = u
        d = crdt_amd.Doc(client_id=me)
        ref = ODoc(me)
        d.apply_update(u_in)
        ref.apply_update(u_in)
        for doc in (d, ref):
            doc.map_set("users", "a", any_int(2))
            doc.array_insert("messages", 1 if me == 5 else 0, [any_int(9)])
            doc.map_delete("users", "a")
        _same(d, ref)
        assert d.root_json("messages", "array") == ref.root_json("messages", "array")


@pytest.mark.parametrize("nclients", [1500, 2500])
def test_small_update_many_clients(nclients):
    """One small update holding many clients' sections (crdt.js's full-state wire shape): the
    count-free small decode takes it; past its one-workgroup client table (2 048 sections) it
    raises a capacity error and the decode reruns counted. Both against the oracle."""
    src = ODoc(0x7FFFFFF0)
    for c in range(1, nclients + 1):
        p = ODoc(c)
        p.map_set("users", "k%d" % (c % 97), any_int(c))
        src.apply_update(p.encode_state_as_update())
    state = src.encode_state_as_update()
    assert len(state) <= 64 << 10
    d, ref = _merge_both([state])
    _same(d, ref)
    assert json.loads(d.root_json("users", "map")) == json.loads(ref.root_json("users", "map"))
