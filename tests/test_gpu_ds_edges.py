"""Delete-set edge shapes that once slipped past the engine (round-6 review), each against the oracle.

1. A SMALL update (<= 16 KiB: the direct / wave decode paths, not the chunk path) carrying more
   than DSA_WAVE = 4 096 ranges. One transaction that deletes every other item of a 10 000-item
   list writes 5 000 three-byte ranges (readDeleteSet, Y@11105) in ~15 KB. k_units' wavefront
   applies the first 4 096 ranges of an update; the rest are spread over extra workgroups for every
   update the delete-set decoders listed (yc_merge.hip unit_ds_apply_big). Before the fix only the
   chunk-path updates were listed, so ranges 4 096.. of such an update were silently dropped.
2. A delete-only update applied to an EMPTY doc after other merges on the same engine: the batch
   has no client section at all, and the quick small decode (no count synchronisation) used to
   leave the previous merge's client hash in place (k_sections_small returned before its fill),
   so find_client could return a stale client index and k_units could write unit flags at stale
   offsets. Yjs keeps such ranges as pendingDs (crdt.js:294 applies peer updates in any order).

Reference: Y.applyUpdate / Y.encodeStateAsUpdate (crdt.js:294 / 347); oracle/yref.c.
"""
import pytest

crdt_amd = pytest.importorskip("crdt_amd")
from oracle.ymerge import merge_updates as o_merge_updates  # noqa: E402
from oracle.yref import Doc as ODoc  # noqa: E402
from tests.histories import any_int  # noqa: E402

pytestmark = pytest.mark.gpu

MODES = ("direct", "wave", "settle", "chunks")


def _mode(monkeypatch, mode):
    wave = mode in ("wave", "settle")
    monkeypatch.setenv("YCRDT_DECODE", "chunks" if mode == "chunks" else "direct")
    if mode != "chunks":
        monkeypatch.setenv("YCRDT_DIRECT_WAVE", "1" if wave else "0")
    monkeypatch.setenv("YCRDT_WDECODE", "settle" if mode == "settle" else "rank")


def _base_and_holes(n=10_000, step=2, client=77):
    """(base update: one client's n-item list; delete-only delta: every step-th item deleted)."""
    d = ODoc(client)
    d.array_insert("messages", 0, [any_int(i % 50) for i in range(n)])
    base = d.encode_state_as_update()
    sv = d.encode_state_vector()
    for i in range(n - 1 - (n - 1) % step, -1, -step):
        d.array_delete("messages", i, 1)
    delta = d.encode_state_as_update(sv)
    return base, delta


def test_delta_shape():
    base, delta = _base_and_holes()
    assert delta[0] == 0  # no struct section: a delete-only update
    assert len(delta) <= 16 * 1024  # a small update (direct / wave decode)
    assert len(delta) > 3 * 4096  # more than DSA_WAVE ranges of >= 3 bytes


def _oracle(updates, client=0x7FFFFFF0):
    ref = ODoc(client)
    for u in updates:
        ref.apply_update(u)
    return ref.encode_state_as_update(), ref.encode_state_vector()


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("grid", (True, False))
def test_small_update_past_dsa_wave(mode, grid, monkeypatch):
    _mode(monkeypatch, mode)
    monkeypatch.setenv("YCRDT_DS_GRID", "1" if grid else "0")
    base, delta = _base_and_holes()
    want = _oracle([base, delta])
    # in one batch
    d = crdt_amd.Doc(client_id=0x7FFFFFF0)
    d.apply_updates([base, delta])
    assert (d.encode_state_as_update(), d.encode_state_vector()) == want, mode
    # one at a time (the delta merges behind the doc's state)
    d = crdt_amd.Doc(client_id=0x7FFFFFF0)
    d.apply_update(base)
    d.encode_state_vector()
    d.apply_update(delta)
    assert (d.encode_state_as_update(), d.encode_state_vector()) == want, mode
    # beside many other small updates (k_direct's lane-per-update grid)
    others = []
    for c in range(1, 300):
        o = ODoc(5000 + c)
        o.map_set("users", f"k{c % 17}", any_int(c))
        others.append(o.encode_state_as_update())
    ups = others[:150] + [base, delta] + others[150:]
    b = crdt_amd.Batch(ups)
    b.merge()
    assert b.result() == _oracle(ups), mode


@pytest.mark.parametrize("mode", ("direct", "wave"))
def test_delete_only_into_empty_doc_after_other_merges(mode, monkeypatch):
    _mode(monkeypatch, mode)
    # earlier merges on the same engine leave a populated client hash behind
    warm = []
    for c in range(40):
        o = ODoc(100 + c)
        o.map_set("users", f"w{c}", any_int(c))
        warm.append(o.encode_state_as_update())
    w = crdt_amd.Doc(client_id=3)
    w.apply_updates(warm)
    w.encode_state_as_update()
    # a delete-only update whose client the receiving (empty) doc has never seen: pendingDs
    base, delta = _base_and_holes(n=300, step=3, client=100)  # client 100 is in the warm hash
    # Yjs: nothing integrates, every range is kept as pendingDs, and encodeStateAsUpdate returns
    # mergeUpdates([main state, pendingDs]) (the oracle's C port has no pending store: the lazy
    # merge restatement gives that state)
    pending_state = o_merge_updates([b"\x00\x00", delta])
    d = crdt_amd.Doc(client_id=0x7FFFFFF0)
    d.apply_update(delta)
    assert (d.encode_state_as_update(), d.encode_state_vector()) == (pending_state, b"\x00")
    assert d.pending() == (False, True)
    # the structs arrive: the pending ranges apply
    d.apply_update(base)
    assert (d.encode_state_as_update(), d.encode_state_vector()) == _oracle([base, delta])
    assert d.pending() == (False, False)
    # an empty update and a delete-only update in one batch of an empty doc
    d = crdt_amd.Doc(client_id=0x7FFFFFF0)
    d.apply_updates([b"\x00\x00", delta])
    assert (d.encode_state_as_update(), d.encode_state_vector()) == (pending_state, b"\x00")


@pytest.mark.parametrize("prewalk", ("1", "0"))
@pytest.mark.parametrize("extra", (0, 3, 70))
def test_large_delta_short_struct_section(prewalk, extra, monkeypatch):
    """A LARGE update whose struct section is a few structs in front of a big delete set — the sync
    reply's shape (Y.encodeStateAsUpdate(doc, sv) writes the whole delete set, crdt.js:288). k_prewalk
    decodes it whole (<= 64 structs) and the chunk chains skip it; with 70 structs (past its budget)
    or YCRDT_PREWALK=0 the chunk path takes it: the same bytes as the oracle either way."""
    monkeypatch.setenv("YCRDT_PREWALK", prewalk)
    d0 = ODoc(77)
    d0.array_insert("messages", 0, [any_int(i % 50) for i in range(30_000)])
    base = d0.encode_state_as_update()
    sv = d0.encode_state_vector()
    for i in range(29_999, -1, -2):
        d0.array_delete("messages", i, 1)
    for k in range(extra):
        d0.map_set("users", f"x{k}", any_int(k))
    delta = d0.encode_state_as_update(sv)
    assert len(delta) > 16 * 1024
    want = _oracle([base, delta])
    d = crdt_amd.Doc(client_id=0x7FFFFFF0)
    d.apply_update(base)
    d.encode_state_vector()
    d.apply_update(delta)
    assert (d.encode_state_as_update(), d.encode_state_vector()) == want
    b = crdt_amd.Batch([delta, base])  # (one batch merge is order-independent)
    b.merge()
    assert b.result() == want
