"""ContentJSON / ContentEmbed / ContentFormat values outside JSON.stringify's form, against Yjs
13.5.16 itself (tests/golden/edges.json "json" cases, tests/golden/gen/gen_edge_fixtures.js).

Yjs parses such a value (Y@72137 readContentJSON, JSON.parse) and writes JSON.stringify of the
parsed value back (Y@71991), so whitespace, escapes, duplicate and array-index keys, long numbers
(0.30000000000000004 stays, 1.50 becomes 1.5, 1e400 becomes null), overlong length prefixes and
deep nesting all come out rewritten. The engine lists such structs while decoding
(yc_decode.hip k_json_structs), computes the canonical contents on the device (k_json_canon,
yc_parse.h json_content_canon) and merges the batch re-staged with them (yc_engine.hip
json_rewrite) — before round 6 it refused these updates (YCRDT_E_UNSUPPORTED).

Paths: Y.applyUpdate into an empty doc and behind a doc state, Y.mergeUpdates, Y.diffUpdate (both
delete-set orders), a multi-document batch, and a large update on the chunk decoder holding every
non-canonical text of tests/golden/json_forms.json — whose result must equal that of the same
update written with Node's JSON.stringify texts (the fixture's third column).
"""
import json
import os
import sys

import pytest

crdt_amd = pytest.importorskip("crdt_amd")
from oracle.yref import Doc as ODoc  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def cases():
    sys.setrecursionlimit(max(sys.getrecursionlimit(), 20000))
    with open(os.path.join(HERE, "golden", "edges.json")) as f:
        return [c for c in json.load(f)["cases"] if c["kind"] == "json"]


@pytest.fixture(scope="module")
def pending_case():
    with open(os.path.join(HERE, "golden", "edges.json")) as f:
        return [c for c in json.load(f)["cases"] if c["kind"] == "json_pending"][0]


@pytest.fixture(scope="module")
def e135():
    e = crdt_amd.Engine(int(os.environ.get("YCRDT_DEVICE", "0")), compat=135)
    yield e
    e.close()


def _check_doc(d, c, sfx=""):
    assert d.encode_state_as_update().hex() == c["state" + sfx], (c["name"], sfx)
    assert d.encode_state_vector().hex() == c["sv" + sfx], (c["name"], sfx)
    for root, kind in c["roots"].items():
        assert json.loads(d.root_json(root, kind)) == c["json" + sfx][root], (c["name"], root, sfx)


def test_json_cases_validate_on_host(cases):
    """The host scanner (Y.applyUpdate's synchronous checks) takes every case: valid Yjs input."""
    assert len(cases) >= 6
    for c in cases:
        assert crdt_amd.validate_update(bytes.fromhex(c["update"])) == (True, True), c["name"]


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["", "chunks", "direct"])
def test_json_apply(cases, mode, monkeypatch):
    if mode:
        monkeypatch.setenv("YCRDT_DECODE", mode)
    for c in cases:
        u, base = bytes.fromhex(c["update"]), bytes.fromhex(c["base"])
        d = crdt_amd.Doc(client_id=0x7FFFFFF0)
        d.apply_update(u)
        _check_doc(d, c)
        d2 = crdt_amd.Doc(client_id=0x7FFFFFF0)
        d2.apply_updates([base, u])
        _check_doc(d2, c, "_with_base")
        d3 = crdt_amd.Doc(client_id=0x7FFFFFF0)  # behind a resident doc state
        d3.apply_update(base)
        d3.encode_state_vector()
        d3.apply_update(u)
        _check_doc(d3, c, "_with_base")


@pytest.mark.gpu
def test_json_pending(pending_case):
    """The texts in an update Yjs parks (its first item follows an item of a client not seen yet):
    Yjs writes the parked structs back re-encoded (pendingStructs, Y@21330), then integrates them
    when the dependency arrives."""
    c = pending_case
    d = crdt_amd.Doc(client_id=0x7FFFFFF0)
    d.apply_update(bytes.fromhex(c["update"]))
    assert d.encode_state_as_update().hex() == c["state_pending"]
    assert d.encode_state_vector().hex() == c["sv_pending"]
    d.apply_update(bytes.fromhex(c["dep"]))
    assert d.encode_state_as_update().hex() == c["state"]
    assert d.encode_state_vector().hex() == c["sv"]
    for root, kind in c["roots"].items():
        assert json.loads(d.root_json(root, kind)) == c["json"][root]


@pytest.mark.gpu
@pytest.mark.parametrize("compat", [136, 135])
def test_json_merge_and_diff(cases, e135, compat):
    eng = e135 if compat == 135 else None
    sfx = "_raw" if compat == 135 else ""
    for c in cases:
        u, base = bytes.fromhex(c["update"]), bytes.fromhex(c["base"])
        assert crdt_amd.merge_updates([base, u], eng).hex() == c["merged_with_base" + sfx], c["name"]
        assert crdt_amd.merge_updates([u, u], eng).hex() == c["merged_pair" + sfx], c["name"]
        assert crdt_amd.diff_update(u, b"\x00", eng).hex() == c["diff_empty" + sfx], c["name"]
        # mergeUpdates of one update returns it unchanged (Y@39011), as Yjs does
        assert crdt_amd.merge_updates([u], eng) == u


@pytest.mark.gpu
def test_json_multi_document_batch(cases):
    docs = [[bytes.fromhex(c["base"]), bytes.fromhex(c["update"])] for c in cases]
    docs.insert(1, [bytes.fromhex(cases[0]["base"])])  # a document without such values between them
    got = crdt_amd.merge_docs(docs)
    k = 0
    for i, (st, sv) in enumerate(got):
        if i == 1:
            continue
        c = cases[k]
        k += 1
        assert st.hex() == c["state_with_base"] and sv.hex() == c["sv_with_base"], c["name"]


def _vs(s: bytes) -> bytes:
    out = bytearray()
    n = len(s)
    while n > 127:
        out.append(0x80 | (n & 0x7F))
        n >>= 7
    out.append(n)
    return bytes(out) + s


def _array_update(client: int, texts) -> bytes:
    """One section of `client`: every text one ContentJSON struct of root array "messages",
    chained by origin (an older Yjs peer's YArray pushes)."""
    out = bytearray()
    out += bytes([1]) + _vu(len(texts)) + _vu(client) + _vu(0)
    for i, t in enumerate(texts):
        if i == 0:
            out += bytes([2]) + _vu(1) + _vs(b"messages")
        else:
            out += bytes([0x82]) + _vu(client) + _vu(i - 1)
        out += _vu(1) + _vs(t)
    out += bytes([0])
    return bytes(out)


def _vu(n: int) -> bytes:
    out = bytearray()
    while n > 127:
        out.append(0x80 | (n & 0x7F))
        n >>= 7
    out.append(n)
    return bytes(out)


@pytest.mark.gpu
def test_json_large_update_equals_node_stringify():
    """Every non-canonical text of json_forms.json (2 166 of them, twice; Node's JSON.stringify
    beside each) as one large update (> 64 KiB: the chunk decoder, many rewrite items in one pass): its
    merge equals the merge of the same update written with Node's texts, which the engine passes
    through unchanged."""
    with open(os.path.join(HERE, "golden", "json_forms.json")) as f:
        forms = json.load(f)["cases"]
    raw = [bytes.fromhex(h) for w, h, _ in forms if w == 2] * 2
    canon = [bytes.fromhex(c) for w, _, c in forms if w == 2] * 2
    assert len(raw) > 4000
    ua, ub = _array_update(4242, raw), _array_update(4242, canon)
    assert len(ua) > 64 * 1024
    da, db = crdt_amd.Doc(client_id=0x7FFFFFF0), crdt_amd.Doc(client_id=0x7FFFFFF0)
    da.apply_update(ua)
    db.apply_update(ub)
    sa, sb = da.encode_state_as_update(), db.encode_state_as_update()
    ref = ODoc(0x7FFFFFF0)  # canonical texts pass through: the oracle's state of Node's texts
    ref.apply_update(ub)
    assert sb == ref.encode_state_as_update()
    assert sa == sb
    assert da.root_json("messages", "array") == db.root_json("messages", "array")
    assert crdt_amd.merge_updates([ua, ub]) == crdt_amd.merge_updates([ub, ub])
    # two clients in one batch, one of each form
    uc = _array_update(4243, raw[::-1])
    ud = _array_update(4243, canon[::-1])
    assert crdt_amd.merge_updates([ua, uc]) == crdt_amd.merge_updates([ub, ud])
