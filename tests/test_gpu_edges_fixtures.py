"""Valid Yjs input at the edges, on the GPU path, against Yjs 13.5.16 itself
(tests/golden/edges.json, tests/golden/gen/gen_edge_fixtures.js):

* `any` values nested up to 2 000 levels (lib0 readAny has no depth limit; crdt.js stores whatever
  JSON the user sets, crdt.js:434): apply, toJSON and mergeUpdates;
* updates whose struct section holds two sections of one client, or sections in ascending client
  order — layouts Yjs never writes but reads: Y.applyUpdate (the last section of a client wins,
  readClientsStructRefs Y@19286), Y.mergeUpdates (the lazy readers' loop, Y@39011 — the engine's
  serial k_lz_merge_seq) and Y.diffUpdate (runs of one client, Y@40711).

compat 136 (default) must give the canonical (13.6 delete-set order) bytes, compat 135 Yjs's raw
bytes.
"""
import json
import os
import sys

import pytest

crdt_amd = pytest.importorskip("crdt_amd")

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def edges():
    sys.setrecursionlimit(max(sys.getrecursionlimit(), 20000))  # 2 000-level JSON values
    with open(os.path.join(HERE, "golden", "edges.json")) as f:
        return json.load(f)["cases"]


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


def test_deep_any_apply_and_json(edges):
    for c in edges:
        if c["kind"] != "deep":
            continue
        ups = [bytes.fromhex(u) for u in c["updates"]]
        d = crdt_amd.Doc(client_id=0x7FFFFFF0)
        d.apply_updates(ups)
        _check_doc(d, c)
        d2 = crdt_amd.Doc(client_id=0x7FFFFFF0)
        for u in ups:
            d2.apply_update(u)
        _check_doc(d2, c)
        st, val = d.map_get("users", "obj2000")
        assert st == 1 and val.startswith('{"a":{"a":')


def test_deep_any_merge_updates(edges, e135):
    for c in edges:
        if c["kind"] != "deep":
            continue
        ups = [bytes.fromhex(u) for u in c["updates"]]
        assert crdt_amd.merge_updates(ups).hex() == c["merged"], c["name"]
        assert crdt_amd.merge_updates(ups, e135).hex() == c["merged_raw"], c["name"]
        # the merged update applies to the same state
        d = crdt_amd.Doc(client_id=0x7FFFFFF0)
        d.apply_update(crdt_amd.merge_updates(ups))
        _check_doc(d, c)


def _sections(edges):
    return [c for c in edges if c["kind"] == "sections"]


def test_sections_apply(edges):
    for c in _sections(edges):
        x = bytes.fromhex(c["update"])
        others = [bytes.fromhex(u) for u in c["others"]]
        d = crdt_amd.Doc(client_id=0x7FFFFFF0)
        d.apply_update(x)
        _check_doc(d, c)
        d.apply_updates(others)
        _check_doc(d, c, "_with_others")
        d2 = crdt_amd.Doc(client_id=0x7FFFFFF0)
        d2.apply_updates([x] + others)
        _check_doc(d2, c, "_with_others")


@pytest.mark.parametrize("compat", [136, 135])
def test_sections_merge_and_diff(edges, e135, compat):
    eng = e135 if compat == 135 else None
    sfx = "_raw" if compat == 135 else ""
    for c in _sections(edges):
        x = bytes.fromhex(c["update"])
        others = [bytes.fromhex(u) for u in c["others"]]
        tag = (c["name"], compat)
        assert crdt_amd.merge_updates([x] + others, eng).hex() == c["merged_with_others" + sfx], tag
        assert crdt_amd.merge_updates(others + [x], eng).hex() == c["merged_others_first" + sfx], tag
        assert crdt_amd.merge_updates([x, x], eng).hex() == c["merged_pair" + sfx], tag
        assert crdt_amd.diff_update(x, b"\x00", eng).hex() == c["diff_empty" + sfx], tag
        assert crdt_amd.diff_update(x, bytes.fromhex(c["diff_sv_of"]), eng).hex() == c["diff_sv" + sfx], tag
        assert crdt_amd.diff_update(x, bytes.fromhex(c["diff_hi1_of"]), eng).hex() == c["diff_hi1" + sfx], tag


def test_sections_batched_diff(edges):
    """The sync responder's batch (ycrdt_diff_updates): the same pairs in one device pass."""
    ups, svs, want = [], [], []
    for c in _sections(edges):
        x = bytes.fromhex(c["update"])
        for sv_key, out_key in (("diff_sv_of", "diff_sv"), ("diff_hi1_of", "diff_hi1")):
            ups.append(x)
            svs.append(bytes.fromhex(c[sv_key]))
            want.append(c[out_key])
    got = crdt_amd.diff_updates(ups, svs)
    assert [g.hex() for g in got] == want
