"""GPU parity of the crdt.c path: materialised toJSON and local ops, through the C ABI.

* toJSON of every root of every Yjs golden case (tests/golden/{kat,map,array,nested}.json hold the
  real Yjs 13.5.16 `toJSON()`), computed from the device view (map winners, YArray list ranking).
* Local-op scripts recorded from Yjs 13.5.16 (tests/golden/ops.json, gen_ops_fixtures.js): YMap
  set / delete, set(key, new Y.Array()) + push / unshift / insert / delete on nested arrays, the
  same on a root YArray, interleaved with remote deltas. After EVERY step the doc's
  encodeStateAsUpdate must be byte-identical to the Yjs doc's (13.6 canonical order).
"""
import json
import os

import pytest

crdt_amd = pytest.importorskip("crdt_amd")

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("setname", ["kat", "map", "array", "nested"])
def test_gpu_json_golden(golden, setname):
    for c in golden[setname]:
        d = crdt_amd.Doc(client_id=0x7FFFFFF0)
        d.apply_updates([bytes.fromhex(u) for u in c["updates"]])
        for root, kind in c["roots"].items():
            got = json.loads(d.root_json(root, kind))
            assert got == c["json"][root], (c["name"], root)


def test_gpu_json_empty_doc():
    d = crdt_amd.Doc(client_id=1)
    assert d.root_json("users", "map") == "{}"
    assert d.root_json("messages", "array") == "[]"


def _ops():
    with open(os.path.join(HERE, "golden", "ops.json")) as f:
        return json.load(f)["cases"]


def _step(d, s):
    op = s["op"]
    pk = s.get("parent_key")
    if op == "apply":
        d.apply_update(bytes.fromhex(s["update"]))
    elif op == "map_set":
        d.map_set(s["root"], s["key"], bytes.fromhex(s["any"]))
    elif op == "map_set_type":
        d.map_set_type(s["root"], s["key"], s["type"])
    elif op == "map_delete":
        d.map_delete(s["root"], s["key"])
    elif op == "array_insert":
        d.array_insert(s["root"], s["index"], [bytes.fromhex(a) for a in s["anys"]], parent_key=pk)
    elif op == "array_delete":
        d.array_delete(s["root"], s["index"], s["length"], parent_key=pk)
    else:
        raise AssertionError(op)


@pytest.mark.parametrize("chunk", range(4))
def test_gpu_local_ops_yjs(chunk):
    """Every step of every recorded Yjs op script, byte for byte, then the final toJSON."""
    cases = _ops()[chunk::4]
    for c in cases:
        d = crdt_amd.Doc(client_id=c["client"])
        for i, s in enumerate(c["steps"]):
            _step(d, s)
            assert d.encode_state_as_update().hex() == s["state"], (c["name"], i, s["op"])
        assert json.loads(d.root_json("users", "map")) == c["json"]["users"], c["name"]
        assert json.loads(d.root_json("messages", "array")) == c["json"]["messages"], c["name"]


def test_gpu_local_op_errors():
    d = crdt_amd.Doc(client_id=3)
    with pytest.raises(crdt_amd.YcrdtError, match="Length exceeded"):
        d.array_insert("messages", 1, [b"\x7d\x01"])
    d.array_insert("messages", 0, [b"\x7d\x01", b"\x7d\x02"])
    with pytest.raises(crdt_amd.YcrdtError, match="Length exceeded"):
        d.array_delete("messages", 1, 5)  # deletes element 1, then throws, as Yjs does
    assert json.loads(d.root_json("messages", "array")) == [1]
    with pytest.raises(crdt_amd.YcrdtError):
        d.map_set("users", "k", b"\xff")  # not a lib0 any value
    with pytest.raises(crdt_amd.YcrdtError):
        d.array_insert("users", 0, [b"\x7d\x01"], parent_key="nolist")  # no shared type there
    d.map_delete("users", "absent")  # a no-op, no struct written
    assert json.loads(d.root_json("users", "map")) == {}


@pytest.mark.parametrize("every", [1, 3])
def test_gpu_local_delta_replay(every):
    """Incremental local-op encode (ycrdt_doc_take_local_update): a peer that receives only the
    local-op deltas (one op, or the merge of up to `every` ops) plus the same remote updates
    reaches the Yjs-recorded state bytes, wherever a delta has been delivered."""
    for c in _ops()[::3]:
        a = crdt_amd.Doc(client_id=c["client"])
        a.track_local(True)  # the host opted in to delta broadcast
        b = crdt_amd.Doc(client_id=0x7FFFFFF1)
        pending = 0
        for i, s in enumerate(c["steps"]):
            _step(a, s)
            if s["op"] == "apply":
                if pending:
                    b.apply_update(a.take_local_update())
                    pending = 0
                b.apply_update(bytes.fromhex(s["update"]))
            else:
                pending += 1
                if pending >= every or i == len(c["steps"]) - 1:
                    b.apply_update(a.take_local_update())
                    pending = 0
            if not pending:
                assert b.encode_state_as_update().hex() == s["state"], (c["name"], i, s["op"])
        assert a.take_local_update() == b"\x00\x00"  # nothing new since the last take


def test_local_ops_untracked_stay_bounded():
    """Without delta tracking, local ops record nothing (the list used to grow for the
    doc's lifetime); a take then turns tracking on for the ops that follow."""
    d = crdt_amd.Doc(client_id=77)
    for i in range(50):
        d.map_set("users", f"k{i % 5}", bytes([125, i]))
    assert d.take_local_update() == b"\x00\x00"
    d.map_set("users", "k0", bytes([125, 99]))
    u = d.take_local_update()
    peer = crdt_amd.Doc(client_id=78)
    peer.apply_update(u)
    assert peer.pending()[0]  # the op's origin is an item the peer never received
