"""Pins the CPU restatement (oracle/) against the Yjs 13.5.16 golden fixtures.

The fixtures were produced by tests/golden/gen/gen_fixtures.js from the real Yjs bundle; the
oracle must reproduce them byte for byte, in both client orders:
  compat 136 (DS/SV sorted by client desc, Yjs 13.6 — the canonical form the engine emits) and
  compat 135 (DS/SV in store-insertion order, exactly what Yjs 13.5.16 wrote).
"""
import json

import pytest

from oracle.yref import Doc, OracleError

SETS = ("kat", "map", "array", "nested")


def _cases(golden):
    for s in SETS:
        for c in golden[s]:
            yield c


def _apply(c, compat):
    d = Doc(0x7FFFFFF0, compat)
    for u in c["updates"]:
        d.apply_update(bytes.fromhex(u))
    return d


@pytest.mark.parametrize("setname", SETS)
def test_oracle_state_canonical(golden, setname):
    for c in golden[setname]:
        d = _apply(c, 136)
        assert d.encode_state_as_update().hex() == c["state"], c["name"]
        assert d.encode_state_vector().hex() == c["sv"], c["name"]


@pytest.mark.parametrize("setname", SETS)
def test_oracle_state_raw_13_5(golden, setname):
    for c in golden[setname]:
        d = _apply(c, 135)
        assert d.encode_state_as_update().hex() == c["state_raw"], c["name"]
        assert d.encode_state_vector().hex() == c["sv_raw"], c["name"]


@pytest.mark.parametrize("setname", SETS)
def test_oracle_json_and_deltas(golden, setname):
    for c in golden[setname]:
        d = _apply(c, 136)
        for root, kind in c["roots"].items():
            assert json.loads(d.root_json(root, kind)) == c["json"][root], (c["name"], root)
        for df in c["diffs"]:
            assert d.encode_state_as_update(bytes.fromhex(df["sv"])).hex() == df["update"], c["name"]


def test_oracle_kats_literal():
    # SURVEY.md App. A.6 literal bytes
    d = Doc(1)
    d.map_set("users", "user1", bytes([118, 1, 4]) + b"name" + bytes([119, 5]) + b"Alice")
    assert list(d.encode_state_as_update()) == [1, 1, 1, 0, 40, 1, 5, 117, 115, 101, 114, 115, 5, 117, 115, 101, 114, 49, 1, 118, 1, 4, 110, 97, 109, 101, 119, 5, 65, 108, 105, 99, 101, 0]
    assert list(d.encode_state_vector()) == [1, 1, 1]
    e = Doc(3)
    for i in range(5):
        e.map_set("u", "x", bytes([125, i]))
    assert list(e.encode_state_as_update()) == [1, 2, 3, 0, 33, 1, 1, 117, 1, 120, 4, 168, 3, 3, 1, 125, 4, 1, 3, 1, 0, 4]


def test_oracle_rejects_garbage():
    for bad in (b"", b"\x00", b"\x01\x05", bytes([1, 1, 1, 0, 40, 1]), b"\xff" * 8):
        d = Doc(1)
        with pytest.raises(OracleError):
            d.apply_update(bad)


def test_oracle_pending_reported():
    a = Doc(1)
    a.map_set("m", "k", bytes([125, 1]))
    sv = a.encode_state_vector()
    a.map_set("m", "k", bytes([125, 2]))
    delta = a.encode_state_as_update(sv)
    d = Doc(9)
    with pytest.raises(OracleError) as ei:
        d.apply_update(delta)
    assert ei.value.code == -2


def test_oracle_local_ops_pinned():
    """The oracle's local ops (typeMapSet / typeListInsertGenerics / typeListDelete restated) replay
    the root-type Yjs op scripts of tests/golden/ops.json byte for byte after every step."""
    import json
    import os

    with open(os.path.join(os.path.dirname(__file__), "golden", "ops.json")) as f:
        cases = [c for c in json.load(f)["cases"] if c["name"].startswith("ops_root_")]
    assert len(cases) == 20
    for c in cases:
        d = Doc(c["client"])
        for i, s in enumerate(c["steps"]):
            op = s["op"]
            if op == "apply":
                d.apply_update(bytes.fromhex(s["update"]))
            elif op == "map_set":
                d.map_set(s["root"], s["key"], bytes.fromhex(s["any"]))
            elif op == "map_delete":
                d.map_delete(s["root"], s["key"])
            elif op == "array_insert":
                d.array_insert(s["root"], s["index"], [bytes.fromhex(a) for a in s["anys"]])
            elif op == "array_delete":
                d.array_delete(s["root"], s["index"], s["length"])
            assert d.encode_state_as_update().hex() == s["state"], (c["name"], i, op)
        assert json.loads(d.root_json("users", "map")) == c["json"]["users"], c["name"]
        assert json.loads(d.root_json("messages", "array")) == c["json"]["messages"], c["name"]


def test_oracle_config_fixtures():
    """Reduced-scale C3 / C4 / C5 cases played through Yjs 13.5.16 (tests/golden/configs.json)."""
    import json as _json
    import os as _os

    from oracle.yref import Doc as _Doc

    with open(_os.path.join(_os.path.dirname(__file__), "golden", "configs.json")) as f:
        cases = _json.load(f)["cases"]
    for c in cases:
        d = _Doc(0x7FFFFFF0)
        for u in c["updates"]:
            d.apply_update(bytes.fromhex(u))
        assert d.encode_state_as_update().hex() == c["state"], c["name"]
        assert d.encode_state_vector().hex() == c["sv"], c["name"]
        for df in c["diffs"]:
            assert d.encode_state_as_update(bytes.fromhex(df["sv"])).hex() == df["update"], c["name"]
        for root, val in c["json"].items():
            kind = "array" if isinstance(val, list) else "map"
            assert _json.loads(d.root_json(root, kind)) == val, (c["name"], root)


def _edges():
    import json as _json
    import os as _os
    import sys as _sys

    _sys.setrecursionlimit(max(_sys.getrecursionlimit(), 20000))  # 2 000-level JSON values
    with open(_os.path.join(_os.path.dirname(__file__), "golden", "edges.json")) as f:
        # (the "json" cases — ContentJSON texts Yjs rewrites with JSON.stringify — are pinned on the
        # GPU side against the fixture itself, test_gpu_json_rewrite.py; the oracle copies such texts)
        return [c for c in _json.load(f)["cases"] if not c["kind"].startswith("json")]


def test_oracle_edge_fixtures_apply():
    """Deep `any` values and non-canonical section layouts (tests/golden/edges.json, Yjs 13.5.16):
    Y.applyUpdate results."""
    import json as _json

    checked = 0
    for c in _edges():
        groups = [(c["updates"], "")] if c["kind"] == "deep" else [([c["update"]], ""), ([c["update"]] + c["others"], "_with_others")]
        for ups, sfx in groups:
            d = Doc(0x7FFFFFF0)
            try:
                for u in ups:
                    d.apply_update(bytes.fromhex(u))
            except OracleError as e:  # the oracle has no pending store: those are pinned on the GPU
                assert e.code == -2, (c["name"], sfx)  # side against the fixture (test_gpu_edges_fixtures)
                continue
            checked += 1
            assert d.encode_state_as_update().hex() == c["state" + sfx], (c["name"], sfx)
            assert d.encode_state_vector().hex() == c["sv" + sfx], (c["name"], sfx)
            for root, kind in c["roots"].items():
                assert _json.loads(d.root_json(root, kind)) == c["json" + sfx][root], (c["name"], root)
    assert checked >= 10


def test_oracle_edge_fixtures_lazy():
    """The same inputs through mergeUpdates / diffUpdate (oracle/ymerge.py), Yjs's raw bytes."""
    from oracle.ymerge import diff_update, merge_updates

    for c in _edges():
        if c["kind"] == "deep":
            ups = [bytes.fromhex(u) for u in c["updates"]]
            assert merge_updates(ups).hex() == c["merged_raw"], c["name"]
            continue
        x = bytes.fromhex(c["update"])
        others = [bytes.fromhex(u) for u in c["others"]]
        assert merge_updates([x] + others).hex() == c["merged_with_others_raw"], c["name"]
        assert merge_updates(others + [x]).hex() == c["merged_others_first_raw"], c["name"]
        assert merge_updates([x, x]).hex() == c["merged_pair_raw"], c["name"]
        assert diff_update(x, b"\x00").hex() == c["diff_empty_raw"], c["name"]
        assert diff_update(x, bytes.fromhex(c["diff_sv_of"])).hex() == c["diff_sv_raw"], c["name"]
        assert diff_update(x, bytes.fromhex(c["diff_hi1_of"])).hex() == c["diff_hi1_raw"], c["name"]
