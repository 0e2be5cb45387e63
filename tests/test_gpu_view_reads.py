"""Per-key reads of the materialised view (YMap.get / has / size, YArray.length / get) agree with
the type's toJSON on every Yjs golden case and on docs built by local ops, nested types included.
These replace the facade's full toJSON + JSON.parse per call (crdt_amd/js/index.js)."""
import json

import pytest

crdt_amd = pytest.importorskip("crdt_amd")

pytestmark = pytest.mark.gpu


def _check_doc(d, roots, tag):
    for name, kind in roots.items():
        full = json.loads(d.root_json(name, kind))
        if kind == "map":
            assert d.map_size(name) >= len(full), tag  # size also counts entries whose value is undefined
            for k, v in full.items():
                st, j = d.map_get(name, k)
                tr = d.map_type_at(name, k)
                if tr == 1:  # a Y.Map under this key reads through its parent key
                    assert d.map_size(name, parent_key=k) == len(v), (tag, k)
                    for kk, vv in v.items():
                        st2, j2 = d.map_get(name, kk, parent_key=k)
                        assert st2 == 1 and json.loads(j2) == vv, (tag, k, kk)
                if tr >= 0:
                    continue  # shared types are handed out as objects by the facade
                assert st == 1 and json.loads(j) == v, (tag, k)
            assert d.map_get(name, "\u0000absent")[0] == 0, tag
        else:
            assert d.array_length(name) == len(full), tag
            for i, v in enumerate(full):
                st, j = d.array_get(name, i)
                assert st in (1, 2), (tag, i)
                assert (json.loads(j) if st == 1 else None) == v, (tag, i)
            assert d.array_get(name, len(full))[0] == 0, tag


@pytest.mark.parametrize("setname", ["kat", "map", "array", "nested"])
def test_reads_match_tojson_golden(golden, setname):
    for c in golden[setname]:
        d = crdt_amd.Doc(client_id=0x7FFFFFF0)
        d.apply_updates([bytes.fromhex(u) for u in c["updates"]])
        _check_doc(d, c["roots"], c["name"])
        # nested arrays under map keys: length / get through the parent key
        for name, kind in c["roots"].items():
            if kind != "map":
                continue
            full = json.loads(d.root_json(name, kind))
            for k, v in full.items():
                if isinstance(v, list) and d.map_type_at(name, k) == 0:
                    assert d.array_length(name, parent_key=k) == len(v), (c["name"], k)
                    for i, x in enumerate(v):
                        st, j = d.array_get(name, i, parent_key=k)
                        assert (json.loads(j) if st == 1 else None) == x, (c["name"], k, i)


def _any_str(v):
    b = v.encode()
    return bytes([119, len(b)]) + b


def test_reads_after_local_ops():
    d = crdt_amd.Doc(client_id=5)
    for i in range(40):
        d.map_set("users", "u%d" % (i % 7), _any_str("v%d" % i))
        if i % 6 == 5:
            d.map_delete("users", "u%d" % (i % 7))
        st, j = d.map_get("users", "u%d" % (i % 7))
        want = json.loads(d.root_json("users", "map")).get("u%d" % (i % 7))
        assert (json.loads(j) if st == 1 else None) == want
    d.map_set_type("docs", "list", 0)
    for i in range(10):
        d.array_insert("docs", d.array_length("docs", parent_key="list"), [bytes([125, i])], parent_key="list")
    assert d.array_length("docs", parent_key="list") == 10
    assert [json.loads(d.array_get("docs", i, parent_key="list")[1]) for i in range(10)] == list(range(10))
    _check_doc(d, {"users": "map"}, "local")


def test_two_docs_one_engine_per_op_loop():
    """crdt.js's per-op loop (bench.py per_op_leg) with both peers writing, on ONE engine: every
    merge of one doc takes the engine workspace from the other, and a doc read through its view
    gets the view built beside its merge (yc_engine.hip commit_merge). Both peers' toJSON, per-key
    reads and encoded states match the oracle's two docs fed the same calls."""
    from oracle.yref import Doc as ODoc
    from tests.v1util import canonical_update

    eng = crdt_amd.default_engine()
    g = [crdt_amd.Doc(client_id=1, engine=eng), crdt_amd.Doc(client_id=2, engine=eng)]
    o = [ODoc(client_id=1), ODoc(client_id=2)]
    for i in range(60):
        w, r = i % 2, 1 - i % 2  # the writer alternates
        key = "user%d" % (i % 9)
        if i % 5 == 4:
            g[w].map_delete("users", key)
            o[w].map_delete("users", key)
        else:
            v = _any_str("v%d" % i)
            g[w].map_set("users", key, v)
            o[w].map_set("users", key, v)
        u = g[w].encode_state_as_update()
        assert canonical_update(u) == canonical_update(o[w].encode_state_as_update()), i
        g[r].apply_update(u)
        o[r].apply_update(u)
        for d, od in zip(g, o):
            assert json.loads(d.root_json("users", "map")) == json.loads(od.root_json("users", "map")), i
        st, j = g[r].map_get("users", key)
        want = json.loads(o[r].root_json("users", "map")).get(key)
        assert (json.loads(j) if st == 1 else None) == want, i
    _check_doc(g[0], {"users": "map"}, "peer0")
    _check_doc(g[1], {"users": "map"}, "peer1")
