"""compat=135 on the GPU path: Yjs 13.5.16's own bytes, client order included.

13.5.16 writes a doc's delete set and state vector in store insertion order (createDeleteSetFromStructStore
/ getStateVector iterate store.clients, Y@10800 / Y@22723), and a merged / diffed update's delete set in
Map insertion order (first appearance, mergeDeleteSets / readDeleteSet, Y@11105). An engine created
with compat=135 reproduces those raw fixture fields (`state_raw`, `sv_raw`, `merged_raw`, the raw
merge.json vectors, pending.json's raw state / delta after every out-of-order apply); compat=136 (the
default) emits the 13.6 canonical descending order that the other GPU tests pin.
"""
import json
import os

import pytest

crdt_amd = pytest.importorskip("crdt_amd")

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SETS = ("kat", "map", "array", "nested")


@pytest.fixture(scope="module")
def e135():
    e = crdt_amd.Engine(int(os.environ.get("YCRDT_DEVICE", "0")), compat=135)
    yield e
    e.close()


def _load(name):
    with open(os.path.join(ROOT, "tests", "golden", name)) as f:
        return json.load(f)["cases"]


@pytest.mark.parametrize("setname", SETS)
def test_135_state_and_sv_raw(golden, setname, e135):
    """Fresh doc, the case's updates applied one at a time (as the generator did), raw bytes."""
    for c in golden[setname]:
        d = crdt_amd.Doc(client_id=0x7FFFFFF0, engine=e135)
        for u in c["updates"]:
            d.apply_update(bytes.fromhex(u))
        assert d.encode_state_as_update().hex() == c["state_raw"], c["name"]
        assert d.encode_state_vector().hex() == c["sv_raw"], c["name"]


@pytest.mark.parametrize("setname", SETS)
def test_135_deltas_vs_oracle(golden, setname, e135):
    """Deltas against each fixture target state vector, vs the 135 oracle (pinned by state_raw)."""
    from oracle.yref import Doc

    for c in golden[setname]:
        d = crdt_amd.Doc(client_id=0x7FFFFFF0, engine=e135)
        o = Doc(0x7FFFFFF0, 135)
        for u in c["updates"]:
            d.apply_update(bytes.fromhex(u))
            o.apply_update(bytes.fromhex(u))
        for df in c["diffs"]:
            sv = bytes.fromhex(df["sv"])
            assert d.encode_state_as_update(sv) == o.encode_state_as_update(sv), (c["name"], df["sv"])


@pytest.mark.parametrize("setname", SETS)
def test_135_merge_updates_raw(golden, setname, e135):
    for c in golden[setname]:
        ups = [bytes.fromhex(u) for u in c["updates"]]
        assert crdt_amd.merge_updates(ups, engine=e135).hex() == c["merged_raw"], c["name"]


def test_135_merge_reverse_pair_and_diff_raw(golden, e135):
    cases = {c["name"]: c for s in SETS for c in golden[s]}
    for m in _load("merge.json"):
        ups = [bytes.fromhex(u) for u in cases[m["name"]]["updates"]]
        assert crdt_amd.merge_updates(list(reversed(ups)), engine=e135).hex() == m["rev"], m["name"]
        if "pair" in m:
            assert crdt_amd.merge_updates(ups[:2], engine=e135).hex() == m["pair"], m["name"]
        merged = crdt_amd.merge_updates(ups, engine=e135)
        srcs, svs, want = [], [], []
        for d in m["diffs"]:
            src = merged if d["src"] == "merged" else ups[0]
            got = crdt_amd.diff_update(src, bytes.fromhex(d["sv"]), engine=e135)
            assert got.hex() == d["out"], (m["name"], d["src"], d["sv"])
            srcs.append(src)
            svs.append(bytes.fromhex(d["sv"]))
            want.append(d["out"])
        # the batched per-update diff (sync responder) keeps each update's own first-appearance order
        got = crdt_amd.diff_updates(srcs, svs, engine=e135)
        assert [g.hex() for g in got] == want, m["name"]


@pytest.mark.parametrize("part", range(3))
def test_135_pending_every_step_raw(part, e135):
    """Out-of-order applies: 13.5.16's raw state, raw state vector and raw delta after every apply."""
    for c in _load("pending.json")[part::3]:
        d = crdt_amd.Doc(client_id=0x7FFFFFF0, engine=e135)
        for k, (u, st) in enumerate(zip(c["updates"], c["steps"])):
            d.apply_update(bytes.fromhex(u))
            tag = (c["name"], k)
            assert d.pending() == (st["pending"], st["pending_ds"]), tag
            assert d.encode_state_as_update().hex() == st["state_raw"], tag
            assert d.encode_state_vector().hex() == st["sv_raw"], tag
            if "delta" in st:
                got = d.encode_state_as_update(bytes.fromhex(st["delta"]["sv"]))
                assert got.hex() == st["delta"]["update_raw"], tag
