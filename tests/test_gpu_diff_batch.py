"""Batched sync responder: n x Y.diffUpdate(update_i, sv_i) in one device pass
(`ycrdt_diff_updates`, crdt.js:286-291 `Y.encodeStateAsUpdate(doc, peerSV)` per joining peer,
batched across peers and topics).

Every output must equal the single-pair path and the oracle's diffUpdate (oracle/ymerge.py, pinned
by the Yjs 13.5.16 vectors in tests/golden/merge.json), in any batch order and mixed with empty,
delete-set-only and fully covered pairs."""
import json
import os
import random

import pytest

crdt_amd = pytest.importorskip("crdt_amd")
from oracle.ymerge import diff_update, merge_updates  # noqa: E402
from tests.histories import array_history  # noqa: E402
from tests.v1util import canonical_update  # noqa: E402

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _golden_pairs(golden):
    cases = {c["name"]: c for s in ("kat", "map", "array", "nested") for c in golden[s]}
    with open(os.path.join(HERE, "golden", "merge.json")) as f:
        vecs = json.load(f)["cases"]
    pairs = []
    for m in vecs:
        ups = [bytes.fromhex(u) for u in cases[m["name"]]["updates"]]
        merged = merge_updates(ups)
        for d in m["diffs"]:
            src = merged if d["src"] == "merged" else ups[0]
            pairs.append((src, bytes.fromhex(d["sv"]), canonical_update(bytes.fromhex(d["out"]))))
    return pairs


def test_diff_batch_golden(golden):
    pairs = _golden_pairs(golden)
    assert len(pairs) > 50
    got = crdt_amd.diff_updates([p[0] for p in pairs], [p[1] for p in pairs])
    for (src, sv, want), g in zip(pairs, got):
        assert g == want, (src.hex()[:40], sv.hex())
    # any batch order gives the same per-pair bytes
    order = list(range(len(pairs)))
    random.Random(7).shuffle(order)
    got2 = crdt_amd.diff_updates([pairs[i][0] for i in order], [pairs[i][1] for i in order])
    for k, i in enumerate(order):
        assert got2[k] == pairs[i][2]


def test_diff_batch_config_fleet():
    """C5-shaped: many small docs, each diffed against every lagging peer state vector."""
    with open(os.path.join(HERE, "golden", "configs.json")) as f:
        cases = [c for c in json.load(f)["cases"] if c["name"].startswith("c5_")]
    ups, svs = [], []
    for c in cases:
        state = bytes.fromhex(c["state"])
        for df in c["diffs"]:
            ups.append(state)
            svs.append(bytes.fromhex(df["sv"]))
        ups.append(state)
        svs.append(b"\x00")  # a fresh joiner: the whole doc
    got = crdt_amd.diff_updates(ups, svs)
    for u, sv, g in zip(ups, svs, got):
        assert g == canonical_update(diff_update(u, sv))
        assert g == crdt_amd.diff_update(u, sv)


@pytest.mark.parametrize("seed", range(4))
def test_diff_batch_random_vs_oracle(seed):
    from oracle.yref import Doc

    rng = random.Random(seed)
    ups, svs = [], []
    for k in range(5):
        states, wire = array_history(300 + 10 * seed + k, n_replicas=3 + k % 3, rounds=3, ops=6, with_map=True)
        merged = merge_updates(states + wire)
        cand = [merged] + states[:2] + wire[:3]
        svl = [b"\x00"]
        for st in states:
            d = Doc(1)
            d.apply_update(st)
            svl.append(d.encode_state_vector())
        d = Doc(1)
        d.apply_update(merged)
        svl.append(d.encode_state_vector())  # fully covered: structs empty, delete set kept
        for _ in range(12):
            ups.append(rng.choice(cand))
            svs.append(rng.choice(svl))
    ups.append(b"\x00\x00")
    svs.append(b"\x00")
    got = crdt_amd.diff_updates(ups, svs)
    assert len(got) == len(ups)
    for u, sv, g in zip(ups, svs, got):
        assert g == canonical_update(diff_update(u, sv))


def test_diff_batch_edges():
    assert crdt_amd.diff_updates([], []) == []
    states, _ = array_history(77, n_replicas=2, rounds=1, ops=3, with_map=False)
    with pytest.raises(Exception):
        crdt_amd.diff_updates([states[0], b"\x05\xff"], [b"\x00", b"\x00"])  # one malformed update fails the batch
    with pytest.raises(Exception):
        crdt_amd.diff_updates([states[0]], [b"\x03"])  # truncated state vector
    # the engine is still usable after a refused batch
    assert crdt_amd.diff_updates([states[0]], [b"\x00"]) == [canonical_update(diff_update(states[0], b"\x00"))]
