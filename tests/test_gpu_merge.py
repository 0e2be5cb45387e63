"""GPU Y.mergeUpdates / Y.diffUpdate vs the Yjs 13.5.16 vectors (canonical 13.6 client order of
the delete set) and vs the restated oracle (oracle/ymerge.py) on random histories."""
import json
import os
import random

import pytest

crdt_amd = pytest.importorskip("crdt_amd")
from oracle.ymerge import diff_update, merge_updates  # noqa: E402
from tests.histories import array_history  # noqa: E402
from tests.v1util import canonical_update  # noqa: E402

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("setname", ["kat", "map", "array", "nested"])
def test_gpu_merge_updates_golden(golden, setname):
    for c in golden[setname]:
        ups = [bytes.fromhex(u) for u in c["updates"]]
        got = crdt_amd.merge_updates(ups)
        want = c["merged"] if len(ups) > 1 else c["merged_raw"]
        assert got.hex() == want, c["name"]


def test_gpu_merge_reverse_pair_and_diff(golden):
    cases = {c["name"]: c for s in ("kat", "map", "array", "nested") for c in golden[s]}
    with open(os.path.join(ROOT, "tests", "golden", "merge.json")) as f:
        vecs = json.load(f)["cases"]
    for m in vecs:
        ups = [bytes.fromhex(u) for u in cases[m["name"]]["updates"]]
        if len(ups) > 1:
            assert crdt_amd.merge_updates(list(reversed(ups))) == canonical_update(bytes.fromhex(m["rev"])), m["name"]
        if "pair" in m:
            assert crdt_amd.merge_updates(ups[:2]) == canonical_update(bytes.fromhex(m["pair"])), m["name"]
        merged = merge_updates(ups)
        for d in m["diffs"]:
            src = merged if d["src"] == "merged" else ups[0]
            got = crdt_amd.diff_update(src, bytes.fromhex(d["sv"]))
            assert got == canonical_update(bytes.fromhex(d["out"])), (m["name"], d["src"], d["sv"])


@pytest.mark.parametrize("seed", range(6))
def test_gpu_merge_random_vs_oracle(seed):
    states, wire = array_history(100 + seed, n_replicas=3 + seed, rounds=3, ops=6, with_map=True)
    batch = states + wire
    random.Random(seed).shuffle(batch)
    assert crdt_amd.merge_updates(batch) == canonical_update(merge_updates(batch))
    merged = crdt_amd.merge_updates(batch)
    for st in states[:2]:
        from oracle.yref import Doc

        d = Doc(1)
        d.apply_update(st)
        sv = d.encode_state_vector()
        assert crdt_amd.diff_update(merged, sv) == canonical_update(diff_update(merged, sv))
