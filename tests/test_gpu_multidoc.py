"""Multi-document batches (ycrdt_merge_docs / ycrdt_batch_stage_docs): many independent Y.Docs in
one device pass (config C5's topic fleet, crdt.js:235 one doc per topic; and many C2 replica sets
per pass). Each document's output must equal merging it alone: the Yjs-recorded golden states,
the C5 fleet fixtures, and single-document merges of generated C1 / C2-shaped sets."""
import json
import os
import random

import pytest

crdt_amd = pytest.importorskip("crdt_amd")

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_multidoc_golden_all_cases_one_pass(golden):
    cases = [c for s in ("kat", "map", "array", "nested") for c in golden[s]]
    docs = [[bytes.fromhex(u) for u in c["updates"]] for c in cases]
    res = crdt_amd.merge_docs(docs)
    for c, (u, sv) in zip(cases, res):
        assert u.hex() == c["state"], c["name"]
        assert sv.hex() == c["sv"], c["name"]


def test_multidoc_c5_fleet_and_empty_docs():
    with open(os.path.join(ROOT, "tests", "golden", "configs.json")) as f:
        cases = [c for c in json.load(f)["cases"]]
    docs = [[bytes.fromhex(u) for u in c["updates"]] for c in cases]
    docs.insert(3, [])                  # a document with no update at all
    docs.insert(5, [b"\x00\x00"])      # and one with only the empty update
    res = crdt_amd.merge_docs(docs)
    assert res[3] == (b"\x00\x00", b"\x00") and res[5] == (b"\x00\x00", b"\x00")
    for c, (u, sv) in zip(cases, [r for i, r in enumerate(res) if i not in (3, 5)]):
        assert u.hex() == c["state"], c["name"]


def test_multidoc_shared_clients_and_batch_api():
    """The same client ids and root names in every document must not mix across documents."""
    from crdt_amd.workload import gen_map

    docs = [gen_map(n_keys=300, n_replicas=12, ops_per_replica=60, seed=100 + i)[0] for i in range(9)]
    random.Random(1).shuffle(docs[4])
    singles = []
    for d in docs:
        b = crdt_amd.Batch(d)
        b.merge()
        singles.append(b.result())
        del b
    mb = crdt_amd.Batch(docs=docs)
    st = mb.merge()
    assert mb.result_docs() == singles
    assert st.items == sum(crdt_amd.Batch(d).merge().items for d in docs)
    with pytest.raises(crdt_amd.YcrdtError):  # other merges ran since: the workspace is not mb's any more
        mb.result_docs()
