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


def test_multidoc_packed_result_golden_and_large(golden):
    """ycrdt_batch_result_docs_packed: the device-side split packed back to back in one host array
    (pipelined D2H) gives every document's Yjs state and state vector; a multi-chunk batch (the
    112-document C2 shape, reduced) equals the per-document result."""
    from crdt_amd.workload import gen_map

    cases = [c for s in ("kat", "map", "array", "nested") for c in golden[s]]
    docs = [[bytes.fromhex(u) for u in c["updates"]] for c in cases]
    docs.insert(2, [])
    b = crdt_amd.Batch(docs=docs)
    b.merge()
    blob, offs = b.result_docs_packed()
    assert len(offs) == 2 * len(docs) + 1 and int(offs[-1]) == len(blob)
    got = [(bytes(blob[offs[2 * d]:offs[2 * d + 1]]), bytes(blob[offs[2 * d + 1]:offs[2 * d + 2]])) for d in range(len(docs))]
    assert got[2] == (b"\x00\x00", b"\x00")
    for c, (u, sv) in zip(cases, got[:2] + got[3:]):
        assert u.hex() == c["state"], c["name"]
        assert sv.hex() == c["sv"], c["name"]
    big = [gen_map(n_keys=20000, n_replicas=200, ops_per_replica=400, seed=700 + i)[0] for i in range(6)]
    os.environ["YCRDT_PIN_CHUNK"] = "65536"  # staging waves in both halves on a few MB
    try:
        b = crdt_amd.Batch(docs=big)
        b.merge()
        blob, offs = b.result_docs_packed()
    finally:
        del os.environ["YCRDT_PIN_CHUNK"]
    assert len(blob) > 2 * 16 * 65536
    per = b.result_docs()
    for d in range(len(big)):
        assert bytes(blob[offs[2 * d]:offs[2 * d + 1]]) == per[d][0]
        assert bytes(blob[offs[2 * d + 1]:offs[2 * d + 2]]) == per[d][1]
    one = crdt_amd.Batch(big[0])
    one.merge()
    blob1, offs1 = one.result_docs_packed()
    assert (bytes(blob1[:offs1[1]]), bytes(blob1[offs1[1]:offs1[2]])) == one.result()


def test_staging_beside_merges_serving_loop():
    """The serving loop of bench.py end_to_end: a second host thread stages batch k+1 (copy stream,
    its own pinned area) while batch k merges and returns its packed result into a reused buffer;
    every batch equals its sequential merge. Multi-wave staging (YCRDT_PIN_CHUNK) on a few MB."""
    from concurrent.futures import ThreadPoolExecutor

    from crdt_amd.workload import gen_map

    sets = [[gen_map(n_keys=3000, n_replicas=40, ops_per_replica=200, seed=900 + 7 * k + i)[0] for i in range(5)]
            for k in range(4)]
    eng = crdt_amd.Engine()
    want = []
    for docs in sets:
        b = crdt_amd.Batch(docs=docs, engine=eng)
        b.merge()
        want.append(b.result_docs())
        del b
    os.environ["YCRDT_PIN_CHUNK"] = "65536"
    try:
        got, buf = [], None
        with ThreadPoolExecutor(1) as stager:
            nxt = stager.submit(lambda: crdt_amd.Batch(docs=sets[0], engine=eng))
            for k in range(len(sets)):
                b = nxt.result()
                if k + 1 < len(sets):
                    nxt = stager.submit(lambda d=sets[k + 1]: crdt_amd.Batch(docs=d, engine=eng))
                b.merge()
                blob, offs = b.result_docs_packed(out=buf)
                got.append([(bytes(blob[offs[2 * d]:offs[2 * d + 1]]), bytes(blob[offs[2 * d + 1]:offs[2 * d + 2]]))
                            for d in range(len(sets[k]))])
                buf = blob.base if blob.base is not None else blob
                del b
    finally:
        del os.environ["YCRDT_PIN_CHUNK"]
    assert got == want


# ---------------------------------------------------------------- fleet ingest (apply_updates_multi)
def _interleaved(cases, rng):
    """(doc index, update) pairs of every case, interleaved across documents, per-doc order kept."""
    queues = [[bytes.fromhex(u) for u in c["updates"]] for c in cases]
    pos = [0] * len(queues)
    out = []
    live = [i for i, q in enumerate(queues) if q]
    while live:
        i = rng.choice(live)
        out.append((i, queues[i][pos[i]]))
        pos[i] += 1
        if pos[i] == len(queues[i]):
            live.remove(i)
    return out


def test_apply_multi_golden_fleet(golden):
    """Every golden case is one document; all their updates arrive interleaved in ONE call."""
    cases = [c for s in ("kat", "map", "array", "nested") for c in golden[s]]
    docs = [crdt_amd.Doc(client_id=0x7FFFFFF0) for _ in cases]
    pairs = _interleaved(cases, random.Random(3))
    crdt_amd.apply_updates_multi([docs[i] for i, _ in pairs], [u for _, u in pairs])
    for c, d in zip(cases, docs):
        assert d.encode_state_as_update().hex() == c["state"], c["name"]
        assert d.encode_state_vector().hex() == c["sv"], c["name"]
        for name, kind in c["roots"].items():
            assert json.loads(d.root_json(name, kind)) == c["json"][name], c["name"]


def test_apply_multi_in_rounds_and_reads_between(golden):
    """Several ingest calls on the same fleet, reads and local ops in between (state stays in HBM)."""
    cases = [c for s in ("map", "nested") for c in golden[s]][:30]
    docs = [crdt_amd.Doc(client_id=0x7FFFFFF0) for _ in cases]
    pairs = _interleaved(cases, random.Random(5))
    k = len(pairs) // 3
    for part in (pairs[:k], pairs[k:2 * k], pairs[2 * k:]):
        crdt_amd.apply_updates_multi([docs[i] for i, _ in part], [u for _, u in part])
        for d in docs[::7]:
            d.encode_state_vector()
    for c, d in zip(cases, docs):
        assert d.encode_state_as_update().hex() == c["state"], c["name"]


def test_apply_multi_pending_docs_fall_back():
    """Out-of-order deltas (Yjs pending structs) in the fleet: each such document takes its own
    pending emulation, the others still merge together; every read equals Yjs's after the batch."""
    with open(os.path.join(ROOT, "tests", "golden", "pending.json")) as f:
        cases = json.load(f)["cases"][:24]
    docs = [crdt_amd.Doc(client_id=0x7FFFFFF0) for _ in cases]
    pairs = _interleaved(cases, random.Random(9))
    crdt_amd.apply_updates_multi([docs[i] for i, _ in pairs], [u for _, u in pairs])
    for c, d in zip(cases, docs):
        st = c["steps"][-1]
        assert d.pending() == (st["pending"], st["pending_ds"]), c["name"]
        assert d.encode_state_as_update().hex() == st["state"], c["name"]


def test_apply_multi_c5_fleet_large():
    """A C5-shaped fleet: 20k documents of 2-3 small replica updates each, one ingest call."""
    from crdt_amd.workload import gen_map

    base = [gen_map(n_keys=20, n_replicas=2 + s % 2, ops_per_replica=4, seed=700 + s)[0] for s in range(50)]
    n_docs = 20000
    fleet = [base[i % len(base)] for i in range(n_docs)]
    docs = [crdt_amd.Doc(client_id=0x7FFFFFF0) for _ in range(n_docs)]
    idx, ups = [], []
    for i, us in enumerate(fleet):
        for u in us:
            idx.append(i)
            ups.append(u)
    crdt_amd.apply_updates_multi(docs, ups, doc_index=idx)
    want = crdt_amd.merge_docs(base)
    for i in range(0, n_docs, 997):
        assert (docs[i].encode_state_as_update(), docs[i].encode_state_vector()) == want[i % len(base)], i
    # every state at once (ycrdt_docs_states_packed), with a few documents holding deferred applies
    # (flushed as one batch) and one with a pending struct (its own encode)
    for i in (3, 4, 5):
        docs[i].apply_update(base[(i + 1) % len(base)][0])
    pend = crdt_amd.Doc(client_id=0x7FFFFFF0)
    pend.apply_update(bytes.fromhex(_PENDING_ONLY))
    allw = docs + [pend, crdt_amd.Doc(client_id=5)]
    blob, offs = crdt_amd.states_packed(allw)
    for i in list(range(0, n_docs, 331)) + [3, 4, 5, n_docs, n_docs + 1]:
        got = (bytes(blob[offs[2 * i]:offs[2 * i + 1]]), bytes(blob[offs[2 * i + 1]:offs[2 * i + 2]]))
        assert got == (allw[i].encode_state_as_update(), allw[i].encode_state_vector()), i


# one struct of client 7 at clock 1 whose clock-0 predecessor never arrived: Yjs keeps it pending
_PENDING_ONLY = "010107012801057573657273016201770178" + "00"


def test_apply_multi_malformed_applies_prefix(golden):
    c = golden["map"][0]
    ups = [bytes.fromhex(u) for u in c["updates"]]
    d1, d2 = crdt_amd.Doc(client_id=1), crdt_amd.Doc(client_id=2)
    with pytest.raises(crdt_amd.YcrdtError):
        crdt_amd.apply_updates_multi([d1] * len(ups) + [d2], ups + [b"\x05\x01"])
    assert d1.encode_state_as_update().hex() == c["state"]
