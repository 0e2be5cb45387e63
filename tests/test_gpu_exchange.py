"""libycrdt's multi-rank exchanges at world size 2: two processes on the one GPU, each with its own
engine, joined by the package's torch-free TCP hub (crdt_amd/hosthub.py) — and, as a second
independent transport, a torch.distributed gloo group (tests/torch_comm.py) — that carries the
library's collectives through the host exchange (ycrdt_comm_create_exchange; RCCL is the same code
with device buffers). The
library's own code runs on both ranks — shard export, the pre-exchange status agreement, the flag
sum, the fleet key-space build and MAX all-reduce, the delete-set all-gather — and every result is
checked against Yjs fixtures / the unsharded merge:

* sharded merge of ONE document (C4 shape): each rank parses only its share of the
  updates (the struct / section bitmaps, delete-set starts and section records are combined), then
  integrates its key-hash shard; the flag words are summed, and both ranks encode bytes equal to
  the unsharded merge (Yjs state);
* fleet state vectors (C5): each rank merges a different part of every document's updates; the
  exchanged state vectors equal Yjs's state vectors of the whole documents;
* delete-set all-gather: each rank's part of a document; the union equals the delete set of
  Y.mergeUpdates over all parts;
* an empty document held by the ranks is in the fleet result (state vector [0]);
* a section table past its estimate on one rank makes every rank re-run the decode alike;
* a malformed update parsed by one rank fails the merge on every rank; a rank that fails on the
  host before the exchange makes the other rank's call fail too (no hang), and the communicator
  keeps working.
"""
import json
import os
import socket

import pytest

crdt_amd = pytest.importorskip("crdt_amd")

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cases(prefix):
    with open(os.path.join(HERE, "golden", "configs.json")) as f:
        return [c for c in json.load(f)["cases"] if c["name"].startswith(prefix)]


def _worker(rank, world, port, q, transport):
    import sys

    sys.path.insert(0, os.path.dirname(HERE))
    hub = None
    if transport == "gloo":
        import torch.distributed as dist

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
    else:
        from crdt_amd.hosthub import HostHub

        hub = HostHub(world, rank, "127.0.0.1", port)
    out = {"rank": rank, "torch_loaded": "torch" in sys.modules}
    try:
        from crdt_amd.workload import gen_nested
        from tests.v1util import delete_set_of

        eng = crdt_amd.Engine()
        if transport == "gloo":
            from tests.torch_comm import comm_over_torch

            comm = comm_over_torch(crdt_amd, eng)
        else:
            comm = crdt_amd.Comm.over_hub(eng, hub)
        # ---- sharded merge of one document: every C4 fixture + a generated C4 history
        docs = [[bytes.fromhex(u) for u in c["updates"]] for c in _cases("c4_")]
        docs.append(gen_nested(40, 1500, 200, seed=5)[0])
        shard_ok = []
        for ups in docs:
            b = crdt_amd.Batch(ups, eng)
            b.merge_sharded(world, comm)
            got = b.result()
            b.merge()
            shard_ok.append(got == b.result())
            del b
        out["shard"] = shard_ok
        # ---- fleet state vectors: rank r holds the updates u[i] with i % world == r of every C5 doc
        c5 = _cases("c5_")
        svs = {}
        for j, c in enumerate(c5):
            mine = [bytes.fromhex(u) for i, u in enumerate(c["updates"]) if i % world == rank]
            d = crdt_amd.Doc(client_id=0x7FFFFFF0, engine=eng)
            d.apply_updates(mine)
            if mine or j % 3:  # some documents only on some ranks
                svs[7 * j + 2] = d.encode_state_vector()
        svs[999_999] = b"\x00"  # a document every rank holds with an empty state vector
        if rank == 1:
            svs[999_998] = b"\x00"  # ... and one only rank 1 holds
        fleet = comm.fleet_sv_allreduce_max(svs)
        out["fleet"] = [(fleet.get(7 * j + 2, b"").hex(), c["sv"]) for j, c in enumerate(c5)]
        out["fleet_empty"] = [fleet.get(999_999), fleet.get(999_998)]
        # ---- delete-set all-gather: each rank's part of every C3 / C4 fixture (Y.mergeUpdates of its
        # replicas' states); the union is the delete set of Y.mergeUpdates over all of them
        ds_ok = []
        for c in _cases("c3_") + _cases("c4_"):
            ups = [bytes.fromhex(u) for u in c["updates"]]
            mine = crdt_amd.merge_updates([u for i, u in enumerate(ups) if i % world == rank], eng)
            union = comm.ds_allgather(mine)
            ds_ok.append(delete_set_of(union) == delete_set_of(crdt_amd.merge_updates(ups, eng)))
        out["ds"] = ds_ok
        # ---- a malformed update parsed by one rank: the error reaches every rank
        ups = list(docs[0])
        ups[3] = b"\x01" + b"\xff" * (len(ups[3]) - 1)  # an endless varuint; same length: the same layout
        try:
            b = crdt_amd.Batch(ups, eng)
            b.merge_sharded(world, comm)
            out["fail"] = "no error"
        except crdt_amd.YcrdtError as e:
            out["fail"] = e.kind
        # ---- rank 1 fails on the host before the exchange: rank 0 gets an error too, nobody hangs
        if rank == 1:
            os.environ["YCRDT_TEST_FAIL_BEFORE_EXCHANGE"] = "1"
        try:
            b = crdt_amd.Batch(docs[0], eng)
            b.merge_sharded(world, comm)
            out["fail2"] = "no error"
        except crdt_amd.YcrdtError as e:
            out["fail2"] = e.kind
        os.environ.pop("YCRDT_TEST_FAIL_BEFORE_EXCHANGE", None)
        # ---- rank 0's section table overflows its (test-shrunk) estimate: both ranks re-run the
        # decode with the worst-case bound and still give the unsharded bytes
        if rank == 0:
            os.environ["YCRDT_TEST_SECTION_CAP"] = "2"
        b = crdt_amd.Batch(docs[-1], eng)
        b.merge_sharded(world, comm)
        got = b.result()
        os.environ.pop("YCRDT_TEST_SECTION_CAP", None)
        b.merge()
        out["overflow"] = got == b.result()
        # ---- and the communicator still works afterwards
        b = crdt_amd.Batch(docs[1], eng)
        b.merge_sharded(world, comm)
        got = b.result()
        b.merge()
        out["after"] = got == b.result()
        comm.close()
    except Exception as e:  # noqa: BLE001 — reported to the parent
        out["error"] = repr(e)
    finally:
        q.put(out)
        if hub is not None:
            hub.close()
        else:
            import torch.distributed as dist

            dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("transport", ["hub", "gloo"])
def test_exchanges_world2_one_gpu(transport):
    import multiprocessing as mp

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, transport)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    codes = [p.exitcode for p in procs]
    res = sorted([q.get() for _ in range(world)], key=lambda r: r["rank"])
    assert codes == [0, 0], (codes, res)
    for r in res:
        assert "error" not in r, r
        assert r["torch_loaded"] == (transport == "gloo"), r  # the package's own transport needs no torch
        assert all(r["shard"]), r["shard"]
        for got, want in r["fleet"]:
            assert got == want
        assert all(r["ds"]), r["ds"]
        assert r["fail"] != "no error", r
        assert r["fail2"] != "no error", r
        assert r["after"], r
        assert r["overflow"], r
        assert r["fleet_empty"] == [b"\x00", b"\x00"], r
    assert res[0]["fleet"] == res[1]["fleet"]
