#!/usr/bin/env python3
"""Benchmark: CRDT items merged/sec on MI355X (BASELINE.json metric) — config C2, at scale.

Workload (BASELINE.json configs[1]): one YMap 'users' with 100k hot keys
(Zipf s=1.1), a base snapshot of every key by one client, then 1,000 replicas x 1,000 concurrent
set/delete ops with no gossip; a document's input is the base update plus every replica's
encodeStateAsUpdate(replica, baseSV) — 1,001 Yjs v1 updates, ≈13.5 MB, ≈0.9 M items.

A step = one device pass that merges `--docs` (default 112) such documents — independent replica
sets with different seeds, ≥ 100 M items — as a multi-document batch (ycrdt_batch_stage_docs:
decode → dedupe → delete sets → YMap winner → canonical re-encode per document), inputs already
resident in HBM, outputs left in HBM. Each document's result is exactly what `for u in doc:
Y.applyUpdate(d, u)` followed by `Y.encodeStateAsUpdate(d)` computes (byte-identical;
tests/test_gpu_parity.py, tests/test_gpu_multidoc.py). Items = Σ struct clock lengths of the
inputs (Item + GC, Skip excluded), the SURVEY §8(d) unit. `single_doc` keeps the one-document
step of round 1 for continuity.

Multi-GPU: one process per GPU — under torch.distributed.run, or `bench.py --gpus N` spawns the N
ranks itself (rank r on device r % devices). The headline shards by document (north_star:
"partitioned ... by document/topic"): every rank merges its own independent documents (seeds
offset per rank) with no data-path collective ⇒ "scaling": "weak". Barriers, the max-over-ranks
step time and the per-rank reports go through libycrdt's own communicator (RCCL; a host exchange
over gloo when ranks share a device). With N > 1 two more legs run by default: C4 key-hash sharded
across the ranks (one 102 M-item document) and the C5 fleet (routed ingest + the fleet
state-vector all-reduce).
"""
import argparse
import csv
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--workload", default="c2", choices=["c2", "c1"])
    p.add_argument("--docs", type=int, default=112,
                   help="independent documents of the workload merged per step in one device pass (>= 100 M items)")
    p.add_argument("--replicas", type=int, default=None, help="override replica count (default: config)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--fleet-pairs", type=int, default=20000,
                   help="C5-shaped sync-responder leg: (doc state, peer SV) pairs in one batched diff (0 = off)")
    p.add_argument("--cpu-replicas", type=int, default=300,
                   help="replicas in the Yjs CPU-baseline sample (bounded: ~10 s of Yjs work)")
    p.add_argument("--port-replicas", type=int, default=1000, help="replicas in the oracle-port timing sample")
    p.add_argument("--profile-phases", action="store_true")
    p.add_argument("--no-per-op", action="store_true", help="skip the crdt.js per-op leg")
    p.add_argument("--fleet-docs", type=int, default=1_000_000, help="documents in the C5 fleet-ingest leg (0 = skip)")
    p.add_argument("--no-c4", action="store_true", help="skip the C4 leg (N = 1: one GPU; N > 1: key-hash sharded over the ranks)")
    p.add_argument("--only-headline", action="store_true",
                   help="time the headline merge only (no side legs): rocprof averages then match the bench line")
    p.add_argument("--c3-items", type=int, default=10_000_000,
                   help="C3 leg: YArray 'messages', 256 replicas x 16 rounds, this many values (0 = off)")
    p.add_argument("--billion", type=int, default=0, metavar="DOCS",
                   help="opt-in leg: DOCS distinct C2 documents (1120 = 1.0 B items, ~15 GB of updates) merged in ONE "
                        "ycrdt_batch_merge (multi-window batch), with its HBM footprint and properties; skips the side legs")
    return p.parse_args()


def _sample(cfg, n_replicas, updates, gen_map):
    c = dict(cfg)
    c["n_replicas"] = min(n_replicas, cfg["n_replicas"])
    return updates if c["n_replicas"] == cfg["n_replicas"] else gen_map(**c)[0], c["n_replicas"]


def cpu_baselines(args, cfg, updates, out_update, st, eng, gen_map):
    """The reference path timed on this box's host cores, beside the GPU number (never `value`).

    kind "reference": Yjs 13.5.16 itself (the library @ypear/crdt delegates to), in Node, on one
    core, over a bounded sample of the same workload (scripts/yjs_baseline.js); its output is
    checked against the GPU merge of the same sample (sha256 of the canonical update).
    `port`: the oracle's sequential C restatement (oracle/yref.c) on the full batch, also 1 core.
    """
    import hashlib
    import shutil
    import struct
    import subprocess
    import tempfile

    import crdt_amd
    from oracle.yref import Doc as ODoc

    res = None
    node = shutil.which("node")
    sups, nrep = _sample(cfg, args.cpu_replicas, updates, gen_map)
    b = crdt_amd.Batch(sups, eng)
    sst = b.merge()
    gpu_out = b.result()[0]
    del b
    if node:
        with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
            f.write(struct.pack("<I", len(sups)))
            for u in sups:
                f.write(struct.pack("<I", len(u)))
                f.write(u)
            fname = f.name
        try:
            r = subprocess.run([node, "--max-old-space-size=16384", os.path.join(ROOT, "scripts", "yjs_baseline.js"), fname],
                               capture_output=True, text=True, timeout=240)
            y = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 and r.stdout.strip() else None
        finally:
            os.unlink(fname)
        if y and y.get("available"):
            res = {
                "value": round(sst.items / (y["ms"] * 1e-3), 1),
                "unit": "items/s",
                "cores": 1,
                "kind": "reference",
                "sample": f"C2 base + {nrep} replicas x {cfg['ops_per_replica']} ops ({sst.items} items): Yjs "
                          f"{y['yjs']} / lib0 {y['lib0']} in Node {y['node']}, for u of batch: Y.applyUpdate(doc, u); "
                          f"Y.encodeStateAsUpdate(doc), {y['ms'] / 1e3:.2f} s",
                "parity": y["out_sha256"] == hashlib.sha256(gpu_out).hexdigest(),
            }
    if res is None:
        res = {"value": None, "unit": "items/s", "cores": 1, "kind": "reference",
               "sample": "reference baseline unavailable (no Node or no Yjs on this machine)"}
    # the sequential C restatement (oracle/yref.c) on the full batch
    pups, prep = _sample(cfg, args.port_replicas, updates, gen_map)
    d = ODoc(0x7FFFFFF0)
    c0 = time.perf_counter()
    for u in pups:
        d.apply_update(u)
    ref = d.encode_state_as_update()
    c1 = time.perf_counter()
    pitems = st.items if pups is updates else None
    if pitems is None:
        b2 = crdt_amd.Batch(pups, eng)
        pitems = b2.merge().items
        del b2
    res["port"] = {
        "value": round(pitems / (c1 - c0), 1), "unit": "items/s", "cores": 1, "kind": "port",
        "sample": f"C2 base + {prep} replicas x {cfg['ops_per_replica']} ops ({pitems} items), oracle/yref.c "
                  f"sequential Yjs restatement, {c1 - c0:.2f} s",
        "parity": (ref == out_update) if pups is updates else None,
    }
    return res


def apply_loop_leg(eng, updates, out_update):
    """crdt.js's own ingest shape (onData per message crdt.js:294, LevelDB replay crdt.js:79-98):
    one Y.applyUpdate call per update of the C2 batch through the C ABI (host buffers), then ONE
    read (Y.encodeStateAsUpdate). Each apply validates on the host and queues; the read merges the
    whole queue in one device pass, so the loop costs about one merge, not 1,001. Output compared
    with the batched merge's."""
    import crdt_amd

    reps = 3
    loop_ms = read_ms = 0.0
    same = True
    for _ in range(reps):
        d = crdt_amd.Doc(client_id=0x7FFFFFF0, engine=eng)
        t0 = time.perf_counter()
        for u in updates:
            d.apply_update(u)
        t1 = time.perf_counter()
        got = d.encode_state_as_update()
        t2 = time.perf_counter()
        loop_ms += (t1 - t0) * 1e3
        read_ms += (t2 - t1) * 1e3
        same = same and got == out_update
        del d
    loop_ms /= reps
    read_ms /= reps
    return {"applies": len(updates), "apply_calls_ms": round(loop_ms, 3), "first_read_ms": round(read_ms, 3),
            "total_ms": round(loop_ms + read_ms, 3), "merges": 1, "parity": same,
            "includes": "per call: ctypes + host validation + queue copy; read: H2D + one merge + D2H"}


def _any_str(v: str) -> bytes:
    """lib0 `any` encoding of one string (tag 119, varString)."""
    b = v.encode()
    n, out = len(b), bytearray([119])
    while n > 0x7F:
        out.append(0x80 | (n & 0x7F))
        n >>= 7
    out.append(n)
    return bytes(out) + b


def per_op_leg(eng, n_ops_list=(500, 2000)):
    """crdt.js's per-op path (SURVEY.md §6 'crdt.js end-to-end', crdt.js:433-445, 294-305): peer A
    does one YMap set (every 5th op a delete) and encodes its FULL state (crdt.js sends
    Y.encodeStateAsUpdate(y.doc) per op); peer B applies it and rebuilds its crdt.c cache
    (toJSON of the root). Reported as ops/s next to the same loop in Yjs 13.5.16 (Node, one core,
    scripts/yjs_baseline.js perop), final states compared byte for byte."""
    import hashlib
    import crdt_amd

    res = {}
    for n_ops in n_ops_list:
        a = crdt_amd.Doc(client_id=1, engine=eng)
        b = crdt_amd.Doc(client_id=2, engine=eng)
        a.track_local(False)
        dev = 0.0
        t0 = time.perf_counter()
        for i in range(n_ops):
            key = "user%d" % (i % 100)
            if i % 5 == 4:
                a.map_delete("users", key)
            else:
                a.map_set("users", key, _any_str("v%d" % i))
            u = a.encode_state_as_update()
            dev += a.last_stats().device_ms
            b.apply_update(u)
            b.root_json("users", "map")
            dev += b.last_stats().device_ms
        dt = time.perf_counter() - t0
        final = b.encode_state_as_update()
        r = {"ops": n_ops, "ms": round(dt * 1e3, 2), "ops_per_s": round(n_ops / dt, 1),
             "breakdown": {"merges_per_op": 2, "wall_ms_per_op": round(dt * 1e3 / n_ops, 4),
                           "device_ms_per_op": round(dev / n_ops, 4),
                           "host_ms_per_op": round((dt * 1e3 - dev) / n_ops, 4),
                           "note": "device = the two merges' kernel time (events on the engine stream); host = "
                                   "launch issue, ~6 host syncs per merge, staging copies, view build, ctypes"},
             "includes": "A: set/delete + full encodeStateAsUpdate; B: applyUpdate + toJSON (crdt.c), ctypes, 1 GPU"}
        y = _yjs_perop(n_ops)
        if y:
            from tests.v1util import canonical_update
            r["yjs"] = {"ops_per_s": round(n_ops / (y["ms"] * 1e-3), 1), "cores": 1, "kind": "reference",
                        "parity": y["state_sha256"] == hashlib.sha256(canonical_update(final)).hexdigest(),
                        "sample": f"the same loop in Yjs {y['yjs']} / Node {y['node']}"}
        res[str(n_ops)] = r
        del a, b
    return res


def _yjs_perop(n_ops, timeout=240):
    import shutil
    import subprocess

    node = shutil.which("node")
    if not node:
        return None
    r = subprocess.run([node, os.path.join(ROOT, "scripts", "yjs_baseline.js"), str(n_ops), "perop"],
                       capture_output=True, text=True, timeout=timeout)
    y = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 and r.stdout.strip() else None
    return y if y and y.get("available") else None


def _yjs_time(ups, timeout=240):
    """Yjs 13.5.16 in Node on one core over a batch (scripts/yjs_baseline.js): (ms, sha256) or None."""
    import shutil
    import struct
    import subprocess
    import tempfile

    node = shutil.which("node")
    if not node:
        return None
    with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
        f.write(struct.pack("<I", len(ups)))
        for u in ups:
            f.write(struct.pack("<I", len(u)))
            f.write(u)
        fname = f.name
    try:
        r = subprocess.run([node, "--max-old-space-size=16384", os.path.join(ROOT, "scripts", "yjs_baseline.js"), fname],
                           capture_output=True, text=True, timeout=timeout)
        y = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 and r.stdout.strip() else None
    finally:
        os.unlink(fname)
    return y if y and y.get("available") else None


def c3_leg(eng, n_items, steps=3):
    """BASELINE.json configs[2] (C3): YArray 'messages', 256 replicas doing push / unshift / insert /
    cut over 16 rounds (crdt_amd/workload/ycw_array.cpp), every replica's per-round update merged
    in one batch (4,096 updates). Properties at full size: the reversed batch and the merge of the
    output give the same bytes. Beside it, on bounded samples of the same generator: the oracle
    port (oracle/yref.c, 1 core) and Yjs 13.5.16 in Node (1 core), outputs compared."""
    import hashlib

    import crdt_amd
    from crdt_amd.workload import gen_array
    from oracle.yref import Doc as ODoc

    g0 = time.perf_counter()
    ups, gst = gen_array(256, 16, n_items, 3)
    gen_s = time.perf_counter() - g0
    b = crdt_amd.Batch(ups, eng)
    st = b.merge()  # warm-up
    eng.set_profiling(True)
    acc, t0 = {}, time.perf_counter()
    for _ in range(steps):
        st = b.merge()
        for n, m in eng.phase_times():
            acc[n] = acc.get(n, 0.0) + m
    wall = (time.perf_counter() - t0) / steps
    eng.set_profiling(False)
    out = b.result()[0]
    del b
    rb = crdt_amd.Batch(list(reversed(ups)), eng)
    rb.merge()
    rev_ok = rb.result()[0] == out
    del rb
    ib = crdt_amd.Batch([out], eng)
    ib.merge()
    idem_ok = ib.result()[0] == out
    del ib
    res = {"full_state_ingest": full_state_leg(eng, "C3 merged state (256 clients) as one update", ups, out)}
    res.update({"workload": "C3: YArray 'messages', 256 replicas x 16 rounds, push 40% / unshift 15% / insert 30% / cut 15%",
           "updates": len(ups), "input_bytes": sum(map(len, ups)), "items": st.items, "structs": st.structs,
           "segments": st.segments, "output_bytes": len(out), "ms_per_merge": round(wall * 1e3, 3),
           "device_ms": round(st.device_ms, 3), "items_per_s": round(st.items / wall, 1),
           "phases_ms": {n: round(m / steps, 3) for n, m in acc.items()},
           "order_independent": rev_ok, "idempotent": idem_ok, "generate_s": round(gen_s, 2)})
    # the oracle port and Yjs on bounded samples of the same generator
    for key, n, runner in (("port", 1_000_000, "port"), ("yjs", 200_000, "yjs")):
        sups, sst = gen_array(256, 16, n, 3)
        gb = crdt_amd.Batch(sups, eng)
        gst2 = gb.merge()
        t0 = time.perf_counter()
        for _ in range(3):
            gst2 = gb.merge()
        gms = (time.perf_counter() - t0) * 1e3 / 3
        gout = gb.result()[0]
        del gb
        if runner == "port":
            d = ODoc(0x7FFFFFF0)
            c0 = time.perf_counter()
            for u in sups:
                d.apply_update(u)
            ref = d.encode_state_as_update()
            cms = (time.perf_counter() - c0) * 1e3
            res[key] = {"items": gst2.items, "cpu_ms": round(cms, 1), "gpu_ms": round(gms, 2), "cores": 1, "kind": "port",
                        "parity": ref == gout, "sample": f"{n} values, oracle/yref.c sequential Yjs restatement"}
        else:
            y = _yjs_time(sups)
            yf = _yjs_time([gout])  # the sample's merged state applied as one update (full-state ingest)
            if yf:
                res["full_state_ingest"]["yjs_sample"] = {
                    "items": gst2.items, "cpu_ms": round(yf["ms"], 1), "cores": 1, "kind": "reference",
                    "parity": yf["out_sha256"] == hashlib.sha256(gout).hexdigest(),
                    "sample": f"the {n}-value sample's merged state ({len(gout)} B) as one update, Yjs {yf['yjs']} in Node {yf['node']}"}
            if y:
                res[key] = {"items": gst2.items, "cpu_ms": round(y["ms"], 1), "gpu_ms": round(gms, 2), "cores": 1,
                            "kind": "reference", "parity": y["out_sha256"] == hashlib.sha256(gout).hexdigest(),
                            "sample": f"{n} values, Yjs {y['yjs']} in Node {y['node']}"}
    return res


def full_state_leg(eng, name, ups, full, reps=3, small_ops=0):
    """crdt.js's wire shape (crdt.js:288 sync step 2, :443 every local op, :79-98 LevelDB replay):
    a peer's FULL state arrives as ONE multi-client update. Timed with the update resident in HBM
    (ycrdt_batch_merge): merged alone (an empty doc applying it) and behind the state of a doc
    that holds the first half of the history (the merge of ups[:n/2]). Both must give the full
    state's bytes back (it is canonical and covers the half). Beside it, the same through the doc
    path (Y.applyUpdate into a fresh doc + encodeStateAsUpdate: host staging included)."""
    import crdt_amd

    half_b = crdt_amd.Batch(ups[: len(ups) // 2], eng)
    half_b.merge()
    half = half_b.result()[0]
    del half_b
    res = {"what": name, "full_bytes": len(full), "half_bytes": len(half)}
    for key, batch in (("into_empty", [full]), ("into_half", [half, full])):
        b = crdt_amd.Batch(batch, eng)
        st = b.merge()
        t0 = time.perf_counter()
        dev = 0.0
        for _ in range(reps):
            st = b.merge()
            dev += st.device_ms
        ms = (time.perf_counter() - t0) * 1e3 / reps
        ok = b.result()[0] == full
        del b
        res[key] = {"ms_per_merge": round(ms, 3), "device_ms": round(dev / reps, 3), "items": st.items,
                    "items_per_s": round(st.items / (ms * 1e-3), 1), "equal_to_full_state": ok}
    d = crdt_amd.Doc(client_id=0x7FFFFFF0, engine=eng)
    t0 = time.perf_counter()
    d.apply_update(full)
    got = d.encode_state_as_update()
    res["doc_apply_ms"] = round((time.perf_counter() - t0) * 1e3, 3)
    res["doc_equal"] = got == full
    if small_ops:
        res["small_into_large"] = small_into_large(eng, d, full, small_ops)
    del d
    return res


def small_into_large(eng, d, full, n_ops, root="users"):
    """crdt.js's steady state on a large document (crdt.js:294 then :297-305): ONE small remote
    update (a peer's map set, sent as a delta) applied to a doc holding the full state, then the
    read that merges it. Per apply: Y.applyUpdate + Y.encodeStateVector (the merge), and separately
    the crdt.c rebuild (toJSON of the root map). The peer's deltas come from the oracle port holding
    the same state; the doc's final state is compared with the oracle's."""
    from oracle.yref import Doc as ODoc

    peer = ODoc(0x5EED0001)
    peer.apply_update(full)
    deltas = []
    for i in range(n_ops):
        sv = peer.encode_state_vector()
        peer.map_set(root, "k%d" % (i * 7919 % 100_000), _any_str("w%d" % i))
        deltas.append(peer.encode_state_as_update(sv))
    d.encode_state_vector()
    merge_ms, json_ms = [], []
    for u in deltas:
        t0 = time.perf_counter()
        d.apply_update(u)
        d.encode_state_vector()
        t1 = time.perf_counter()
        merge_ms.append((t1 - t0) * 1e3)
    for u in deltas[:3]:  # (toJSON of a 100 k-key map: timed on a few applies)
        t1 = time.perf_counter()
        d.root_json(root, "map")
        json_ms.append((time.perf_counter() - t1) * 1e3)
    merge_ms.sort()
    same = d.encode_state_as_update() == peer.encode_state_as_update()
    return {"applies": n_ops, "delta_bytes": len(deltas[-1]), "apply_merge_ms_median": round(merge_ms[len(merge_ms) // 2], 3),
            "apply_merge_ms_min": round(merge_ms[0], 3), "tojson_ms": round(min(json_ms), 3), "parity": same,
            "includes": "per apply: host validation + queue, the merge of (doc state + delta) on the device (the state is "
                        "re-decoded: record mode + step table), the state-vector read-back"}


def billion_leg(eng, cfg, gen_map, n_docs, reps=3):
    """north_star 'bit-exact Yjs merge of >= 1 B CRDT items': n_docs distinct C2 documents (seeds
    disjoint from the headline's) merged in ONE ycrdt_batch_merge — a batch of ~15 GB laid out in
    4 GiB windows (yc_work.h) — timed with its inputs resident in HBM. Properties at full size:
    three documents merged alone (forward and reversed update order) give their bytes in the big
    merge; the merge of all outputs as one batch returns them unchanged (idempotence)."""
    from concurrent.futures import ThreadPoolExecutor

    import crdt_amd

    def log(msg):  # progress on stderr: a multi-minute leg must not look hung
        print(f"[billion {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)

    log(f"engine holds {eng.device_bytes() / 2**30:.1f} GiB after the headline; trimming")
    eng.trim()
    seeds = [cfg["seed"] + 7_000_003 + i * 1_009 for i in range(n_docs)]
    g0 = time.perf_counter()
    docs = []
    with ThreadPoolExecutor(16) as ex:
        for i, d in enumerate(ex.map(lambda sd: gen_map(**dict(cfg, seed=sd))[0], seeds)):
            docs.append(d)
            if i % 100 == 99:
                log(f"generated {i + 1}/{n_docs} documents")
    gen_s = time.perf_counter() - g0
    in_bytes = sum(len(u) for d in docs for u in d)
    log(f"{in_bytes / 1e9:.2f} GB of updates in {gen_s:.1f} s; staging")
    s0 = time.perf_counter()
    b = crdt_amd.Batch(docs=docs, engine=eng)
    stage_s = time.perf_counter() - s0
    log(f"staged in {stage_s:.1f} s; first merge")
    st = b.merge()  # first merge: workspace allocation
    log(f"first merge: {st.items} items, device {st.device_ms:.1f} ms, HBM {eng.device_bytes() / 2**30:.1f} GiB")
    t0 = time.perf_counter()
    for _ in range(reps):
        st = b.merge()
    ms = (time.perf_counter() - t0) * 1e3 / reps
    log(f"{reps} merges: {ms:.1f} ms each")
    hbm = eng.device_bytes()
    outs = [u for u, _ in b.result_docs()]
    out_bytes = sum(map(len, outs))
    del b
    alone = True
    for k in (0, n_docs // 2, n_docs - 1):
        for ups in (docs[k], list(reversed(docs[k]))):
            sb = crdt_amd.Batch(ups, eng)
            sb.merge()
            alone = alone and sb.result()[0] == outs[k]
            del sb
    ib = crdt_amd.Batch(docs=[[o] for o in outs], engine=eng)
    ist = ib.merge()
    idem = [u for u, _ in ib.result_docs()] == outs
    del ib
    return {"docs": n_docs, "updates": sum(map(len, docs)), "input_bytes": in_bytes, "items": st.items,
            "structs": st.structs, "segments": st.segments, "output_bytes": out_bytes, "merges": 1,
            "ms_per_merge": round(ms, 2), "items_per_s": round(st.items / (ms * 1e-3), 1),
            "windows": (in_bytes >> 32) + 1, "hbm_footprint_bytes": hbm,
            "alone_equal_fwd_and_reversed": alone, "idempotent": idem, "idempotence_merge_items": ist.items,
            "generate_s": round(gen_s, 1), "stage_s": round(stage_s, 1),
            "includes": "one multi-document device pass, inputs resident in HBM (staging and D2H not timed)"}


def c4_leg(eng, reps=3):
    """C4 (BASELINE configs[3], nested YArrays under YMap keys) on one GPU at BASELINE scale: the
    whole document (crdt_amd/workload C4_FULL: 1 M keys, 64 replicas, ~100 items per nested array,
    102 M items, base snapshot, ~10 % of keys overwritten by a fresh array — nested GC —, deletes)
    merged in one device pass; the merge of the reversed update list and of its own output give the
    same bytes; and the same merge as 8 logical key-hash shards (each shard's integrate phases run
    in turn, flag words summed as the RCCL all-reduce would) — byte-identical to the unsharded result."""
    import crdt_amd
    from crdt_amd.workload import C4_FULL as C4, gen_nested

    t0 = time.perf_counter()
    ups, st = gen_nested(**C4)
    gen_s = time.perf_counter() - t0
    b = crdt_amd.Batch(ups, eng)
    b.merge()
    t0 = time.perf_counter()
    for _ in range(reps):
        s1 = b.merge()
    ms = (time.perf_counter() - t0) * 1e3 / reps
    full = b.result()
    eng.set_profiling(True)
    b.merge()
    phases = {n: round(m, 3) for n, m in eng.phase_times()}
    eng.set_profiling(False)
    t0 = time.perf_counter()
    b.merge_sharded(8)
    sh_ms = (time.perf_counter() - t0) * 1e3
    same = b.result() == full
    del b
    rb = crdt_amd.Batch(list(reversed(ups)), eng)
    rb.merge()
    rev_ok = rb.result() == full
    del rb
    ib = crdt_amd.Batch([full[0]], eng)
    ib.merge()
    idem_ok = ib.result() == full
    del ib
    return {"workload": f"C4 (BASELINE scale): YMap 'docs' of {C4['n_keys']} nested YArrays, {C4['n_replicas']} replicas x "
                        f"{C4['pushes']} ops (push of 1-4 values, overwrite with a new array {C4['p_over']:.2%}, delete "
                        f"{C4['p_del']:.0%}), base snapshot",
            "order_independent": rev_ok, "idempotent": idem_ok,
            "updates": len(ups), "input_bytes": sum(len(u) for u in ups), "items": s1.items, "structs": s1.structs,
            "segments": s1.segments, "output_bytes": len(full[0]), "ms_per_merge": round(ms, 3),
            "items_per_s": round(s1.items / (ms * 1e-3), 1), "phases_ms": phases,
            "sharded_8_logical": {"ms": round(sh_ms, 3), "identical": same,
                                  "includes": "8 x (mask + winner + dead types + YATA + merge flags + export), "
                                              "sum, GC merge settle, one encode, on this GPU"},
            "generate_s": round(gen_s, 2)}


def c4_sharded_leg(eng, comm, world, rank, reps=2):
    """C4 (BASELINE configs[3]) at BASELINE scale, key-hash sharded across the ranks: every rank
    stages the same C4_FULL updates (102 M items), parses its share of them and integrates its
    shard; the parse results and the flag words are combined inside libycrdt over its own
    communicator (RCCL between GPUs, the host exchange when ranks share a device). Checked against
    the unsharded merge of the same batch on every rank."""
    import crdt_amd
    from crdt_amd.workload import C4_FULL, gen_nested

    ups, _ = gen_nested(**C4_FULL)
    b = crdt_amd.Batch(ups, eng)
    eng.set_profiling(True)
    b.merge_sharded(world, comm)  # warm-up (workspace)
    comm.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        s1 = b.merge_sharded(world, comm)
    ms = (time.perf_counter() - t0) * 1e3 / reps
    phases = {n: round(m, 3) for n, m in eng.phase_times()}
    eng.set_profiling(False)
    full = b.result()
    b.merge()
    same = b.result() == full
    del b
    ms_all = [struct_unpack_d(x) for x in comm.allgather(struct_pack_d(ms))]
    return {"ranks": world, "ms_per_merge": round(max(ms_all), 3), "ms_per_rank": [round(x, 3) for x in ms_all],
            "items": s1.items, "items_per_s": round(s1.items / (max(ms_all) * 1e-3), 1),
            "identical_to_unsharded": same, "phases_ms_rank": phases,
            "transport": comm.transport}


def struct_pack_d(x):
    import struct

    return struct.pack("<d", float(x))


def struct_unpack_d(b):
    import struct

    return struct.unpack("<d", b)[0]


def fleet_ranks_leg(eng, comm, world, rank, n_docs):
    """C5 (BASELINE configs[4]) across the ranks: a fleet of n_docs topics (one Y.Doc each,
    crdt.js:221,235; the updates of the 60 Yjs-generated C5 fixture documents, cycled).
    (1) routed ingest: every rank applies, in ONE ycrdt_apply_updates_multi call, the updates of
    the topics ycrdt_route assigns to it (no data collective; fleet documents/s = all topics over
    the slowest rank's time). (2) gossip without routing: every rank holds every topic, but only the
    updates u_i with i % world == rank; ycrdt_comm_fleet_sv_allreduce_max gives every rank the state
    vector of the union for every topic (sampled topics compared with Yjs's state vectors)."""
    import numpy as np

    import crdt_amd

    with open(os.path.join(ROOT, "tests", "golden", "configs.json")) as f:
        cases = [c for c in json.load(f)["cases"] if c["name"].startswith("c5_")]
    base = [[bytes.fromhex(u) for u in c["updates"]] for c in cases]
    # (1) routed ingest
    mine = [d for d in range(n_docs) if crdt_amd.route(str(d).encode(), world) == rank]
    idx, ups = [], []
    for j, d in enumerate(mine):
        for u in base[d % len(base)]:
            idx.append(j)
            ups.append(u)
    docs = [crdt_amd.Doc(client_id=0x7FFFFFF0, engine=eng) for _ in mine]
    comm.barrier()
    t0 = time.perf_counter()
    crdt_amd.apply_updates_multi(docs, ups, engine=eng, doc_index=np.asarray(idx, dtype=np.int64))
    ingest_ms = (time.perf_counter() - t0) * 1e3
    ok = True
    for j, d in enumerate(mine[:50]):
        ok = ok and docs[j].encode_state_vector().hex() == cases[d % len(cases)]["sv"]
    del docs
    ing = [struct_unpack_d(x) for x in comm.allgather(struct_pack_d(ingest_ms))]
    # (2) un-routed gossip: the fleet's state vectors over the ranks (a sample of the topics: every
    # rank holds a part of each)
    n_sv = min(n_docs, 100_000)
    svs = {}
    idx, ups, held = [], [], []
    for d in range(n_sv):
        part = [u for i, u in enumerate(base[d % len(base)]) if i % world == rank]
        if part:
            held.append(d)
            for u in part:
                idx.append(len(held) - 1)
                ups.append(u)
    docs = [crdt_amd.Doc(client_id=0x7FFFFFF0, engine=eng) for _ in held]
    crdt_amd.apply_updates_multi(docs, ups, engine=eng, doc_index=np.asarray(idx, dtype=np.int64))
    blob, offs = crdt_amd.states_packed(docs, eng)
    for j, d in enumerate(held):
        svs[d] = bytes(blob[int(offs[2 * j + 1]):int(offs[2 * j + 2])])
    del docs
    comm.barrier()
    t0 = time.perf_counter()
    fleet = comm.fleet_sv_allreduce_max(svs)
    sv_ms = (time.perf_counter() - t0) * 1e3
    sv_ok = len(fleet) == n_sv and all(fleet[d].hex() == cases[d % len(cases)]["sv"] for d in range(0, n_sv, 97))
    svm = [struct_unpack_d(x) for x in comm.allgather(struct_pack_d(sv_ms))]
    return {"docs": n_docs, "routed_ingest": {"ms": round(max(ing), 2), "ms_per_rank": [round(x, 2) for x in ing],
                                             "docs_per_s": round(n_docs / (max(ing) * 1e-3), 1), "parity": ok,
                                             "docs_this_rank": len(mine)},
            "sv_allreduce": {"docs": n_sv, "ms": round(max(svm), 2), "parity": sv_ok,
                             "includes": "host pack + device sort/reduce + key-space all-gather + one MAX all-reduce"}}


def fleet_ingest_leg(eng, n_docs):
    """C5 fleet ingest (crdt.js:235 one Y.Doc per topic, crdt.js:294 Y.applyUpdate per message):
    n_docs documents, each receiving the replica updates of one of the C5 fixtures (Yjs-generated,
    tests/golden/configs.json, cycled), all applied with ONE ycrdt_apply_updates_multi call (host
    buffers in, one device pass, every document's state left in HBM). Parity: every document's
    encodeStateAsUpdate / encodeStateVector equals the fixture's Yjs state. Beside it: Yjs 13.5.16
    in Node, worker_threads on W cores (each worker applies and encodes its share of the documents),
    final states compared (sha256 over the canonical states in document order)."""
    import hashlib

    import crdt_amd

    with open(os.path.join(ROOT, "tests", "golden", "configs.json")) as f:
        cases = [c for c in json.load(f)["cases"] if c["name"].startswith("c5_")]
    base = [[bytes.fromhex(u) for u in c["updates"]] for c in cases]
    idx, ups = [], []
    for d in range(n_docs):
        for u in base[d % len(base)]:
            idx.append(d)
            ups.append(u)
    in_bytes = sum(len(u) for u in ups)
    import numpy as np

    idx_np = np.asarray(idx, dtype=np.int64)
    reps, ms = 2, []
    docs = None
    for _ in range(reps):
        docs = [crdt_amd.Doc(client_id=0x7FFFFFF0, engine=eng) for _ in range(n_docs)]
        t0 = time.perf_counter()
        crdt_amd.apply_updates_multi(docs, ups, engine=eng, doc_index=idx_np)
        ms.append((time.perf_counter() - t0) * 1e3)
    gpu_ms = min(ms)
    # every document's state and state vector in one call (ycrdt_docs_states_packed): one gather on
    # the device, one pipelined D2H
    r0 = time.perf_counter()
    blob, offs = crdt_amd.states_packed(docs, eng)
    read_ms = (time.perf_counter() - r0) * 1e3
    mv = memoryview(blob)
    parity = True
    h = hashlib.sha256()
    from tests.v1util import canonical_update
    for d in range(n_docs):
        c = cases[d % len(cases)]
        st = mv[int(offs[2 * d]):int(offs[2 * d + 1])]
        if d < len(cases) or d % 4099 == 0:
            # the engine writes the canonical (13.6) order, so the Yjs side's canonical form is the state itself
            parity = parity and bytes(st).hex() == c["state"] and canonical_update(bytes(st)) == bytes(st)
            parity = parity and bytes(mv[int(offs[2 * d + 1]):int(offs[2 * d + 2])]).hex() == c["sv"]
        h.update(hashlib.sha256(st).digest())
    res = {"docs": n_docs, "updates": len(ups), "in_bytes": in_bytes, "ms": round(gpu_ms, 2),
           "read_all_states_ms": round(read_ms, 2), "out_bytes": int(offs[-1]),
           "docs_per_s": round(n_docs / (gpu_ms * 1e-3), 1), "updates_per_s": round(len(ups) / (gpu_ms * 1e-3), 1),
           "calls": 1, "parity": parity,
           "includes": "ctypes + host validation + H2D + one multi-document merge + per-document split in HBM, 1 GPU"}
    y = _yjs_fleet(idx, ups, n_docs)
    if y:
        res["yjs"] = {"docs_per_s": round(n_docs / (y["ms"] * 1e-3), 1), "workers": y["workers"], "kind": "reference",
                      "cores": y["workers"], "ms": round(y["ms"], 2), "parity": y["state_sha256"] == h.hexdigest(),
                      "sample": f"Yjs {y['yjs']} in Node {y['node']}, worker_threads W={y['workers']} (os.cpus() = "
                                f"{y['cpus']}, capped at the box's CPU share), each: new Y.Doc + Y.applyUpdate per "
                                "update + Y.encodeStateAsUpdate per document"}
    del docs
    return res


def _yjs_fleet(idx, ups, n_docs, timeout=400):
    import shutil
    import struct
    import subprocess
    import tempfile

    node = shutil.which("node")
    if not node:
        return None
    with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
        f.write(struct.pack("<I", len(ups)))
        for d, u in zip(idx, ups):
            f.write(struct.pack("<II", d, len(u)) + u)
        fname = f.name
    try:
        w = str(int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1))
        r = subprocess.run([node, os.path.join(ROOT, "scripts", "yjs_baseline.js"), fname, "fleet", w, str(n_docs)],
                           capture_output=True, text=True, timeout=timeout)
        y = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 and r.stdout.strip() else None
    finally:
        os.unlink(fname)
    return y if y and y.get("available") else None


def fleet_sync_leg(eng, n_pairs):
    """Batched sync responder: n_pairs (doc state, lagging
    peer state vector) pairs from the reduced C5 fixtures (60 docs of 2-4 clients, Yjs-generated),
    cycled to n_pairs, answered with ONE ycrdt_diff_updates call (host buffers in and out, PCIe and
    per-pair host split included). Beside it: Yjs 13.5.16's Y.diffUpdate over the same pairs in Node
    on one core, outputs compared (sha256 of the canonical updates)."""
    import hashlib
    import shutil
    import struct
    import subprocess
    import tempfile

    import crdt_amd

    with open(os.path.join(ROOT, "tests", "golden", "configs.json")) as f:
        cases = [c for c in json.load(f)["cases"] if c["name"].startswith("c5_")]
    base = []
    for c in cases:
        st = bytes.fromhex(c["state"])
        base += [(st, bytes.fromhex(df["sv"])) for df in c["diffs"]] + [(st, b"\x00")]
    pairs = [base[i % len(base)] for i in range(n_pairs)]
    ups, svs = [p[0] for p in pairs], [p[1] for p in pairs]
    crdt_amd.diff_updates(ups[:64], svs[:64], eng)  # warm
    reps = 3
    t0 = time.perf_counter()
    for _ in range(reps):
        outs = crdt_amd.diff_updates(ups, svs, eng)
    gpu_ms = (time.perf_counter() - t0) * 1e3 / reps
    eng.set_profiling(True)  # one more pass with the engine's phase events: the device-side share
    crdt_amd.diff_updates(ups, svs, eng)
    phases = eng.phase_times()
    eng.set_profiling(False)
    res = {"pairs": n_pairs, "docs": len(cases), "in_bytes": sum(map(len, ups)) + sum(map(len, svs)),
           "out_bytes": sum(map(len, outs)), "ms": round(gpu_ms, 3), "pairs_per_s": round(n_pairs / (gpu_ms * 1e-3), 1),
           "includes": "host pack + H2D + lazy decode + diff + encode + D2H + per-pair split, 1 GPU",
           "engine_phases_ms": {n: round(m, 4) for n, m in phases}, "yjs": None}
    node = shutil.which("node")
    if node:
        with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
            f.write(struct.pack("<I", 2 * n_pairs))
            for u, v in pairs:
                f.write(struct.pack("<I", len(u)) + u + struct.pack("<I", len(v)) + v)
            fname = f.name
        try:
            wd = str(int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1))
            r = subprocess.run([node, os.path.join(ROOT, "scripts", "yjs_baseline.js"), fname, "diff", wd],
                               capture_output=True, text=True, timeout=240)
            y = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 and r.stdout.strip() else None
        finally:
            os.unlink(fname)
        if y and y.get("available"):
            h = hashlib.sha256()
            for o in outs:
                h.update(o)
            res["yjs"] = {"pairs_per_s": round(y["pairs"] / (y["ms"] * 1e-3), 1), "cores": y["workers"], "kind": "reference",
                          "ms": round(y["ms"], 2), "parity": y["out_sha256"] == h.hexdigest(),
                          "sample": f"Yjs {y['yjs']} Y.diffUpdate over the same {y['pairs']} pairs in Node {y['node']}, "
                                    f"worker_threads W={y['workers']} (os.cpus() = {y.get('cpus', 1)}, capped at the box's CPU share)"}
    return res


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args))  # no GPU call in this process before the ranks exist
    sys.exit(run_rank(args))


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_entry(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), YCRDT_HUB_PORT=str(port))
    sys.exit(run_rank(parse(), report=q))


def spawn_ranks(args):
    """`bench.py --gpus N` without a launcher: N fresh processes (multiprocessing spawn), rank r on
    device r % devices, the same code path as under torch.distributed.run. Fails unless exactly N
    ranks came up and all of them finished cleanly."""
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_entry, args=(r, args.gpus, port, q)) for r in range(args.gpus)]
    for p in procs:
        p.start()
    for p in procs:
        p.join()
    seen = set()
    while not q.empty():
        seen.add(q.get())
    codes = [p.exitcode for p in procs]
    if any(codes):
        print(f"bench: rank exit codes {codes}", file=sys.stderr, flush=True)
        return 1
    if seen != set(range(args.gpus)):
        print(f"bench: {len(seen)} of {args.gpus} ranks reported ({sorted(seen)})", file=sys.stderr, flush=True)
        return 1
    return 0


def setup_ranks(rank, world, local, report):
    """The engine on this rank's device and libycrdt's communicator. The package's TCP hub
    (crdt_amd/hosthub.py: rank 0 listens on MASTER_PORT + 1, or YCRDT_HUB_PORT; no torch) only
    bootstraps — it carries the RCCL unique id — and is the host transport when ranks share a device
    (RCCL takes one rank per GPU). Barriers, the max-over-ranks step time and every data exchange go
    through libycrdt's Comm."""
    import crdt_amd
    from crdt_amd.hosthub import HostHub

    ndev = crdt_amd.device_count()
    if ndev < 1:
        raise RuntimeError("no HIP device")
    dev = int(os.environ.get("YCRDT_DEVICE", "0")) if world == 1 else local % ndev
    eng = crdt_amd.Engine(device=dev)
    if world == 1:
        return eng, None, ndev
    port = int(os.environ.get("YCRDT_HUB_PORT") or int(os.environ["MASTER_PORT"]) + 1)
    hub = HostHub(world, rank, os.environ.get("MASTER_ADDR", "127.0.0.1"), port)
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if local_world > ndev:  # ranks share a device: the library's collectives over the hub
        comm = crdt_amd.Comm.over_hub(eng, hub)
        comm.transport = f"host exchange over the TCP hub ({local_world} ranks on {ndev} device(s))"
    else:
        uid = hub.bcast(crdt_amd.Comm.unique_id() if rank == 0 else None)
        comm = crdt_amd.Comm(eng, world, rank, uid)
        comm.transport = "rccl"
    comm.hub = hub
    comm.barrier()
    if report is not None:
        report.put(rank)
    return eng, comm, ndev


def run_rank(args, report=None):
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    eng, comm, ndev = setup_ranks(rank, world, local, report)

    import crdt_amd
    from crdt_amd.workload import C1, C2, gen_map

    cfg = dict(C2 if args.workload == "c2" else C1)
    if args.replicas:
        cfg["n_replicas"] = args.replicas
    # every rank merges its own documents (weak scaling); document 0 of rank 0 is the pinned C2
    seeds = [cfg["seed"] + rank * 100_003 + i * 1_009 for i in range(max(1, args.docs))]
    from concurrent.futures import ThreadPoolExecutor

    with ThreadPoolExecutor(16) as ex:
        docs = list(ex.map(lambda sd: gen_map(**dict(cfg, seed=sd))[0], seeds))
    cfg["seed"] = seeds[0]
    updates = docs[0]
    ndocs = len(docs)
    in_bytes = sum(len(u) for d in docs for u in d)

    batch = crdt_amd.Batch(docs=docs, engine=eng) if ndocs > 1 else crdt_amd.Batch(updates, eng)
    st = None
    for _ in range(max(1, args.warmup)):
        st = batch.merge()
    if ndocs > 1:
        results = batch.result_docs()
        out_update, out_sv = results[0]
        out_bytes = sum(len(u) + len(v) for u, v in results)
        del results
    else:
        out_update, out_sv = batch.result()
        out_bytes = len(out_update) + len(out_sv)

    def barrier():
        if comm is not None:
            comm.barrier()  # libycrdt's own transport (RCCL / host exchange)

    # ---- timed region: K merges, inputs resident in HBM. The engine's phase events stay on: they
    # time the dominant kernel live, on the engine stream it runs on (roofline below).
    eng.set_profiling(True)
    phase_acc = {}
    barrier()
    t0 = time.perf_counter()
    dev_ms = 0.0
    for _ in range(args.steps):
        st = batch.merge()  # synchronous: returns after the device finished
        dev_ms += st.device_ms
        for name, ms in eng.phase_times():
            phase_acc[name] = phase_acc.get(name, 0.0) + ms
    barrier()
    t1 = time.perf_counter()
    eng.set_profiling(False)
    dt = t1 - t0
    rank_reports = None
    if comm is not None:
        # the max over the ranks of the step time, the items of all ranks, and each rank's report
        mine = {"rank": rank, "device": local % ndev, "dt_s": dt, "items": int(st.items),
                "ms_per_step": round(dt * 1e3 / args.steps, 4),
                "phases_ms": {n: round(m / args.steps, 4) for n, m in phase_acc.items()}}
        rank_reports = [json.loads(x) for x in comm.allgather(json.dumps(mine).encode())]
        if len(rank_reports) != world:
            raise RuntimeError(f"{len(rank_reports)} rank reports for world {world}")
        dt = max(r["dt_s"] for r in rank_reports)
        items_step = float(sum(r["items"] for r in rank_reports))
    else:
        items_step = float(st.items)
    ms_per_step = dt * 1e3 / args.steps
    value = items_step * args.steps / dt
    phases = [(n, m / args.steps) for n, m in phase_acc.items()]

    # ---- roofline of the dominant kernel. Every single-kernel phase of the merge (one launch,
    # timed by the engine's HIP events on the stream it runs on) with its algorithmic bytes per
    # unit: `roofline` is the one with the longest average launch, `kernels` lists
    # them all. `traffic` is the HBM bytes per launch from the committed rocprofv3 PMC pass
    # (2 x FETCH_SIZE + WRITE_SIZE, gfx950 correction; scripts/pmc.sh + scripts/pmc_summary.py).
    S, G, OS = st.structs, st.segments, st.out_structs
    roof_models = [
        # phase, kernel, algorithmic bytes per launch, per-unit statement
        ("decode.direct", "yc::k_direct", in_bytes + in_bytes * 3 // 8,
         "every input byte read once + spec / final / section-start bitmaps (3 bits per input byte)"),
        ("decode.structs", "yc::k_struct_decode", 42 * S + in_bytes,
         "42 B per struct (position + section read, 34 B of struct columns written) + the struct's own bytes"),
        ("merge.units", "yc::k_units", 37 * S + 5 * st.units,
         "37 B of struct columns per struct + owner (4 B) and flag byte per unit"),
        ("merge.segment_props", "yc::k_seg_props", 85 * G,
         "85 B per segment (unit owner / flags + 7 source-struct columns + origin segment lookup read; "
         "hop record, cidx / src / origin / right origin, winner slot written)"),
        ("merge.resolve", "yc::k_resolve", 28 * G,
         "28 B per segment (hop record read, flags / key written, winner slot read-modify-write)"),
        ("encode.sizes", "yc::k_out_sizes", 8 * G + 46 * OS,
         "8 B per segment (output number, flags) + 46 B per output struct (segment bounds, source + 6 struct "
         "columns read; first segment, client, size written)"),
        ("encode.write", "yc::k_write_structs", 46 * OS + 2 * st.out_bytes,
         "46 B of columns per output struct + every output byte copied (read from the input, written)"),
    ]
    ph = dict(phases)
    kernels = []
    for phase, kname, alg_b, per in roof_models:
        k_ms = ph.get(phase, 0.0)
        if k_ms <= 0:
            continue
        gbs = alg_b / (k_ms * 1e-3) / 1e9
        kernels.append({"kernel": kname, "phase": phase, "avg_launch_ms": round(k_ms, 4), "alg_bytes_per_launch": int(alg_b),
                        "alg_bytes_per_unit": per, "achieved_GBs": round(gbs, 2), "frac": round(gbs / HBM_PEAK_GBS, 5)})
    dom = max(kernels, key=lambda k: k["avg_launch_ms"]) if kernels else None
    ROOF_KERNEL = dom["kernel"] if dom else "yc::k_resolve"
    traffic, traffic_src = None, None
    pmc = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_c2_pmc.csv")))
    rows = []
    if pmc:
        with open(pmc[-1]) as f:
            rows = list(csv.DictReader(f))
        traffic_src = os.path.basename(pmc[-1])
    for k in kernels:
        for r in rows:
            if r["kernel"] == k["kernel"]:
                k["traffic"] = int(float(r["hbm_bytes"]))
    traffic = dom.get("traffic") if dom else None
    # the whole merge's counter traffic from the same PMC pass (sum over its kernels, per merge)
    # (per-dispatch averages x dispatches / merges when the summary counts dispatches: kernels
    # launched several times per merge — scans — count every launch)
    pipe_traffic = None
    if rows:
        merges = max([int(r.get("dispatches") or 1) for r in rows if r["kernel"] == "yc::k_resolve"] or [1])
        pipe_traffic = int(sum(float(r["hbm_bytes"]) * int(r.get("dispatches") or merges) for r in rows) / merges)
    dominant = max(phases, key=lambda p: p[1]) if phases else ("merge", st.device_ms)
    roofline = {
        "bound": "hbm",
        "kernel": ROOF_KERNEL,
        "achieved": dom["achieved_GBs"] if dom else 0.0,
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": dom["frac"] if dom else 0.0,
        "traffic": traffic,
        "traffic_unit": "HBM bytes per launch",
        "traffic_source": traffic_src,
        "alg_bytes_per_launch": dom["alg_bytes_per_launch"] if dom else 0,
        "alg_bytes_per_unit": dom["alg_bytes_per_unit"] if dom else None,
        "avg_launch_ms": dom["avg_launch_ms"] if dom else 0.0,
        "largest_phase": {"name": dominant[0], "ms": round(dominant[1], 4)},
        "kernels": kernels,
    }
    # algorithmic bytes of the whole merge: B_in + B_out + 64·S
    b_alg = in_bytes + out_bytes + 64 * st.structs
    steps_items = st.items

    # ---- end to end (host buffers in, host buffers out): pack + H2D + merge + D2H + per-document
    # split; never `value`
    # A serving loop: batch k+1 is staged (host pack + pinned H2D on the engine's copy stream) by a
    # second host thread while batch k merges and its result comes back; one result buffer is
    # reused. One untimed warm-up batch (pinned areas, first touch of the result buffer).
    e2e_steps = 0 if args.only_headline or args.billion or world > 1 else 4
    make = (lambda: crdt_amd.Batch(docs=docs, engine=eng)) if ndocs > 1 else (lambda: crdt_amd.Batch(updates, eng))
    e2e_ms = 0.0
    if e2e_steps:
        from concurrent.futures import ThreadPoolExecutor

        res_buf = None
        with ThreadPoolExecutor(1) as stager:
            for i in range(e2e_steps + 1):
                if i == 1:
                    e0 = time.perf_counter()
                nxt = stager.submit(make) if i == 0 else nxt
                b2 = nxt.result()
                if i < e2e_steps:
                    nxt = stager.submit(make)  # staged beside this batch's merge and result
                b2.merge()
                blob, _ = b2.result_docs_packed(out=res_buf)  # every document's update + state vector
                res_buf = blob.base if blob.base is not None else blob
                del b2, blob
        e2e_ms = (time.perf_counter() - e0) * 1e3 / e2e_steps
    del batch
    # ---- one C2 document per step (the round-1 headline shape), for continuity
    single = None
    if ndocs > 1 and rank == 0 and not args.only_headline and not args.billion:
        sb = crdt_amd.Batch(updates, eng)
        sst = sb.merge()
        s0 = time.perf_counter()
        for _ in range(10):
            sst = sb.merge()
        sms = (time.perf_counter() - s0) * 1e3 / 10
        single = {"ms_per_step": round(sms, 4), "items_per_step": sst.items, "items_per_s": round(sst.items / (sms * 1e-3), 1)}
        del sb

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.only_headline and not args.billion:
        cpu = cpu_baselines(args, cfg, updates, out_update, crdt_amd.Batch(updates, eng).merge(), eng, gen_map)
    fleet = None
    if rank == 0 and world == 1 and args.fleet_pairs > 0 and not args.only_headline and not args.billion:
        fleet = fleet_sync_leg(eng, args.fleet_pairs)
    ingest = None
    if rank == 0 and world == 1 and args.fleet_docs > 0 and not args.only_headline and not args.billion:
        ingest = fleet_ingest_leg(eng, args.fleet_docs)
    side = rank == 0 and world == 1 and not args.only_headline and not args.billion
    loop = apply_loop_leg(eng, updates, out_update) if side else None
    full_c2 = full_state_leg(eng, "one C2 document's merged state (1 001 clients) as one update", updates, out_update, small_ops=30) if side else None
    per_op = per_op_leg(eng) if side and not args.no_per_op else None
    c3 = c3_leg(eng, args.c3_items) if side and args.c3_items > 0 else None
    c4 = c4_leg(eng) if side and not args.no_c4 else None
    # N > 1: the multi-GPU legs (on by default): C4 key-hash sharded over the ranks, the C5 fleet
    multi = comm is not None and not args.only_headline and not args.billion
    c4s = c4_sharded_leg(eng, comm, world, rank) if multi and not args.no_c4 else None
    fleet_ranks = fleet_ranks_leg(eng, comm, world, rank, args.fleet_docs) if multi and args.fleet_docs > 0 else None
    billion = billion_leg(eng, cfg, gen_map, args.billion) if args.billion and rank == 0 else None
    line = {
        "metric": "CRDT items merged/sec at 1/2/4/8 MI355X + % of HBM roofline",
        "value": round(value, 1),
        "unit": "items/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8/u32 (integer byte-stream + index work)",
        "data": "synthetic (seeded C2 generator, pinned byte-exact against Yjs 13.5.16)",
        "config": {
            "workload": f"{args.workload.upper()} x {ndocs} documents per step, one device pass: YMap 'users', "
                        f"{cfg['n_keys']} keys, {cfg['n_replicas']} replicas x {cfg['ops_per_replica']} set/del ops per "
                        "document" + (", base snapshot" if cfg["base_snapshot"] else ""),
            "docs_per_step": ndocs,
            "updates_per_step": sum(len(d) for d in docs),
            "input_bytes": in_bytes,
            "items_per_step_per_gpu": st.items,
            "structs": st.structs,
            "segments": st.segments,
            "output_bytes": out_bytes,
            "parallelism": f"doc-sharded x{world}",
            "transport": comm.transport if comm is not None else None,
        },
        "ranks": rank_reports,
        "single_doc": single,
        "device_ms_per_step": round(dev_ms / args.steps, 4),
        "unique_items_per_step_per_gpu": st.units,
        "end_to_end": {"ms_per_step": round(e2e_ms, 3), "items_per_s": round(steps_items / (e2e_ms * 1e-3), 1),
                       "x_device": round(e2e_ms / (dev_ms / args.steps), 2) if dev_ms else None,
                       "includes": "host buffers in (no-copy ycrdt_buf packing, pinned pipelined H2D) + merge + "
                                   "per-document split in HBM + pipelined D2H of every document's update and state "
                                   "vector into one reused host array (ycrdt_batch_result_docs_packed); batch k+1 staged by a second host "
                                   "thread beside batch k's merge and result (the engine's copy stream), 1 GPU"} if e2e_steps else None,
        "pipeline_roofline": {
            "b_alg_bytes": b_alg,
            "achieved_GBs": round(b_alg / (ms_per_step * 1e-3) / 1e9, 2),
            "frac": round(b_alg / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
            # HBM / fabric bytes the merge actually moves (PMC, every kernel of one merge) over this
            # step time: how busy the memory system is, against the algorithmic bytes above
            "traffic_bytes": pipe_traffic,
            "traffic_GBs": round(pipe_traffic / (ms_per_step * 1e-3) / 1e9, 2) if pipe_traffic else None,
            "traffic_frac": round(pipe_traffic / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if pipe_traffic else None,
            "traffic_source": traffic_src,
        },
        "roofline": roofline,
        "cpu_baseline": cpu,
        "fleet_sync": fleet,
        "fleet_ingest": ingest,
        "apply_loop": loop,
        "full_state_ingest": full_c2,
        "per_op": per_op,
        "c3": c3,
        "c4": c4,
        "c4_sharded": c4s,
        "fleet_ranks": fleet_ranks,
        "billion": billion,
        "phases_ms": {n: round(m, 4) for n, m in phases},
    }
    # no PyTorch anywhere in a rank (north_star: the host side is libycrdt + its C ABI)
    assert "torch" not in sys.modules, "torch was imported"
    line["torch_loaded"] = False
    if rank == 0:
        print(json.dumps(line), flush=True)
    if comm is not None:
        comm.barrier()
        comm.close()
        comm.hub.close()
    return 0


if __name__ == "__main__":
    main()
