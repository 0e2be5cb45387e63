"""bench.py's per-op loop (crdt.js:433-445 then 294-305) with the doc-state marks on and off, and the
single-document merge (one C2 document's 1 000 replica updates in one batch)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import crdt_amd  # noqa: E402

eng = crdt_amd.Engine()
for mode in ("1", "0", "1"):
    os.environ["YCRDT_PREDECODE"] = mode
    res = bench.per_op_leg.__wrapped__(eng, (500, 2000)) if hasattr(bench.per_op_leg, "__wrapped__") else None
    if res is None:
        import bench as B
        saved = B._yjs_perop
        B._yjs_perop = lambda n: None  # (the Yjs loop is timed by bench.py itself)
        res = B.per_op_leg(eng, (500, 2000))
        B._yjs_perop = saved
    print("PREDECODE", mode, {k: (v["ops_per_s"], v["breakdown"]["device_ms_per_op"], v["breakdown"]["host_ms_per_op"]) for k, v in res.items()}, flush=True)
