"""One workload merged three times (the last one traced by rocprofv3 --kernel-trace; the caller
prints it with scripts/trace_last.py): c4 (BASELINE C4 scale), c3, c2full (a C2 document's merged
state as one update), c2x112 (the headline batch), perop (bench.py's per-op loop)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import crdt_amd  # noqa: E402
from crdt_amd import workload as W  # noqa: E402

which = sys.argv[1]
if which == "c4":
    ups, _ = W.gen_nested(**W.C4_FULL)
elif which == "c3":
    ups, _ = W.gen_array(256, 16, 10_000_000, 3)
elif which == "c2full":
    b = crdt_amd.Batch(W.gen_map(**W.C2)[0])
    b.merge()
    ups = [b.result()[0]]
    del b
elif which == "c2x112":
    from concurrent.futures import ThreadPoolExecutor
    seeds = [W.C2["seed"] + i * 1_009 for i in range(112)]  # bench.py's documents (rank 0)
    with ThreadPoolExecutor(16) as ex:
        docs = list(ex.map(lambda sd: W.gen_map(**dict(W.C2, seed=sd))[0], seeds))
elif which == "perop":  # bench.py's per-op loop (crdt.js set + full encode, apply + toJSON)
    import bench
    print(bench.per_op_leg(crdt_amd.Engine(), (300,)), flush=True)
    raise SystemExit(0)
else:
    raise SystemExit("workload?")
eng = crdt_amd.Engine()
b = crdt_amd.Batch(docs=docs, engine=eng) if which == "c2x112" else crdt_amd.Batch(ups, eng)
for _ in range(3):
    st = b.merge()
print(which, st.as_dict(), flush=True)
