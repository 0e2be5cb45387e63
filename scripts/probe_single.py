#!/usr/bin/env python3
"""One C2 document (BASELINE configs[1]) merged alone, per phase: the latency-bound single-document
shape of bench.py's `single_doc`. Usage: probe_single.py [reps]. YCRDT_DECODE=direct|chunks forces a
decode path for the small updates."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import crdt_amd  # noqa: E402
from crdt_amd.workload import C2, gen_map  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
subset = sys.argv[2] if len(sys.argv) > 2 else "all"  # all | base | replicas
ups = gen_map(**C2)[0]
if subset == "base":
    ups = ups[:1]
elif subset == "replicas":
    ups = ups[1:]
eng = crdt_amd.Engine()
b = crdt_amd.Batch(ups, eng)
st = b.merge()
ref = b.result()[0]
t0 = time.perf_counter()
for _ in range(reps):
    st = b.merge()
ms = (time.perf_counter() - t0) * 1e3 / reps
eng.set_profiling(True)
acc = {}
for _ in range(reps):
    b.merge()
    for n, m in eng.phase_times():
        acc[n] = acc.get(n, 0.0) + m / reps
eng.set_profiling(False)
print("updates", len(ups), "bytes", sum(map(len, ups)), "items", st.items, "structs", st.structs)
print("wall ms/merge %.3f device ms %.3f" % (ms, st.device_ms))
print({k: round(v, 3) for k, v in acc.items()})
print("parity(self)", b.result()[0] == ref)
