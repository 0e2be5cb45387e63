"""One C2 document's merged state (1 001 clients) merged alone — crdt.js's full-state wire shape —
with the engine's phase times and YCRDT_DEBUG_DECODE lines (diagnostics)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import crdt_amd  # noqa: E402
from crdt_amd.workload import C2, gen_map  # noqa: E402

ups = gen_map(**C2)[0]
eng = crdt_amd.Engine()
b = crdt_amd.Batch(ups, eng)
b.merge()
full = b.result()[0]
del b
print("full state", len(full), flush=True)
os.environ["YCRDT_DEBUG_DECODE"] = "1"
fb = crdt_amd.Batch([full], eng)
fb.merge()
os.environ.pop("YCRDT_DEBUG_DECODE")
eng.set_profiling(True)
for _ in range(3):
    t0 = time.perf_counter()
    st = fb.merge()
    print(f"merge {1e3 * (time.perf_counter() - t0):.2f} ms, device {st.device_ms:.2f}", flush=True)
print(", ".join(f"{n} {m:.3f}" for n, m in eng.phase_times() if m > 0.05), flush=True)
