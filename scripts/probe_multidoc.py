"""K independent C2 documents (different seeds) merged in ONE device pass (multi-document batch):
device time, items/s and phases vs K.

    python scripts/probe_multidoc.py [K ...]
"""
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import crdt_amd  # noqa: E402
from crdt_amd.workload import C2, gen_map  # noqa: E402

ks = [int(x) for x in sys.argv[1:]] or [1, 10, 50, 100]
t0 = time.time()
with ThreadPoolExecutor(16) as ex:
    docs = list(ex.map(lambda i: gen_map(**dict(C2, seed=1000 + i))[0], range(max(ks))))
print(f"generated {len(docs)} C2 docs in {time.time() - t0:.1f} s", flush=True)
eng = crdt_amd.Engine()
for k in ks:
    b = crdt_amd.Batch(docs=docs[:k], engine=eng)
    st = b.merge()
    eng.set_profiling(True)
    best = None
    for _ in range(3):
        t1 = time.perf_counter()
        st = b.merge()
        wall = time.perf_counter() - t1
        if best is None or wall < best[0]:
            best = (wall, eng.phase_times())
    eng.set_profiling(False)
    inb = sum(len(u) for d in docs[:k] for u in d)
    print(f"K={k:4d}: {st.items / 1e6:7.1f} M items, {inb / 1e6:8.1f} MB in, wall {best[0] * 1e3:8.2f} ms, "
          f"{st.items / best[0] / 1e6:8.1f} M items/s | " + ", ".join(f"{n} {m:.2f}" for n, m in best[1] if m > 0.2), flush=True)
    del b
