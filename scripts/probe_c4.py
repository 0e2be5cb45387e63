"""C4 decode probe on the GPU: phase times of the base snapshot alone, the replica updates alone and
the whole C4 batch (crdt_amd/workload C4).

    python scripts/probe_c4.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import crdt_amd  # noqa: E402
from crdt_amd.workload import C4, gen_nested  # noqa: E402

ups, st = gen_nested(**C4)
print(f"{len(ups)} updates, base {len(ups[0]) / 1e6:.2f} MB, replicas {sum(map(len, ups[1:])) / 1e6:.1f} MB, {st}", flush=True)
eng = crdt_amd.Engine()
for name, sel in (("base", ups[:1]), ("all", ups)):
    b = crdt_amd.Batch(sel, eng)
    b.merge()
    eng.set_profiling(True)
    s = b.merge()
    ph = eng.phase_times()
    eng.set_profiling(False)
    t0 = time.perf_counter()
    b.merge()
    ms = (time.perf_counter() - t0) * 1e3
    print(f"{name}: {ms:.1f} ms wall, device {s.device_ms:.2f} ms;", ", ".join(f"{n} {m:.3f}" for n, m in ph if m > 0.05), flush=True)
    del b
