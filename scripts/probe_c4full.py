#!/usr/bin/env python3
"""C4 at BASELINE scale (crdt_amd.workload.C4_FULL) merged a few times, per phase (rocprof target)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import crdt_amd  # noqa: E402
from crdt_amd.workload import C4_FULL, gen_nested  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
ups, st = gen_nested(**C4_FULL)
eng = crdt_amd.Engine()
b = crdt_amd.Batch(ups, eng)
b.merge()
eng.set_profiling(True)
for _ in range(reps):
    t0 = time.perf_counter()
    s = b.merge()
    print("merge ms %.2f" % ((time.perf_counter() - t0) * 1e3), {n: round(m, 2) for n, m in eng.phase_times()}, flush=True)
