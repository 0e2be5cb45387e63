"""Throughput of concurrent engines on one GPU: the C2 x 112-document batch merged K times by one
engine, then by E engines (own HIP streams and workspaces) from E host threads (ctypes releases
the GIL), each merging its own copy of the batch K/E times.

    python scripts/probe_engines.py [docs] [K] [E]
"""
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import crdt_amd  # noqa: E402
from crdt_amd.workload import C2, gen_map  # noqa: E402

ndocs = int(sys.argv[1]) if len(sys.argv) > 1 else 112
K = int(sys.argv[2]) if len(sys.argv) > 2 else 8
E = int(sys.argv[3]) if len(sys.argv) > 3 else 2
seeds = [C2["seed"] + i * 1_009 for i in range(ndocs)]
with ThreadPoolExecutor(16) as ex:
    docs = list(ex.map(lambda sd: gen_map(**dict(C2, seed=sd))[0], seeds))
engs = [crdt_amd.Engine() for _ in range(E)]
batches = [crdt_amd.Batch(docs=docs, engine=e) for e in engs]
for b in batches:
    b.merge()
items = batches[0].merge().items
t0 = time.perf_counter()
for _ in range(K):
    batches[0].merge()
t1 = time.perf_counter()
print(f"1 engine: {K} merges {1e3 * (t1 - t0) / K:.2f} ms/merge, {items * K / (t1 - t0) / 1e9:.3f} G items/s", flush=True)


def run(b):
    for _ in range(K // E):
        b.merge()


with ThreadPoolExecutor(E) as ex:
    t0 = time.perf_counter()
    list(ex.map(run, batches))
    t1 = time.perf_counter()
n = (K // E) * E
print(f"{E} engines: {n} merges {1e3 * (t1 - t0) / n:.2f} ms/merge, {items * n / (t1 - t0) / 1e9:.3f} G items/s", flush=True)
outs = [b.result_docs()[0][0] for b in batches]
print("same output:", all(o == outs[0] for o in outs), flush=True)
