#!/usr/bin/env python3
"""Where the end-to-end C2 step (bench.py `end_to_end`) spends its time: batch staging (pack + pinned
H2D), the merge, and the per-document packed result (device split + D2H). probe_e2e.py [ndocs]"""
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import crdt_amd  # noqa: E402
from crdt_amd.workload import C2, gen_map  # noqa: E402

nd = int(sys.argv[1]) if len(sys.argv) > 1 else 112
with ThreadPoolExecutor(16) as ex:
    base = list(ex.map(lambda sd: gen_map(**dict(C2, seed=sd))[0], range(2, 2 + min(nd, 16))))
docs = [base[i % len(base)] for i in range(nd)]
eng = crdt_amd.Engine()
for it in range(3):
    t0 = time.perf_counter()
    b = crdt_amd.Batch(docs=docs, engine=eng)
    t1 = time.perf_counter()
    st = b.merge()
    t2 = time.perf_counter()
    blob, offs = b.result_docs_packed()
    t3 = time.perf_counter()
    del b
    t4 = time.perf_counter()
    print("stage %.1f ms, merge %.1f ms (device %.1f), result %.1f ms (%.0f MB), free %.1f ms, total %.1f ms" % (
        (t1 - t0) * 1e3, (t2 - t1) * 1e3, st.device_ms, (t3 - t2) * 1e3, blob.nbytes / 1e6, (t4 - t3) * 1e3, (t4 - t0) * 1e3), flush=True)

# the bench's serving loop: batch k+1 staged by a second host thread beside batch k's merge + result
res = None
with ThreadPoolExecutor(1) as stager:
    nxt = stager.submit(lambda: crdt_amd.Batch(docs=docs, engine=eng))
    for i in range(6):
        if i == 2:
            t0 = time.perf_counter()
        b = nxt.result()
        nxt = stager.submit(lambda: crdt_amd.Batch(docs=docs, engine=eng))
        st = b.merge()
        blob, offs = b.result_docs_packed(out=res)
        res = blob.base if blob.base is not None else blob
        del b, blob
    print("pipelined: %.1f ms per batch (device %.1f)" % ((time.perf_counter() - t0) * 1e3 / 4, st.device_ms), flush=True)
    nxt.result()
