"""Host/device split of one batched diff call (bench fleet_sync shape); diagnostic only."""
import ctypes
import json
import os
import time

import crdt_amd
from crdt_amd import _bufs, _Out, _check, _take, lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
cases = [c for c in json.load(open(os.path.join(ROOT, "tests", "golden", "configs.json")))["cases"] if c["name"].startswith("c5_")]
base = []
for c in cases:
    st = bytes.fromhex(c["state"])
    base += [(st, bytes.fromhex(d["sv"])) for d in c["diffs"]] + [(st, b"\x00")]
n = 20000
ups = [base[i % len(base)][0] for i in range(n)]
svs = [base[i % len(base)][1] for i in range(n)]
eng = crdt_amd.default_engine()
crdt_amd.diff_updates(ups, svs, eng)
for _ in range(3):
    t0 = time.perf_counter()
    ua, uk = _bufs(ups)
    va, vk = _bufs(svs)
    t1 = time.perf_counter()
    outs = (_Out * n)()
    _check(lib().ycrdt_diff_updates(eng._h, ua, va, n, outs))
    t2 = time.perf_counter()
    res = [_take(outs[i]) for i in range(n)]
    t3 = time.perf_counter()
    print(f"bufs {1e3*(t1-t0):.2f} ms  C call {1e3*(t2-t1):.2f} ms  take {1e3*(t3-t2):.2f} ms", flush=True)
