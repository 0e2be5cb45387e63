"""One C2 document's merged state (1 001 clients) merged alone — crdt.js's full-state wire shape —
with the engine's phase times and YCRDT_DEBUG_DECODE lines (diagnostics)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import crdt_amd  # noqa: E402
from crdt_amd.workload import C2, gen_map  # noqa: E402

if os.environ.get("PROBE_WL") == "c3":  # (a C3 state: 256 sections of ~600 KB; with PROBE_HALF=1 behind half of it)
    from crdt_amd.workload import gen_array
    ups = gen_array(256, 16, 10_000_000, 3)[0]
else:
    ups = gen_map(**C2)[0]
eng = crdt_amd.Engine()
b = crdt_amd.Batch(ups, eng)
b.merge()
full = b.result()[0]
del b
print("full state", len(full), flush=True)
src = [full]
if os.environ.get("PROBE_HALF") == "1":
    hb = crdt_amd.Batch(ups[: len(ups) // 2], eng)
    hb.merge()
    src = [hb.result()[0], full]
    del hb
eng.set_profiling(True)
res = {}
CONFIGS = {"1": {}, "0": {}}  # record mode on (the default) and off; more from argv: name:VAR=v,VAR=v
for a in sys.argv[1:]:
    name, kv = a.split(":", 1)
    CONFIGS[name] = dict(x.split("=", 1) for x in kv.split(","))
for fwc, env in CONFIGS.items():
    for k in ("YCRDT_FWC_WALK", "YCRDT_SPEC_HINT", "YCRDT_SCHUNK", "YCRDT_RTAB", "YCRDT_RANK_LAST"):
        os.environ.pop(k, None)
    os.environ.update(env)
    os.environ["YCRDT_FWC"] = fwc if fwc in ("0", "1") else env.get("YCRDT_FWC", "1")
    fb = crdt_amd.Batch(src, eng)
    os.environ["YCRDT_DEBUG_DECODE"] = "1"
    print(fwc, env, flush=True)
    fb.merge()
    os.environ.pop("YCRDT_DEBUG_DECODE")
    for _ in range(3):
        t0 = time.perf_counter()
        st = fb.merge()
        print(f"YCRDT_FWC={fwc}: merge {1e3 * (time.perf_counter() - t0):.2f} ms, device {st.device_ms:.2f}", flush=True)
    res[fwc] = fb.result()
    print(", ".join(f"{n} {m:.3f}" for n, m in eng.phase_times() if m > 0.05), flush=True)
print("all configs equal:", all(r == res["0"] for r in res.values()), "state equal:", res["1"][0] == full, flush=True)
