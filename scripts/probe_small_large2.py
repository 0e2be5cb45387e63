"""One small peer delta at a time into a doc holding a C2 document's state (crdt.js:294): per-apply
merge time and the engine's phase times, with the doc-state marks on (default) and off."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import crdt_amd  # noqa: E402
from crdt_amd.workload import C2, gen_map  # noqa: E402
from oracle.yref import Doc as ODoc  # noqa: E402

ups = gen_map(**C2)[0]
eng = crdt_amd.Engine()
b = crdt_amd.Batch(ups, eng)
b.merge()
full = b.result()[0]
del b
peer = ODoc(0x5EED0001)
peer.apply_update(full)
deltas = []
for i in range(12):
    sv = peer.encode_state_vector()
    peer.map_set("users", "k%d" % (i * 7919 % 100_000), bench._any_str("w%d" % i))
    deltas.append(peer.encode_state_as_update(sv))
for mode in sys.argv[1:] or ["1", "0"]:
    os.environ["YCRDT_PREDECODE"] = mode
    d = crdt_amd.Doc(client_id=0x7FFFFFF0, engine=eng)
    d.apply_update(full)
    d.encode_state_vector()
    eng.set_profiling(True)
    ts = []
    for u in deltas:
        t0 = time.perf_counter()
        d.apply_update(u)
        d.encode_state_vector()
        ts.append((time.perf_counter() - t0) * 1e3)
    ph = eng.phase_times()
    eng.set_profiling(False)
    print("PREDECODE", mode, "apply+merge ms", " ".join(f"{t:.2f}" for t in ts), "device", f"{d.last_stats().device_ms:.2f}", flush=True)
    print("  ", ", ".join(f"{n} {m:.3f}" for n, m in ph if m > 0.03), flush=True)
    print("   equal:", d.encode_state_as_update() == peer.encode_state_as_update(), flush=True)
