"""Phases of one small remote delta merged into a doc holding a C2 document's state (bench
small_into_large): which passes the 1.4 ms of device time go to."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import crdt_amd  # noqa: E402
from bench import _any_str  # noqa: E402
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
for i in range(40):
    sv = peer.encode_state_vector()
    peer.map_set("users", "k%d" % (i * 7919 % 100_000), _any_str("w%d" % i))
    deltas.append(peer.encode_state_as_update(sv))
d = crdt_amd.Doc(client_id=0x7FFFFFF0, engine=eng)
d.apply_update(full)
d.encode_state_vector()
for u in deltas[:10]:
    d.apply_update(u)
    d.encode_state_vector()
eng.set_profiling(True)
acc, n = {}, 0
t0 = time.perf_counter()
for u in deltas[10:]:
    d.apply_update(u)
    d.encode_state_vector()
    for k, m in eng.phase_times():
        acc[k] = acc.get(k, 0.0) + m
    n += 1
ms = (time.perf_counter() - t0) * 1e3 / n
eng.set_profiling(False)
st = d.last_stats()
print("wall ms/apply (profiling on) %.3f device ms %.3f" % (ms, st.device_ms))
print({k: round(v / n, 3) for k, v in acc.items()})
print("parity", d.encode_state_as_update() == peer.encode_state_as_update())
