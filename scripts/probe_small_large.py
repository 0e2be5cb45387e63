"""bench.py's C2 full-state leg alone (a C2 document's merged state as one update; then one small
remote delta at a time applied to a doc holding it, crdt.js:294), printed as JSON."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import crdt_amd  # noqa: E402
from crdt_amd.workload import C2, gen_map  # noqa: E402

ups = gen_map(**C2)[0]
eng = crdt_amd.Engine()
b = crdt_amd.Batch(ups, eng)
b.merge()
full = b.result()[0]
del b
print(json.dumps(bench.full_state_leg(eng, "C2 document state", ups, full, small_ops=int(sys.argv[1]) if len(sys.argv) > 1 else 30)), flush=True)
