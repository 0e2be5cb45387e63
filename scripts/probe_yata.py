"""Times the YArray integration (tree vs sequential kernels) on seeded many-replica array histories
(tests/histories.py, built with the CPU oracle) and checks both against the oracle's merge."""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if len(sys.argv) > 1 and sys.argv[1] == "child":
    import pickle

    import crdt_amd

    batch, want = pickle.load(open(sys.argv[2], "rb"))
    eng = crdt_amd.Engine()
    eng.set_profiling(True)
    b = crdt_amd.Batch(batch, eng)
    b.merge()
    best = 1e9
    for _ in range(3):
        st = b.merge()
        ph = dict(eng.phase_times())
        best = min(best, ph.get("merge.yata", 0.0))
    out = b.result()[0]
    print(f"  {os.environ.get('YCRDT_YATA', 'tree'):5s} merge.yata {best:8.3f} ms  total {st.device_ms:8.3f} ms  "
          f"segments {st.segments}  equal_oracle {out == want}")
    sys.exit(0)

import pickle  # noqa: E402

from oracle.yref import Doc  # noqa: E402
from tests.histories import array_history  # noqa: E402

for reps, rounds, ops in ((16, 4, 20), (64, 4, 10), (128, 3, 8)):
    t0 = time.time()
    states, wire = array_history(900 + reps, n_replicas=reps, rounds=rounds, ops=ops)
    batch = states + wire
    d = Doc(0x7FFFFFF0)
    t1 = time.time()
    for u in batch:
        d.apply_update(u)
    want = d.encode_state_as_update()
    t2 = time.time()
    print(f"{reps} replicas x {rounds} rounds x {ops} ops: {len(batch)} updates; oracle merge {1e3 * (t2 - t1):.1f} ms (gen {t1 - t0:.1f} s)")
    f = f"/tmp/yata_{reps}.pkl"
    pickle.dump((batch, want), open(f, "wb"))
    for mode in ("tree", "seq"):
        env = dict(os.environ)
        if mode == "seq":
            env["YCRDT_YATA"] = "seq"
        subprocess.run([sys.executable, __file__, "child", f], env=env, check=True)
