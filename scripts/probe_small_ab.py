"""Per-op loop (bench.py per_op_leg) with the single-workgroup small-batch kernels on / off,
alternated in ONE process (the switches are read per merge): ops/s per mode and round."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import crdt_amd  # noqa: E402

MODES = {
    "all_on": {},
    "quick_off": {"YCRDT_DECODE_QUICK": "0"},
    "fence": {"YCRDT_PHASE_FENCE": "1"},
    "merge_off": {"YCRDT_MERGE_SMALL": "0"},
    "all_off": {"YCRDT_MERGE_SMALL": "0", "YCRDT_ENCODE_SMALL": "0", "YCRDT_DECODE_SMALL": "0", "YCRDT_VIEW_SMALL": "0"},
}
bench._yjs_perop = lambda n: None  # (the Yjs leg is not compared here)
eng = crdt_amd.Engine()
bench.per_op_leg(eng, (100,))  # warm-up
res = {m: [] for m in MODES}
for rnd in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    for m, env in MODES.items():
        for k in ("YCRDT_MERGE_SMALL", "YCRDT_ENCODE_SMALL", "YCRDT_DECODE_SMALL", "YCRDT_VIEW_SMALL", "YCRDT_DECODE_QUICK", "YCRDT_PHASE_FENCE"):
            os.environ.pop(k, None)
        os.environ.update(env)
        r = bench.per_op_leg(eng, (500,))["500"]
        res[m].append((r["ops_per_s"], r["breakdown"]["device_ms_per_op"]))
        print(rnd, m, r["ops_per_s"], r["breakdown"]["device_ms_per_op"], flush=True)
for m, v in res.items():
    print(m, "ops/s", [x[0] for x in v], "device ms/op", [x[1] for x in v])
