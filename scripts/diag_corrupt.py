"""Diagnostics for tests/test_gpu_corrupt.py: every case in every decode mode; mismatches (with the
engine's state bytes) written to gpurun_out/corrupt_diag.json."""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import crdt_amd  # noqa: E402

fx = json.load(open(os.path.join(ROOT, "tests", "golden", "corrupt.json")))
base = bytes.fromhex(fx["base"])
out = []
for mode in ("direct", "wave", "chunks"):
    os.environ["YCRDT_DECODE"] = "direct" if mode == "wave" else mode
    os.environ["YCRDT_DIRECT_WAVE"] = "1" if mode == "wave" else "0"
    for c in fx["cases"]:
        u = bytearray(bytes.fromhex(fx["sources"][c["src"]]))
        bad = bytes(u[: c["cut"]]) if "cut" in c else bytes(u[: c["at"]] + bytes([c["val"]]) + u[c["at"] + 1:])
        d = crdt_amd.Doc(client_id=5)
        d.apply_update(base)
        err = None
        try:
            d.apply_update(bad)
        except crdt_amd.YcrdtError as e:
            err = str(e)
        try:
            st = d.encode_state_as_update()
        except crdt_amd.YcrdtError as e:
            out.append({"mode": mode, "name": c["name"], "threw": c["threw"], "engine_err": err, "read_err": str(e)})
            continue
        ok = ((err is not None) == (c["threw"] is not None)) and (not c["state_sha256"] or hashlib.sha256(st).hexdigest() == c["state_sha256"]) \
            and d.encode_state_vector().hex() == c["sv"]
        if not ok:
            out.append({"mode": mode, "name": c["name"], "threw": c["threw"], "engine_err": err, "state": st.hex(),
                        "sv": d.encode_state_vector().hex(), "want_sv": c["sv"]})
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(out, open(os.path.join(ROOT, "gpurun_out", "corrupt_diag.json"), "w"))
print(len(out), "mismatches;", sorted({(o["mode"], o["name"]) for o in out})[:40])
