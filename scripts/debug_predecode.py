"""YCRDT_PREDECODE=check over the pending.json replays: the first case / step whose doc-state marks
differ from the state's decode, with the state bytes (from a doc without marks) printed."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import crdt_amd  # noqa: E402

cases = json.load(open(os.path.join(ROOT, "tests", "golden", "pending.json")))["cases"]
for c in cases:
    os.environ["YCRDT_PREDECODE"] = "check"
    d = crdt_amd.Doc(client_id=0x7FFFFFF0)
    for k, u in enumerate(c["updates"]):
        d.apply_update(bytes.fromhex(u))
        try:
            d.pending()
            d.encode_state_as_update()
        except crdt_amd.YcrdtError as e:
            print("case", c["name"], "step", k, e)
            os.environ["YCRDT_PREDECODE"] = "0"
            s = crdt_amd.Doc(client_id=0x7FFFFFF0)
            for j in range(k):
                s.apply_update(bytes.fromhex(c["updates"][j]))
                print(" after", j, "pending", s.pending(), "state", s.encode_state_as_update().hex())
            print(" update", k, c["updates"][k])
            raise SystemExit(0)
print("no mismatch")
