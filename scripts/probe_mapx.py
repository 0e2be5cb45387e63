"""A corrupt.json case: the engine's state vs the oracle's, struct by struct (diagnostics)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import crdt_amd  # noqa: E402
from oracle.yref import Doc as ODoc  # noqa: E402
from oracle.ymerge import Dec, lazy_structs, read_delete_set  # noqa: E402

fx = json.load(open(os.path.join(ROOT, "tests", "golden", "corrupt.json")))
name = sys.argv[1] if len(sys.argv) > 1 else "small2_b1340_127"
c = [x for x in fx["cases"] if x["name"] == name][0]
u = bytearray(bytes.fromhex(fx["sources"][c["src"]]))
u[c["at"]] = c["val"]
base = bytes.fromhex(fx["base"])


def show(st):
    d = Dec(st)
    ss = lazy_structs(d)
    ds = read_delete_set(d)
    return [f"{s.kind} {s.client}:{s.clock}+{s.length} ref{s.ref} o={s.origin} r={s.right_origin} p={s.parent} ps={s.parent_sub}" for s in ss], ds


o = ODoc(5)
o.apply_update(base)
o.apply_update(bytes(u))
want = o.encode_state_as_update()
g = crdt_amd.Doc(client_id=5)
g.apply_update(base)
g.apply_update(bytes(u))
got = g.encode_state_as_update()
ws, wd = show(want)
gs, gd = show(got)
print("equal", want == got, len(ws), len(gs))
for i in range(max(len(ws), len(gs))):
    a = ws[i] if i < len(ws) else "-"
    b = gs[i] if i < len(gs) else "-"
    print(("   " if a == b else "!! ") + a + ("" if a == b else "   |   " + b))
print("ds want", wd)
print("ds got ", gd)
print("the update:")
for line in show(bytes(u))[0]:
    print("  ", line)
