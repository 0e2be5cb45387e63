"""Per-op loop breakdown (bench.py per_op_leg): time spent in each facade call, per call type."""
import sys
import time

sys.path.insert(0, ".")
import crdt_amd  # noqa: E402
from bench import _any_str  # noqa: E402


def run(n_ops):
    eng = crdt_amd.default_engine()
    a = crdt_amd.Doc(client_id=1, engine=eng)
    b = crdt_amd.Doc(client_id=2, engine=eng)
    a.track_local(False)
    t = {"set": 0.0, "encode": 0.0, "apply": 0.0, "json": 0.0}
    ph = {}
    for i in range(n_ops):
        key = "user%d" % (i % 100)
        t0 = time.perf_counter()
        if i % 5 == 4:
            a.map_delete("users", key)
        else:
            a.map_set("users", key, _any_str("v%d" % i))
        t1 = time.perf_counter()
        u = a.encode_state_as_update()
        t2 = time.perf_counter()
        b.apply_update(u)
        t3 = time.perf_counter()
        b.root_json("users", "map")
        t4 = time.perf_counter()
        t["set"] += t1 - t0; t["encode"] += t2 - t1; t["apply"] += t3 - t2; t["json"] += t4 - t3
        if i == n_ops - 1:
            for d, name in ((a, "a"), (b, "b")):
                try:
                    st = d.last_stats()
                    ph[name] = {f: getattr(st, f) for f, _ in st._fields_}
                except Exception as e:  # noqa: BLE001
                    ph[name] = repr(e)
    eng.set_profiling(True)
    b.apply_update(u)
    b.root_json("users", "map")
    print("b phases", [(n, round(m, 3)) for n, m in eng.phase_times()], flush=True)
    a.map_set("users", "x", _any_str("y"))
    a.encode_state_as_update()
    print("a phases", [(n, round(m, 3)) for n, m in eng.phase_times()], flush=True)
    eng.set_profiling(False)
    print(n_ops, {k: round(v / n_ops * 1e3, 3) for k, v in t.items()}, "ms/op", flush=True)
    print(ph, flush=True)


if __name__ == "__main__":
    import os
    for n in [int(x) for x in os.environ.get("PEROP_N", "500,2000").split(",")]:
        run(n)
