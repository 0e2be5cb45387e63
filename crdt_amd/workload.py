"""Seeded synthetic replica-update workloads for tests and bench.py.

Thin ctypes wrapper over crdt_amd/workload/ycw.cpp (built as crdt_amd/libycrdt_workload.so).
"""
import ctypes
import json
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
_L = None


def _lib():
    global _L
    if _L is None:
        L = ctypes.CDLL(os.path.join(_HERE, "libycrdt_workload.so"))
        P = ctypes.POINTER
        L.ycw_gen_map.argtypes = [
            ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_double, ctypes.c_double, ctypes.c_int,
            ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int,
            P(ctypes.c_void_p), P(ctypes.c_size_t), P(ctypes.c_void_p), P(ctypes.c_size_t), P(ctypes.c_void_p),
        ]
        L.ycw_gen_array.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32,
                                    P(ctypes.c_void_p), P(ctypes.c_size_t), P(ctypes.c_void_p), P(ctypes.c_size_t),
                                    P(ctypes.c_uint64), P(ctypes.c_void_p), P(ctypes.c_size_t)]
        L.ycw_gen_nested.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_double,
                                     ctypes.c_double, ctypes.c_uint32, P(ctypes.c_void_p), P(ctypes.c_size_t),
                                     P(ctypes.c_void_p), P(ctypes.c_size_t), P(ctypes.c_uint64)]
        L.ycw_free.argtypes = [ctypes.c_void_p]
        _L = L
    return _L


# SURVEY.md §8(d)
C1 = dict(n_keys=1000, n_replicas=2, ops_per_replica=10000, zipf_s=0.0, p_set=0.8, base_snapshot=False,
          base_client=1, client_mode=1, value_mode=1, seed=42)
C2 = dict(n_keys=100_000, n_replicas=1000, ops_per_replica=1000, zipf_s=1.1, p_set=0.8, base_snapshot=True,
          base_client=1, client_mode=0, value_mode=0, seed=2)
C3 = dict(n_replicas=256, rounds=16, items=10_000_000, seed=3)
# C4 (nested YArrays under YMap keys): 100k keys, 2 000 replicas x 10 000 ops ~= 50 M items per
# document; BASELINE's 100 M items is two such documents' worth per GPU pair, key-hash sharded
C4 = dict(n_replicas=2000, n_keys=100_000, pushes=10_000, init_len=4, p_over=0.02, p_del=0.05, seed=4)
# C4 at BASELINE scale: 1 M keys, 64 replicas, ~100 items per nested array (102 M
# items, 41 M structs, 716 MB of updates), ~10 % of the keys overwritten by a fresh array
C4_FULL = dict(n_replicas=64, n_keys=1_000_000, pushes=640_000, init_len=4, p_over=0.0025, p_del=0.05, seed=4)


def gen_nested(n_replicas, n_keys, pushes, init_len=4, p_over=0.02, p_del=0.05, seed=4):
    """C4-shaped workload (crdt_amd/workload/ycw_nested.cpp): the base snapshot + one update per
    replica. Returns (updates: list[bytes], stats: dict(items, structs, deletes))."""
    L = _lib()
    data, dlen, offs, nupd = ctypes.c_void_p(), ctypes.c_size_t(), ctypes.c_void_p(), ctypes.c_size_t()
    st = (ctypes.c_uint64 * 3)()
    rc = L.ycw_gen_nested(n_replicas, n_keys, pushes, init_len, p_over, p_del, seed, ctypes.byref(data),
                          ctypes.byref(dlen), ctypes.byref(offs), ctypes.byref(nupd), st)
    if rc != 0:
        raise ValueError("bad workload config")
    try:
        raw = ctypes.string_at(data.value, dlen.value) if dlen.value else b""
        o = (ctypes.c_uint64 * (nupd.value + 1)).from_address(offs.value)
        ups = [raw[o[i]:o[i + 1]] for i in range(nupd.value)]
    finally:
        L.ycw_free(data)
        L.ycw_free(offs)
    return ups, {"items": st[0], "structs": st[1], "deletes": st[2]}


def gen_array(n_replicas=256, rounds=16, items=10_000_000, seed=3, order=False):
    """C3-shaped YArray workload (crdt_amd/workload/ycw_array.cpp): every replica's per-round wire
    update. Returns (updates: list[bytes], stats: dict); with order=True stats["order"] lists the
    final live values as (client, clock) in the generator's list order."""
    L = _lib()
    data, dlen, offs, nupd = ctypes.c_void_p(), ctypes.c_size_t(), ctypes.c_void_p(), ctypes.c_size_t()
    st = (ctypes.c_uint64 * 4)()
    op, no = ctypes.c_void_p(), ctypes.c_size_t()
    rc = L.ycw_gen_array(n_replicas, rounds, items, seed, ctypes.byref(data), ctypes.byref(dlen), ctypes.byref(offs),
                         ctypes.byref(nupd), st, ctypes.byref(op) if order else None, ctypes.byref(no) if order else None)
    if rc != 0:
        raise ValueError("bad workload config")
    try:
        raw = ctypes.string_at(data.value, dlen.value) if dlen.value else b""
        o = (ctypes.c_uint64 * (nupd.value + 1)).from_address(offs.value)
        ups = [raw[o[i]:o[i + 1]] for i in range(nupd.value)]
        stats = {"ops": st[0], "items": st[1], "deleted": st[2], "length": st[3]}
        if order:
            a = (ctypes.c_uint32 * (2 * no.value + 1)).from_address(op.value)
            stats["order"] = [(a[2 * i], a[2 * i + 1]) for i in range(no.value)]
            L.ycw_free(op)
    finally:
        L.ycw_free(data)
        L.ycw_free(offs)
    return ups, stats


def gen_map(n_keys, n_replicas, ops_per_replica, zipf_s=1.1, p_set=0.8, base_snapshot=True, base_client=1,
            client_mode=0, value_mode=0, seed=2, script=False):
    """Returns (updates: list[bytes], script: dict|None)."""
    L = _lib()
    data, dlen, offs, nupd, sc = ctypes.c_void_p(), ctypes.c_size_t(), ctypes.c_void_p(), ctypes.c_size_t(), ctypes.c_void_p()
    rc = L.ycw_gen_map(n_keys, n_replicas, ops_per_replica, zipf_s, p_set, 1 if base_snapshot else 0, base_client,
                       client_mode, value_mode, seed, 1 if script else 0, ctypes.byref(data), ctypes.byref(dlen),
                       ctypes.byref(offs), ctypes.byref(nupd), ctypes.byref(sc) if script else None)
    if rc != 0:
        raise ValueError("bad workload config")
    try:
        raw = ctypes.string_at(data.value, dlen.value) if dlen.value else b""
        o = (ctypes.c_uint64 * (nupd.value + 1)).from_address(offs.value)
        ups = [raw[o[i]:o[i + 1]] for i in range(nupd.value)]
        js = json.loads(ctypes.string_at(sc.value).decode()) if script else None
    finally:
        L.ycw_free(data)
        L.ycw_free(offs)
        if script:
            L.ycw_free(sc)
    return ups, js

