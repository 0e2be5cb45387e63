"""crdt_amd — MI355X-native batched Yjs merge engine (Python mirror of the `Y` surface).

The reference (@ypear/crdt) talks to its CRDT engine only through the object injected as
`router.options.Y` (reference crdt.js:175-180). This module exposes the same surface on top of
the C ABI in include/ycrdt.h (libycrdt.so, hand-written gfx950 HIP kernels):

    Doc()                         new Y.Doc()                      crdt.js:33,54,56,80,221
    apply_update(doc, u8)         Y.applyUpdate(doc, u8)           crdt.js:35,56,58,85,294
    apply_updates(doc, [u8])      n × Y.applyUpdate, one batch     crdt.js:79-98 (LevelDB replay)
    encode_state_as_update(doc[, sv])  Y.encodeStateAsUpdate       crdt.js:56,260,288,347,443,...
    encode_state_vector(doc)      Y.encodeStateVector(doc)         crdt.js:59,239,258,289
    merge_updates([u8])           Y.mergeUpdates                   north_star (Y@39011)
    diff_update(u8, sv)           Y.diffUpdate                     Y@40711
    diff_updates(u8s, svs)        n x Y.diffUpdate, one batched pass (crdt.js:286-291 sync responder)

Errors raise YcrdtError (the reference only reads `e.message`, crdt.js:38-39). There is no CPU
fallback: importing works without a GPU, but every compute call needs the HIP device.
"""
import ctypes
import os

__all__ = [
    "YcrdtError", "Engine", "Doc", "Batch", "MergeStats", "apply_update", "apply_updates",
    "encode_state_as_update", "encode_state_vector", "merge_updates", "diff_update", "diff_updates", "default_engine", "library_path",
]

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

YCRDT_OK = 0
ERRORS = {
    -1: "DECODE",
    -2: "PENDING",
    -3: "UNSUPPORTED",
    -4: "CAPACITY",
    -5: "DEVICE",
    -6: "ARG",
}


class YcrdtError(Exception):
    def __init__(self, code, message):
        super().__init__(message)
        self.code = code
        self.kind = ERRORS.get(code, "UNKNOWN")


class _Buf(ctypes.Structure):
    _fields_ = [("ptr", ctypes.c_void_p), ("len", ctypes.c_size_t)]


class _Out(ctypes.Structure):
    _fields_ = [("ptr", ctypes.c_void_p), ("len", ctypes.c_size_t)]


class MergeStats(ctypes.Structure):
    _fields_ = [
        ("in_bytes", ctypes.c_uint64),
        ("items", ctypes.c_uint64),
        ("structs", ctypes.c_uint64),
        ("units", ctypes.c_uint64),
        ("segments", ctypes.c_uint64),
        ("out_structs", ctypes.c_uint64),
        ("out_bytes", ctypes.c_uint64),
        ("clients", ctypes.c_uint64),
        ("device_ms", ctypes.c_double),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


def library_path():
    # YCRDT_LIB: another build of the library (A/B experiments); the in-tree one by default
    return os.environ.get("YCRDT_LIB") or os.path.join(_HERE, "libycrdt.so")


EXPORTS = (
    "ycrdt_engine_create", "ycrdt_engine_destroy", "ycrdt_engine_set_profiling", "ycrdt_engine_phase_times",
    "ycrdt_engine_device_bytes", "ycrdt_engine_trim",
    "ycrdt_doc_create", "ycrdt_doc_destroy", "ycrdt_apply_update", "ycrdt_apply_updates",
    "ycrdt_encode_state_as_update", "ycrdt_encode_state_vector", "ycrdt_doc_last_stats",
    "ycrdt_batch_stage", "ycrdt_batch_merge", "ycrdt_batch_result", "ycrdt_batch_destroy",
    "ycrdt_merge_updates", "ycrdt_diff_update", "ycrdt_diff_updates", "ycrdt_free", "ycrdt_last_error", "ycrdt_version",
    "ycrdt_doc_json", "ycrdt_type_json", "ycrdt_map_entries", "ycrdt_map_set", "ycrdt_map_set_type", "ycrdt_map_delete", "ycrdt_array_insert",
    "ycrdt_array_delete", "ycrdt_doc_client_id", "ycrdt_map_type_at", "ycrdt_doc_take_local_update",
    "ycrdt_doc_flush", "ycrdt_doc_pending", "ycrdt_doc_track_local", "ycrdt_validate_update", "ycrdt_debug_replay",
    "ycrdt_batch_stage_docs", "ycrdt_batch_result_docs", "ycrdt_batch_result_docs_packed", "ycrdt_merge_docs",
    "ycrdt_map_get", "ycrdt_map_size", "ycrdt_array_length", "ycrdt_array_get", "ycrdt_apply_updates_multi",
    "ycrdt_comm_unique_id", "ycrdt_comm_create", "ycrdt_comm_destroy", "ycrdt_batch_merge_sharded",
    "ycrdt_comm_sv_allreduce_max", "ycrdt_comm_ds_allgather", "ycrdt_comm_create_exchange", "ycrdt_route",
    "ycrdt_comm_fleet_sv_allreduce_max", "ycrdt_docs_states_packed", "ycrdt_comm_allgather", "ycrdt_device_count",
)

MERGE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p)
ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32), ctypes.c_size_t, ctypes.c_int)
ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint8), ctypes.c_size_t,
                                ctypes.POINTER(ctypes.c_uint8))


class _Exchange(ctypes.Structure):
    _fields_ = [("ctx", ctypes.c_void_p), ("allreduce_u32", ALLREDUCE_FN), ("allgather", ALLGATHER_FN)]


def lib():
    """Loads libycrdt.so (built in-tree by __graft_entry__.build()); fails loudly if absent."""
    global _LIB
    if _LIB is not None:
        return _LIB
    path = library_path()
    if not os.path.exists(path):
        raise RuntimeError(f"{path} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
    L = ctypes.CDLL(path)
    vp, sz, u32, i32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_int
    P = ctypes.POINTER
    L.ycrdt_engine_create.argtypes = [i32, i32, P(vp)]
    L.ycrdt_engine_destroy.argtypes = [vp]
    L.ycrdt_engine_set_profiling.argtypes = [vp, i32]
    L.ycrdt_engine_phase_times.argtypes = [vp, P(ctypes.c_char_p), P(ctypes.c_double), i32]
    L.ycrdt_engine_device_bytes.argtypes = [vp, P(ctypes.c_uint64)]
    L.ycrdt_engine_trim.argtypes = [vp]
    L.ycrdt_doc_create.argtypes = [vp, u32, P(vp)]
    L.ycrdt_doc_destroy.argtypes = [vp]
    L.ycrdt_apply_update.argtypes = [vp, _Buf]
    L.ycrdt_apply_updates.argtypes = [vp, P(_Buf), sz]
    L.ycrdt_encode_state_as_update.argtypes = [vp, _Buf, P(_Out)]
    L.ycrdt_encode_state_vector.argtypes = [vp, P(_Out)]
    L.ycrdt_doc_last_stats.argtypes = [vp, P(MergeStats)]
    L.ycrdt_batch_stage.argtypes = [vp, P(_Buf), sz, P(vp)]
    L.ycrdt_batch_merge.argtypes = [vp, P(MergeStats)]
    L.ycrdt_batch_result.argtypes = [vp, P(_Out), P(_Out)]
    L.ycrdt_batch_destroy.argtypes = [vp]
    L.ycrdt_merge_updates.argtypes = [vp, P(_Buf), sz, P(_Out)]
    L.ycrdt_diff_update.argtypes = [vp, _Buf, _Buf, P(_Out)]
    L.ycrdt_diff_updates.argtypes = [vp, P(_Buf), P(_Buf), sz, P(_Out)]
    L.ycrdt_doc_take_local_update.argtypes = [vp, P(_Out)]
    L.ycrdt_doc_flush.argtypes = [vp]
    L.ycrdt_doc_pending.argtypes = [vp, P(i32), P(i32)]
    L.ycrdt_doc_track_local.argtypes = [vp, i32]
    L.ycrdt_validate_update.argtypes = [_Buf, P(i32)]
    L.ycrdt_batch_stage_docs.argtypes = [vp, P(_Buf), P(u32), sz, u32, P(vp)]
    L.ycrdt_batch_result_docs.argtypes = [vp, P(_Out), P(_Out)]
    L.ycrdt_batch_result_docs_packed.argtypes = [vp, vp, ctypes.c_uint64, P(ctypes.c_uint64), P(ctypes.c_uint64)]
    L.ycrdt_merge_docs.argtypes = [vp, P(_Buf), P(u32), sz, u32, P(_Out), P(_Out)]
    L.ycrdt_debug_replay.argtypes = [P(_Buf), sz, MERGE_FN, vp, P(_Out), P(_Out), P(_Out)]
    L.ycrdt_free.argtypes = [P(_Out)]
    cs = ctypes.c_char_p
    L.ycrdt_doc_json.argtypes = [vp, cs, i32, P(_Out)]
    L.ycrdt_type_json.argtypes = [vp, cs, cs, i32, P(_Out)]
    L.ycrdt_map_entries.argtypes = [vp, cs, cs, P(_Out)]
    L.ycrdt_map_type_at.argtypes = [vp, cs, cs, P(i32)]
    L.ycrdt_map_set.argtypes = [vp, cs, cs, cs, ctypes.c_char_p, sz]
    L.ycrdt_map_set_type.argtypes = [vp, cs, cs, cs, u32]
    L.ycrdt_map_delete.argtypes = [vp, cs, cs, cs]
    L.ycrdt_array_insert.argtypes = [vp, cs, cs, u32, ctypes.c_char_p, sz, u32]
    L.ycrdt_array_delete.argtypes = [vp, cs, cs, u32, u32]
    L.ycrdt_doc_client_id.argtypes = [vp, P(u32)]
    L.ycrdt_map_get.argtypes = [vp, cs, cs, cs, P(i32), P(_Out)]
    L.ycrdt_apply_updates_multi.argtypes = [vp, P(vp), P(_Buf), sz]
    L.ycrdt_comm_unique_id.argtypes = [ctypes.c_char_p]
    L.ycrdt_comm_create.argtypes = [vp, i32, i32, ctypes.c_char_p, P(vp)]
    L.ycrdt_comm_destroy.argtypes = [vp]
    L.ycrdt_batch_merge_sharded.argtypes = [vp, vp, u32, P(MergeStats)]
    L.ycrdt_comm_sv_allreduce_max.argtypes = [vp, vp, _Buf, P(_Out)]
    L.ycrdt_comm_ds_allgather.argtypes = [vp, vp, _Buf, P(_Out)]
    L.ycrdt_comm_allgather.argtypes = [vp, vp, _Buf, P(_Out), P(_Out)]
    L.ycrdt_device_count.argtypes = [P(i32)]
    L.ycrdt_comm_create_exchange.argtypes = [vp, i32, i32, P(_Exchange), P(vp)]
    L.ycrdt_docs_states_packed.argtypes = [vp, P(vp), sz, vp, ctypes.c_uint64, P(ctypes.c_uint64), P(ctypes.c_uint64)]
    L.ycrdt_route.argtypes = [ctypes.c_char_p, sz, u32]
    L.ycrdt_route.restype = u32
    L.ycrdt_comm_fleet_sv_allreduce_max.argtypes = [vp, vp, P(u32), P(_Buf), sz, P(_Out), P(_Out), P(_Out)]
    L.ycrdt_map_size.argtypes = [vp, cs, cs, P(u32)]
    L.ycrdt_array_length.argtypes = [vp, cs, cs, P(ctypes.c_uint64)]
    L.ycrdt_array_get.argtypes = [vp, cs, cs, ctypes.c_uint64, P(i32), P(_Out)]
    L.ycrdt_last_error.restype = ctypes.c_char_p
    L.ycrdt_version.restype = ctypes.c_char_p
    _LIB = L
    return L


def _check(rc):
    if rc != YCRDT_OK:
        raise YcrdtError(rc, lib().ycrdt_last_error().decode(errors="replace"))


def _pack():
    """The in-tree host-glue extension (crdt_amd/_ycpack.c, built with libycrdt.so)."""
    try:
        from . import _ycpack
    except ImportError as e:
        raise RuntimeError("crdt_amd/_ycpack not built: run `python -c 'import __graft_entry__ as g; g.build()'`") from e
    return _ycpack


def _bufs(updates):
    """ycrdt_buf[] over the updates, pointing into the bytes objects themselves (no join / copy;
    _ycpack.c). The array keeps the objects it points into alive."""
    keep = updates if isinstance(updates, (list, tuple)) else list(updates)
    raw, conv = _pack().bufs(keep)
    n = len(keep)
    arr = (_Buf * max(1, n)).from_buffer_copy(raw)
    arr._keep = (keep, conv)
    return arr, keep


def _opt(s):
    return None if s is None else s.encode()


def _take(out):
    try:
        return ctypes.string_at(out.ptr, out.len) if out.len else b""
    finally:
        lib().ycrdt_free(ctypes.byref(out))


class Engine:
    """One HIP device + stream + HBM workspace (compat 136 = Yjs 13.6 canonical client order)."""

    def __init__(self, device=0, compat=136):
        h = ctypes.c_void_p()
        _check(lib().ycrdt_engine_create(device, compat, ctypes.byref(h)))
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().ycrdt_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_profiling(self, on=True):
        _check(lib().ycrdt_engine_set_profiling(self._h, 1 if on else 0))

    def device_bytes(self) -> int:
        """HBM held by the engine (merge workspace + doc-state arena + staging batch)."""
        v = ctypes.c_uint64()
        _check(lib().ycrdt_engine_device_bytes(self._h, ctypes.byref(v)))
        return v.value

    def trim(self):
        """Releases the merge workspace (ycrdt_engine_trim): HBM back after a giant merge."""
        _check(lib().ycrdt_engine_trim(self._h))

    def phase_times(self):
        names = (ctypes.c_char_p * 64)()
        ms = (ctypes.c_double * 64)()
        n = lib().ycrdt_engine_phase_times(self._h, names, ms, 64)
        return [(names[i].decode(), ms[i]) for i in range(n)]


_DEFAULT = None


def default_engine():
    global _DEFAULT
    if _DEFAULT is None:
        _DEFAULT = Engine(int(os.environ.get("YCRDT_DEVICE", "0")))
    return _DEFAULT


class Doc:
    """Y.Doc backed by the GPU engine. The canonical encoded state lives in HBM."""

    def __init__(self, client_id=None, engine=None):
        self.engine = engine or default_engine()
        h = ctypes.c_void_p()
        cid = client_id if client_id is not None else int.from_bytes(os.urandom(4), "little")
        _check(lib().ycrdt_doc_create(self.engine._h, cid, ctypes.byref(h)))
        self._h = h
        self.client_id = cid

    def __del__(self):
        if getattr(self, "_h", None):
            try:
                lib().ycrdt_doc_destroy(self._h)
            except Exception:  # interpreter teardown: module globals already cleared
                pass
            self._h = None

    def apply_update(self, update: bytes):
        u = bytes(update)
        b = _Buf(ctypes.cast(ctypes.c_char_p(u), ctypes.c_void_p), len(u))
        _check(lib().ycrdt_apply_update(self._h, b))

    def apply_updates(self, updates):
        arr, keep = _bufs(updates)
        _check(lib().ycrdt_apply_updates(self._h, arr, len(keep)))

    def encode_state_as_update(self, sv: bytes = b"") -> bytes:
        s = bytes(sv or b"")
        b = _Buf(ctypes.cast(ctypes.c_char_p(s), ctypes.c_void_p), len(s))
        out = _Out()
        _check(lib().ycrdt_encode_state_as_update(self._h, b, ctypes.byref(out)))
        return _take(out)

    def encode_state_vector(self) -> bytes:
        out = _Out()
        _check(lib().ycrdt_encode_state_vector(self._h, ctypes.byref(out)))
        return _take(out)

    def flush(self):
        """Runs the deferred Y.applyUpdate calls now (every read does this implicitly)."""
        _check(lib().ycrdt_doc_flush(self._h))

    def pending(self):
        """(structs, delete_set): whether Yjs would hold store.pendingStructs / store.pendingDs."""
        a, b = ctypes.c_int(), ctypes.c_int()
        _check(lib().ycrdt_doc_pending(self._h, ctypes.byref(a), ctypes.byref(b)))
        return bool(a.value), bool(b.value)

    def track_local(self, on=True):
        """Record local-op updates for take_local_update (off until this or the first take)."""
        _check(lib().ycrdt_doc_track_local(self._h, 1 if on else 0))

    def last_stats(self) -> MergeStats:
        st = MergeStats()
        _check(lib().ycrdt_doc_last_stats(self._h, ctypes.byref(st)))
        return st

    # ---- crdt.c materialisation + local ops (same signatures as oracle/yref.py's Doc) ----------
    # `parent_key` addresses the shared type stored in root map `root` under that key.
    def root_json(self, name: str, kind: str) -> str:
        """YMap.toJSON / YArray.toJSON of root `name` (kind "map" | "array") as JSON text."""
        out = _Out()
        _check(lib().ycrdt_doc_json(self._h, name.encode(), 0 if kind == "map" else 1, ctypes.byref(out)))
        return _take(out).decode()

    def type_json(self, root: str, kind: str, parent_key: str = None) -> str:
        """toJSON of the root type, or of the YMap / YArray stored in root map `root`[parent_key]
        (only that type's own list is read)."""
        out = _Out()
        _check(lib().ycrdt_type_json(self._h, root.encode(), _opt(parent_key), 0 if kind == "map" else 1, ctypes.byref(out)))
        return _take(out).decode()

    def map_type_at(self, root: str, key: str) -> int:
        """type ref of the shared type under root map `root`[key] (0 YArray, 1 YMap), -1 if none."""
        t = ctypes.c_int32()
        _check(lib().ycrdt_map_type_at(self._h, root.encode(), key.encode(), ctypes.byref(t)))
        return t.value

    def map_get(self, root: str, key: str, parent_key: str = None):
        """YMap.get without a toJSON of the map: (state, json) — state 0 absent, 1 value, 2 undefined."""
        st, out = ctypes.c_int32(), _Out()
        _check(lib().ycrdt_map_get(self._h, root.encode(), _opt(parent_key), key.encode(), ctypes.byref(st), ctypes.byref(out)))
        return st.value, _take(out).decode()

    def map_size(self, root: str, parent_key: str = None) -> int:
        n = ctypes.c_uint32()
        _check(lib().ycrdt_map_size(self._h, root.encode(), _opt(parent_key), ctypes.byref(n)))
        return n.value

    def array_length(self, root: str, parent_key: str = None) -> int:
        n = ctypes.c_uint64()
        _check(lib().ycrdt_array_length(self._h, root.encode(), _opt(parent_key), ctypes.byref(n)))
        return n.value

    def array_get(self, root: str, index: int, parent_key: str = None):
        st, out = ctypes.c_int32(), _Out()
        _check(lib().ycrdt_array_get(self._h, root.encode(), _opt(parent_key), index, ctypes.byref(st), ctypes.byref(out)))
        return st.value, _take(out).decode()

    def map_set(self, root: str, key: str, any_bytes: bytes, parent_key: str = None):
        a = bytes(any_bytes)
        _check(lib().ycrdt_map_set(self._h, root.encode(), _opt(parent_key), key.encode(), a, len(a)))

    def map_set_type(self, root: str, key: str, type_ref: int = 0, parent_key: str = None):
        """YMap.set(key, new Y.Array()) (type_ref 0) / new Y.Map() (1)."""
        _check(lib().ycrdt_map_set_type(self._h, root.encode(), _opt(parent_key), key.encode(), type_ref))

    def map_delete(self, root: str, key: str, parent_key: str = None):
        _check(lib().ycrdt_map_delete(self._h, root.encode(), _opt(parent_key), key.encode()))

    def array_insert(self, root: str, index: int, anys: list, parent_key: str = None):
        a = b"".join(bytes(x) for x in anys)
        _check(lib().ycrdt_array_insert(self._h, root.encode(), _opt(parent_key), index, a, len(a), len(anys)))

    def take_local_update(self) -> bytes:
        """The local ops since the previous call as one update (incremental wire delta)."""
        out = _Out()
        _check(lib().ycrdt_doc_take_local_update(self._h, ctypes.byref(out)))
        return _take(out)

    def array_delete(self, root: str, index: int, length: int, parent_key: str = None):
        _check(lib().ycrdt_array_delete(self._h, root.encode(), _opt(parent_key), index, length))


def _docs_arrays(docs):
    docs = docs if isinstance(docs, (list, tuple)) else list(docs)
    raw, dof, conv = _pack().docs(docs)
    n = len(raw) // ctypes.sizeof(_Buf) if any(len(d) for d in docs) else 0
    arr = (_Buf * max(1, n)).from_buffer_copy(raw)
    do = (ctypes.c_uint32 * max(1, n)).from_buffer_copy(dof)
    arr._keep = (docs, conv)
    return arr, range(n), do


class Batch:
    """A set of updates staged in HBM; merge() runs the whole merge on the device. With
    `docs=[[u8, ...], ...]` instead of `updates` the batch holds many independent documents
    (ycrdt_batch_stage_docs) merged in the same device pass; result_docs() splits them."""

    def __init__(self, updates=None, engine=None, docs=None):
        self.engine = engine or default_engine()
        h = ctypes.c_void_p()
        self.ndocs = 1
        if docs is not None:
            arr, keep, do = _docs_arrays(docs)
            self.ndocs = max(1, len(docs))
            _check(lib().ycrdt_batch_stage_docs(self.engine._h, arr, do, len(keep), self.ndocs, ctypes.byref(h)))
        else:
            arr, keep = _bufs(updates)
            _check(lib().ycrdt_batch_stage(self.engine._h, arr, len(keep), ctypes.byref(h)))
        self._h = h

    def __del__(self):
        if getattr(self, "_h", None):
            try:
                lib().ycrdt_batch_destroy(self._h)
            except Exception:  # interpreter teardown: module globals already cleared
                pass
            self._h = None

    def merge(self) -> MergeStats:
        st = MergeStats()
        _check(lib().ycrdt_batch_merge(self._h, ctypes.byref(st)))
        return st

    def merge_sharded(self, nshards: int, comm: "Comm" = None) -> MergeStats:
        """Key-hash sharded merge (C4): every logical shard on this GPU (comm None) or this rank's
        shard with the flag words summed over RCCL. Same bytes as merge()."""
        st = MergeStats()
        _check(lib().ycrdt_batch_merge_sharded(self._h, comm._h if comm else None, nshards, ctypes.byref(st)))
        return st

    def result(self):
        u, s = _Out(), _Out()
        _check(lib().ycrdt_batch_result(self._h, ctypes.byref(u), ctypes.byref(s)))
        return _take(u), _take(s)

    def result_docs(self):
        """[(encoded update, state vector)] per document of a multi-document batch."""
        us, ss = (_Out * self.ndocs)(), (_Out * self.ndocs)()
        _check(lib().ycrdt_batch_result_docs(self._h, us, ss))
        return [(_take(us[i]), _take(ss[i])) for i in range(self.ndocs)]

    def result_docs_packed(self, out=None):
        """(blob, offs): every document's update and state vector back to back in one numpy uint8
        array, split on the device — document d's update is blob[offs[2d]:offs[2d+1]], its state
        vector blob[offs[2d+1]:offs[2d+2]] (ycrdt_batch_result_docs_packed). `out`: a uint8 array to
        write into when it is large enough (a serving loop reuses one: no page faults of a fresh
        gigabyte per batch); blob is then a view of it."""
        import numpy as np

        offs = np.zeros(2 * self.ndocs + 1, dtype=np.uint64)
        total = ctypes.c_uint64()
        op = offs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))
        _check(lib().ycrdt_batch_result_docs_packed(self._h, None, 0, op, ctypes.byref(total)))
        if out is not None and out.dtype == np.uint8 and out.flags.c_contiguous and out.size >= max(1, total.value):
            blob = out
        else:
            blob = np.empty(max(1, total.value), dtype=np.uint8)
        _check(lib().ycrdt_batch_result_docs_packed(self._h, blob.ctypes.data, total.value, op, ctypes.byref(total)))
        return blob[: total.value], offs


def merge_docs(docs, engine=None):
    """Many independent documents' update lists merged in ONE device pass (ycrdt_merge_docs):
    [(encodeStateAsUpdate, encodeStateVector)] of a fresh doc per list."""
    eng = engine or default_engine()
    arr, keep, do = _docs_arrays(docs)
    n = max(1, len(docs))
    us, ss = (_Out * n)(), (_Out * n)()
    _check(lib().ycrdt_merge_docs(eng._h, arr, do, len(keep), n, us, ss))
    return [(_take(us[i]), _take(ss[i])) for i in range(len(docs))]


# ---- the `Y` functions the reference calls ---------------------------------------------------
def apply_update(doc: Doc, update: bytes):
    doc.apply_update(update)


def apply_updates(doc: Doc, updates):
    doc.apply_updates(updates)


def encode_state_as_update(doc: Doc, sv: bytes = b"") -> bytes:
    return doc.encode_state_as_update(sv)


def encode_state_vector(doc: Doc) -> bytes:
    return doc.encode_state_vector()


class Comm:
    """Communicator inside libycrdt (one rank per GPU). RCCL: Comm.unique_id() on rank 0, the bytes
    handed to every rank by any channel, then Comm(engine, nranks, rank, uid) on each. Or
    Comm.over(engine, nranks, rank, allreduce, allgather): the library's collectives over host
    callbacks (ycrdt_exchange) — e.g. the package's TCP hub, Comm.over_hub (crdt_amd/hosthub.py)."""

    @staticmethod
    def unique_id() -> bytes:
        buf = ctypes.create_string_buffer(128)
        _check(lib().ycrdt_comm_unique_id(buf))
        return buf.raw

    ID_BYTES = 128  # YCRDT_COMM_ID_BYTES: ycrdt_comm_create copies exactly this many bytes

    def __init__(self, engine, nranks: int, rank: int, uid: bytes):
        uid = bytes(uid)
        if len(uid) != Comm.ID_BYTES:
            raise ValueError(f"communicator id must be {Comm.ID_BYTES} bytes (got {len(uid)})")
        h = ctypes.c_void_p()
        _check(lib().ycrdt_comm_create(engine._h, nranks, rank, uid, ctypes.byref(h)))
        self._h, self.engine, self.nranks, self.rank = h, engine, nranks, rank

    @classmethod
    def over(cls, engine, nranks: int, rank: int, allreduce, allgather):
        """allreduce(numpy u32 array, op) -> None, in place, op 0 = sum / 1 = max, over every rank;
        allgather(bytes) -> bytes, the ranks' equal-length payloads concatenated in rank order."""
        import numpy as np

        self = cls.__new__(cls)

        def ar(_ctx, words, n, op):
            try:
                a = np.ctypeslib.as_array(words, shape=(n,)) if n else np.zeros(0, np.uint32)
                allreduce(a, op)
                return 0
            except Exception:  # noqa: BLE001 — surfaces as YCRDT_E_DEVICE in the library call
                return -1

        def ag(_ctx, send, nbytes, recv):
            try:
                got = allgather(ctypes.string_at(send, nbytes) if nbytes else b"")
                if len(got) != nbytes * nranks:
                    return -1
                if got:
                    ctypes.memmove(recv, got, len(got))
                return 0
            except Exception:  # noqa: BLE001
                return -1

        self._cbs = (ALLREDUCE_FN(ar), ALLGATHER_FN(ag))
        self._x = _Exchange(None, self._cbs[0], self._cbs[1])
        h = ctypes.c_void_p()
        _check(lib().ycrdt_comm_create_exchange(engine._h, nranks, rank, ctypes.byref(self._x), ctypes.byref(h)))
        self._h, self.engine, self.nranks, self.rank = h, engine, nranks, rank
        return self

    @classmethod
    def over_hub(cls, engine, hub):
        """The host exchange over a crdt_amd.hosthub.HostHub (TCP through rank 0, no torch)."""
        return cls.over(engine, hub.world, hub.rank, hub.allreduce_u32, lambda b: b"".join(hub.allgather(b)))

    def close(self):
        if getattr(self, "_h", None):
            lib().ycrdt_comm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def fleet_sv_allreduce_max(self, svs: dict) -> dict:
        """{doc id (u32): state vector bytes} held by this rank -> {doc id: state vector of the union
        over the ranks} for every document any rank holds (ycrdt_comm_fleet_sv_allreduce_max)."""
        import numpy as np

        ids = list(svs)
        arr, keep = _bufs([svs[i] for i in ids])
        docs = (ctypes.c_uint32 * max(1, len(ids)))(*ids)
        d, o, b = _Out(), _Out(), _Out()
        _check(lib().ycrdt_comm_fleet_sv_allreduce_max(self._h, self.engine._h, docs, arr, len(ids),
                                                        ctypes.byref(d), ctypes.byref(o), ctypes.byref(b)))
        dd = np.frombuffer(_take(d), dtype=np.uint32)
        oo = np.frombuffer(_take(o), dtype=np.uint64)
        blob = _take(b)
        return {int(dd[j]): blob[int(oo[j]):int(oo[j + 1])] for j in range(len(dd))}

    def sv_allreduce_max(self, sv: bytes) -> bytes:
        out = _Out()
        b = bytes(sv)
        _check(lib().ycrdt_comm_sv_allreduce_max(self._h, self.engine._h, _Buf(ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p), len(b)), ctypes.byref(out)))
        return _take(out)

    def allgather(self, payload: bytes) -> list:
        """Every rank's bytes, in rank order (ycrdt_comm_allgather, the library's own transport)."""
        import numpy as np

        b, o = _Out(), _Out()
        p = bytes(payload)
        _check(lib().ycrdt_comm_allgather(self._h, self.engine._h, _Buf(ctypes.cast(ctypes.c_char_p(p), ctypes.c_void_p), len(p)),
                                          ctypes.byref(b), ctypes.byref(o)))
        blob = _take(b)
        offs = np.frombuffer(_take(o), dtype=np.uint64)
        return [blob[int(offs[r]):int(offs[r + 1])] for r in range(len(offs) - 1)]

    def barrier(self):
        self.allgather(b"")

    def ds_allgather(self, update: bytes) -> bytes:
        out = _Out()
        b = bytes(update)
        _check(lib().ycrdt_comm_ds_allgather(self._h, self.engine._h, _Buf(ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p), len(b)), ctypes.byref(out)))
        return _take(out)


def device_count() -> int:
    """HIP devices visible to this process (ycrdt_device_count); 0 without a GPU."""
    n = ctypes.c_int32()
    rc = lib().ycrdt_device_count(ctypes.byref(n))
    return n.value if rc == 0 else 0


def route(doc_id, world: int) -> int:
    """Owner rank of a document / topic id (ycrdt_route): stable across ranks, processes and runs."""
    b = doc_id.encode() if isinstance(doc_id, str) else bytes(doc_id)
    return int(lib().ycrdt_route(b, len(b), world))


def apply_updates_multi(docs, updates, engine=None, doc_index=None):
    """Y.applyUpdate(docs[i], updates[i]) for every i — a fleet ingest batch — merged in one device
    pass for every document with nothing pending (ycrdt_apply_updates_multi). With doc_index
    (integer array, one per update) `docs` lists the documents once and update i goes to
    docs[doc_index[i]]."""
    import numpy as np

    hv = np.fromiter((d._h.value for d in docs), dtype=np.uint64, count=len(docs)) if docs else np.zeros(1, np.uint64)
    if doc_index is not None:
        hv = hv[np.asarray(doc_index, dtype=np.int64)] if len(updates) else np.zeros(1, np.uint64)
    if (len(hv) if len(updates) else 0) != len(updates):
        raise ValueError("one document per update")
    eng = engine or (docs[0].engine if docs else default_engine())
    arr, keep = _bufs(updates)
    hs = hv.ctypes.data_as(ctypes.POINTER(ctypes.c_void_p))
    _check(lib().ycrdt_apply_updates_multi(eng._h, hs, arr, len(keep)))


def states_packed(docs, engine=None):
    """(blob, offs): every document's encodeStateAsUpdate and encodeStateVector back to back in one
    numpy uint8 array (ycrdt_docs_states_packed) — doc i's update blob[offs[2i]:offs[2i+1]], its
    state vector blob[offs[2i+1]:offs[2i+2]]."""
    import numpy as np

    eng = engine or (docs[0].engine if docs else default_engine())
    hv = np.fromiter((d._h.value for d in docs), dtype=np.uint64, count=len(docs)) if docs else np.zeros(1, np.uint64)
    hs = hv.ctypes.data_as(ctypes.POINTER(ctypes.c_void_p))
    offs = np.zeros(2 * len(docs) + 1, dtype=np.uint64)
    op = offs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))
    total = ctypes.c_uint64()
    _check(lib().ycrdt_docs_states_packed(eng._h, hs, len(docs), None, 0, op, ctypes.byref(total)))
    blob = np.empty(max(1, total.value), dtype=np.uint8)
    _check(lib().ycrdt_docs_states_packed(eng._h, hs, len(docs), blob.ctypes.data, total.value, op, ctypes.byref(total)))
    return blob[: total.value], offs


def merge_updates(updates, engine=None) -> bytes:
    """Y.mergeUpdates(updates) on the GPU (lazy k-way struct merge + delete-set union)."""
    eng = engine or default_engine()
    arr, keep = _bufs(updates)
    out = _Out()
    _check(lib().ycrdt_merge_updates(eng._h, arr, len(keep), ctypes.byref(out)))
    return _take(out)


def diff_update(update: bytes, sv: bytes, engine=None) -> bytes:
    """Y.diffUpdate(update, sv) on the GPU."""
    eng = engine or default_engine()
    u, v = bytes(update), bytes(sv)
    bu = _Buf(ctypes.cast(ctypes.c_char_p(u), ctypes.c_void_p), len(u))
    bv = _Buf(ctypes.cast(ctypes.c_char_p(v), ctypes.c_void_p), len(v))
    out = _Out()
    _check(lib().ycrdt_diff_update(eng._h, bu, bv, ctypes.byref(out)))
    return _take(out)


def validate_update(update: bytes):
    """Host-side validation of one update (no GPU): (ok, structs_ok)."""
    u = bytes(update)
    b = _Buf(ctypes.cast(ctypes.c_char_p(u), ctypes.c_void_p), len(u))
    so = ctypes.c_int()
    rc = lib().ycrdt_validate_update(b, ctypes.byref(so))
    return rc == YCRDT_OK, bool(so.value)


def debug_replay(updates, merge):
    """Test hook (no GPU): replays Y.applyUpdate x n on struct headers with `merge(list[bytes]) ->
    bytes` as Y.mergeUpdates; returns (state vector ascending, pending update, pending delete set)."""
    keep = []

    def cb(_ctx, ups, n, out):
        try:
            arr = ctypes.cast(ups, ctypes.POINTER(_Buf))
            ins = [ctypes.string_at(arr[i].ptr, arr[i].len) if arr[i].len else b"" for i in range(n)]
            res = bytes(merge(ins))
            buf = ctypes.create_string_buffer(res, max(1, len(res)))
            keep.append(buf)
            o = ctypes.cast(out, ctypes.POINTER(_Out))
            o[0].ptr = ctypes.cast(buf, ctypes.c_void_p)
            o[0].len = len(res)
            return 0
        except Exception:  # noqa: BLE001 — surfaces as an error code in the replay
            return -6

    fn = MERGE_FN(cb)
    arr, kept = _bufs(updates)
    sv, p, pd = _Out(), _Out(), _Out()
    _check(lib().ycrdt_debug_replay(arr, len(kept), fn, None, ctypes.byref(sv), ctypes.byref(p), ctypes.byref(pd)))
    return _take(sv), _take(p), _take(pd)


def diff_updates(updates, svs, engine=None) -> list:
    """[Y.diffUpdate(u, sv) for u, sv in zip(updates, svs)] in one batched GPU pass (the sync
    responder of crdt.js:286-291 batched across peers / topics)."""
    eng = engine or default_engine()
    if len(updates) != len(svs):
        raise ValueError("diff_updates: one state vector per update")
    ua, ukeep = _bufs(updates)
    va, vkeep = _bufs(svs)
    outs = (_Out * max(len(ukeep), 1))()
    _check(lib().ycrdt_diff_updates(eng._h, ua, va, len(ukeep), outs))
    return [_take(outs[i]) for i in range(len(ukeep))]
