"""ctypes binding of oracle/libyref.so — the CPU restatement of Yjs 13.5.16.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg. The product path (crdt_amd) never imports this module.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "libyref.so")
        if not os.path.exists(path):
            raise RuntimeError("oracle/libyref.so not built (run `make -C oracle`)")
        L = ctypes.CDLL(path)
        vp, u8p, sz = ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t
        outp, outl = ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t)
        L.yo_doc_new.restype = vp
        L.yo_doc_new.argtypes = [ctypes.c_uint32, ctypes.c_int]
        L.yo_doc_free.argtypes = [vp]
        L.yo_apply_update.argtypes = [vp, u8p, sz]
        L.yo_encode_state_as_update.argtypes = [vp, u8p, sz, outp, outl]
        L.yo_encode_state_vector.argtypes = [vp, outp, outl]
        L.yo_root_json.argtypes = [vp, ctypes.c_char_p, ctypes.c_int, outp, outl]
        L.yo_map_set.argtypes = [vp, ctypes.c_char_p, ctypes.c_char_p, u8p, sz]
        L.yo_map_delete.argtypes = [vp, ctypes.c_char_p, ctypes.c_char_p]
        L.yo_array_insert.argtypes = [vp, ctypes.c_char_p, ctypes.c_uint32, u8p, sz, ctypes.c_uint32]
        L.yo_array_delete.argtypes = [vp, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32]
        L.yo_client_id.restype = ctypes.c_uint32
        L.yo_client_id.argtypes = [vp]
        L.yo_free.argtypes = [vp]
        L.yo_last_error.restype = ctypes.c_char_p
        _LIB = L
    return _LIB


class OracleError(Exception):
    def __init__(self, code, msg):
        super().__init__(f"oracle error {code}: {msg}")
        self.code = code


def _take(p, n):
    try:
        return ctypes.string_at(p.value, n.value) if n.value else b""
    finally:
        lib().yo_free(p)


class Doc:
    """One Y.Doc replica restated in C. compat=136 → DS/SV client order sorted desc (Yjs 13.6);
    compat=135 → store insertion order (Yjs 13.5.16)."""

    def __init__(self, client_id=0x7FFFFFF0, compat=136):
        self._d = lib().yo_doc_new(client_id, compat)

    def __del__(self):
        if getattr(self, "_d", None):
            lib().yo_doc_free(self._d)
            self._d = None

    def _chk(self, rc):
        if rc != 0:
            raise OracleError(rc, lib().yo_last_error().decode(errors="replace"))

    def apply_update(self, u: bytes):
        self._chk(lib().yo_apply_update(self._d, bytes(u), len(u)))

    def encode_state_as_update(self, sv: bytes = b"") -> bytes:
        p, n = ctypes.c_void_p(), ctypes.c_size_t()
        self._chk(lib().yo_encode_state_as_update(self._d, bytes(sv), len(sv), ctypes.byref(p), ctypes.byref(n)))
        return _take(p, n)

    def encode_state_vector(self) -> bytes:
        p, n = ctypes.c_void_p(), ctypes.c_size_t()
        self._chk(lib().yo_encode_state_vector(self._d, ctypes.byref(p), ctypes.byref(n)))
        return _take(p, n)

    def root_json(self, name: str, kind: str) -> str:
        p, n = ctypes.c_void_p(), ctypes.c_size_t()
        self._chk(lib().yo_root_json(self._d, name.encode(), 0 if kind == "map" else 1, ctypes.byref(p), ctypes.byref(n)))
        return _take(p, n).decode()

    def map_set(self, root: str, key: str, any_bytes: bytes):
        self._chk(lib().yo_map_set(self._d, root.encode(), key.encode(), any_bytes, len(any_bytes)))

    def map_delete(self, root: str, key: str):
        self._chk(lib().yo_map_delete(self._d, root.encode(), key.encode()))

    def array_insert(self, root: str, index: int, anys: list):
        b = b"".join(anys)
        self._chk(lib().yo_array_insert(self._d, root.encode(), index, b, len(b), len(anys)))

    def array_delete(self, root: str, index: int, length: int):
        self._chk(lib().yo_array_delete(self._d, root.encode(), index, length))

    @property
    def client_id(self):
        return lib().yo_client_id(self._d)
