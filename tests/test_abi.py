"""CPU-side checks of the C ABI boundary: the library loads and exports every declared symbol."""
import os
import re

import crdt_amd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_header_symbols_exported():
    hdr = open(os.path.join(ROOT, "include", "ycrdt.h")).read()
    declared = set(re.findall(r"\b(ycrdt_[a-z_]+)\s*\(", hdr))
    assert declared == set(crdt_amd.EXPORTS), declared ^ set(crdt_amd.EXPORTS)
    L = crdt_amd.lib()
    for sym in declared:
        assert hasattr(L, sym), sym


def test_version_string():
    assert b"gfx950" in crdt_amd.lib().ycrdt_version()


def test_library_is_fresh():
    """libycrdt.so must be rebuilt after every source edit (the GPU box runs the in-tree build)."""
    so = os.path.getmtime(os.path.join(ROOT, "crdt_amd", "libycrdt.so"))
    src = os.path.join(ROOT, "crdt_amd", "csrc")
    for f in os.listdir(src):
        if f.endswith((".hip", ".h")):
            assert os.path.getmtime(os.path.join(src, f)) <= so, f"{f} is newer than libycrdt.so: rebuild"


def test_buf_arrays_point_at_the_inputs():
    """The mirror's ycrdt_buf[] (one joined blob, numpy-filled columns) addresses every input,
    empty ones included."""
    import ctypes

    ups = [b"", b"\x00\x00", bytes(range(200)), b"", b"\x01" * 7]
    arr, keep = crdt_amd._bufs(ups)
    assert len(keep) == len(ups)
    for i, u in enumerate(ups):
        assert arr[i].len == len(u)
        assert ctypes.string_at(arr[i].ptr, arr[i].len) == u
    empty, k = crdt_amd._bufs([])
    assert k == [] and len(empty) == 1
