#!/usr/bin/env python3
"""Times the batched merge of a saved batch (u32 count, then u32 len + bytes per update) on the GPU,
per phase, and checks the output against a saved expected update. Usage: probe_batch.py <bin> [<out>]"""
import struct
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import crdt_amd  # noqa: E402

b = open(sys.argv[1], "rb").read()
n = struct.unpack_from("<I", b, 0)[0]
p, ups = 4, []
for _ in range(n):
    ln = struct.unpack_from("<I", b, p)[0]
    ups.append(b[p + 4:p + 4 + ln])
    p += 4 + ln
eng = crdt_amd.Engine()
bt = crdt_amd.Batch(ups, eng)
st = bt.merge()
eng.set_profiling(True)
st = bt.merge()
ph = eng.phase_times()
eng.set_profiling(False)
out = bt.result()[0]
print("items", st.items, "structs", st.structs, "segments", st.segments, "device_ms", round(st.device_ms, 3))
print({k: round(v, 3) for k, v in ph})
if len(sys.argv) > 2:
    print("parity", out == open(sys.argv[2], "rb").read())
