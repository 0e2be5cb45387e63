#!/usr/bin/env python3
"""Dumps a generated workload batch (C1/C2) as one binary file for native decode experiments.

Format: u32 n, then n × (u32 len, len bytes). Usage: python scripts/dump_workload.py c2 out.bin
"""
import struct
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from crdt_amd.workload import C1, C2, gen_map  # noqa: E402


def main():
    name, out = sys.argv[1], sys.argv[2]
    ups, _ = gen_map(**(C2 if name == "c2" else C1))
    with open(out, "wb") as f:
        f.write(struct.pack("<I", len(ups)))
        for u in ups:
            f.write(struct.pack("<I", len(u)))
            f.write(u)
    print(len(ups), sorted(len(u) for u in ups)[-3:])


if __name__ == "__main__":
    main()
