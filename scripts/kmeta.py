#!/usr/bin/env python3
"""Per-kernel register / scratch / LDS metadata from a hipcc -S output (dev tool).
usage: kmeta.py file.s [name_substring]"""
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else ""
meta = s[s.index("amdhsa.kernels:"):]
for blk in re.split(r"\n  - ", meta)[1:]:
    f = dict(re.findall(r"^\s*\.(\w+):\s+(\S+)", blk, flags=re.M))
    name = f.get("name", "?")
    if pat in name:
        print(f"{name[:70]:70s} vgpr {f.get('vgpr_count')} agpr {f.get('agpr_count')} "
              f"scratch {f.get('private_segment_fixed_size')} lds {f.get('group_segment_fixed_size')} "
              f"spill_v {f.get('vgpr_spill_count')}")
