#!/usr/bin/env python3
"""Instruction histogram of one kernel in a hipcc -S output (dev tool).
usage: isa_stats.py file.s kernel_substring [top]"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
names = [m.group(1) for m in re.finditer(r"^(\S+):(?:\s|$)", s, flags=re.M) if pat in m.group(1) and not m.group(1).startswith(".")]
name = names[0]
i = s.index("\n" + name + ":") + 1
j = s.index(".Lfunc_end", i)
c = collections.Counter()
for line in s[i:j].split("\n"):
    t = line.strip()
    if not t or t.startswith((".", ";")) or t.endswith(":"):
        continue
    c[t.split()[0]] += 1
print(name, "static instrs", sum(c.values()))
for k, v in c.most_common(top):
    print(f"  {k:30s}{v}")
m = re.search(r"\.vgpr_count:\s+(\d+)", s[j:j + 200000])
