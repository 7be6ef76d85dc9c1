#!/usr/bin/env python3
"""Static spill / reload instructions of a kernel by loop depth (scratch and SGPR-to-VGPR-lane):
  python3 tools/spills_in_loops.py <file.s> [kernel-symbol-substring]"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else "render_kernel"
for m in re.finditer(r"\n(_Z\w*" + re.escape(pat) + r"\w*):[^\n]*\n", s):
    sym = m.group(1)
    body = s[m.end():s.index(".Lfunc_end", m.end())].split("\n")
    depth = 0
    c = collections.Counter()
    for l in body:
        if l.startswith(".LBB") or l.startswith("; %bb"):
            d = re.search(r"Depth=(\d+)", l)
            depth = int(d.group(1)) if d else 0
        t = l.strip()
        op = t.split()[0] if t else ""
        if op.startswith("scratch_") or op in ("v_readlane_b32", "v_writelane_b32"):
            c[(op, depth)] += 1
    print(sym[:70])
    for (op, d), n in sorted(c.items(), key=lambda x: (x[0][1], x[0][0])):
        print(f"  depth {d}  {op:24s} {n}")
