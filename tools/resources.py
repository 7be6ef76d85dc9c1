#!/usr/bin/env python3
"""Per-kernel register / occupancy table from `make -C raytrace2_amd/csrc asm` remarks (stdin)."""
import re
import sys

txt = sys.stdin.read()
rows = []
for blk in re.split(r"remark: Function Name: ", txt)[1:]:
    name = blk.split()[0]
    def g(k):
        m = re.search(re.escape(k) + r": (\d+)", blk)
        return int(m.group(1)) if m else -1
    m = re.search(r"render_kernelILj(\d+)ELi(\d)ELb(\d)E", name)
    tag = f"F={m.group(1):>3} mode={m.group(2)} stats={m.group(3)}" if m else name[:40]
    rows.append((tag, g("VGPRs"), g("SGPRs"), g("SGPRs Spill"), g("VGPRs Spill"), g("ScratchSize [bytes/lane]"),
                 g("Occupancy [waves/SIMD]")))
print(f"{'kernel':40} {'vgpr':>5} {'sgpr':>5} {'sspill':>6} {'vspill':>6} {'scratch':>7} {'occ':>4}")
for r in rows:
    print(f"{r[0]:40} {r[1]:5} {r[2]:5} {r[3]:6} {r[4]:6} {r[5]:7} {r[6]:4}")
