"""Static instruction mix of the basic blocks inside one loop of a kernel dump (tools/asm_mix.py
output): blocks whose loop annotations name the loop header."""
import collections
import re
import sys

L = open(sys.argv[1]).read().split("\n")
depth = sys.argv[2] if len(sys.argv) > 2 else "2"
blocks = []  # (label, [comment lines], [instr lines])
cur = None
for l in L:
    if l.startswith(".LBB") or l.startswith("; %bb"):
        cur = [l.split()[0] if l.startswith(".LBB") else l.split()[1], [l], []]
        blocks.append(cur)
    elif cur is not None and l.strip().startswith(";"):
        if not cur[2]:
            cur[1].append(l)
    elif cur is not None and l.startswith("\t") and not l.strip().startswith("."):
        cur[2].append(l.split()[0])
# loop headers: blocks annotated "=> ... Loop Header: Depth=<depth>"
hdrs = [b[0].rstrip(":") for b in blocks if any(("Loop Header: Depth=" + depth) in c for c in b[1])]
for h in hdrs:
    name = h.lstrip(".L")
    c = collections.Counter()
    nb = 0
    for b in blocks:
        txt = " ".join(b[1])
        if b[0].rstrip(":") == h or ("Header=" + name + " ") in txt or ("Parent Loop " + name + " ") in txt:
            nb += 1
            c.update(b[2])
    valu = sum(v for k, v in c.items() if k.startswith("v_"))
    salu = sum(v for k, v in c.items() if k.startswith("s_") and not k.startswith(("s_load", "s_waitcnt", "s_nop", "s_cbranch", "s_branch")))
    print(h, "blocks", nb, "VALU", valu, "SALU", salu,
          {k: v for k, v in c.most_common() if k.startswith(("v_mov", "v_readlane", "v_writelane", "v_cndmask", "s_nop"))})
