"""Instruction mix of one render_kernel variant in build/rt2/render.s (make -C raytrace2_amd/csrc asm)."""
import collections
import re
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "ILj4ELi2ELb0E"
s = open("build/rt2/render.s").read()
name = [m for m in re.findall(r"^(_Z\S+):", s, re.M) if tag in m][0]
st = s.index("\n" + name + ":") + 1
en = s.index(".Lfunc_end", st)
body = s[st:en].split("\n")
ins = [l for l in body if l.startswith("\t") and not l.strip().startswith((".", ";"))]
print(name, len(ins), "instructions")
c = collections.Counter(l.split()[0] for l in ins)
print(c.most_common(50))
out = sys.argv[2] if len(sys.argv) > 2 else "/tmp/kernel.s"
open(out, "w").write("\n".join(body))
