"""Where a render kernel reloads spilled SGPRs inside its loops (each reload is a v_readlane, one VALU
instruction): maps every spill lane back to the kernel-argument field it holds when the prologue
loaded it from the argument segment, and counts the reloads per field at loop depth >= 1.
  python3 tools/spill_map.py build/rt2/render.s <kernel symbol>   (make -C raytrace2_amd/csrc asm)"""
import collections
import re
import sys

FIELDS = [("nodes", 0), ("materials", 8), ("textures", 16), ("perlin_vec", 24), ("perlin_perm", 32), ("root", 40),
          ("background", 44), ("cam", 56), ("width", 140), ("height", 144), ("local_rows", 148), ("band_h", 152),
          ("rank", 156), ("world", 160), ("tile_shift", 164), ("tiles_x", 168), ("tile_items", 172),
          ("n_items", 176), ("batch_max", 180), ("batch_div", 184), ("frame_begin", 188), ("n_frames", 192),
          ("max_depth", 196), ("chunks", 200), ("n_chunks", 208), ("div_tile_items", 212), ("div_tiles_x", 220),
          ("div_band_h", 228), ("div_band_w", 236), ("div_world", 244), ("seed_lo", 252), ("seed_hi", 256),
          ("samples", 264), ("local_pixels", 272), ("ray_counts", 280), ("work_counter", 288), ("stats", 296),
          ("stack_depth", 304), ("lds_nodes", 308), ("lds_partial", 312), ("lin", 320), ("lind", 328),
          ("lin_wide", 336), ("lin_len", 344)]


def field(off):
    name = None
    for n, o in FIELDS:
        if o <= off:
            name = f"{n}+{off - o}" if off > o else n
    return name


src, sym = sys.argv[1], sys.argv[2]
s = open(src).read()
i = s.index("\n" + sym + ":")
j = s.index(".Lfunc_end", i)
L = s[i:j].split("\n")
kseg = {"s[0:1]"}  # kernarg segment pointer copies
sgpr_src = {}       # sgpr -> kernarg offset
lane_src = {}       # (vgpr, lane) -> kernarg offset or '?'
depth = 0
reloads = collections.Counter()
for l in L:
    if l.startswith(".LBB") or l.startswith("; %bb"):
        m = re.search(r"Depth=(\d+)", l)
        depth = int(m.group(1)) if m else 0
        continue
    t = l.strip()
    if t.startswith(";"):
        m = re.search(r"Depth=(\d+)", t)
        if m:
            depth = int(m.group(1))
        continue
    m = re.match(r"s_mov_b64 (s\[\d+:\d+\]), s\[0:1\]", t)
    if m:
        kseg.add(m.group(1))
    m = re.match(r"s_load_dword(?:x(\d+))? (s\[(\d+):(\d+)\]|s(\d+)), (s\[\d+:\d+\]), (0x[0-9a-f]+|\d+)$", t)
    if m and m.group(6) in kseg:
        base = int(m.group(3) or m.group(5))
        n = int(m.group(1) or 1)
        off = int(m.group(7), 0)
        for k in range(n):
            sgpr_src[f"s{base + k}"] = off + 4 * k
        continue
    m = re.match(r"s_mov_b32 (s\d+), (s\d+)$", t)
    if m:
        if m.group(2) in sgpr_src:
            sgpr_src[m.group(1)] = sgpr_src[m.group(2)]
        else:
            sgpr_src.pop(m.group(1), None)
        continue
    m = re.match(r"v_writelane_b32 (v\d+), (s\d+), (\d+)$", t)
    if m:
        lane_src[(m.group(1), m.group(3))] = sgpr_src.get(m.group(2), "?")
        continue
    m = re.match(r"v_readlane_b32 (s\d+), (v\d+), (\d+)$", t)
    if m and depth >= 1:
        o = lane_src.get((m.group(2), m.group(3)), "?")
        reloads[(field(o) if o != "?" else "?(computed)", depth)] += 1
    m = re.match(r"\S+ (s\d+)", t)  # any other write of an sgpr ends its kernarg identity
    if m and not t.startswith(("v_", "s_waitcnt", "s_cbranch", "s_branch", "s_cmp")):
        sgpr_src.pop(m.group(1), None)
tot = sum(reloads.values())
print(f"{tot} static v_readlane reloads inside loops")
for (f, d), c in sorted(reloads.items(), key=lambda x: -x[1]):
    print(f"  depth {d}  {c:4d}  {f}")
