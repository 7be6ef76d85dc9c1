"""Static checks on the gfx950 kernel's generated ISA (hipcc cross-compiles here, no GPU):
 * no inline-asm block issues a scalar load whose base/offset registers an earlier load of the same
   block writes (that load's data may land first: a wrong address, i.e. a GPU memory fault);
 * no scratch (spill) memory in the variants the benchmark uses."""
import os
import re
import subprocess

import pytest

from conftest import ROOT

SRC = os.path.join(ROOT, "raytrace2_amd", "csrc", "render.hip")


def makefile_hipflags():
    """The kernel's compile flags as the build uses them (raytrace2_amd/csrc/Makefile HIPFLAGS)."""
    mk = open(os.path.join(ROOT, "raytrace2_amd", "csrc", "Makefile")).read()
    line = re.search(r"^HIPFLAGS\s*:=(.*)$", mk, re.M).group(1)
    return [f for f in line.split() if not f.startswith("$(") and f not in ("-fPIC", "-Wall")]


@pytest.fixture(scope="module")
def isa(tmp_path_factory):
    out = tmp_path_factory.mktemp("isa") / "render.s"
    flags = makefile_hipflags()
    assert "--offload-arch=gfx950" in flags
    r = subprocess.run(["/opt/rocm/bin/hipcc", *flags, "--cuda-device-only", "-S", "-o", str(out), SRC,
                        "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    return out.read_text(), r.stderr


def test_inline_scalar_loads_have_no_register_hazards(isa):
    s, _ = isa
    checked = 0
    for blk in re.findall(r";;#ASMSTART\n(.*?);;#ASMEND", s, re.S):
        loads = [l.strip() for l in blk.split("\n") if l.strip().startswith("s_load")]
        if len(loads) < 2:
            continue
        checked += 1
        written = set()
        for l in loads:
            ops = []
            for a, b, c in re.findall(r"s\[(\d+):(\d+)\]|\bs(\d+)\b", l.split(None, 1)[1]):
                ops.append(set(range(int(a), int(b) + 1)) if a else {int(c)})
            assert not (set().union(*ops[1:]) & written), loads
            written |= ops[0]
    assert checked > 0


def test_no_scratch_in_bench_variants(isa):
    """The Cornell kernel the benchmark times (threaded, no stats) writes no spill inside its loops.
    At 8 waves (64 VGPRs) the compiler parks a few loop-invariant values in scratch (at most 16 B per
    lane) once before the path loop and reloads them (L1-hit loads, no store traffic)."""
    s, remarks = isa
    blocks = re.split(r"remark: Function Name: ", remarks)[1:]
    seen = 0
    for b in blocks:
        name = b.split()[0]
        if "ILj4ELi2ELb0E" not in name:
            continue
        seen += 1
        scratch = int(re.search(r"ScratchSize \[bytes/lane\]: (\d+)", b).group(1))
        assert scratch <= 16, (name, scratch)
        body = s.split(f"\n{name}:", 1)[1].split(".Lfunc_end", 1)[0]
        head = re.search(r"^\.LBB\d+_\d+:.*Loop Header: Depth=1", body, re.M)
        stores = [m.start() for m in re.finditer(r"scratch_store|buffer_store.*Spill", body)]
        assert head is not None and all(p < head.start() for p in stores), (name, len(stores))
    assert seen == 1


def _loop_depth_scratch(body):
    """(loop depth, instruction) of every scratch (spill) access in a kernel body."""
    out, depth = [], 0
    for line in body.split("\n"):
        if line.startswith(".LBB") or line.startswith("; %bb"):
            m = re.search(r"Depth=(\d+)", line)
            depth = int(m.group(1)) if m else 0
        t = line.strip()
        if t.startswith("scratch_"):
            out.append((depth, t.split()[0]))
    return out


def _kernel(isa, tag):
    s, remarks = isa
    blk = [b for b in re.split(r"remark: Function Name: ", remarks)[1:] if tag in b.split()[0]]
    assert len(blk) == 1, tag
    name = blk[0].split()[0]
    scratch = int(re.search(r"ScratchSize \[bytes/lane\]: (\d+)", blk[0]).group(1))
    body = s.split(f"\n{name}:", 1)[1].split(".Lfunc_end", 1)[0]
    return scratch, body


def test_cornell_volume_bench_kernel_spills_at_most_one_pair(isa):
    """the Cornell volume kernel the C4 bench runs (threaded, 8 waves) spills at most one
    8-byte register pair (the path's pixel word, stored once per work item, reloaded at the Philox
    refills) and no spill store sits inside the trace's loops (round 3's one-pass box boundaries had
    pushed it to 25 spilled VGPRs, 56 B per lane, stored and reloaded in the trace)."""
    scratch, body = _kernel(isa, "ILj6ELi2ELb0E")
    deep = [x for x in _loop_depth_scratch(body) if x[0] >= 2 and x[1].startswith("scratch_store")]
    assert scratch <= 16 and not deep, (scratch, deep[:5])


def test_book2_bench_kernel_spills_stay_out_of_the_trace(isa):
    """The book 2 kernel (C5) runs at 8 waves with VGPRs spilled (occupancy beats spills there, DESIGN
    §4): its scratch stays at most 96 B per lane and no spill store or reload sits inside the trace's
    loops (loop depth >= 2); the reloads left are the marble texture's double-precision sin constants
    on the shading path (depth 1)."""
    scratch, body = _kernel(isa, "ILj303ELi2ELb0E")
    deep = [x for x in _loop_depth_scratch(body) if x[0] >= 2]
    assert scratch <= 96 and not deep, (scratch, deep[:5])
