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
