"""bench.py in the launch forms the round-end runs use, at a small Cornell size.

* `python bench.py` (N = 1): the one-process tracer, ncclGather over a communicator of size 1;
* `python -m torch.distributed.run --nproc-per-node 1 ... bench.py --gpus 1` with RT2_BENCH_RANKS=1:
  the one-process-per-GPU path of the scaling runs (rt2_tracer_join = ncclCommInitRank, the gather
  to rank 0, max-over-ranks timing) at world 1;
* the same launcher with 2 ranks and RT2_BENCH_SHARE_GPU=1: both ranks on GPU 0, each rendering its
  row bands, the bands gathered over gloo (a rehearsal of N = 2: RCCL cannot put two ranks on one GPU).

Each run prints one JSON line with the contract's fields, and writes the gathered image, which must
equal the plain one-GPU tracer's image byte for byte (the band split is invisible in the result)."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

ARGS = ["--scene", "cornell_box_original.json", "--width", "96", "--height", "80", "--spp", "16",
        "--steps", "2", "--warmup", "1", "--no-cpu", "--stats-frames", "1"]


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(tmp_path, name, env_extra, nproc=None, extra=()):
    img = str(tmp_path / f"{name}.png")
    cmd = [sys.executable, "-u"]
    if nproc is not None:
        cmd += ["-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}", "--master-addr",
                "127.0.0.1", "--master-port", str(_port())]
    cmd += [os.path.join(ROOT, "bench.py"), "--gpus", str(nproc or 1), *ARGS, "--out-image", img, *extra]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", **env_extra)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT, env=env)
    assert r.returncode == 0, (name, r.stdout[-2000:], r.stderr[-3000:])
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, (name, r.stdout[-2000:])
    return json.loads(lines[0]), open(img, "rb").read()


@pytest.fixture(scope="module")
def plain(tmp_path_factory, have_gpu):
    return _run(tmp_path_factory.mktemp("bench"), "plain", {}, extra=["--plain"])


def _check_line(d, n):
    # (BASELINE.json's metric name is printed for the headline workload only; one image split over the
    # ranks is strong scaling)
    assert d["metric"] == "Mray/s (samples x bounces) cornell_box_original.json 96x80 @ 16 spp"
    assert d["n_gpus"] == n and d["steps"] == 2 and d["warmup"] == 1 and d["unit"] == "Mray/s"
    assert d["value"] > 0 and d["ms_per_step"] > 0 and d["higher_is_better"] is True and d["scaling"] == "strong"
    assert d["config"]["workload"].startswith("cornell_box_original.json 96x80 @ 16 spp")
    assert sum(r["rows"] for r in d["detail"]["per_rank"]) == 80 and len(d["detail"]["per_rank"]) == (n if n > 1 else 1)


def test_bench_single_process(tmp_path, plain):
    d, img = _run(tmp_path, "multi1", {})
    _check_line(d, 1)
    assert img == plain[1]


def test_bench_rank_per_gpu_world1_rccl(tmp_path, plain):
    d, img = _run(tmp_path, "ranks1", {"RT2_BENCH_RANKS": "1"}, nproc=1)
    _check_line(d, 1)
    assert img == plain[1]


def test_bench_two_ranks_share_one_gpu(tmp_path, plain):
    d, img = _run(tmp_path, "share2", {"RT2_BENCH_SHARE_GPU": "1"}, nproc=2)
    _check_line(d, 2)
    assert img == plain[1]
