"""Frame-per-GPU path with a real peer, on the GPU.

Two and eight ranks (torch.distributed.run, gloo, all on device 0; eight is SURVEY.md §8e's "8 simulated
ranks on one GPU" parity case) each render their own camera through the HIP
render graph: PRE_EXPOSURE -> histogram all-reduce -> POST_EXPOSURE (wide resolve over 2*W*H pixels).
Checks, per frame:
  * each rank's local bins are the oracle's histogram of that rank's own GPU colour image (bit-exact);
  * the exchanged bins are the sum of the local ones on every rank;
  * every rank's exposure equals the oracle's wide resolve of the summed bins (|d| <= 1e-5), frame after
    frame (the exposure carries over: resolve_luminance_histogram.inl:75-79).
Config C5 at its own size (`test_c5_4k_exchange_vs_oracle`): eight ranks on device 0, each rendering the bench's
own C3 inputs for its camera (the Sponza-proxy mesh at 3840x2160, bench.build_inputs), two frames with the same checks;
the local-bin check runs on each rank against the oracle histogram of its own 4K colour. Reference exchange point:
renderer.cpp:1155-1168.
And `bench.py --gpus 2` (self-launching its ranks) prints one line with n_gpus == 2.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env(**kw):
    env = dict(os.environ)
    env.update({"SOC_BENCH_SHARE_DEVICE": "1", "SOC_DIST_BACKEND": "gloo", "HSA_ENABLE_IPC_MODE_LEGACY": "0",
                "OMP_NUM_THREADS": "2", **kw})
    return env


@pytest.mark.parametrize("ranks,backend", [(1, "nccl"), (2, "gloo"), (8, "gloo")])
def test_rank_frames_exchange_vs_oracle(tmp_path, soc, oracle, ranks, backend):
    """(1, nccl): the real collective (RCCL) at world size 1 -- PRE -> dist.all_reduce on the device AutoExposure bins ->
    POST, the renderer's second (sky) lane on -- on the 1-GPU box; the multi-rank cases share device 0 over gloo."""
    from helpers import globals_for
    from soc_real_time_renderer_amd import multi_gpu
    out = tmp_path / "dist.npz"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
           "--master-addr", "127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "tests", "dist_frame_worker.py")]
    extra = dict(SOC_DIST_BACKEND="nccl", SOC_DIST_FORCE="1", SOC_BENCH_SHARE_DEVICE="0") if backend == "nccl" else {}
    p = subprocess.run(cmd, env=_env(SOC_DIST_OUT=str(out), **extra), capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    d = np.load(out)
    world, W, H = int(d["world"]), int(d["W"]), int(d["H"])
    assert world == ranks
    local, reduced, exposure, color = d["local"], d["reduced"], d["exposure"], d["color"]
    frames = local.shape[1]
    g = globals_for(W, H, elapsed=10.0, frame_counter=2)
    ae = soc.AutoExposure()   # exposure 0 at start, like the renderer's buffer
    for f in range(frames):
        for r in range(world):
            ref = soc.AutoExposure()
            oracle.generate_luminance_histogram(g, color[r, f], ref)
            assert np.array_equal(np.array(ref.histogram_buckets, np.uint32), local[r, f]), (r, f)
            assert int(local[r, f].astype(np.int64).sum()) == W * H
        summed = local[:, f].astype(np.uint64).sum(axis=0)
        for r in range(world):
            assert np.array_equal(reduced[r, f].astype(np.uint64), summed), (r, f)
        ae.histogram_buckets[:] = [int(v) for v in summed]
        total, wide = multi_gpu.exposure_pixels(world, W, H)
        oracle.resolve_luminance_histogram(g, ae, total, wide)
        for r in range(world):
            assert abs(float(exposure[r, f]) - ae.exposure) <= 1e-5, (r, f, float(exposure[r, f]), ae.exposure)
        assert all(exposure[r, f] == exposure[0, f] for r in range(world))
    # the ranks rendered different cameras
    for r in range(1, world):
        assert not np.array_equal(local[0, 0], local[r, 0]), r


def test_c5_4k_exchange_vs_oracle(tmp_path, soc, oracle):
    import bench
    from soc_real_time_renderer_amd import multi_gpu
    ranks = 8
    out = tmp_path / "c5.npz"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
           "--master-addr", "127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "tests", "dist_frame_worker.py")]
    p = subprocess.run(cmd, env=_env(SOC_DIST_OUT=str(out), SOC_DIST_CONFIG="c3"), capture_output=True, text=True,
                       timeout=400)
    errs = [ln for ln in p.stderr.splitlines() if "Error" in ln or "error" in ln]
    assert p.returncode == 0, "\n".join(errs[:20]) + p.stdout[-2000:] + p.stderr[-4000:]
    d = np.load(out)
    world, W, H = int(d["world"]), int(d["W"]), int(d["H"])
    assert (world, W, H) == (ranks, 3840, 2160)
    local, reduced, exposure, local_ok = d["local"], d["reduced"], d["exposure"], d["local_ok"]
    assert local_ok.all(), local_ok          # each rank: bins == the oracle histogram of its own GPU colour
    assert (d["sky"] < 0.5).all()
    g = bench.make_globals(W, H, multi_gpu.camera_for_rank(0))
    ae = soc.AutoExposure()
    for f in range(local.shape[1]):
        for r in range(world):
            assert int(local[r, f].astype(np.int64).sum()) == W * H
        summed = local[:, f].astype(np.uint64).sum(axis=0)
        assert int(summed.sum()) == world * W * H
        for r in range(world):
            assert np.array_equal(reduced[r, f].astype(np.uint64), summed), (r, f)
        ae.histogram_buckets[:] = [int(v) for v in summed]
        total, wide = multi_gpu.exposure_pixels(world, W, H)
        oracle.resolve_luminance_histogram(g, ae, total, wide)
        for r in range(world):
            assert abs(float(exposure[r, f]) - ae.exposure) <= 1e-5, (r, f, float(exposure[r, f]), ae.exposure)
    for r in range(1, world):
        assert not np.array_equal(local[0, 0], local[r, 0]), r


def test_bench_exchange_rccl_world1():
    """bench.py --exchange at N = 1: the frames take PRE -> RCCL all-reduce (a world-size-1 group) -> POST and the line
    carries the backend and the all-reduce time per frame (SURVEY.md §8e's report)."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--exchange", "--steps", "20", "--warmup", "5",
           "--width", "640", "--height", "360", "--no-cpu-baseline", "--profile-frames", "2"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    # the line is the whole of stdout: RCCL's version banner and other native prints go to stderr (bench.emit)
    lines = p.stdout.splitlines()
    assert len(lines) == 1 and lines[0].startswith("{"), p.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 1
    assert out["config"]["histogram_allreduce"] is True
    assert out["config"]["collective_backend"] == "nccl"
    assert out["allreduce_us_per_frame"] is not None and out["allreduce_us_per_frame"] > 0


def test_bench_gpus2_self_launch():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "4", "--warmup", "1",
           "--width", "320", "--height", "180", "--no-cpu-baseline", "--profile-frames", "2"]
    p = subprocess.run(cmd, env=_env(), capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2
    assert out["config"]["histogram_allreduce"] is True
    assert [x["rank"] for x in out["ranks"]] == [0, 1]
    assert out["allreduce_us_per_frame"] is not None and out["allreduce_us_per_frame"] > 0
    assert out["value"] > 0
