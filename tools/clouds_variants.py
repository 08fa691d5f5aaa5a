"""Time the cloud pass split into its parts (atmosphere / cloud march / sun-visibility march).

Builds profiling variants of clouds.hip (-DSOC_CLOUDS_PROFILE=k) linked with the other objects into
build/variants/libsoc_rt_clouds<k>.so, then times each on the bench workload with HIP events.
Usage: python tools/clouds_variants.py [--build-only]
"""
import ctypes as C
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "soc_real_time_renderer_amd", "csrc")
BUILD = os.path.join(ROOT, "soc_real_time_renderer_amd", "build")
VAR = os.path.join(BUILD, "variants")
MODES = {0: "full", 1: "atmosphere only", 2: "cloud march only", 3: "cloud march, no sun march"}


def build():
    os.makedirs(VAR, exist_ok=True)
    objs = [os.path.join(BUILD, f) for f in os.listdir(BUILD) if f.endswith(".o") and f != "clouds.o"]
    for k in MODES:
        o = os.path.join(VAR, f"clouds{k}.o")
        so = os.path.join(VAR, f"libsoc_rt_clouds{k}.so")
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17",
                               "-mcode-object-version=5", f"-DSOC_CLOUDS_PROFILE={k}", "-I" + os.path.join(ROOT, "include"),
                               "-c", os.path.join(CSRC, "clouds.hip"), "-o", o])
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", so, o] + objs)


def run():
    sys.path.insert(0, ROOT)
    import torch
    import bench
    import soc_real_time_renderer_amd as soc
    from soc_real_time_renderer_amd import _abi, multi_gpu, scene
    W, H = 3840, 2160
    g = bench.make_globals(W, H, multi_gpu.camera_for_rank(0))
    gb = scene.gbuffer(g, W, H)
    dev = torch.device("cuda", 0)
    depth = torch.from_numpy(gb["depth"]).to(dev)
    noise = torch.from_numpy(scene.noise_texture()).to(dev)
    out = torch.zeros(H, W, 4, dtype=torch.uint8, device=dev)
    ws = soc.cloud_rendering_workspace(W, H, dev)
    s = torch.cuda.current_stream()
    for k, name in MODES.items():
        lib = C.CDLL(os.path.join(VAR, f"libsoc_rt_clouds{k}.so"))
        lib.soc_cloud_rendering.restype = C.c_int
        lib.soc_cloud_rendering.argtypes = [C.c_void_p, _abi.SocImg, _abi.SocImg, _abi.SocImg, C.c_void_p, C.c_void_p]
        args = (C.byref(g), soc.img(depth), soc.img(noise), soc.img(out), C.c_void_p(ws.data_ptr()), C.c_void_p(s.cuda_stream))
        for _ in range(3):
            assert lib.soc_cloud_rendering(*args) == 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(20):
            lib.soc_cloud_rendering(*args)
        e1.record(s)
        torch.cuda.synchronize()
        print(f"mode {k} ({name}): {e0.elapsed_time(e1) / 20 * 1e3:.1f} us", flush=True)


if __name__ == "__main__":
    if "--run-only" not in sys.argv:
        build()
    if "--build-only" not in sys.argv:
        run()
