"""Time profiling builds of one kernel source (-D<MACRO>=k) on a fixed workload.

Each variant is clouds.hip / bloom_fused.hip compiled with the macro and linked with the other
objects into build/variants/libsoc_rt_<name><k>.so (ctypes loads them side by side).
Usage: python tools/kernel_variants.py {clouds|comp|bloom4} [--build-only | --run-only] [--modes 0,2]
"""
import ctypes as C
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "soc_real_time_renderer_amd", "csrc")
BUILD = os.path.join(ROOT, "soc_real_time_renderer_amd", "build")
VAR = os.path.join(BUILD, "variants")
CASES = {
    "clouds": ("clouds.hip", "SOC_CLOUDS_PROFILE",
               {0: "full", 1: "atmosphere only", 2: "cloud march only", 3: "cloud march, no sun march",
                4: "classify only", 5: "classify only, no atomic"}),
    "comp": ("composition.hip", "SOC_COMP_PROFILE",
             {0: "full", 1: "no shadow tap", 2: "no AO tap", 3: "no shadow, no AO"}),
    "bloom4": ("bloom_fused.hip", "SOC_BLOOM_PROFILE",
               {0: "K4 full", 1: "K4 no quad phase", 2: "K4 no output phase", 3: "K4 no global stores"}),
}


def build(case):
    src, macro, modes = CASES[case]
    os.makedirs(VAR, exist_ok=True)
    obj = src.replace(".hip", ".o")
    objs = [os.path.join(BUILD, f) for f in os.listdir(BUILD) if f.endswith(".o") and f != obj]
    for k in modes:
        o = os.path.join(VAR, f"{case}{k}.o")
        so = os.path.join(VAR, f"libsoc_rt_{case}{k}.so")
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17",
                               "-mcode-object-version=5", "-fno-slp-vectorize", f"-D{macro}={k}", "-I" + os.path.join(ROOT, "include"),
                               "-c", os.path.join(CSRC, src), "-o", o])
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", so, o] + objs)


def workload(case, lib, dev):
    """Returns a callable issuing one launch of the variant's pass on the bench workload."""
    import torch
    import bench
    import soc_real_time_renderer_amd as soc
    from soc_real_time_renderer_amd import _abi, multi_gpu, scene
    W, H = 3840, 2160
    g = bench.make_globals(W, H, multi_gpu.camera_for_rank(0))
    s = torch.cuda.current_stream()
    P = C.c_void_p
    if case == "comp":
        gb = scene.gbuffer(g, W, H)
        shadow = torch.from_numpy(scene.shadow_map(g, 4096)).to(dev)
        t = {k: torch.from_numpy(gb[k]).to(dev) for k in ("albedo", "emissive", "normal", "depth")}
        ssao = torch.full((H // 2, W // 2), 200, dtype=torch.uint8, device=dev)
        clouds = torch.zeros(H, W, 4, dtype=torch.uint8, device=dev)
        out = torch.zeros(H, W, 4, dtype=torch.float16, device=dev)
        lib.soc_composition.argtypes = [P, P] + [_abi.SocImg] * 8 + [P]
        args = (C.byref(g), None, soc.img(out), soc.img(t["albedo"]), soc.img(t["emissive"]), soc.img(t["normal"]),
                soc.img(t["depth"]), soc.img(ssao), soc.img(shadow), soc.img(clouds), P(s.cuda_stream))
        return lambda: lib.soc_composition(*args), (shadow, t, ssao, clouds, out)
    if case == "clouds":
        gb = scene.gbuffer(g, W, H)
        depth = torch.from_numpy(gb["depth"]).to(dev)
        noise = torch.from_numpy(scene.noise_texture()).to(dev)
        out = torch.zeros(H, W, 4, dtype=torch.uint8, device=dev)
        ws = soc.cloud_rendering_workspace(W, H, dev)
        lib.soc_cloud_rendering.argtypes = [P, _abi.SocImg, _abi.SocImg, _abi.SocImg, P, P]
        args = (C.byref(g), soc.img(depth), soc.img(noise), soc.img(out), P(ws.data_ptr()), P(s.cuda_stream))
        keep = (depth, noise, out, ws)
        return lambda: lib.soc_cloud_rendering(*args), keep
    em = (torch.rand(H, W, 4, device=dev) * 4).half()
    mips = [torch.zeros(H >> i, W >> i, 4, dtype=torch.float16, device=dev) for i in range(4)]
    out = torch.zeros_like(em)
    arr = (_abi.SocImg * 4)(*[soc.img(m) for m in mips])
    lib.soc_bloom_fused_stage.argtypes = [P, _abi.SocImg, C.POINTER(_abi.SocImg), C.c_int32, _abi.SocImg, C.c_int32, P]
    lib.soc_bloom_fused_stage(C.byref(g), soc.img(em), arr, 4, soc.img(out), 0, P(s.cuda_stream))
    args = (C.byref(g), soc.img(em), arr, 4, soc.img(out), 4, P(s.cuda_stream))
    return lambda: lib.soc_bloom_fused_stage(*args), (em, mips, out, arr)


def run(case, only=None):
    sys.path.insert(0, ROOT)
    import torch
    dev = torch.device("cuda", 0)
    for k, name in CASES[case][2].items():
        if only is not None and k not in only:
            continue
        lib = C.CDLL(os.path.join(VAR, f"libsoc_rt_{case}{k}.so"))
        fn, keep = workload(case, lib, dev)
        for _ in range(3):
            assert fn() == 0
        s = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(20):
            fn()
        e1.record(s)
        torch.cuda.synchronize()
        print(f"{case} mode {k} ({name}): {e0.elapsed_time(e1) / 20 * 1e3:.1f} us", flush=True)
        del keep


if __name__ == "__main__":
    case = sys.argv[1]
    if "--run-only" not in sys.argv:
        build(case)
    only = None
    if "--modes" in sys.argv:
        only = [int(m) for m in sys.argv[sys.argv.index("--modes") + 1].split(",")]
    if "--build-only" not in sys.argv:
        run(case, only)
