"""SSAO tap-layout probe at 4K on the C3 Sponza-proxy MESH G-buffer (rasterised by the HIP rasteriser, as bench.py):
times SSAOGeneration reading the taps from the D32 image and from the depth layouts of ssao.hip (LAY_*), the layout
build pass separately, and checks every variant's output against the default's bits.
usage: python tools/ssao_layout_probe.py [W H]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import soc_real_time_renderer_amd as soc  # noqa: E402
from soc_real_time_renderer_amd import multi_gpu, raster, scene  # noqa: E402
from bench import make_globals  # noqa: E402


def timed(fn, n=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


def main():
    W, H = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (3840, 2160)
    dev = torch.device("cuda", 0)
    g = make_globals(W, H, multi_gpu.camera_for_rank(0))
    sc = raster.scene_setup(g, scene.SPONZA_MESH, tex_size=256, device=dev)
    gbd = raster.render_gbuffer(g, sc, W, H, 1024, dev)
    depth, normal = gbd["depth"], gbd["normal"]
    lib = soc.lib()
    lib.soc_depth_layout_bytes.restype = C.c_int64
    lib.soc_depth_layout.argtypes = [soc.SocImg, C.c_void_p, C.c_int32, C.c_void_p]
    lib.soc_ssao_generation_layout.argtypes = [C.c_void_p, soc.SocImg, C.c_void_p, C.c_int32, soc.SocImg, soc.SocImg,
                                               C.c_void_p, C.c_void_p]
    table = torch.zeros((H // 2) * (W // 2) * 2, dtype=torch.float32, device=dev)
    ref = torch.zeros(H // 2, W // 2, dtype=torch.uint8, device=dev)
    soc.ssao_prepare_noise(normal, ref, table)
    soc.ssao_generation(g, depth, normal, ref, table)
    torch.cuda.synchronize()
    us = timed(lambda: soc.ssao_generation(g, depth, normal, ref, table))
    print(f"D32 (default): {us:.1f} us", flush=True)
    st = soc._stream(None)
    for lay, name in ((1, "row pairs both parities"), (2, "quads"), (8, "PROBE taps on the lane's rows (wrong result)"),
                      (9, "PROBE taps at the lane's own texels (wrong result)")):
        nbytes = lib.soc_depth_layout_bytes(W, H, lay if lay < 8 else 1)
        buf = torch.zeros(nbytes, dtype=torch.uint8, device=dev)
        bp = C.c_void_p(buf.data_ptr())

        def build():
            assert lib.soc_depth_layout(soc.img(depth), bp, lay if lay < 8 else 1, st) == 0

        build_us = timed(build)
        out = torch.zeros_like(ref)

        def run():
            assert lib.soc_ssao_generation_layout(C.addressof(g), soc.img(depth), bp, lay, soc.img(normal), soc.img(out),
                                                  soc._ptr(table), st) == 0

        us2 = timed(run)
        same = bool(torch.equal(out, ref))
        print(f"{name}: ssao {us2:.1f} us, layout build {build_us:.1f} us ({nbytes / 1e6:.1f} MB), "
              f"bit-identical {same}", flush=True)


if __name__ == "__main__":
    main()
