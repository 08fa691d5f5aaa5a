"""Hi-Z pyramid (GenerateMin/MaxHIZTask, generate_hiz.glsl:17-98; terrain row f3). CPU: the oracle equals
the plain 2x2 min / max pyramid where the extents halve exactly. GPU: bit-exact against the oracle at
every size, odd extents included (the reference's window quirks are reproduced on both sides)."""
import numpy as np
import pytest
import torch

from helpers import globals_for
from soc_real_time_renderer_amd import raster


def mips_for(W, H, lib="np"):
    n = raster.hiz_mip_count(W, H)
    shapes = [(max(1, (H // 2) >> i), max(1, (W // 2) >> i)) for i in range(n)]
    if lib == "np":
        return [np.full(s, -7.0, np.float32) for s in shapes]
    return [torch.full(s, -7.0, dtype=torch.float32, device="cuda") for s in shapes]


def depth_field(W, H, seed):
    rng = np.random.default_rng(seed)
    d = rng.uniform(0.2, 1.0, (H, W)).astype(np.float32)
    d[rng.uniform(size=d.shape) < 0.1] = 1.0
    return d


@pytest.mark.parametrize("op_max", [False, True])
def test_oracle_hiz_is_the_pyramid(oracle, op_max):
    W, H = 512, 256
    g = globals_for(W, H, frames=1)
    d = depth_field(W, H, 1)
    mips = mips_for(W, H)
    oracle.generate_hiz(g, d, mips, op_max)
    f = np.maximum if op_max else np.minimum
    cur = d
    for i, m in enumerate(mips):
        cur = f(f(cur[0::2, 0::2], cur[1::2, 0::2]), f(cur[0::2, 1::2], cur[1::2, 1::2]))
        assert np.array_equal(m, cur), i
    assert mips[-1].shape == (1, 2)


@pytest.mark.gpu
@pytest.mark.parametrize("W,H", [(512, 256), (97, 55), (1920, 1080), (3840, 2160)])
@pytest.mark.parametrize("op_max", [False, True])
def test_hiz_bit_exact(soc, oracle, W, H, op_max):
    g = globals_for(W, H, frames=1)
    d = depth_field(W, H, W)
    ref = mips_for(W, H)
    oracle.generate_hiz(g, d, ref, op_max)
    out = mips_for(W, H, "torch")
    raster.generate_hiz(g, torch.from_numpy(d).cuda(), out, op_max)
    torch.cuda.synchronize()
    for i, (a, b) in enumerate(zip(out, ref)):
        assert np.array_equal(a.cpu().numpy(), b), (i, a.shape)
