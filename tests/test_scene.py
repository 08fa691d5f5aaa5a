"""Input generator checks (CPU): the Sponza-proxy and terrain G-buffers follow the reference's G-buffer
contract (g_buffer_generation.inl:180-230, draw_terrain.inl:196-222) and are deterministic."""
import hashlib

import numpy as np

from helpers import sponza_inputs, terrain_inputs


def _digest(gb):
    h = hashlib.sha256()
    for k in ("albedo", "normal", "emissive", "velocity", "depth"):
        h.update(np.ascontiguousarray(gb[k]).tobytes())
    return h.hexdigest()


def test_terrain_gbuffer_contract():
    W, H = 192, 108
    g, gb = terrain_inputs(W, H)
    depth = gb["depth"]
    sky = depth == 1.0
    assert 0.35 < sky.mean() < 0.65                      # C4: about half the frame is sky
    assert ((depth > 0.0) & (depth <= 1.0)).all()          # z_ndc clipped to [0, 1] (Q1)
    n = gb["normal"][~sky].astype(np.float32)
    assert np.allclose(np.linalg.norm(n[:, :3], axis=1), 1.0, atol=2e-3)
    assert (n[:, 1] > 0.0).all()                           # a height field's normals point up
    assert (gb["velocity"][~sky] == 0).all()               # out_velocity = vec4(0) (draw_terrain.inl:221)
    em = gb["emissive"].astype(np.float32)
    assert (em[..., :3] == 0).all() and (em[..., 3] == 1).all()
    alb = gb["albedo"][~sky].astype(np.float32)
    assert (alb[:, 3] == 1).all() and (alb[:, :3] > 0).all()
    # the clear values on sky pixels (g_buffer_generation.inl clears)
    assert (gb["albedo"][sky].astype(np.float32) == np.float32([0.2, 0.4, 1.0, 1.0]).astype(np.float16)).all()
    # the terrain lies below the reference sun's ortho box (y in [24, 56]): nothing is rasterised into
    # the shadow map, which keeps its clear depth, as in the reference frame
    assert (gb["shadow"] == 1.0).all()


def test_terrain_depth_monotone_with_distance():
    """Nearer terrain (bottom rows, camera looking down) has smaller depth than the horizon rows."""
    _, gb = terrain_inputs(160, 90)
    d = gb["depth"]
    col = d[:, 80]
    land = col[col < 1.0]
    assert land.size > 20
    assert land[-1] < land[0]


def test_scene_generation_is_deterministic():
    a = terrain_inputs(96, 54)[1]
    b = terrain_inputs(96, 54)[1]
    assert _digest(a) == _digest(b)
    c = sponza_inputs(96, 54)[1]
    d = sponza_inputs(96, 54)[1]
    assert _digest(c) == _digest(d)
