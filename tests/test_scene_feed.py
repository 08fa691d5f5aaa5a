"""ECS scene feed: Scene::update (src/ecs/scene.cpp:47-118) restated in the C ABI (soc_scene_update), checked
against float64 glm math written independently: translate * (Rz Ry Rx) * scale for glm::toMat4(glm::quat(euler))
(glm's Euler quaternion is the z-y-x composition), transpose(inverse(model)), rotateX/Y/Z of (0, -1, 0) and
cos(radians(angle)). No GPU."""
import numpy as np
import pytest


def _R(ax, a):
    c, s = np.cos(a), np.sin(a)
    if ax == "x":
        return np.array([[1, 0, 0], [0, c, -s], [0, s, c]])
    if ax == "y":
        return np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])
    return np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]])


def _model64(p, rot_deg, sc):
    r = np.radians(np.float64(rot_deg))
    M = np.eye(4)
    M[:3, :3] = _R("z", r[2]) @ _R("y", r[1]) @ _R("x", r[0]) @ np.diag(sc)
    M[:3, 3] = p
    return M


def test_transforms_and_lights(soc):
    rng = np.random.default_rng(0x5CE)
    ents, want = [], []
    for i in range(40):
        p = rng.uniform(-20, 20, 3)
        rot = rng.uniform(-180, 180, 3)
        sc = rng.uniform(0.2, 3.0, 3)
        kind = i % 3     # 0: plain transform, 1: point light, 2: spot light
        e = soc.entity(p, rot, sc, point_light=kind == 1, spot_light=kind == 2, color=rng.uniform(0, 1, 3),
                       intensity=float(rng.uniform(1, 20)), cut_off=float(rng.uniform(5, 30)),
                       outer_cut_off=float(rng.uniform(30, 45)))
        ents.append(e)
        want.append((kind, np.float32(p), np.float32(rot), np.float32(sc), e))
    g = soc.globals_defaults(64, 64)
    g.point_light_count = 7      # cleared by the update
    models, normals = soc.scene_update(g, ents)
    pl, sl = 0, 0
    for i, (kind, p, rot, sc, e) in enumerate(want):
        M = _model64(np.float64(p), rot, np.float64(sc))
        got = models[i].T.astype(np.float64)          # stored glm-style: [column][row]
        assert np.abs(got - M).max() <= 2e-6 * max(1.0, np.abs(M).max()), i
        N = np.linalg.inv(M).T
        assert np.abs(normals[i].T - N).max() <= 2e-5 * max(1.0, np.abs(N).max()), i
        if kind == 1:
            L = g.point_lights[pl]
            pl += 1
            assert list(L.position) == list(p) and list(L.color) == list(np.float32(e.color)) and L.intensity == e.intensity
        if kind == 2:
            L = g.spot_lights[sl]
            sl += 1
            r = np.radians(np.float64(rot))
            d = _R("z", r[2]) @ (_R("y", r[1]) @ (_R("x", r[0]) @ np.array([0.0, -1.0, 0.0])))
            assert np.abs(np.array(L.direction) - d).max() < 1e-6
            assert L.cut_off == pytest.approx(np.cos(np.radians(e.cut_off)), abs=1e-6)
            assert L.outer_cut_off == pytest.approx(np.cos(np.radians(e.outer_cut_off)), abs=1e-6)
    assert (g.point_light_count, g.spot_light_count) == (pl, sl) == (13, 13)


def test_defaults_and_capacity(soc):
    e = soc.entity(point_light=True)
    assert (e.intensity, e.cut_off, e.outer_cut_off) == (16.0, 20.0, 30.0)     # components.hpp:55-66
    g = soc.globals_defaults(64, 64)
    soc.scene_update(g, [soc.entity(point_light=True) for _ in range(128)])
    assert g.point_light_count == 128
    with pytest.raises(soc.SocError, match="exceed"):
        soc.scene_update(g, [soc.entity(point_light=True) for _ in range(129)])
    soc.scene_update(g, [])
    assert g.point_light_count == 0 and g.spot_light_count == 0
