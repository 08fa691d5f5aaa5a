"""Accuracy of the atmosphere's sky-view table (clouds.hip clouds_sky_table / atmosphere_table) against evaluating the
atmosphere for every view direction (cloud_rendering.inl:353-439, float64 restatement with marched secondary rays),
over the view frusta of the bench's C3 and C4 cameras at 3840x2160.

The in-scattering integrals (totalRlh, totalMie) of a view ray depend, for the frame's camera, sun and elapsed time, on
the ray's elevation sine e and its azimuth away from the sun (mirror symmetry), in three branches at the grazing
elevations +-eh (ground hit ahead / miss / ground hit behind, as the reference's rsi and min decide). Each branch is
tabulated on NT x NU entries (rows dense towards the grazing direction, a margin DL inside the branch), interpolated
bilinearly, and the exact phase functions are applied; the error is reported in RGBA8 levels of the atmosphere colour.

    python tools/sky_table_check.py [--nt 128] [--nu 64] [--sub 4] [--configs c3,c4]
"""
import argparse
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from soc_real_time_renderer_amd import multi_gpu  # noqa: E402
RP, RA = 6371e3, 6471e3
kRlh = np.array([5.5e-6, 13.0e-6, 22.4e-6]); kMie = 21e-6; iSun = 22.0; g0 = 0.758
def rsi(p, d, R):
    PoD = (p * d).sum(-1); delta = PoD * PoD + R * R - (p * p).sum(-1)
    s = np.sqrt(np.maximum(delta, 0))
    return np.where(delta < 0, -1.0, -PoD - s), np.where(delta < 0, -1.0, -PoD + s)
def integrals(r, r0, pSun, iTime):
    r = r / np.linalg.norm(r, axis=-1, keepdims=True)
    r0b = np.broadcast_to(r0, r.shape)
    px, py = rsi(r0b, r, RA)
    py = np.minimum(py, rsi(r0b, r, RP)[0])
    iStep = (py - px) / 16.0
    tR = np.zeros(r.shape); tM = np.zeros(r.shape); iOdR = np.zeros(len(r)); iOdM = np.zeros(len(r))
    t = np.full(len(r), iTime)
    for i in range(16):
        iPos = r0b + r * (t + iStep * 0.5)[:, None]
        h = np.linalg.norm(iPos, axis=-1) - RP
        odR = np.exp(-h / 8e3) * iStep; odM = np.exp(-h / 1.2e3) * iStep
        iOdR += odR; iOdM += odM
        jx, jy = rsi(iPos, np.broadcast_to(pSun, iPos.shape), RA)
        jStep = jy / 8.0; jT = np.zeros(len(r)); jR = np.zeros(len(r)); jM = np.zeros(len(r))
        for j in range(8):
            jPos = iPos + pSun * (jT + jStep * 0.5)[:, None]
            jh = np.linalg.norm(jPos, axis=-1) - RP
            jR += np.exp(-jh / 8e3) * jStep; jM += np.exp(-jh / 1.2e3) * jStep; jT += jStep
        attn = np.exp(-(kMie * (iOdM + jM)[:, None] + kRlh * (iOdR + jR)[:, None]))
        tR += odR[:, None] * attn; tM += odM[:, None] * attn
        t = t + iStep
    return tR, tM
def color(r, tR, tM, pSun):
    r = r / np.linalg.norm(r, axis=-1, keepdims=True)
    mu = (r * pSun).sum(-1); mumu = mu * mu; gg = g0 * g0
    pR = 3 / (16 * math.pi) * (1 + mumu)
    pM = 3 / (8 * math.pi) * ((1 - gg) * (mumu + 1)) / ((1 + gg - 2 * mu * g0) ** 1.5 * (2 + gg))
    return (kRlh * pR[:, None] * tR + tM * (pM * kMie)[:, None]) * iSun

DL = 3e-5   # clouds.hip SkyTab.dl


def study(cfg, NT, NU, sub=4):
    W, H = 3840, 2160
    cam = multi_gpu.terrain_camera_for_rank(0) if cfg == 'c4' else multi_gpu.camera_for_rank(0)
    g = bench.make_globals(W, H, cam)
    ip = np.ctypeslib.as_array(g.camera_inverse_projection_matrix).reshape(4, 4).T.astype(np.float64)
    iv = np.ctypeslib.as_array(g.camera_inverse_view_matrix).reshape(4, 4).T.astype(np.float64)
    xs, ys = np.meshgrid(np.arange(0, W, sub), np.arange(0, H, sub))
    ndx = xs.ravel() / (W - 1) * 2 - 1; ndy = ys.ravel() / (H - 1) * 2 - 1
    rv = ip @ np.stack([ndx, ndy, -np.ones_like(ndx), np.zeros_like(ndx)])
    rw = iv @ np.stack([rv[0], rv[1], -np.ones_like(ndx), np.zeros_like(ndx)])
    d = rw[:3].T; d /= np.linalg.norm(d, axis=1, keepdims=True)
    d = d[d[:, 1] > -0.3]    # sky-ish and near-horizon directions
    cp = np.array(g.camera_position[:3], np.float64)
    r0 = np.array([cp[0], 6372e3 + cp[1], cp[2]])
    pSun = -np.array(g.sun_info.direction[:3], np.float64)
    iTime = float(g.elapsed_time)
    up = r0 / np.linalg.norm(r0); eh = math.sqrt(1 - (RP / np.linalg.norm(r0)) ** 2)
    sh = pSun - up * (pSun @ up); sh /= np.linalg.norm(sh); bt = np.cross(up, sh)
    def params(dd):
        e = dd @ up
        dh = dd - np.outer(e, up); nh = np.linalg.norm(dh, axis=1)
        c = np.clip((dh @ sh) / np.maximum(nh, 1e-30), -1, 1)
        u = np.sqrt((1 - c) / 2)
        br = np.where(e <= -eh, 0, np.where(e < eh, 1, 2))
        t = np.where(br == 0, np.sqrt(np.clip((-(eh + DL) - e) / (1 - eh - DL), 0, 1)),
                     np.where(br == 1, np.clip((e + (eh - DL)) / (2 * (eh - DL)), 0, 1),
                              np.sqrt(np.clip((e - (eh + DL)) / (1 - eh - DL), 0, 1))))
        return br, t, u
    def dir_of(br, t, u):
        e = np.where(br == 0, -(eh + DL) - t * t * (1 - eh - DL),
                     np.where(br == 1, -(eh - DL) + t * 2 * (eh - DL), (eh + DL) + t * t * (1 - eh - DL)))
        c = 1 - 2 * u * u; s = np.sqrt(np.maximum(1 - c * c, 0))
        ce = np.sqrt(np.maximum(1 - e * e, 0))
        return np.outer(e, up) + (ce * c)[:, None] * sh + (ce * s)[:, None] * bt
    tabs = []
    for br in range(3):
        T, U = np.meshgrid(np.linspace(0, 1, NT), np.linspace(0, 1, NU), indexing='ij')
        dd = dir_of(np.full(T.size, br), T.ravel(), U.ravel())
        tR, tM = integrals(dd, r0, pSun, iTime)
        tabs.append((tR.reshape(NT, NU, 3), tM.reshape(NT, NU, 3)))
    br, t, u = params(d)
    ref_R, ref_M = integrals(d, r0, pSun, iTime)
    ref = color(d, ref_R, ref_M, pSun)
    out = np.zeros_like(ref)
    for b in range(3):
        m = br == b
        ft = t[m] * (NT - 1); fu = u[m] * (NU - 1)
        i0 = np.clip(ft.astype(int), 0, NT - 2); j0 = np.clip(fu.astype(int), 0, NU - 2)
        wt = (ft - i0)[:, None]; wu = (fu - j0)[:, None]
        def bil(A):
            a = A[i0, j0]; b_ = A[i0, j0 + 1]; c_ = A[i0 + 1, j0]; d_ = A[i0 + 1, j0 + 1]
            top = a + wu * (b_ - a); bot = c_ + wu * (d_ - c_); return top + wt * (bot - top)
        out[m] = color(d[m], bil(tabs[b][0]), bil(tabs[b][1]), pSun)
    err = np.abs(out - ref) * 255
    print(f"{cfg} {NT}x{NU}: {len(d)} directions (branches {np.bincount(br, minlength=3).tolist()}), colour max "
          f"{ref.max():.3f}; error in RGBA8 levels: median {np.median(err):.5f} p99.9 {np.percentile(err, 99.9):.4f} "
          f"max {err.max():.4f}")
    return float(err.max())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nt", type=int, default=128)
    ap.add_argument("--nu", type=int, default=64)
    ap.add_argument("--sub", type=int, default=4, help="pixel stride of the sampled view directions")
    ap.add_argument("--configs", default="c3,c4")
    a = ap.parse_args()
    worst = max(study(c, a.nt, a.nu, a.sub) for c in a.configs.split(","))
    print(f"max error {worst:.4f} levels")


if __name__ == "__main__":
    main()
