"""Accuracy of the atmosphere's secondary-ray optical-depth table (clouds.hip clouds_od_lut / secondary_od_lut) against
marching the secondary ray (cloud_rendering.inl:399-423), in numpy fp32 on the CPU.

The secondary ray of a primary sample depends on the sample only through r = |iPos| and mu = iPos.pSun / r (for a unit
sun direction), so one kOdR x kOdM table of (log2 odR, log2 odM) over r in [rPlanet, rAtmos], mu in [-1, 1] serves
every sky pixel. This draws random (r, mu), marches them, interpolates the table bilinearly in (r, mu) on the logs, and
reports the error of the attenuation exponent kMie odM + kRlh.z odR that the atmosphere takes exp() of.

    python tools/od_lut_check.py [--samples 300000]
"""
import argparse

import numpy as np

R, RA = np.float32(6371e3), np.float32(6471e3)
SH_R, SH_M = np.float32(8e3), np.float32(1.2e3)
K_MIE, K_RLH_B = 21e-6, 22.4e-6
N_R, N_M = 256, 512          # clouds.hip kOdR, kOdM


def march(r, mu):
    """8-step midpoint optical depths of the sun ray from radius r at cosine mu (the reference's loop), fp32."""
    r = r.astype(np.float32)
    mu = mu.astype(np.float32)
    A = r * r
    pod = r * mu
    delta = pod * pod + RA * RA - A
    with np.errstate(invalid="ignore", over="ignore"):
        jst = np.where(delta < 0, np.float32(-1.0), -pod + np.sqrt(np.maximum(delta, 0))) / np.float32(8)
        t = np.zeros_like(r)
        o_r = np.zeros_like(r)
        o_m = np.zeros_like(r)
        for _ in range(8):
            tt = t + jst * np.float32(0.5)
            h = np.sqrt(A + tt * (2 * pod + tt)) - R
            o_r += np.exp(-h / SH_R) * jst
            o_m += np.exp(-h / SH_M) * jst
            t += jst
    return o_r.astype(np.float64), o_m.astype(np.float64)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--samples", type=int, default=300000)
    a = ap.parse_args()
    ri = np.arange(N_R)
    mi = np.arange(N_M)
    rr, mm = np.meshgrid(R + ri * (RA - R) / (N_R - 1), -1.0 + mi * 2.0 / (N_M - 1), indexing="ij")
    tr, tm = march(rr, mm)
    with np.errstate(divide="ignore", invalid="ignore"):
        ok = np.isfinite(tr) & np.isfinite(tm) & (tr >= 0) & (tm >= 0)
        lr = np.where(ok, np.log2(np.maximum(tr, 1e-30)), np.nan)
        lm = np.where(ok, np.log2(np.maximum(tm, 1e-30)), np.nan)
    rng = np.random.default_rng(7)
    r = R + rng.uniform(0, 1, a.samples) * (RA - R)
    mu = rng.uniform(-1, 1, a.samples)
    er, em = march(r, mu)
    fr = (r - R) / (RA - R) * (N_R - 1)
    fm = (mu + 1) / 2 * (N_M - 1)
    i0 = np.clip(np.floor(fr).astype(int), 0, N_R - 2)
    j0 = np.clip(np.floor(fm).astype(int), 0, N_M - 2)
    wr, wm = fr - i0, fm - j0

    def interp(t):
        top = t[i0, j0] + wm * (t[i0, j0 + 1] - t[i0, j0])
        bot = t[i0 + 1, j0] + wm * (t[i0 + 1, j0 + 1] - t[i0 + 1, j0])
        return np.exp2(top + wr * (bot - top))
    vr, vm = interp(lr), interp(lm)
    table = np.isfinite(vr) & np.isfinite(vm)
    # what the atmosphere uses: the attenuation exp(-(kMie odM + kRlh odR)) of the secondary part (blue channel, the
    # largest kRlh), compared as attenuations (deep-shadow samples have huge exponents whose attenuation is 0 either way)
    with np.errstate(over="ignore", invalid="ignore"):
        at_t = np.exp(-(K_RLH_B * vr + K_MIE * vm))
        at_m = np.exp(-(K_RLH_B * er + K_MIE * em))
    d = np.abs(at_t - at_m)[table]
    print(f"table entries finite: {ok.mean():.4f}; samples served by the table: {table.mean():.4f} "
          f"(the rest march their secondary ray)")
    print(f"secondary attenuation error (absolute, of [0, 1]): median {np.median(d):.2e}, "
          f"p99.9 {np.percentile(d, 99.9):.2e}, max {d.max():.2e}")
    up = (mu > 0.9)[table]
    print(f"  mu > 0.9 (the reference sun near the camera): max {d[up].max():.2e}")


if __name__ == "__main__":
    main()
