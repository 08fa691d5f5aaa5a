/*
 * scene_synth.c — deterministic synthetic G-buffer + sun shadow map producer (host, OpenMP).
 *
 * Stands in for the reference's raster producers (depth_prepass.inl, g_buffer_generation.inl:152-230,
 * sun_shadow_draw.inl) which are out of scope for this tier. The
 * reference's Sponza.bin is missing from the mount, so the benchmark frame is a documented
 * "Sponza-proxy": an analytic atrium of axis-aligned boxes spanning Sponza's bounds at the app's 0.01
 * scale (x -19.2..18.0, y -1.26..14.3, z -11.8..11.05, from Sponza.gltf accessor min/max), with an open
 * nave roof (sky), two colonnades, galleries and a few emissive lamps, ray-cast per pixel.
 *
 * Outputs follow the G-buffer contract of g_buffer_generation.inl:180-230: albedo = base + emissive,
 * emissive, world normal (alpha 1), velocity = current uv - previous uv (clip positions through the
 * current / previous jittered view-projections), depth = NDC z of the RH_NO projection (quirk Q1),
 * clears: albedo (0.2,0.4,1,1), others (0,0,0,1), depth 1.0. The shadow map is the same scene ray-cast
 * through the sun's ortho view-projection (depth = NDC z, cleared to 1.0, z outside [0,1] clipped).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/soc_rt.h"

typedef struct { float x, y, z; } v3;
static v3 V(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static v3 add(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
static v3 sub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
static v3 mul(v3 a, float s) { return V(a.x * s, a.y * s, a.z * s); }
static float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static v3 nrm(v3 a) { float l = sqrtf(dot(a, a)); return V(a.x / l, a.y / l, a.z / l); }

typedef struct { v3 lo, hi; int mat; } box;

#define MAX_BOXES 256
typedef struct {
    box b[MAX_BOXES];
    int n;
} scene;

enum { SCENE_SPONZA_PROXY = 0, SCENE_TERRAIN = 1 };

enum { M_FLOOR = 0, M_WALL, M_PILLAR, M_GALLERY, M_ROOF, M_LAMP, M_BANNER, M_STATUE, M_COUNT };

static void addbox(scene* s, float x0, float y0, float z0, float x1, float y1, float z1, int mat) {
    if (s->n >= MAX_BOXES) return;
    box* b = &s->b[s->n++];
    b->lo = V(x0 < x1 ? x0 : x1, y0 < y1 ? y0 : y1, z0 < z1 ? z0 : z1);
    b->hi = V(x0 < x1 ? x1 : x0, y0 < y1 ? y1 : y0, z0 < z1 ? z1 : z0);
    b->mat = mat;
}

static void build_sponza_proxy(scene* s) {
    s->n = 0;
    const float X0 = -19.2f, X1 = 18.0f, Z0 = -11.8f, Z1 = 11.05f, Y0 = -1.26f, YT = 14.3f;
    addbox(s, X0, Y0, Z0, X1, 0.0f, Z1, M_FLOOR);                 /* floor slab */
    addbox(s, X0, 0.0f, Z1 - 0.6f, X1, YT, Z1, M_WALL);           /* long walls */
    addbox(s, X0, 0.0f, Z0, X1, YT, Z0 + 0.6f, M_WALL);
    addbox(s, X0, 0.0f, Z0, X0 + 0.6f, YT, Z1, M_WALL);           /* end walls */
    addbox(s, X1 - 0.6f, 0.0f, Z0, X1, YT, Z1, M_WALL);
    /* colonnades (z = +-4) ground + first floor */
    for (int i = 0; i < 11; ++i) {
        float x = -15.0f + 3.0f * (float)i;
        for (int side = -1; side <= 1; side += 2) {
            float z = 4.0f * (float)side;
            addbox(s, x - 0.45f, 0.0f, z - 0.45f, x + 0.45f, 6.0f, z + 0.45f, M_PILLAR);
            addbox(s, x - 0.35f, 6.5f, z - 0.35f, x + 0.35f, 11.8f, z + 0.35f, M_PILLAR);
        }
    }
    /* galleries, arcade beams and side-aisle roofs */
    addbox(s, X0, 6.0f, 3.6f, X1, 6.5f, Z1, M_GALLERY);
    addbox(s, X0, 6.0f, Z0, X1, 6.5f, -3.6f, M_GALLERY);
    addbox(s, X0, 5.4f, 3.55f, X1, 6.0f, 4.45f, M_GALLERY);
    addbox(s, X0, 5.4f, -4.45f, X1, 6.0f, -3.55f, M_GALLERY);
    addbox(s, X0, 11.8f, 3.6f, X1, 12.4f, Z1, M_ROOF);
    addbox(s, X0, 11.8f, Z0, X1, 12.4f, -3.6f, M_ROOF);
    addbox(s, X0, 12.4f, 3.4f, X1, 13.0f, 4.6f, M_ROOF);          /* cornices over the nave edge */
    addbox(s, X0, 12.4f, -4.6f, X1, 13.0f, -3.4f, M_ROOF);
    /* hanging banners between upper pillars */
    for (int i = 0; i < 5; ++i) {
        float x = -13.5f + 6.0f * (float)i;
        addbox(s, x - 1.1f, 7.0f, 3.85f, x + 1.1f, 11.0f, 3.95f, M_BANNER);
        addbox(s, x - 1.1f, 7.0f, -3.95f, x + 1.1f, 11.0f, -3.85f, M_BANNER);
    }
    /* emissive lamps on the ground-floor pillars */
    for (int i = 0; i < 6; ++i) {
        float x = -15.0f + 6.0f * (float)i;
        addbox(s, x - 0.25f, 3.0f, 3.3f, x + 0.25f, 3.6f, 3.55f, M_LAMP);
        addbox(s, x - 0.25f, 3.0f, -3.55f, x + 0.25f, 3.6f, -3.3f, M_LAMP);
    }
    /* statues / props in the nave */
    addbox(s, -2.0f, 0.0f, -1.0f, 0.0f, 1.6f, 1.0f, M_STATUE);
    addbox(s, 6.0f, 0.0f, -0.6f, 7.2f, 2.4f, 0.6f, M_STATUE);
    addbox(s, -9.0f, 0.0f, -1.5f, -7.5f, 0.8f, 1.5f, M_STATUE);
    /* floating canopy frames above the atrium (inside the sun frustum, y 24..40) */
    addbox(s, -10.0f, 27.0f, -6.0f, -2.0f, 27.4f, 6.0f, M_ROOF);
    addbox(s, 2.0f, 30.0f, -8.0f, 9.0f, 30.4f, 2.0f, M_ROOF);
}

static const float k_base[M_COUNT][3] = {
    {0.55f, 0.50f, 0.42f}, {0.62f, 0.55f, 0.45f}, {0.70f, 0.66f, 0.58f}, {0.50f, 0.46f, 0.40f},
    {0.45f, 0.40f, 0.35f}, {0.90f, 0.85f, 0.70f}, {0.60f, 0.12f, 0.10f}, {0.35f, 0.38f, 0.42f}};

static inline float hash3(int x, int y, int z) {
    uint32_t h = (uint32_t)x * 73856093u ^ (uint32_t)y * 19349663u ^ (uint32_t)z * 83492791u;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    return (float)(h & 0xffffu) / 65535.0f;
}

/* ray vs boxes; returns material or -1 */
static int trace(const scene* s, v3 o, v3 d, float tmin, float* t_out, v3* n_out) {
    float best = 1e30f;
    int hit = -1;
    v3 bn = V(0, 0, 0);
    const float ix = 1.0f / d.x, iy = 1.0f / d.y, iz = 1.0f / d.z;
    for (int i = 0; i < s->n; ++i) {
        const box* b = &s->b[i];
        float tx0 = (b->lo.x - o.x) * ix, tx1 = (b->hi.x - o.x) * ix;
        float ty0 = (b->lo.y - o.y) * iy, ty1 = (b->hi.y - o.y) * iy;
        float tz0 = (b->lo.z - o.z) * iz, tz1 = (b->hi.z - o.z) * iz;
        float tn_x = fminf(tx0, tx1), tf_x = fmaxf(tx0, tx1);
        float tn_y = fminf(ty0, ty1), tf_y = fmaxf(ty0, ty1);
        float tn_z = fminf(tz0, tz1), tf_z = fmaxf(tz0, tz1);
        float tn = fmaxf(fmaxf(tn_x, tn_y), tn_z), tf = fminf(fminf(tf_x, tf_y), tf_z);
        if (tf < tn || tf < tmin) continue;
        float t = tn >= tmin ? tn : tf;
        if (t < best) {
            best = t;
            hit = b->mat;
            if (tn == tn_x) bn = V(d.x > 0 ? -1.0f : 1.0f, 0, 0);
            else if (tn == tn_y) bn = V(0, d.y > 0 ? -1.0f : 1.0f, 0);
            else bn = V(0, 0, d.z > 0 ? -1.0f : 1.0f);
        }
    }
    *t_out = best;
    *n_out = bn;
    return hit;
}

static inline void mat_vec(const float* m, float x, float y, float z, float w, float* o) {
    for (int r = 0; r < 4; ++r) o[r] = m[r] * x + m[4 + r] * y + m[8 + r] * z + m[12 + r] * w;
}

/* f32 -> f16 RNE (same routine as the oracle's) */
static uint16_t f2h(float f) {
    const uint32_t f32infty = 255u << 23, f16max = (127u + 16u) << 23;
    const uint32_t denorm_magic = ((127u - 15u) + (23u - 10u) + 1u) << 23;
    uint32_t u, sign, o;
    memcpy(&u, &f, 4);
    sign = u & 0x80000000u;
    u ^= sign;
    if (u >= f16max) o = (u > f32infty) ? 0x7e00u : 0x7c00u;
    else if (u < (113u << 23)) {
        float fu, dm;
        memcpy(&fu, &u, 4);
        memcpy(&dm, &denorm_magic, 4);
        fu += dm;
        uint32_t r;
        memcpy(&r, &fu, 4);
        o = r - denorm_magic;
    } else {
        uint32_t mant_odd = (u >> 13) & 1u;
        u += ((uint32_t)(15 - 127) << 23) + 0xfffu;
        u += mant_odd;
        o = u >> 13;
    }
    return (uint16_t)(o | (sign >> 16));
}

static void put4(uint16_t* p, float a, float b, float c, float d) { p[0] = f2h(a); p[1] = f2h(b); p[2] = f2h(c); p[3] = f2h(d); }

static void material(int mat, v3 p, v3 n, float* alb, float* emi) {
    /* procedural tiling: 0.5-unit blocks with per-block tint + mortar lines */
    float u = fabsf(n.x) > 0.5f ? p.z : p.x, v = fabsf(n.y) > 0.5f ? p.z : p.y;
    int bu = (int)floorf(u * 2.0f), bv = (int)floorf(v * 4.0f);
    float tint = 0.8f + 0.4f * hash3(bu, bv, mat);
    float fu = u * 2.0f - floorf(u * 2.0f), fv = v * 4.0f - floorf(v * 4.0f);
    float mortar = (fu < 0.04f || fv < 0.06f) ? 0.55f : 1.0f;
    for (int c = 0; c < 3; ++c) { alb[c] = k_base[mat][c] * tint * mortar; emi[c] = 0.0f; }
    if (mat == M_LAMP) { emi[0] = 4.0f; emi[1] = 2.6f; emi[2] = 1.2f; }
    if (mat == M_BANNER && fv > 0.45f && fv < 0.55f) { emi[0] = 0.9f; emi[1] = 0.6f; emi[2] = 0.1f; }
}

/* ---------------------------------------------------------------------------------------------------
 * Scene 1: terrain proxy for config C4. The reference draws a 100 x 100 vertex grid of
 * quad patches over [0, terrain_scale]^2 (renderer.cpp:194-220), tessellated at the maximum level 3
 * (draw_terrain.inl:150-163) and displaced by (height - terrain_midpoint) * terrain_height_scale
 * (:185-191); its Terrain/heightmap.exr is missing from the mount, so the height is a deterministic
 * fBm (seed 0x7E44). The tessellated grid (298 x 298 vertices, 176,418 triangles) is rasterised on the
 * host: pixel centres, edge functions with a top-left fill rule, z_ndc interpolated affinely in screen
 * space, LESS_OR_EQUAL in draw order (later triangles win ties), fragments with z_ndc outside [0, 1]
 * clipped. The G-buffer follows draw_terrain.inl:196-222: albedo (procedural grass / rock / snow by
 * height and slope, alpha 1), normal = the surface normal (the reference writes its normal map's
 * texel; the map is generated from the missing heightmap), velocity 0 (as the reference writes),
 * emissive left at its clear (0, 0, 0, 1).
 * ------------------------------------------------------------------------------------------------- */
#define T_SEGS 297                 /* 99 patches x tessellation level 3 */
#define T_NV (T_SEGS + 1)

static inline float vnoise_hash(int x, int y, uint32_t seed) {
    uint32_t h = (uint32_t)x * 0x8da6b343u ^ (uint32_t)y * 0xd8163841u ^ seed * 0xcb1ab31fu;
    h ^= h >> 15; h *= 0x2c1b3c6du; h ^= h >> 12; h *= 0x297a2d39u; h ^= h >> 15;
    return (float)(h & 0xffffffu) / 16777215.0f;
}

static float vnoise(float x, float y, uint32_t seed) {
    const float fx = floorf(x), fy = floorf(y);
    const int ix = (int)fx, iy = (int)fy;
    float tx = x - fx, ty = y - fy;
    tx = tx * tx * (3.0f - 2.0f * tx);
    ty = ty * ty * (3.0f - 2.0f * ty);
    const float a = vnoise_hash(ix, iy, seed), b = vnoise_hash(ix + 1, iy, seed);
    const float c = vnoise_hash(ix, iy + 1, seed), d = vnoise_hash(ix + 1, iy + 1, seed);
    return (a + (b - a) * tx) + ((c + (d - c) * tx) - (a + (b - a) * tx)) * ty;
}

/* heightmap value in [0.15, 0.65) at terrain uv in [0, 1]^2: squared fBm (valleys and ridges) */
static float terrain_height(float u, float v) {
    float h = 0.0f, amp = 0.5f, freq = 4.0f;
    for (int o = 0; o < 6; ++o) {
        h += amp * vnoise(u * freq, v * freq, 0x7E44u + (uint32_t)o);
        amp *= 0.5f;
        freq *= 2.03f;
    }
    h /= 0.984375f;
    return 0.15f + 0.5f * h * h;
}

typedef struct {
    v3 p[T_NV * T_NV];           /* world positions */
    int built;
    float scale_x, scale_z, hscale, mid, off[3];
} terrain_mesh;
static terrain_mesh g_terrain;

static const terrain_mesh* get_terrain(const soc_globals* g) {
    terrain_mesh* t = &g_terrain;
    if (t->built && t->scale_x == g->terrain_scale[0] && t->scale_z == g->terrain_scale[1] && t->hscale == g->terrain_height_scale &&
        t->mid == g->terrain_midpoint && t->off[0] == g->terrain_offset[0] && t->off[1] == g->terrain_offset[1] &&
        t->off[2] == g->terrain_offset[2])
        return t;
    t->scale_x = g->terrain_scale[0];
    t->scale_z = g->terrain_scale[1];
    t->hscale = g->terrain_height_scale;
    t->mid = g->terrain_midpoint;
    memcpy(t->off, g->terrain_offset, sizeof t->off);
#pragma omp parallel for
    for (int j = 0; j < T_NV; ++j)
        for (int i = 0; i < T_NV; ++i) {
            const float u = (float)i / (float)T_SEGS, v = (float)j / (float)T_SEGS;
            const float h = (terrain_height(u, v) - t->mid) * t->hscale;
            t->p[j * T_NV + i] = V(u * t->scale_x - t->off[0], t->off[1] + h, v * t->scale_z - t->off[2]);
        }
    t->built = 1;
    return t;
}

static v3 terrain_normal(const terrain_mesh* t, float u, float v) {
    const float e = 1.0f / 1024.0f;
    const float hx = (terrain_height(u + e, v) - terrain_height(u - e, v)) * t->hscale / (2.0f * e * t->scale_x);
    const float hz = (terrain_height(u, v + e) - terrain_height(u, v - e)) * t->hscale / (2.0f * e * t->scale_z);
    return nrm(V(-hx, 1.0f, -hz));
}

static void terrain_material(float height, v3 n, float u, float v, float* alb) {
    const float slope = 1.0f - n.y;
    const float grain = 0.85f + 0.3f * vnoise(u * 900.0f, v * 900.0f, 0x51u);
    float c[3] = {0.24f, 0.36f, 0.12f};                                   /* grass */
    if (slope > 0.25f) { c[0] = 0.42f; c[1] = 0.38f; c[2] = 0.33f; }     /* rock */
    if (height > 24.0f && slope < 0.35f) { c[0] = 0.88f; c[1] = 0.90f; c[2] = 0.93f; }   /* snow */
    for (int k = 0; k < 3; ++k) alb[k] = c[k] * grain;
}

/* Rasterise the terrain grid through `pv` (column-major clip transform) into W x H: per pixel the
 * winning triangle id (-1: none) and its perspective-correct barycentrics (b1, b2). */
static void terrain_raster(const terrain_mesh* t, const float* pv, int W, int H, float* depth, int* tri, float* b1o,
                           float* b2o) {
    const int ntri = 2 * T_SEGS * T_SEGS;
    float* sx = (float*)malloc(sizeof(float) * 4 * T_NV * T_NV);   /* screen x, y, z_ndc, 1/w per vertex */
#pragma omp parallel for
    for (int k = 0; k < T_NV * T_NV; ++k) {
        float c[4];
        mat_vec(pv, t->p[k].x, t->p[k].y, t->p[k].z, 1.0f, c);
        float* o = sx + 4 * k;
        if (c[3] <= 1e-6f) { o[3] = 0.0f; continue; }
        const float iw = 1.0f / c[3];
        o[0] = (c[0] * iw * 0.5f + 0.5f) * (float)W;   /* uv = ndc * 0.5 + 0.5, y = 0 at the top row */
        o[1] = (c[1] * iw * 0.5f + 0.5f) * (float)H;
        o[2] = c[2] * iw;
        o[3] = iw;
    }
    const int TS = 32, tx_n = (W + TS - 1) / TS, ty_n = (H + TS - 1) / TS;
#pragma omp parallel for schedule(dynamic, 1)
    for (int tile = 0; tile < tx_n * ty_n; ++tile) {
        const int x0 = (tile % tx_n) * TS, y0 = (tile / tx_n) * TS;
        const int x1 = x0 + TS < W ? x0 + TS : W, y1 = y0 + TS < H ? y0 + TS : H;
        for (int y = y0; y < y1; ++y)
            for (int x = x0; x < x1; ++x) {
                depth[(size_t)y * W + x] = 1.0f;
                tri[(size_t)y * W + x] = -1;
            }
        for (int id = 0; id < ntri; ++id) {
            const int q = id >> 1, qi = q % T_SEGS, qj = q / T_SEGS;
            const int v00 = qj * T_NV + qi, v10 = v00 + 1, v01 = v00 + T_NV, v11 = v01 + 1;
            const int a = v00, b = (id & 1) ? v11 : v10, c = (id & 1) ? v01 : v11;
            const float* A = sx + 4 * a; const float* B = sx + 4 * b; const float* Cv = sx + 4 * c;
            if (A[3] == 0.0f || B[3] == 0.0f || Cv[3] == 0.0f) continue;
            float minx = fminf(A[0], fminf(B[0], Cv[0])), maxx = fmaxf(A[0], fmaxf(B[0], Cv[0]));
            float miny = fminf(A[1], fminf(B[1], Cv[1])), maxy = fmaxf(A[1], fmaxf(B[1], Cv[1]));
            if (maxx < (float)x0 || minx > (float)x1 || maxy < (float)y0 || miny > (float)y1) continue;
            const float area = (B[0] - A[0]) * (Cv[1] - A[1]) - (B[1] - A[1]) * (Cv[0] - A[0]);
            if (area == 0.0f) continue;
            const float sgn = area > 0.0f ? 1.0f : -1.0f, inv_area = 1.0f / area;
            int px0 = (int)floorf(minx - 0.5f), px1 = (int)ceilf(maxx - 0.5f);
            int py0 = (int)floorf(miny - 0.5f), py1 = (int)ceilf(maxy - 0.5f);
            if (px0 < x0) px0 = x0;
            if (py0 < y0) py0 = y0;
            if (px1 > x1 - 1) px1 = x1 - 1;
            if (py1 > y1 - 1) py1 = y1 - 1;
            for (int y = py0; y <= py1; ++y)
                for (int x = px0; x <= px1; ++x) {
                    const float fx = (float)x + 0.5f, fy = (float)y + 0.5f;
                    /* edge functions, oriented so that inside is >= 0 for either winding */
                    float e0 = ((Cv[0] - B[0]) * (fy - B[1]) - (Cv[1] - B[1]) * (fx - B[0])) * sgn;
                    float e1 = ((A[0] - Cv[0]) * (fy - Cv[1]) - (A[1] - Cv[1]) * (fx - Cv[0])) * sgn;
                    float e2 = ((B[0] - A[0]) * (fy - A[1]) - (B[1] - A[1]) * (fx - A[0])) * sgn;
                    if (e0 < 0.0f || e1 < 0.0f || e2 < 0.0f) continue;
                    /* top-left rule for pixels exactly on an edge: keep only the edge whose outward
                       normal points up or left (shared edges are then covered once) */
                    if (e0 == 0.0f || e1 == 0.0f || e2 == 0.0f) {
                        const float* P0[3] = {B, Cv, A};
                        const float* P1[3] = {Cv, A, B};
                        const float ev[3] = {e0, e1, e2};
                        int ok = 1;
                        for (int k = 0; k < 3; ++k) {
                            if (ev[k] != 0.0f) continue;
                            const float dx = (P1[k][0] - P0[k][0]) * sgn, dy = (P1[k][1] - P0[k][1]) * sgn;
                            if (!((dy < 0.0f) || (dy == 0.0f && dx > 0.0f))) ok = 0;
                        }
                        if (!ok) continue;
                    }
                    const float w0 = e0 * sgn * inv_area, w1 = e1 * sgn * inv_area, w2 = e2 * sgn * inv_area;
                    const float z = w0 * A[2] + w1 * B[2] + w2 * Cv[2];
                    if (z < 0.0f || z > 1.0f) continue;                      /* depth clipping */
                    const size_t i = (size_t)y * W + x;
                    if (!(z <= depth[i])) continue;                         /* LESS_OR_EQUAL */
                    depth[i] = z;
                    tri[i] = id;
                    if (b1o) {
                        const float q0 = w0 * A[3], q1 = w1 * B[3], q2 = w2 * Cv[3], qs = q0 + q1 + q2;
                        b1o[i] = q1 / qs;
                        b2o[i] = q2 / qs;
                    }
                }
        }
    }
    free(sx);
}

static void terrain_gbuffer(const soc_globals* g, int W, int H, uint16_t* albedo, uint16_t* emissive, uint16_t* normal,
                            float* depth, uint16_t* velocity) {
    const terrain_mesh* t = get_terrain(g);
    int* tri = (int*)malloc(sizeof(int) * (size_t)W * H);
    float* b1 = (float*)malloc(sizeof(float) * (size_t)W * H);
    float* b2 = (float*)malloc(sizeof(float) * (size_t)W * H);
    terrain_raster(t, g->camera_projection_view_matrix, W, H, depth, tri, b1, b2);
#pragma omp parallel for schedule(static)
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const size_t i = (size_t)y * W + x;
            put4(emissive + 4 * i, 0, 0, 0, 1);
            put4(velocity + 4 * i, 0, 0, 0, 1);
            if (tri[i] < 0) {
                put4(albedo + 4 * i, 0.2f, 0.4f, 1.0f, 1.0f);
                put4(normal + 4 * i, 0, 0, 0, 1);
                continue;
            }
            put4(velocity + 4 * i, 0, 0, 0, 0);   /* out_velocity = vec4(0) (draw_terrain.inl:221) */
            const int id = tri[i], q = id >> 1, qi = q % T_SEGS, qj = q / T_SEGS;
            /* the triangle's vertex uvs: a = (qi, qj), b = (qi+1, qj+1) or (qi+1, qj), c = (qi, qj+1) or (qi+1, qj+1) */
            const float ua = (float)qi, va = (float)qj;
            const float ub = ua + 1.0f, vb = (id & 1) ? va + 1.0f : va;
            const float uc = (id & 1) ? ua : ua + 1.0f, vc = va + 1.0f;
            const float w1 = b1[i], w2 = b2[i], w0 = 1.0f - w1 - w2;
            const float u = (w0 * ua + w1 * ub + w2 * uc) / (float)T_SEGS, v = (w0 * va + w1 * vb + w2 * vc) / (float)T_SEGS;
            const v3 n = terrain_normal(t, u, v);
            const float hgt = (terrain_height(u, v) - t->mid) * t->hscale;
            float alb[3];
            terrain_material(hgt, n, u, v, alb);
            put4(albedo + 4 * i, alb[0], alb[1], alb[2], 1.0f);
            put4(normal + 4 * i, n.x, n.y, n.z, 1.0f);
        }
    free(tri);
    free(b1);
    free(b2);
}

static scene g_scene;
static int g_scene_built = 0;

static const scene* get_scene(int id) {
    (void)id;
    if (!g_scene_built) { build_sponza_proxy(&g_scene); g_scene_built = 1; }
    return &g_scene;
}

/* G-buffer at W x H (tight rows): albedo/emissive/normal/velocity RGBA16F (uint16 bits), depth f32. */
int soc_scene_gbuffer(int scene_id, const soc_globals* g, int W, int H, uint16_t* albedo, uint16_t* emissive,
                      uint16_t* normal, float* depth, uint16_t* velocity) {
    if (!g || W <= 0 || H <= 0 || !albedo || !emissive || !normal || !depth || !velocity) return -1;
    if (scene_id == SCENE_TERRAIN) {
        terrain_gbuffer(g, W, H, albedo, emissive, normal, depth, velocity);
        return 0;
    }
    const scene* s = get_scene(scene_id);
    /* NB: the reference's camera_inverse_projection_view_matrix is inv(P) * inv(V) (application.cpp:136), not
       inv(P*V); unproject with inv(V) * (inv(P) * ndc) as the shaders do. */
    const float* ip = g->camera_inverse_projection_matrix;
    const float* iv = g->camera_inverse_view_matrix;
    const float* pv = g->camera_projection_view_matrix;
    const float* ppv = g->camera_previous_projection_view_matrix;
    const v3 cam = V(g->camera_position[0], g->camera_position[1], g->camera_position[2]);
#pragma omp parallel for schedule(dynamic, 8)
    for (int y = 0; y < H; ++y) {
        for (int x = 0; x < W; ++x) {
            const size_t i = (size_t)y * W + x;
            float ndx = ((float)x + 0.5f) / (float)W * 2.0f - 1.0f, ndy = ((float)y + 0.5f) / (float)H * 2.0f - 1.0f;
            float e[4], f[4];
            mat_vec(ip, ndx, ndy, 1.0f, 1.0f, e);
            mat_vec(iv, e[0] / e[3], e[1] / e[3], e[2] / e[3], 1.0f, f);
            v3 dir = nrm(sub(V(f[0], f[1], f[2]), cam));
            float t;
            v3 n;
            int m = trace(s, cam, dir, 0.25f, &t, &n);
            if (m < 0) {
                depth[i] = 1.0f;
                put4(albedo + 4 * i, 0.2f, 0.4f, 1.0f, 1.0f);
                put4(emissive + 4 * i, 0, 0, 0, 1);
                put4(normal + 4 * i, 0, 0, 0, 1);
                put4(velocity + 4 * i, 0, 0, 0, 1);
                continue;
            }
            v3 p = add(cam, mul(dir, t));
            float c[4], q[4];
            mat_vec(pv, p.x, p.y, p.z, 1.0f, c);
            mat_vec(ppv, p.x, p.y, p.z, 1.0f, q);
            float z = c[2] / c[3];
            if (z < 0.0f || z > 1.0f) {  /* clipped by Vulkan depth clipping */
                depth[i] = 1.0f;
                put4(albedo + 4 * i, 0.2f, 0.4f, 1.0f, 1.0f);
                put4(emissive + 4 * i, 0, 0, 0, 1);
                put4(normal + 4 * i, 0, 0, 0, 1);
                put4(velocity + 4 * i, 0, 0, 0, 1);
                continue;
            }
            depth[i] = z;
            float alb[3], emi[3];
            material(m, p, n, alb, emi);
            put4(albedo + 4 * i, alb[0] + emi[0], alb[1] + emi[1], alb[2] + emi[2], 1.0f);
            put4(emissive + 4 * i, emi[0], emi[1], emi[2], 1.0f);
            put4(normal + 4 * i, n.x, n.y, n.z, 1.0f);
            float cu = (c[0] / c[3]) * 0.5f + 0.5f, cv = (c[1] / c[3]) * 0.5f + 0.5f;
            float pu = (q[0] / q[3]) * 0.5f + 0.5f, pvv = (q[1] / q[3]) * 0.5f + 0.5f;
            put4(velocity + 4 * i, cu - pu, cv - pvv, 0.0f, 1.0f);
        }
    }
    return 0;
}

/* Sun shadow map S x S (D32, tight rows). */
int soc_scene_shadow(int scene_id, const soc_globals* g, int S, float* shadow) {
    if (!g || S <= 0 || !shadow) return -1;
    if (scene_id == SCENE_TERRAIN) {   /* depth only, through the sun's ortho projection * view */
        int* tri = (int*)malloc(sizeof(int) * (size_t)S * S);
        terrain_raster(get_terrain(g), g->sun_info.projection_view_matrix, S, S, shadow, tri, NULL, NULL);
        free(tri);
        return 0;
    }
    const scene* s = get_scene(scene_id);
    float ivp[16];
    /* inverse of the sun's projection*view via the library-free closed form is not needed: march the
       ortho box corners instead. Ortho: view-space x,y in [-16,16], view z in [-16, 16] (near=-16,far=16). */
    const float* V_ = g->sun_info.view_matrix;
    const float* P_ = g->sun_info.projection_matrix;
    (void)ivp;
    /* camera basis from the view matrix rows (orthonormal lookAt) */
    v3 sx = V(V_[0], V_[4], V_[8]), sy = V(V_[1], V_[5], V_[9]), sz = V(V_[2], V_[6], V_[10]);
    v3 eye = V(g->sun_info.position[0], g->sun_info.position[1], g->sun_info.position[2]);
    const float l = -1.0f / P_[0] * (1.0f + P_[12]), r = 1.0f / P_[0] * (1.0f - P_[12]);
    const float b = -1.0f / P_[5] * (1.0f + P_[13]), t = 1.0f / P_[5] * (1.0f - P_[13]);
#pragma omp parallel for schedule(dynamic, 16)
    for (int y = 0; y < S; ++y) {
        for (int x = 0; x < S; ++x) {
            float u = ((float)x + 0.5f) / (float)S, v = ((float)y + 0.5f) / (float)S;
            float vx = l + (r - l) * u, vy = b + (t - b) * v;
            /* start on the view-space plane z = +16 (behind the light) and march along -sz */
            v3 o = add(add(eye, mul(sx, vx)), add(mul(sy, vy), mul(sz, 16.0f)));
            v3 d = mul(sz, -1.0f);
            float th;
            v3 n;
            int m = trace(s, o, d, 0.0f, &th, &n);
            float out = 1.0f;
            if (m >= 0) {
                v3 p = add(o, mul(d, th));
                float c[4];
                mat_vec(g->sun_info.projection_view_matrix, p.x, p.y, p.z, 1.0f, c);
                float z = c[2] / c[3];
                if (z >= 0.0f && z <= 1.0f) out = z;
            }
            shadow[(size_t)y * S + x] = out;
        }
    }
    return 0;
}

int soc_scene_box_count(int scene_id) { return get_scene(scene_id)->n; }

/* ---------------------------------------------------------------------------------------------------
 * Scenes as triangle meshes, for the GPU rasteriser (include/soc_rt.h "Rasterisation"):
 *  - terrain: the tessellated grid above (T_NV^2 vertices, 2*T_SEGS^2 triangles, in terrain_raster's
 *    order, each wound counter-clockwise seen from above), analytic vertex normals, uv in [0, 1]^2, and its albedo baked into an RGBA8 texture (the
 *    reference samples its terrain albedo from an image, draw_terrain.inl:196-222);
 *  - Sponza-proxy: the same boxes, 12 triangles each (faces wound counter-clockwise seen from outside),
 *    per-face normals, planar uvs in world units (the material() mapping), one material per box kind
 *    with a tiled procedural texture (0.5 x 0.25 blocks + mortar) of 4 x 4 world units.
 * ------------------------------------------------------------------------------------------------- */
int soc_scene_mesh_counts(int scene_id, int* vertices, int* triangles) {
    if (!vertices || !triangles) return -1;
    if (scene_id == SCENE_TERRAIN) { *vertices = T_NV * T_NV; *triangles = 2 * T_SEGS * T_SEGS; return 0; }
    const scene* s = get_scene(scene_id);
    *vertices = 24 * s->n;
    *triangles = 12 * s->n;
    return 0;
}

int soc_scene_mesh(int scene_id, const soc_globals* g, float* positions, float* normals, float* uvs, uint32_t* indices,
                   uint32_t* materials) {
    if (!g || !positions || !normals || !uvs || !indices || !materials) return -1;
    if (scene_id == SCENE_TERRAIN) {
        const terrain_mesh* t = get_terrain(g);
#pragma omp parallel for
        for (int j = 0; j < T_NV; ++j)
            for (int i = 0; i < T_NV; ++i) {
                const int k = j * T_NV + i;
                const float u = (float)i / (float)T_SEGS, v = (float)j / (float)T_SEGS;
                const v3 n = terrain_normal(t, u, v);
                positions[3 * k] = t->p[k].x; positions[3 * k + 1] = t->p[k].y; positions[3 * k + 2] = t->p[k].z;
                normals[3 * k] = n.x; normals[3 * k + 1] = n.y; normals[3 * k + 2] = n.z;
                uvs[2 * k] = u; uvs[2 * k + 1] = v;
            }
        for (int id = 0; id < 2 * T_SEGS * T_SEGS; ++id) {
            const int q = id >> 1, qi = q % T_SEGS, qj = q / T_SEGS;
            const int v00 = qj * T_NV + qi, v10 = v00 + 1, v01 = v00 + T_NV, v11 = v01 + 1;
            /* counter-clockwise seen from above (outward = up, like the boxes' faces) */
            indices[3 * id] = (uint32_t)v00;
            indices[3 * id + 1] = (uint32_t)((id & 1) ? v01 : v11);
            indices[3 * id + 2] = (uint32_t)((id & 1) ? v11 : v10);
            materials[id] = 0;
        }
        return 0;
    }
    const scene* s = get_scene(scene_id);
    /* face f: axis a = f/2, side = f&1 (0: lo, 1: hi); its 4 corners counter-clockwise seen from outside */
    for (int bi = 0; bi < s->n; ++bi) {
        const box* b = &s->b[bi];
        for (int f = 0; f < 6; ++f) {
            const int a = f >> 1, hi = f & 1;
            const int a1 = (a + 1) % 3, a2 = (a + 2) % 3;
            float lo3[3] = {b->lo.x, b->lo.y, b->lo.z}, hi3[3] = {b->hi.x, b->hi.y, b->hi.z};
            float nrm[3] = {0, 0, 0};
            nrm[a] = hi ? 1.0f : -1.0f;
            /* corners in (a1, a2): (0,0) (1,0) (1,1) (0,1); that order is CCW around +a; reverse for -a */
            const int c1[4] = {0, 1, 1, 0}, c2[4] = {0, 0, 1, 1};
            const int base = 24 * bi + 4 * f;
            for (int k = 0; k < 4; ++k) {
                const int kk = hi ? k : (3 - k);
                float p[3];
                p[a] = hi ? hi3[a] : lo3[a];
                p[a1] = c1[kk] ? hi3[a1] : lo3[a1];
                p[a2] = c2[kk] ? hi3[a2] : lo3[a2];
                float* P = positions + 3 * (base + k);
                P[0] = p[0]; P[1] = p[1]; P[2] = p[2];
                float* N = normals + 3 * (base + k);
                N[0] = nrm[0]; N[1] = nrm[1]; N[2] = nrm[2];
                /* material(): u = |n.x| > 0.5 ? p.z : p.x, v = |n.y| > 0.5 ? p.z : p.y */
                uvs[2 * (base + k)] = a == 0 ? p[2] : p[0];
                uvs[2 * (base + k) + 1] = a == 1 ? p[2] : p[1];
            }
            const int tb = 12 * bi + 2 * f;
            indices[3 * tb] = (uint32_t)base; indices[3 * tb + 1] = (uint32_t)(base + 1); indices[3 * tb + 2] = (uint32_t)(base + 2);
            indices[3 * tb + 3] = (uint32_t)base; indices[3 * tb + 4] = (uint32_t)(base + 2); indices[3 * tb + 5] = (uint32_t)(base + 3);
            materials[tb] = materials[tb + 1] = (uint32_t)b->mat;
        }
    }
    return 0;
}

/* Material textures: terrain -> one size x size RGBA8 albedo over uv [0,1]^2 (terrain_material at texel
   centres); Sponza-proxy -> M_COUNT stacked size x size RGBA8 tiles covering 4 x 4 world units
   (block tint + mortar of material(), linear values stored as UNORM). Emissive factors per material
   go to emissive_rgb (3 floats per material; terrain: 1 material). */
int soc_scene_material_count(int scene_id) { return scene_id == SCENE_TERRAIN ? 1 : M_COUNT; }

int soc_scene_material_textures(int scene_id, const soc_globals* g, int size, uint8_t* rgba, float* emissive_rgb) {
    if (!g || size <= 0 || !rgba || !emissive_rgb) return -1;
    if (scene_id == SCENE_TERRAIN) {
        const terrain_mesh* t = get_terrain(g);
#pragma omp parallel for schedule(dynamic, 8)
        for (int y = 0; y < size; ++y)
            for (int x = 0; x < size; ++x) {
                const float u = ((float)x + 0.5f) / (float)size, v = ((float)y + 0.5f) / (float)size;
                const v3 n = terrain_normal(t, u, v);
                const float hgt = (terrain_height(u, v) - t->mid) * t->hscale;
                float alb[3];
                terrain_material(hgt, n, u, v, alb);
                uint8_t* o = rgba + 4 * ((size_t)y * size + x);
                for (int c = 0; c < 3; ++c) {
                    float cl = alb[c] < 0.0f ? 0.0f : (alb[c] > 1.0f ? 1.0f : alb[c]);
                    o[c] = (uint8_t)lrintf(cl * 255.0f);
                }
                o[3] = 255;
            }
        emissive_rgb[0] = emissive_rgb[1] = emissive_rgb[2] = 0.0f;
        return 0;
    }
    for (int m = 0; m < M_COUNT; ++m) {
#pragma omp parallel for
        for (int y = 0; y < size; ++y)
            for (int x = 0; x < size; ++x) {
                /* texel centre -> world (u, v) in [0, 4): the tile repeats every 4 units */
                const float u = ((float)x + 0.5f) / (float)size * 4.0f, v = ((float)y + 0.5f) / (float)size * 4.0f;
                const int bu = (int)floorf(u * 2.0f), bv = (int)floorf(v * 4.0f);
                const float tint = 0.8f + 0.4f * hash3(bu, bv, m);
                const float fu = u * 2.0f - floorf(u * 2.0f), fv = v * 4.0f - floorf(v * 4.0f);
                const float mortar = (fu < 0.04f || fv < 0.06f) ? 0.55f : 1.0f;
                uint8_t* o = rgba + 4 * (((size_t)m * size + y) * size + x);
                for (int c = 0; c < 3; ++c) {
                    float cl = k_base[m][c] * tint * mortar;
                    cl = cl < 0.0f ? 0.0f : (cl > 1.0f ? 1.0f : cl);
                    o[c] = (uint8_t)lrintf(cl * 255.0f);
                }
                o[3] = 255;
            }
        emissive_rgb[3 * m] = m == M_LAMP ? 4.0f : 0.0f;
        emissive_rgb[3 * m + 1] = m == M_LAMP ? 2.6f : 0.0f;
        emissive_rgb[3 * m + 2] = m == M_LAMP ? 1.2f : 0.0f;
    }
    return 0;
}

/* Terrain heightmap as the reference loads it (R8G8B8A8_UNORM, renderer.cpp:155): terrain_height at
   texel centres, 8-bit in r = g = b, a = 255 (input of HeightToNormalTask). */
int soc_scene_terrain_heightmap(int size, uint8_t* rgba) {
    if (size <= 0 || !rgba) return -1;
#pragma omp parallel for schedule(static)
    for (int y = 0; y < size; ++y)
        for (int x = 0; x < size; ++x) {
            const float h = terrain_height(((float)x + 0.5f) / (float)size, ((float)y + 0.5f) / (float)size);
            const uint8_t v = (uint8_t)lrintf((h < 0.0f ? 0.0f : (h > 1.0f ? 1.0f : h)) * 255.0f);
            uint8_t* o = rgba + 4 * ((size_t)y * size + x);
            o[0] = o[1] = o[2] = v;
            o[3] = 255;
        }
    return 0;
}
