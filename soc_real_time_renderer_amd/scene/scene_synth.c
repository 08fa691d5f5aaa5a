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
