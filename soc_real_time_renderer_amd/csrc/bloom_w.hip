// bloom_w.hip — the bloom chain of renderer.cpp:1024-1062 (BloomDownsampleTask x4,
// bloom_downsample.inl:107-141; BloomUpsampleTask x4, bloom_upsample.inl:98-127) in WEIGHTED form.
//
// At the chain's fixed ratios (1:1 and 2:1 down, 1:2 and 1:1 up) every bilinear tap of the sampling
// contract lands on an exact weight (0, 1/2, 1/4 or 3/4) of clamped texel indices, so
// each pass is a fixed weighted sum over a small footprint of clamp-to-edge texels:
//   down 1:1  13 point taps: 1/8 centre, 1/32 (+-2,+-2), 1/16 (0,+-2) (+-2,0), 1/8 (+-1,+-1)
//   down 2:1  6x6 texels 2X-2..2X+3: (A (x) A + 4 B (x) B) / 128,  A = 1 1 2 2 1 1,  B = 0 1 1 1 1 0
//   up 1:2    4x4 texels: w (x) w / 256, w = 1 5 7 3 on X-2..X+1 (even output) or 3 7 5 1 on X-1..X+2 (odd)
//   up 1:1    3x3 texels: (1 2 1) (x) (1 2 1) / 16
// These are evaluated as fp32 FMAs straight from the RGBA16F texels (v_fma_mix_f32) instead of the
// reference's lerp-by-lerp order, which bloom.hip / bloom_fused.hip reproduce bit-exactly: same
// weights, different rounding order, within the RGBA16F tolerance, ~1/4 of the VALU
// work. Four kernels; the intermediates mip0 and mip2 live only in LDS (with recomputed halos):
//   W1  emissive -> [mip0] -> mip1        W2  mip1 -> [mip2] -> mip3
//   W3  mip3 -> [mip2] -> mip1            W4  mip1 -> [mip0] -> output
// The downsweep's mip0 / mip2 are read only by the next downsample and the upsweep's mip2 / mip0 only
// by the next upsample (quirk Q5 overwrites them), so mips[0] and mips[2] are not written: their final
// contents are unobservable in the reference graph. An intermediate tile entry at an out-of-image
// coordinate holds the value of the clamped coordinate, which is what the next pass's clamped taps read.
#include "bloom_w.hpp"

namespace soc {
// The chain's fixed-ratio fast paths apply when the four mips halve exactly (the reference's mip chain at even
// extents, renderer.cpp:492-513) and the extents fit the 8-bit fixed-point tap range.
bool bloom_fused_applicable(const soc_img& emissive, const soc_img* mips, int mip_count, const soc_img& output) {
    if (mip_count != 4 || output.width != emissive.width || output.height != emissive.height) return false;
    if (emissive.width > 8192 || emissive.height > 8192) return false;
    if (mips[0].width != emissive.width || mips[0].height != emissive.height) return false;
    for (int i = 1; i < 4; ++i)
        if (mips[i - 1].width != 2 * mips[i].width || mips[i - 1].height != 2 * mips[i].height || mips[i].width < 2 ||
            mips[i].height < 2)
            return false;
    return true;
}
}  // namespace soc

namespace soc {
namespace {

// Two horizontally adjacent outputs, one 16-B store when the row allows it.
__device__ __forceinline__ void store2(const DImg& im, int x, int y, uint2 a, uint2 b, bool vec) {
    uint2* row = row_ptr_w<uint2>(im, y);
    if (vec && x + 1 < im.w) {
        *reinterpret_cast<uint4*>(row + x) = uint4{a.x, a.y, b.x, b.y};
        return;
    }
    row[x] = a;
    if (x + 1 < im.w) row[x + 1] = b;
}

// ---- pass footprints (tile-relative; the caller guarantees every index lies inside its tile) -------
// down 1:1 at tile texel (cx, cy)
template <int TW>
__device__ __forceinline__ C3 down11(const uint2 (*t)[TW], int cx, int cy) {
    C3 a{0.0f, 0.0f, 0.0f};
    madd(a, t[cy][cx], 0.125f);
    madd(a, t[cy - 2][cx - 2], 0.03125f);
    madd(a, t[cy - 2][cx + 2], 0.03125f);
    madd(a, t[cy + 2][cx - 2], 0.03125f);
    madd(a, t[cy + 2][cx + 2], 0.03125f);
    madd(a, t[cy - 2][cx], 0.0625f);
    madd(a, t[cy][cx - 2], 0.0625f);
    madd(a, t[cy][cx + 2], 0.0625f);
    madd(a, t[cy + 2][cx], 0.0625f);
    madd(a, t[cy - 1][cx - 1], 0.125f);
    madd(a, t[cy - 1][cx + 1], 0.125f);
    madd(a, t[cy + 1][cx - 1], 0.125f);
    madd(a, t[cy + 1][cx + 1], 0.125f);
    return a;
}

// down 2:1 from the 6x6 block whose top-left tile texel is (c0, r0)
__device__ __forceinline__ constexpr float d21_w(int i, int j) {
    constexpr int A[6] = {1, 1, 2, 2, 1, 1}, B[6] = {0, 1, 1, 1, 1, 0};
    return (float)(A[i] * A[j] + 4 * B[i] * B[j]) * (1.0f / 128.0f);
}
template <int TW>
__device__ __forceinline__ C3 down21(const uint2 (*t)[TW], int c0, int r0) {
    C3 a{0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int j = 0; j < 6; ++j)
#pragma unroll
        for (int i = 0; i < 6; ++i) madd(a, t[r0 + j][c0 + i], d21_w(i, j));
    return a;
}

// up 1:2: the pair of horizontally adjacent outputs (2X, 2X+1) of output row y (parity py) from the
// 5x4 lower-texel block whose top-left tile texel is (X - 2, Y - 2 + py)
template <int TW>
__device__ __forceinline__ void up12_pair(const uint2 (*t)[TW], int c0, int r0, int py, C3& even, C3& odd) {
    even = C3{0.0f, 0.0f, 0.0f};
    odd = C3{0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float wy = u12_w(py, j);
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const uint2 v = t[r0 + j][c0 + i];
            if (i < 4) madd(even, v, u12_w(0, i) * wy);
            if (i > 0) madd(odd, v, u12_w(1, i - 1) * wy);
        }
    }
}

// up 1:1: the pair of outputs at tile texels (cx, cy), (cx + 1, cy)
template <int TW>
__device__ __forceinline__ void up11_pair(const uint2 (*t)[TW], int cx, int cy, C3& a, C3& b) {
    a = C3{0.0f, 0.0f, 0.0f};
    b = C3{0.0f, 0.0f, 0.0f};
    constexpr float w[3] = {1.0f, 2.0f, 1.0f};
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint2 v = t[cy - 1 + j][cx - 1 + i];
            if (i < 3) madd(a, v, w[i] * w[j] * (1.0f / 16.0f));
            if (i > 0) madd(b, v, w[i - 1] * w[j] * (1.0f / 16.0f));
        }
}

// ================================================================================================
// W1: emissive (W x H) -> [mip0, W x H, LDS] -> mip1 (W/2 x H/2)
// ================================================================================================
// MODE (tuning knob SOC_BLOOM_W1_REG): 1 = the 1:1 stage register-blocked (down11_runs): 30 x 8 mip1 outputs per
// workgroup, so the mip0 tile is 64 x 20 and each lane filters a run of 5 mip0 entries of one column at row stride 2
// (r, r + 2, ...), whose footprints share 3 of their 5 rows: 5 new LDS reads per entry instead of 13 (the stage is bound
// by its LDS reads); 2 = 30 x 16 outputs (mip0 tile 64 x 36, runs of 9) and the 2:1 stage in vertical output pairs
// (down21_vpair: 240 lanes, 48 LDS reads per pair instead of 72); 0 = 32 x 8 outputs, every mip0 entry from its 13 LDS
// taps and every output from its 36. Each entry's and output's fmas in down11's / down21's order: the same bits in every
// mode (tests/test_gpu_parity.py).
template <int MODE>
struct W1 {
    static constexpr int OW = MODE ? 30 : 32, OH = MODE == 2 ? 16 : 8;   // mip1 outputs per workgroup
    static constexpr int MW = 2 * OW + 4, MH = 2 * OH + 4;  // mip0 tile, origin (2 X0 - 2, 2 Y0 - 2)
    static constexpr int EW = MW + 4, EH = MH + 4;          // emissive tile, origin (2 X0 - 4, 2 Y0 - 4)
    static constexpr int RUN = MH / 4;                      // mip0 entries per lane run (64 columns x 2 parities x 2 runs)
    static_assert(!MODE || (MW == 64 && MH % 4 == 0), "down11_runs: 64 columns x 2 row parities x 2 runs");
};

// down11 of the mip0 entries (c, r), (c, r + 2), ..., (c, r + 8) of the tile (rows r..r+8 inside the tile: no vertical
// clamping in this workgroup), centre column cx (the clamped image column, tile-relative): a sliding window of the five
// footprint rows (three texels on the centre's row parity, two on the other), two rows loaded per entry after the first.
// Each entry's 13 fmas in down11's order.
template <int TW, int MW, int RUN>
__device__ __forceinline__ void down11_runs(const uint2 (*t)[TW], uint2 (*mt)[MW], int c, int r, int cx) {
    uint2 e0[3], o1[2], e2[3], o3[2], e4[3];
    const int cy0 = r + 2;   // emissive-tile row of the first entry's centre
    auto even = [&](int y, uint2 (&e)[3]) { e[0] = t[y][cx - 2]; e[1] = t[y][cx]; e[2] = t[y][cx + 2]; };
    auto odd = [&](int y, uint2 (&o)[2]) { o[0] = t[y][cx - 1]; o[1] = t[y][cx + 1]; };
    even(cy0 - 2, e0);
    odd(cy0 - 1, o1);
    even(cy0, e2);
    odd(cy0 + 1, o3);
    even(cy0 + 2, e4);
#pragma unroll
    for (int j = 0; j < RUN; ++j) {
        C3 a{0.0f, 0.0f, 0.0f};
        madd(a, e2[1], 0.125f);
        madd(a, e0[0], 0.03125f);
        madd(a, e0[2], 0.03125f);
        madd(a, e4[0], 0.03125f);
        madd(a, e4[2], 0.03125f);
        madd(a, e0[1], 0.0625f);
        madd(a, e2[0], 0.0625f);
        madd(a, e2[2], 0.0625f);
        madd(a, e4[1], 0.0625f);
        madd(a, o1[0], 0.125f);
        madd(a, o1[1], 0.125f);
        madd(a, o3[0], 0.125f);
        madd(a, o3[1], 0.125f);
        mt[r + 2 * j][c] = pack3(a);
        if (j < RUN - 1) {
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                e0[k] = e2[k];
                e2[k] = e4[k];
            }
            o1[0] = o3[0];
            o1[1] = o3[1];
            const int cy = cy0 + 2 * (j + 1);
            odd(cy + 1, o3);
            even(cy + 2, e4);
        }
    }
}

// down21 of the vertically adjacent outputs whose 6x6 blocks start at tile rows r0 and r0 + 2 (column c0): the 8 rows
// r0..r0+7 read once (6 texels each, 48 reads instead of 72), each row's texels added to the outputs it belongs to, so
// each output still sums its 36 taps in down21's order (rows outer, columns inner): the same bits.
template <int TW>
__device__ __forceinline__ void down21_vpair(const uint2 (*t)[TW], int c0, int r0, C3& a, C3& b) {
    a = C3{0.0f, 0.0f, 0.0f};
    b = C3{0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        uint2 v[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) v[i] = t[r0 + j][c0 + i];
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            if (j < 6) madd(a, v[i], d21_w(i, j));
            if (j >= 2) madd(b, v[i], d21_w(i, j - 2));
        }
        // one row's texels live at a time (without it the compiler hoists all 48 reads: 168 VGPRs)
        asm volatile("" : "+v"(a.r), "+v"(a.g), "+v"(a.b), "+v"(b.r), "+v"(b.g), "+v"(b.b)::"memory");
    }
}

// W1, persistent: each workgroup walks tiles t = blockIdx.x, + gridDim.x, ... (XCD-aware contiguous eighths, as
// swz = 1), and loads the NEXT tile's emissive texels into registers while it filters the current one from LDS, so
// the tile loads' latency hides behind the filter instead of being waited on (the one-tile kernel waits on its
// loads and barriers for 61 % of its wave cycles, profiles/r03_sq_stalls.json: 47.5 -> 42.9 us serial at 4K). The
// same arithmetic and bits as that one-tile-per-workgroup kernel.
template <int MODE>
__global__ __launch_bounds__(kWorkgroup) void bloomw_down01p(DImg E, DImg M1, int ntx, int nty) {
    constexpr int W1_OW = W1<MODE>::OW, W1_OH = W1<MODE>::OH, W1_MW = W1<MODE>::MW, W1_MH = W1<MODE>::MH,
                  W1_EW = W1<MODE>::EW, W1_EH = W1<MODE>::EH, RUN = W1<MODE>::RUN;
    __shared__ uint2 et[W1_EH][W1_EW];
    __shared__ uint2 mt[W1_MH][W1_MW];
    constexpr int NT = W1_EW * W1_EH, KR = (NT + 255) / 256;
    const int tid = threadIdx.x, n = ntx * nty, G = (int)gridDim.x;
    int er[KR], ec[KR];
#pragma unroll
    for (int k = 0; k < KR; ++k) {
        const int i = tid + 256 * k;
        er[k] = i / W1_EW;
        ec[k] = i - er[k] * W1_EW;
    }
    auto tile_origin = [&](int t, int& X0, int& Y0) {
        const int q = n >> 3, r = n & 7, k = t & 7;
        const int id = k * q + min(k, r) + (t >> 3);
        const int ty = id / ntx;
        X0 = (id - ty * ntx) * W1_OW;
        Y0 = ty * W1_OH;
    };
    uint2 v[KR];
    auto fetch = [&](int t) {
        int X0, Y0;
        tile_origin(t, X0, Y0);
        const int ex0 = 2 * X0 - 4, ey0 = 2 * Y0 - 4;
#pragma unroll
        for (int k = 0; k < KR; ++k)
            if (tid + 256 * k < NT)
                v[k] = row_ptr<uint2>(E, clampi(ey0 + er[k], 0, E.h - 1))[clampi(ex0 + ec[k], 0, E.w - 1)];
    };
    int t = (int)blockIdx.x;
    if (t < n) fetch(t);
    for (; t < n; t += G) {
#pragma unroll
        for (int k = 0; k < KR; ++k)
            if (tid + 256 * k < NT) et[er[k]][ec[k]] = v[k];
        __syncthreads();
        if (t + G < n) fetch(t + G);   // in flight while this tile is filtered
        int X0, Y0;
        tile_origin(t, X0, Y0);
        const int mx0 = 2 * X0 - 2, my0 = 2 * Y0 - 2, ex0 = mx0 - 2, ey0 = my0 - 2;
        // register-blocked runs unless the tile's mip0 rows reach past the image's top or bottom (there a clamped row
        // repeats, which the fixed row stride does not follow): a uniform branch
        if (MODE && my0 >= 0 && my0 + W1_MH <= E.h) {
            const int c = tid & 63, par = (tid >> 6) & 1, half = tid >> 7;
            if constexpr (MODE != 0)
                down11_runs<W1_EW, W1_MW, RUN>(et, mt, c, par + 2 * RUN * half, clampi(mx0 + c, 0, E.w - 1) - ex0);
        } else
        for (int i = tid; i < W1_MW * W1_MH; i += 256) {
            const int r = i / W1_MW, c = i - r * W1_MW;
            const int cx = clampi(mx0 + c, 0, E.w - 1) - ex0, cy = clampi(my0 + r, 0, E.h - 1) - ey0;
            mt[r][c] = pack3(down11<W1_EW>(et, cx, cy));
        }
        __syncthreads();
        if constexpr (MODE == 2) {   // vertical output pairs: lanes 0..239, outputs (ox, 2 q) and (ox, 2 q + 1)
            if (tid < W1_OW * W1_OH / 2) {
                const int q = tid / W1_OW, ox = tid - q * W1_OW;
                const int X = X0 + ox, Y = Y0 + 2 * q;
                C3 a, b;
                down21_vpair<W1_MW>(mt, 2 * ox, 4 * q, a, b);
                if (X < M1.w && Y < M1.h) row_ptr_w<uint2>(M1, Y)[X] = pack3(a);
                if (X < M1.w && Y + 1 < M1.h) row_ptr_w<uint2>(M1, Y + 1)[X] = pack3(b);
            }
        } else {
            const int oy = tid / W1_OW, ox = tid - oy * W1_OW;
            const int X = X0 + ox, Y = Y0 + oy;
            if (oy < W1_OH && X < M1.w && Y < M1.h) row_ptr_w<uint2>(M1, Y)[X] = pack3(down21<W1_MW>(mt, 2 * ox, 2 * oy));
        }
        __syncthreads();   // et / mt are rewritten by the next tile
    }
}

// ================================================================================================
// W2: mip1 -> [mip2, LDS] -> mip3
// ================================================================================================
constexpr int W2_OW = 16, W2_OH = 8;                          // mip3 outputs per workgroup
constexpr int W2_MW = 2 * W2_OW + 4, W2_MH = 2 * W2_OH + 4;   // mip2 tile 36 x 20
constexpr int W2_SW = 2 * W2_MW + 4, W2_SH = 2 * W2_MH + 4;   // mip1 tile 76 x 44

// down21 of the mip2 entries (c, r0 .. r0 + K - 1) of one column (no vertical clamping in this workgroup): the run's
// 6 + 2 (K - 1) mip1 rows read once (6 texels each; entries one row apart share 4 of their 6 rows), each row's texels
// added to the entries whose block holds it, so each entry sums its 36 taps in down21's order: the same bits.
template <int TW, int MW, int K>
__device__ __forceinline__ void down21_runs(const uint2 (*t)[TW], uint2 (*mt)[MW], int c, int r0, int n, int sc) {
    C3 acc[K];
#pragma unroll
    for (int e = 0; e < K; ++e) acc[e] = C3{0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int R = 0; R < 6 + 2 * (K - 1); ++R) {
        // a shorter last run (n < K entries) skips the rows only its missing entries need (reads inside the tile)
        if (R >= 6 + 2 * (n - 1)) continue;
        uint2 v[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) v[i] = t[2 * r0 + R][sc + i];
#pragma unroll
        for (int e = 0; e < K; ++e) {
            const int j = R - 2 * e;
            if (j >= 0 && j < 6) {
#pragma unroll
                for (int i = 0; i < 6; ++i) madd(acc[e], v[i], d21_w(i, j));
            }
        }
        // one row's texels live at a time (the row's fmas complete before the next row's reads)
#pragma unroll
        for (int e = 0; e < K; ++e) asm volatile("" : "+v"(acc[e].r), "+v"(acc[e].g), "+v"(acc[e].b)::"memory");
    }
#pragma unroll
    for (int e = 0; e < K; ++e)
        if (e < n) mt[r0 + e][c] = pack3(acc[e]);
}

// REG (tuning knob SOC_BLOOM_W2_REG, default 1): the 2:1 mip1 -> mip2 stage in vertical runs of 3 entries per lane
// (down21_runs: 36 columns x 7 runs, 60 LDS reads per run instead of 108) unless the tile's mip2 rows reach past the
// image's top or bottom; the same bits (tests/test_gpu_parity.py).
template <bool REG>
__global__ __launch_bounds__(kWorkgroup) void bloomw_down23(DImg S1, DImg M3, int W2, int H2, int swz) {
    __shared__ uint2 st[W2_SH][W2_SW];
    __shared__ uint2 mt[W2_MH][W2_MW];
    const int tid = threadIdx.x;
    int tbx, tby;
    xcd_order(swz, tbx, tby);   // swz: XCD-aware order (neighbouring tiles share an XCD's L2 for their halos)
    const int X0 = tbx * W2_OW, Y0 = tby * W2_OH;
    const int mx0 = 2 * X0 - 2, my0 = 2 * Y0 - 2, sx0 = 2 * mx0 - 2, sy0 = 2 * my0 - 2;
    load_tile<W2_SW, W2_SH>(S1, sx0, sy0, st, tid);
    __syncthreads();
    constexpr int K = 3, NR = (W2_MH + K - 1) / K;   // 7 runs per column, the last one of 2
    static_assert(W2_MW * NR <= 256, "one run per lane");
    if (REG && my0 >= 0 && my0 + W2_MH <= H2) {
        if (tid < W2_MW * NR) {
            const int c = tid % W2_MW, k = tid / W2_MW, r0 = k * K;
            const int qx = clampi(mx0 + c, 0, W2 - 1);
            down21_runs<W2_SW, W2_MW, K>(st, mt, c, r0, min(K, W2_MH - r0), 2 * qx - 2 - sx0);
        }
    } else
    for (int i = tid; i < W2_MW * W2_MH; i += 256) {
        const int r = i / W2_MW, c = i - r * W2_MW;
        const int qx = clampi(mx0 + c, 0, W2 - 1), qy = clampi(my0 + r, 0, H2 - 1);
        mt[r][c] = pack3(down21<W2_SW>(st, 2 * qx - 2 - sx0, 2 * qy - 2 - sy0));
    }
    __syncthreads();
    if (tid < W2_OW * W2_OH) {
        const int ox = tid % W2_OW, oy = tid / W2_OW;
        const int X = X0 + ox, Y = Y0 + oy;
        if (X < M3.w && Y < M3.h) row_ptr_w<uint2>(M3, Y)[X] = pack3(down21<W2_MW>(mt, 2 * ox, 2 * oy));
    }
}

// ================================================================================================
// W3: mip3 -> [mip2, LDS] -> mip1 (64 x 16 mip1 outputs per workgroup)
// ================================================================================================
constexpr int U_OW = 64, U_OH = 16;
constexpr int W3_MW = U_OW / 2 + 4, W3_MH = U_OH / 2 + 4;   // mip2 tile 36 x 12, origin (X0/2 - 2, Y0/2 - 2)
constexpr int W3_SW = W3_MW / 2 + 4, W3_SH = W3_MH / 2 + 4; // mip3 tile 22 x 10, origin (X0/4 - 3, Y0/4 - 3)

// One lower-res texel pair / row of the 1:2 upsample into the LDS tile entries (c, r), (c + 1, r) at
// intermediate coordinates (qx, qy), (qx + 1, qy), qx even.
template <int SW, int MW>
__device__ __forceinline__ void up12_into(const uint2 (*s)[SW], int sx0, int sy0, uint2 (*m)[MW], int c, int r, int qx, int qy,
                                          int Wq, int Hq) {
    // a clamped coordinate can break the (even, odd) pairing at the image edges: evaluate each entry
    // at its own clamped coordinate
    const int cy = clampi(qy, 0, Hq - 1), py = cy & 1;
    const int q0 = clampi(qx, 0, Wq - 1), q1 = clampi(qx + 1, 0, Wq - 1);
    const int r0 = (cy >> 1) - 2 + py - sy0;
    if ((q0 & 1) == 0 && q1 == q0 + 1) {
        C3 e, o;
        up12_pair<SW>(s, (q0 >> 1) - 2 - sx0, r0, py, e, o);
        m[r][c] = pack3(e);
        m[r][c + 1] = pack3(o);
    } else {
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int q = k ? q1 : q0;
            C3 e, o;
            up12_pair<SW>(s, ((q & ~1) >> 1) - 2 - sx0, r0, py, e, o);
            m[r][c + k] = pack3((q & 1) ? o : e);
        }
    }
}

__global__ __launch_bounds__(kWorkgroup) void bloomw_up32(DImg S3, DImg M1, int W2, int H2, bool vec, int swz) {
    __shared__ uint2 st[W3_SH][W3_SW];
    __shared__ uint2 mt[W3_MH][W3_MW];
    const int tid = threadIdx.x;
    int tbx, tby;
    xcd_order(swz, tbx, tby);   // swz: XCD-aware order (neighbouring tiles share an XCD's L2 for their halos)
    const int X0 = tbx * U_OW, Y0 = tby * U_OH;
    const int mx0 = X0 / 2 - 2, my0 = Y0 / 2 - 2;       // even
    const int sx0 = mx0 / 2 - 2, sy0 = my0 / 2 - 2;     // mx0 / 2 = floor since mx0 is even
    load_tile<W3_SW, W3_SH>(S3, sx0, sy0, st, tid);
    __syncthreads();
    for (int i = tid; i < (W3_MW / 2) * W3_MH; i += 256) {
        const int r = i / (W3_MW / 2), c = 2 * (i - r * (W3_MW / 2));
        up12_into<W3_SW, W3_MW>(st, sx0, sy0, mt, c, r, mx0 + c, my0 + r, W2, H2);
    }
    __syncthreads();
    // mip1 outputs: 32 pairs x 16 rows = 512 pairs, 2 per thread
    for (int i = tid; i < (U_OW / 2) * U_OH; i += 256) {
        const int r = i / (U_OW / 2), pc = i - r * (U_OW / 2);
        const int x = X0 + 2 * pc, y = Y0 + r;
        if (x >= M1.w || y >= M1.h) continue;
        const int py = y & 1;
        C3 e, o;
        up12_pair<W3_MW>(mt, (x >> 1) - 2 - mx0, (y >> 1) - 2 + py - my0, py, e, o);
        store2(M1, x, y, pack3(e), pack3(o), vec);
    }
}

// W3 in separable form (both 1:2 filters are w (x) w): each 1:2 stage as a horizontal pass into an fp32 LDS tile and a
// vertical pass, 4 + 4 taps instead of 16; mip2 still rounded to RGBA16F (within the RGBA16F tolerance, as bloomw_up10s).
struct P3u {
    float r[W3_MH][U_OW], g[W3_MH][U_OW], b[W3_MH][U_OW];   // 10 x 36 (first stage) and 12 x 64 (second) fit
};
template <bool RUNS>
__global__ __launch_bounds__(kWorkgroup) void bloomw_up32s(DImg S3, DImg M1, int W2, int H2, bool vec, int swz) {
    __shared__ uint2 st[W3_SH][W3_SW];
    __shared__ uint2 mt[W3_MH][W3_MW];
    __shared__ P3u hp;
    const int tid = threadIdx.x;
    int tbx, tby;
    xcd_order(swz, tbx, tby);
    const int X0 = tbx * U_OW, Y0 = tby * U_OH;
    const int mx0 = X0 / 2 - 2, my0 = Y0 / 2 - 2;
    const int sx0 = mx0 / 2 - 2, sy0 = my0 / 2 - 2;
    load_tile<W3_SW, W3_SH>(S3, sx0, sy0, st, tid);
    __syncthreads();
    for (int i = tid; i < W3_SH * W3_MW; i += 256) {   // mip3 rows x mip2 columns (clamped coordinates)
        const int sr = i / W3_MW, c = i - sr * W3_MW;
        const int q = clampi(mx0 + c, 0, W2 - 1), px = q & 1, c0 = (q >> 1) - 2 + px - sx0;
        C3 a{0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int k = 0; k < 4; ++k) madd(a, st[sr][c0 + k], u12_w(px, k));
        hp.r[sr][c] = a.r;
        hp.g[sr][c] = a.g;
        hp.b[sr][c] = a.b;
    }
    __syncthreads();
    for (int i = tid; i < W3_MH * W3_MW; i += 256) {   // the mip2 entries
        const int r = i / W3_MW, c = i - r * W3_MW;
        const int cy = clampi(my0 + r, 0, H2 - 1), py = cy & 1, r0 = (cy >> 1) - 2 + py - sy0;
        C3 a{0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float w = u12_w(py, k);
            a.r = __builtin_fmaf(hp.r[r0 + k][c], w, a.r);
            a.g = __builtin_fmaf(hp.g[r0 + k][c], w, a.g);
            a.b = __builtin_fmaf(hp.b[r0 + k][c], w, a.b);
        }
        mt[r][c] = pack3(a);
    }
    __syncthreads();
    for (int i = tid; i < W3_MH * U_OW; i += 256) {   // mip2 rows x mip1 output columns
        const int r = i / U_OW, ox = i - r * U_OW;
        const int x = X0 + ox, px = x & 1, c0 = (x >> 1) - 2 + px - mx0;
        C3 a{0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int k = 0; k < 4; ++k) madd(a, mt[r][c0 + k], u12_w(px, k));
        hp.r[r][ox] = a.r;
        hp.g[r][ox] = a.g;
        hp.b[r][ox] = a.b;
    }
    __syncthreads();
    if constexpr (RUNS) {
        static_assert(U_OW == 64 && U_OH == 16, "64 columns x 4 runs of 4 output rows");
        // SOC_BLOOM_W3_RUNS (default 1): the last vertical 1:2 phase in runs of 4 outputs of one column per lane
        // (outputs Y0 + 4 m .. + 3 read the hp rows 2 m .. 2 m + 5 once: 18 LDS reads instead of 48); each output's 4
        // fmas in the same order: the same bits
        const int ox = tid & 63, m = tid >> 6, x = X0 + ox;
        float hr[6], hg[6], hb[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            hr[k] = hp.r[2 * m + k][ox];
            hg[k] = hp.g[2 * m + k][ox];
            hb[k] = hp.b[2 * m + k][ox];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int y = Y0 + 4 * m + i, py = i & 1, rr = (i >> 1) + (i & 1);
            C3 a{0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float w = u12_w(py, j);
                a.r = __builtin_fmaf(hr[rr + j], w, a.r);
                a.g = __builtin_fmaf(hg[rr + j], w, a.g);
                a.b = __builtin_fmaf(hb[rr + j], w, a.b);
            }
            if (x < M1.w && y < M1.h) row_ptr_w<uint2>(M1, y)[x] = pack3(a);
        }
        return;
    }
    for (int i = tid; i < (U_OW / 2) * U_OH; i += 256) {
        const int r = i / (U_OW / 2), pc = i - r * (U_OW / 2);
        const int x = X0 + 2 * pc, y = Y0 + r;
        if (x >= M1.w || y >= M1.h) continue;
        const int py = y & 1, r0 = (y >> 1) - 2 + py - my0;
        C3 o[2];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int c = 2 * pc + k;
            C3 a{0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float w = u12_w(py, j);
                a.r = __builtin_fmaf(hp.r[r0 + j][c], w, a.r);
                a.g = __builtin_fmaf(hp.g[r0 + j][c], w, a.g);
                a.b = __builtin_fmaf(hp.b[r0 + j][c], w, a.b);
            }
            o[k] = a;
        }
        store2(M1, x, y, pack3(o[0]), pack3(o[1]), vec);
    }
}

// ================================================================================================
// W4: mip1 -> [mip0, LDS] -> output (64 x 16 outputs per workgroup)
// ================================================================================================
constexpr int W4_MW = U_OW + 2, W4_MH = U_OH + 2;             // mip0 tile 66 x 18, origin (X0 - 1, Y0 - 1)
constexpr int W4_SW = U_OW / 2 + 6, W4_SH = U_OH / 2 + 6;     // mip1 tile 38 x 14, origin (X0/2 - 3, Y0/2 - 3)

__global__ __launch_bounds__(kWorkgroup) void bloomw_up10(DImg S1, DImg O, bool vec, int swz) {
    __shared__ uint2 st[W4_SH][W4_SW];
    __shared__ uint2 mt[W4_MH][W4_MW + 2];   // +2: the pair loop writes whole pairs
    const int tid = threadIdx.x;
    int tbx, tby;
    xcd_order(swz, tbx, tby);   // swz: XCD-aware order (neighbouring tiles share an XCD's L2 for their halos)
    const int X0 = tbx * U_OW, Y0 = tby * U_OH;
    const int mx0 = X0 - 1, my0 = Y0 - 1;
    const int sx0 = X0 / 2 - 3, sy0 = Y0 / 2 - 3;
    const int W0 = O.w, H0 = O.h;   // mip0 extent = output extent
    load_tile<W4_SW, W4_SH>(S1, sx0, sy0, st, tid);
    __syncthreads();
    // mip0 entries (c, r) for c = 0..65: pairs start at odd mip0 coordinates (mx0 is odd), so pair
    // entries as (c + 1, c + 2) with even coordinate first, and entry 0 on its own
    for (int i = tid; i < (W4_MW / 2) * W4_MH; i += 256) {
        const int r = i / (W4_MW / 2), k = i - r * (W4_MW / 2);
        const int c = 2 * k + 1;   // mip0 coordinate mx0 + c = X0 + 2k: even
        up12_into<W4_SW, W4_MW + 2>(st, sx0, sy0, mt, c, r, mx0 + c, my0 + r, W0, H0);
    }
    for (int r = tid; r < W4_MH; r += 256) {   // column 0 (coordinate X0 - 1)
        const int cy = clampi(my0 + r, 0, H0 - 1), py = cy & 1;
        const int q = clampi(mx0, 0, W0 - 1);
        C3 e, o;
        up12_pair<W4_SW>(st, ((q & ~1) >> 1) - 2 - sx0, (cy >> 1) - 2 + py - sy0, py, e, o);
        mt[r][0] = pack3((q & 1) ? o : e);
    }
    __syncthreads();
    for (int i = tid; i < (U_OW / 2) * U_OH; i += 256) {
        const int r = i / (U_OW / 2), pc = i - r * (U_OW / 2);
        const int x = X0 + 2 * pc, y = Y0 + r;
        if (x >= O.w || y >= O.h) continue;
        C3 a, b;
        up11_pair<W4_MW + 2>(mt, x - mx0, y - my0, a, b);
        store2(O, x, y, pack3(a), pack3(b), vec);
    }
}

// W4 in separable form: both filters of the pass are rank 1 (up 1:2: w (x) w; up 1:1: (1 2 1) (x) (1 2 1)), so each is a
// horizontal pass into an fp32 LDS tile and a vertical pass: per mip0 entry 4 + 4 taps instead of 16, per output 3 + 3
// instead of 9. The same weights and footprints (the mip0 entries still rounded to RGBA16F, as the chain stores them);
// the sums are grouped by rows, so the last fp32 bits may differ from bloomw_up10 (within the RGBA16F tolerance).
__global__ __launch_bounds__(kWorkgroup) void bloomw_up10s(DImg S1, DImg O, bool vec, int swz) {
    __shared__ Up10Tile<U_OW, U_OH> t;   // bloom_w.hpp (shared with Composition's in-kernel upsample)
    const int tid = threadIdx.x;
    int tbx, tby;
    xcd_order(swz, tbx, tby);
    const int X0 = tbx * U_OW, Y0 = tby * U_OH;
    t.build(S1, X0, Y0, O.w, O.h, tid);
    // 1:1 vertical and the stores (pairs)
    for (int i = tid; i < (U_OW / 2) * U_OH; i += 256) {
        const int r = i / (U_OW / 2), pc = i - r * (U_OW / 2);
        const int x = X0 + 2 * pc, y = Y0 + r;
        if (x >= O.w || y >= O.h) continue;
        C3 o[2];
        t.out(r, 2 * pc, o);
        store2(O, x, y, pack3(o[0]), pack3(o[1]), vec);
    }
}

// W4 in register form (SOC_BLOOM_UP10_REG, default): no LDS and no barriers. Each wave owns a strip of 62 output columns
// (lanes 1..62; lanes 0 and 63 hold the clamped neighbour columns) and walks down R_TH output rows; a lane keeps its
// column's last five 1:2-horizontal sums (one mip1 row more every second output row) and the last three 1:1-horizontal
// sums in registers, and takes its neighbours' mip0 texels by DPP wave shifts. The same operations in the same order as
// Up10Tile (bloomw_up10s), so the same bits, without its four LDS phases (~180 B of LDS traffic per output pixel). Alone
// at C3 36.4-36.8 us against 38.3-39.3 for bloomw_up10s, in the frame within noise; 8 / 32 rows per wave and 64-column
// aligned strips measured the same (the 66 MB output stream is what is left).
#ifndef SOC_BLOOM_UP10_ROWS
#define SOC_BLOOM_UP10_ROWS 16
#endif
constexpr int R_OW = 62, R_TH = SOC_BLOOM_UP10_ROWS;
__device__ __forceinline__ uint32_t up_from_left(uint32_t v) {   // lane i <- lane i-1 (wave_shr:1)
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t up_from_right(uint32_t v) {  // lane i <- lane i+1 (wave_shl:1)
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xf, 0xf, false);
}
__global__ __launch_bounds__(kWorkgroup) void bloomw_up10r(DImg S1, DImg O, int nwx, int nwaves) {
    const int lane = (int)(threadIdx.x & 63);
    const int wid = (int)blockIdx.x * (kWorkgroup / 64) + (int)(threadIdx.x >> 6);
    if (wid >= nwaves) return;   // wave-uniform
    const int W0 = O.w, H0 = O.h, W1 = S1.w, H1 = S1.h;
    const int wx = wid % nwx, Y0 = (wid / nwx) * R_TH;
    const int x = wx * R_OW - 1 + lane;
    const int cx = clampi(x, 0, W0 - 1);
    const int px = cx & 1, c0 = (cx >> 1) - 2 + px;
    int tc[4];
    float wk[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        tc[k] = clampi(c0 + k, 0, W1 - 1);
        wk[k] = px ? u12_w(1, k) : u12_w(0, k);
    }
    // the 1:2 horizontal sum of mip1 row clamp(s) at this lane's mip0 column (Up10Tile::build's first pass): the row's
    // four taps are loaded one mip1 row ahead of their use (two output rows of arithmetic cover their latency)
    auto taps = [&](int s, uint2 (&t)[4]) {
        const uint2* row = row_ptr<uint2>(S1, clampi(s, 0, H1 - 1));
#pragma unroll
        for (int k = 0; k < 4; ++k) t[k] = row[tc[k]];
    };
    auto h12 = [&](const uint2 (&t)[4]) {
        C3 a{0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int k = 0; k < 4; ++k) madd(a, t[k], wk[k]);
        return a;
    };
    // ring[i]: the sum of mip1 row base + i; pend: the taps of row base + 5
    C3 ring[5];
    uint2 pend[4];
    int base = (max(Y0 - 1, 0) >> 1) - 2;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        taps(base + i, pend);
        ring[i] = h12(pend);
    }
    taps(base + 5, pend);
    // this lane's mip0 texel of row cy (the second pass, rounded to RGBA16F), then the row's 1:1 horizontal sum
    auto hrow = [&](int cy) {
        const int jb = (cy >> 1) - 2;   // rows only move down, at most one mip1 row per call
        if (jb > base) {
#pragma unroll
            for (int i = 0; i < 4; ++i) ring[i] = ring[i + 1];
            ring[4] = h12(pend);   // row base + 5 = jb + 4
            base = jb;
            taps(base + 5, pend);
        }
        const int py = cy & 1;
        C3 a{0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float w = u12_w(py, k);
            const C3 h = py ? ring[k + 1] : ring[k];
            a.r = __builtin_fmaf(h.r, w, a.r);
            a.g = __builtin_fmaf(h.g, w, a.g);
            a.b = __builtin_fmaf(h.b, w, a.b);
        }
        const uint2 m = pack3(a);
        const uint2 l = uint2{up_from_left(m.x), up_from_left(m.y)}, r = uint2{up_from_right(m.x), up_from_right(m.y)};
        C3 hs{0.0f, 0.0f, 0.0f};
        madd(hs, l, 1.0f);
        madd(hs, m, 2.0f);
        madd(hs, r, 1.0f);
        return hs;
    };
    C3 hq0 = hrow(max(Y0 - 1, 0)), hq1 = hrow(min(Y0, H0 - 1));
    const bool out_lane = lane >= 1 && lane <= R_OW && x < W0;
    for (int y = Y0; y < min(Y0 + R_TH, H0); ++y) {
        const C3 hq2 = hrow(min(y + 1, H0 - 1));
        C3 o;
        o.r = __builtin_fmaf(hq2.r, 1.0f / 16.0f, __builtin_fmaf(hq1.r, 2.0f / 16.0f, hq0.r * (1.0f / 16.0f)));
        o.g = __builtin_fmaf(hq2.g, 1.0f / 16.0f, __builtin_fmaf(hq1.g, 2.0f / 16.0f, hq0.g * (1.0f / 16.0f)));
        o.b = __builtin_fmaf(hq2.b, 1.0f / 16.0f, __builtin_fmaf(hq1.b, 2.0f / 16.0f, hq0.b * (1.0f / 16.0f)));
        if (out_lane) row_ptr_w<uint2>(O, y)[x] = pack3(o);
        hq0 = hq1;
        hq1 = hq2;
    }
}

// Workgroups of 256 lanes of bloomw_down01p resident on the whole device at once (the persistent kernel's grid bound),
// queried once per device and cached (the occupancy query is not on the per-frame enqueue path).
template <int MODE>
int down01p_resident_set() {
    constexpr int kMaxDevices = 64;
    static int cached[kMaxDevices] = {};
    int dev = 0, cus = 256, per = 0;
    (void)hipGetDevice(&dev);
    if (dev >= 0 && dev < kMaxDevices && cached[dev]) return cached[dev];
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, bloomw_down01p<MODE>, 256, 0);
    const int n = std::max(per, 1) * cus;
    if (dev >= 0 && dev < kMaxDevices) cached[dev] = n;
    return n;
}

bool a16(const soc_img& im) { return im.pitch_bytes % 16 == 0 && reinterpret_cast<uintptr_t>(im.data) % 16 == 0; }

}  // namespace

int launch_bloom_weighted(const soc_img& emissive, const soc_img* mips, const soc_img& output, hipStream_t s, int stage) {
    const DImg E = dimg(emissive), M1 = dimg(mips[1]), M3 = dimg(mips[3]), O = dimg(output);
    const int swz = 1;   // XCD-aware order: halo re-reads served by L2 (2.0x -> 1.0x HBM traffic)
    if (stage == 0 || stage == 1) {
        // persistent: one resident set of workgroups (a multiple of 8, so a workgroup's tiles stay on its XCD)
        auto w1 = [&](auto mode) {
            constexpr int R = decltype(mode)::value;
            const int ntx = ceil_div(mips[1].width, W1<R>::OW), nty = ceil_div(mips[1].height, W1<R>::OH);
            const int grid = std::max(8, (std::min(ntx * nty, down01p_resident_set<R>()) / 8) * 8);
            launch("bloomw_down01p", kWorkgroup, bloomw_down01p<R>, grid, kWorkgroup, 0, s, E, M1, ntx, nty);
        };
        const int mode = tuning_knob("SOC_BLOOM_W1_REG", 1);
        if (mode == 2) w1(std::integral_constant<int, 2>{});
        else if (mode == 1) w1(std::integral_constant<int, 1>{});
        else w1(std::integral_constant<int, 0>{});
    }
    if (stage == 0 || stage == 2) {
        dim3 g(ceil_div(mips[3].width, W2_OW), ceil_div(mips[3].height, W2_OH));
        if (tuning_knob("SOC_BLOOM_W2_REG", 1))
            launch("bloomw_down23", kWorkgroup, bloomw_down23<true>, g, kWorkgroup, 0, s, M1, M3, mips[2].width, mips[2].height, swz);
        else
            launch("bloomw_down23", kWorkgroup, bloomw_down23<false>, g, kWorkgroup, 0, s, M1, M3, mips[2].width, mips[2].height, swz);
    }
    if (stage == 0 || stage == 3) {
        dim3 g(ceil_div(mips[1].width, U_OW), ceil_div(mips[1].height, U_OH));
        if (tuning_knob("SOC_BLOOM_UP_SEP", 1))
            if (tuning_knob("SOC_BLOOM_W3_RUNS", 1))
                launch("bloomw_up32s", kWorkgroup, bloomw_up32s<true>, g, kWorkgroup, 0, s, M3, M1, mips[2].width, mips[2].height, a16(mips[1]), swz);
            else
                launch("bloomw_up32s", kWorkgroup, bloomw_up32s<false>, g, kWorkgroup, 0, s, M3, M1, mips[2].width, mips[2].height, a16(mips[1]), swz);
        else
            launch("bloomw_up32", kWorkgroup, bloomw_up32, g, kWorkgroup, 0, s, M3, M1, mips[2].width, mips[2].height, a16(mips[1]), swz);
    }
    if (stage == 0 || stage == 4) {
        dim3 g(ceil_div(output.width, U_OW), ceil_div(output.height, U_OH));
        if (tuning_knob("SOC_BLOOM_UP10_REG", 1)) {
            const int nwx = ceil_div(output.width, R_OW), nwaves = nwx * ceil_div(output.height, R_TH);
            launch("bloomw_up10r", kWorkgroup, bloomw_up10r, ceil_div(nwaves, kWorkgroup / 64), kWorkgroup, 0, s, M1, O, nwx, nwaves);
        } else if (tuning_knob("SOC_BLOOM_UP_SEP", 1))
            launch("bloomw_up10s", kWorkgroup, bloomw_up10s, g, kWorkgroup, 0, s, M1, O, a16(output), swz);
        else
            launch("bloomw_up10", kWorkgroup, bloomw_up10, g, kWorkgroup, 0, s, M1, O, a16(output), swz);
    }
    return check_launch("bloom_weighted");
}

}  // namespace soc
