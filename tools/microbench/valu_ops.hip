// Issue cost of the individual VALU opcodes of the clouds / SSAO inner loops on gfx950, in the method of valu_rate.hip:
// 16 independent chains per lane, inline asm (the stream is exactly what is written), 8 waves per SIMD over the
// full chip, cycles per wave64 instruction per SIMD from the event time and the in-kernel clock (s_memtime /
// s_memrealtime). v_fma_f32 is the reference (2.44 cycles in profiles/r06_valu_model.json).
// Build: hipcc --offload-arch=gfx950 -O3 -o valu_ops valu_ops.hip ; run on the GPU box.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

constexpr int kChains = 16;

// name, asm body, operand pattern: F = "+v"(x) : a, b;  F1 = "+v"(x);  U = "+v"(n) : ua, ub;  U1 = "+v"(n);
// C = "=v"(x), "+v"(n) : ua (convert + u32 add: 2 instructions);  FU = "+v"(x), "=v"(n) : ua, a, b (2 instructions)
#define OPS(X)                                                                                                      \
    X(FMA, "v_fma_f32 %0, %1, %2, %0", F)                                                                         \
    X(DOT2_U16, "v_dot2_u32_u16 %0, %1, %2, %0", U)                                                               \
    X(CVT_UBYTE0, "v_cvt_f32_ubyte0 %0, %1\n v_add_u32 %1, %2, %1", C)                                           \
    X(CVT_F32_U32, "v_cvt_f32_u32 %0, %1\n v_add_u32 %1, %2, %1", C)                                             \
    X(CVT_FLR, "v_cvt_flr_i32_f32 %1, %0\n v_fma_f32 %0, %0, %3, %4", FU)                                         \
    X(PERM, "v_perm_b32 %0, %0, %0, %1", U)                                                                       \
    X(BFE, "v_bfe_u32 %0, %0, 8, 6", U1)                                                                          \
    X(MAD_U24, "v_mad_u32_u24 %0, %0, %1, %2", U)                                                                 \
    X(LSHL_OR, "v_lshl_or_b32 %0, %0, 16, %1", U)                                                                 \
    X(FLOOR, "v_floor_f32 %0, %0", F1)                                                                            \
    X(SQRT, "v_sqrt_f32 %0, %0", F1)                                                                              \
    X(RCP, "v_rcp_f32 %0, %0", F1)                                                                                \
    X(MED3, "v_med3_f32 %0, %0, %1, %2", F)                                                                       \
    X(CNDMASK, "v_cndmask_b32 %0, %0, %1, vcc", F)                                                                \
    X(CMP_CNDMASK, "v_cmp_gt_f32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %2, vcc", F2)                               \
    X(CMP_FMA, "v_cmp_gt_f32 vcc, %0, %1\n v_fma_f32 %0, %0, %1, %2", F2)                                        \
    X(FMA_MIX, "v_fma_mix_f32 %0, %1, %0, %2 op_sel_hi:[1,0,1]", F)                                               \
    X(ADD_U32, "v_add_u32 %0, %1, %0", U)                                                                         \
    X(AND_B32, "v_and_b32 %0, %1, %0", U)                                                                         \
    X(LSHR, "v_lshrrev_b32 %0, 5, %0", U1)                                                                        \
    X(SUB_F32, "v_sub_f32 %0, %1, %0", F)                                                                         \
    X(MUL_F32, "v_mul_f32 %0, %1, %0", F)                                                                         \
    X(CVT_F32_I32, "v_cvt_f32_i32 %0, %1\n v_add_u32 %1, %2, %1", C)                                             \
    X(CVT_I32_F32, "v_cvt_i32_f32 %1, %0\n v_fma_f32 %0, %0, %3, %4", FU)                                         \
    X(EXP, "v_exp_f32 %0, %0", F1)                                                                                \
    X(PK_FMA, "v_pk_fma_f32 %0, %1, %2, %0", P)                                                                   \
    X(PK_MUL, "v_pk_mul_f32 %0, %1, %0", P)                                                                       \
    X(ADD3, "v_add3_u32 %0, %1, %2, %0", U)                                                                       \
    X(MUL_U24, "v_mul_u32_u24 %0, %1, %0", U)                                                                     \
    X(FMAC, "v_fmac_f32 %0, %1, %2", F)                                                                           \
    X(MAD_I64_I32, "v_mad_i64_i32 %0, s[0:1], %1, %2, %0", D)                                                     \
    X(LSHL_ADD_U64, "v_lshl_add_u64 %0, %0, 0, %1", D64)                                                          \
    X(ADD_CO_U32, "v_add_co_u32 %0, vcc, %1, %0", U)                                                              \
    X(PK_MAX_F16, "v_pk_max_f16 %0, %1, %0", U)                                                                   \
    X(CVT_F32_F16, "v_cvt_f32_f16 %0, %1\n v_add_u32 %1, %2, %1", C)                                            \
    X(LDEXP, "v_ldexp_f32 %0, %0, %1", FI)                                                                        \
    X(MAX_F32, "v_max_f32 %0, %1, %0", F)                                                                         \
    X(MIN_F32, "v_min_f32 %0, %1, %0", F)                                                                         \
    X(CVT_PKRTZ, "v_cvt_pkrtz_f16_f32 %1, %0, %0\n v_fma_f32 %0, %0, %3, %4", FU)                                \
    X(LOG, "v_log_f32 %0, %0", F1)

#define ASM_F(s) asm volatile(s : "+v"(x[c]) : "v"(a), "v"(b))
#define ASM_F1(s) asm volatile(s : "+v"(x[c]))
#define ASM_U(s) asm volatile(s : "+v"(n[c]) : "v"(ua), "v"(ub))
#define ASM_U1(s) asm volatile(s : "+v"(n[c]))
#define ASM_C(s) asm volatile(s : "=v"(x[c]), "+v"(n[c]) : "v"(ua))
#define ASM_FU(s) asm volatile(s : "+v"(x[c]), "=v"(n[c]) : "v"(ua), "v"(a), "v"(b))
#define ASM_D(s) asm volatile(s : "+v"(w[c]) : "v"(ua), "v"(ub) : "s0", "s1")
#define ASM_D64(s) asm volatile(s : "+v"(w[c]) : "v"(w2))
#define ASM_FI(s) asm volatile(s : "+v"(x[c]) : "v"(ua))
#define ASM_F2(s) asm volatile(s : "+v"(x[c]) : "v"(a), "v"(b) : "vcc")
#define ASM_P(s) if (c < kChains / 2) asm volatile(s : "+v"(p[c]) : "v"(a2), "v"(b2))
#define STEPS_F 1
#define STEPS_F1 1
#define STEPS_U 1
#define STEPS_U1 1
#define STEPS_C 2
#define STEPS_FU 2
#define STEPS_F2 2
#define STEPS_D 1
#define STEPS_D64 1
#define STEPS_FI 1
#define STEPS_P 1   // 8 chains: the printed figure is half the per-instruction cost

enum Kind {
#define KIND(name, s, t) name,
    OPS(KIND)
#undef KIND
};

template <Kind K>
__global__ __launch_bounds__(256) void chains(const float* __restrict__ in, unsigned long long* __restrict__ stamps,
                                              float* __restrict__ out, int iters) {
    const float a = in[threadIdx.x & 63], b = in[64 + (threadIdx.x & 63)];
    const unsigned int ua = __float_as_uint(a) | 1u, ub = __float_as_uint(b) | 3u;
    float x[kChains];
    unsigned int n[kChains];
#pragma unroll
    for (int c = 0; c < kChains; ++c) {
        x[c] = in[128 + c] + threadIdx.x * 1e-6f;
        n[c] = threadIdx.x + c;
    }
    typedef float v2 __attribute__((ext_vector_type(2)));
    v2 p[kChains / 2];
#pragma unroll
    for (int c = 0; c < kChains / 2; ++c) p[c] = v2{x[2 * c], x[2 * c + 1]};
    const v2 a2 = v2{a, a}, b2 = v2{b, b};
    unsigned long long w[kChains];
#pragma unroll
    for (int c = 0; c < kChains; ++c) w[c] = n[c] * 3ull;
    const unsigned long long w2 = ua * 7ull;
    __syncthreads();
    unsigned long long t0 = 0, r0 = 0;
    if (threadIdx.x == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < kChains; ++c) {
#define BODY(name, s, t)                                                                                            \
    if constexpr (K == name) ASM_##t(s);
            OPS(BODY)
#undef BODY
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        stamps[2 * blockIdx.x] = t1 - t0;
        stamps[2 * blockIdx.x + 1] = r1 - r0;
    }
    float s = 0.0f;
#pragma unroll
    for (int c = 0; c < kChains; ++c) s += x[c] + (float)n[c];
#pragma unroll
    for (int c = 0; c < kChains / 2; ++c) s += p[c].x + p[c].y;
#pragma unroll
    for (int c = 0; c < kChains; ++c) s += (float)w[c];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

// instructions per chain step: the two-instruction bodies (an add or fma keeps the chain dependent) count 2
template <Kind K>
void run(const float* d_in, int wps, const char* name, int per_step) {
    const int blocks = 256 * wps, iters = 2048;
    unsigned long long* st;
    float* out;
    (void)hipMalloc(&st, sizeof(unsigned long long) * 2 * blocks);
    (void)hipMalloc(&out, sizeof(float) * blocks * 256);
    hipLaunchKernelGGL(chains<K>, dim3(blocks), dim3(256), 0, 0, d_in, st, out, iters);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, 0);
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(chains<K>, dim3(blocks), dim3(256), 0, 0, d_in, st, out, iters);
    (void)hipEventRecord(e1, 0);
    (void)hipDeviceSynchronize();
    float ms = 0.0f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= 3.0f;
    std::vector<unsigned long long> h(2 * blocks);
    (void)hipMemcpy(h.data(), st, sizeof(unsigned long long) * 2 * blocks, hipMemcpyDeviceToHost);
    std::vector<double> clk(blocks);
    for (int b = 0; b < blocks; ++b) clk[b] = h[2 * b + 1] ? (double)h[2 * b] / (double)h[2 * b + 1] * 0.1 : 0.0;
    std::sort(clk.begin(), clk.end());
    const double per_simd = (double)blocks * 4.0 * iters * kChains * per_step / 1024.0 / (per_step == 0 ? 1 : 1);
    printf("%-12s waves/SIMD=%d  cycles per wave-instr per SIMD %.2f (%d instr per step; %.3f ms, %.2f GHz)\n", name, wps,
           ms * 1e-3 * clk[blocks / 2] * 1e9 / per_simd, per_step, ms, clk[blocks / 2]);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipFree(st);
    (void)hipFree(out);
}

int main() {
    std::vector<float> h(256, 1.0f);
    for (int i = 0; i < 64; ++i) { h[i] = 0.9999f; h[64 + i] = 1e-4f; }
    float* d_in;
    (void)hipMalloc(&d_in, sizeof(float) * 256);
    (void)hipMemcpy(d_in, h.data(), sizeof(float) * 256, hipMemcpyHostToDevice);
    for (int wps : {8}) {
#define RUN(name, s, t) if (name == FMA || name >= MAD_I64_I32) run<name>(d_in, wps, #name, STEPS_##t);
        OPS(RUN)
#undef RUN
    }
    (void)hipFree(d_in);
    return 0;
}
