// Issue cost of the VALU instruction kinds the clouds kernels use, on gfx950: 8 independent chains per lane,
// 8 waves per SIMD (full chip), cycles per wave-instruction per SIMD at 2.4 GHz. Build:
//   hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize -o valu_mix valu_mix.hip ; run on the GPU box.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

enum Kind { FMA, EXP, SQRT, RCP, CVT_I32, CVT_F32, FLOOR, DOT2, PERM, MIX_EXP_2FMA, MIX_SQRT_4FMA };

template <Kind K>
__device__ __forceinline__ float step(float v, float a, float b) {
    if constexpr (K == FMA) return __builtin_fmaf(v, a, b);
    if constexpr (K == EXP) return __builtin_amdgcn_exp2f(v);
    if constexpr (K == SQRT) return __builtin_amdgcn_sqrtf(v);
    if constexpr (K == RCP) return __builtin_amdgcn_rcpf(v);
    if constexpr (K == CVT_I32) return __builtin_bit_cast(float, (int)v);
    if constexpr (K == CVT_F32) return (float)__builtin_bit_cast(unsigned, v);
    if constexpr (K == FLOOR) return __builtin_floorf(v);
    if constexpr (K == DOT2) {
        const unsigned u = __builtin_bit_cast(unsigned, v);
        return __builtin_bit_cast(float, __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, u), __builtin_bit_cast(u16x2, u), 7u, false));
    }
    if constexpr (K == PERM) {
        const unsigned u = __builtin_bit_cast(unsigned, v);
        return __builtin_bit_cast(float, __builtin_amdgcn_perm(u, u ^ 0x55u, 0x0c010c00u));
    }
    return v;
}

template <Kind K>
__global__ __launch_bounds__(256) void chains(float* out, int iters, float a, float b) {
    constexpr int C = 8;
    float v[C];
#pragma unroll
    for (int c = 0; c < C; ++c) v[c] = threadIdx.x * 0.001f + c + 0.5f;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < C; ++c) {
            if constexpr (K == MIX_EXP_2FMA) {
                v[c] = __builtin_fmaf(v[c], a, b);
                v[c] = __builtin_fmaf(v[c], a, b);
                v[c] = __builtin_amdgcn_exp2f(v[c]);
            } else if constexpr (K == MIX_SQRT_4FMA) {
                v[c] = __builtin_fmaf(v[c], a, b);
                v[c] = __builtin_fmaf(v[c], a, b);
                v[c] = __builtin_fmaf(v[c], a, b);
                v[c] = __builtin_fmaf(v[c], a, b);
                v[c] = __builtin_amdgcn_sqrtf(v[c]);
            } else {
                v[c] = step<K>(v[c], a, b);
            }
        }
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < C; ++c) s += v[c];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <Kind K>
void run(const char* name, int per_iter) {
    const int blocks = 256 * 8;   // 8 waves per SIMD
    float* out;
    (void)hipMalloc(&out, sizeof(float) * blocks * 256);
    const int iters = 2048;
    chains<K><<<blocks, 256>>>(out, iters, 0.999f, 0.001f);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) chains<K><<<blocks, 256>>>(out, iters, 0.999f, 0.001f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= 5;
    const double instr = (double)blocks * 4 * iters * 8 * per_iter;   // wave-instructions
    const double per_simd = instr / 1024.0;
    printf("%-22s %.3f ms  cycles per wave-instr per SIMD @2.4GHz = %.2f\n", name, ms, (ms * 1e6 * 2.4) / per_simd);
    (void)hipFree(out);
}

int main() {
    run<FMA>("v_fma_f32", 1);
    run<EXP>("v_exp_f32", 1);
    run<SQRT>("v_sqrt_f32", 1);
    run<RCP>("v_rcp_f32", 1);
    run<CVT_I32>("v_cvt_i32_f32", 1);
    run<CVT_F32>("v_cvt_f32_u32", 1);
    run<FLOOR>("v_floor_f32", 1);
    run<DOT2>("v_dot2_u32_u16", 1);
    run<PERM>("v_perm_b32(+xor)", 2);
    run<MIX_EXP_2FMA>("2 fma + exp", 3);
    run<MIX_SQRT_4FMA>("4 fma + sqrt", 5);
    return 0;
}
