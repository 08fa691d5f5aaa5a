// Packed vs unpacked f32 VALU throughput on gfx950 (8 independent chains per lane, 1..8 waves per SIMD, full chip).
// Build WITHOUT SLP vectorisation, so the scalar variants stay scalar (round 3's first version of this benchmark was
// built with plain -O3: the compiler packed its "scalar" chains, and both variants measured v_pk_fma_f32):
//   hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize -o pk_rate pk_rate.hip ; run on the GPU box.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float v2 __attribute__((ext_vector_type(2)));

enum Kind { FMA, PK_FMA, PK_MUL, PK_ADD, MIX_PK_CVT, MIX_FMA_CVT, FMA_DEP2, PK_FMA_DEP2 };

template <Kind K>
__global__ __launch_bounds__(256) void chains(float* out, int iters, float a, float b) {
    float v[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) v[c] = threadIdx.x * 0.001f + c + 0.5f;
    int iv[4] = {1, 2, 3, 4};
    for (int i = 0; i < iters; ++i) {
        if constexpr (K == FMA) {
#pragma unroll
            for (int c = 0; c < 8; ++c) v[c] = __builtin_fmaf(v[c], a, b);
        } else if constexpr (K == FMA_DEP2) {   // 2 chains: dependency latency bound per wave
#pragma unroll
            for (int c = 0; c < 8; ++c) v[c & 1] = __builtin_fmaf(v[c & 1], a, b);
        } else if constexpr (K == PK_FMA_DEP2) {
#pragma unroll
            for (int c = 0; c < 8; c += 2) {
                v2 x = {v[0], v[1]};
                x = __builtin_elementwise_fma(x, v2{a, a}, v2{b, b});
                v[0] = x.x;
                v[1] = x.y;
            }
        } else if constexpr (K == MIX_FMA_CVT) {   // 8 v_fma_f32 + 4 v_cvt_i32_f32 per iteration
#pragma unroll
            for (int c = 0; c < 8; ++c) v[c] = __builtin_fmaf(v[c], a, b);
#pragma unroll
            for (int c = 0; c < 4; ++c) iv[c] += (int)v[2 * c];
        } else {
#pragma unroll
            for (int c = 0; c < 8; c += 2) {
                v2 x = {v[c], v[c + 1]};
                if constexpr (K == PK_FMA || K == MIX_PK_CVT) x = __builtin_elementwise_fma(x, v2{a, a}, v2{b, b});
                if constexpr (K == PK_MUL) x = x * v2{a, a};
                if constexpr (K == PK_ADD) x = x + v2{b, b};
                v[c] = x.x;
                v[c + 1] = x.y;
            }
            if constexpr (K == MIX_PK_CVT) {   // 4 v_pk_fma_f32 + 4 v_cvt_i32_f32 per iteration
#pragma unroll
                for (int c = 0; c < 4; ++c) iv[c] += (int)v[2 * c];
            }
        }
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c) s += v[c];
    out[blockIdx.x * 256 + threadIdx.x] = s + (float)(iv[0] + iv[1] + iv[2] + iv[3]);
}

template <Kind K>
void run(int wps, const char* name, double instr_per_iter) {
    const int blocks = 256 * wps;   // 4 waves per block -> wps waves per SIMD over 1024 SIMDs
    float* out;
    (void)hipMalloc(&out, sizeof(float) * blocks * 256);
    const int iters = 4096;
    hipLaunchKernelGGL((chains<K>), dim3(blocks), dim3(256), 0, 0, out, iters, 0.999f, 0.001f);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((chains<K>), dim3(blocks), dim3(256), 0, 0, out, iters, 0.999f, 0.001f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= 5;
    const double per_simd = (double)blocks * 4 * iters * instr_per_iter / 1024.0;   // VALU wave-instructions per SIMD
    printf("%-34s waves/SIMD=%d  %.3f ms  cycles per VALU wave-instr per SIMD @2.4GHz = %.2f\n", name, wps, ms,
           (ms * 1e6 * 2.4) / per_simd);
    (void)hipFree(out);
}

int main() {
    for (int wps : {2, 4, 8}) {
        run<FMA>(wps, "v_fma_f32 x8", 8);
        run<PK_FMA>(wps, "v_pk_fma_f32 x4 (8 fma)", 4);
        run<PK_MUL>(wps, "v_pk_mul_f32 x4", 4);
        run<PK_ADD>(wps, "v_pk_add_f32 x4", 4);
        run<MIX_FMA_CVT>(wps, "8 v_fma_f32 + 4 cvt/add", 16);
        run<MIX_PK_CVT>(wps, "4 v_pk_fma_f32 + 4 cvt/add", 12);
        run<FMA_DEP2>(wps, "v_fma_f32 x8, 2 chains", 8);
        run<PK_FMA_DEP2>(wps, "v_pk_fma_f32 x4, 1 chain", 4);
    }
    return 0;
}
