// VALU issue rate on gfx950: cycles per wave64 VALU instruction per SIMD, measured in SHADER cycles
// (s_memtime stamps inside the kernel, not events at an assumed 2.4 GHz) with 16 independent chains per lane and
// VGPR operands only (no SGPR constant-bus limit), at 1 / 2 / 4 / 8 waves per SIMD over the full chip.
//
// Every instruction is an inline-asm statement, so the stream is exactly what is written: no SLP packing, no
// reordering, no dead-code removal. A block is 256 lanes (4 waves, one per SIMD of its CU); 256 x wps blocks put
// wps waves on every SIMD (all resident: a few VGPRs per lane). Each block's first lane stamps s_memtime and
// s_memrealtime before and after the loop (after a barrier, so every wave of the block has arrived); the effective
// clock is dmemtime / dmemrealtime x 100 MHz (MI355X_MICROARCH.md, DVFS (6)).
//   cycles per wave-instruction per SIMD = median block dmemtime / (wps x instructions per wave)
// Build: hipcc --offload-arch=gfx950 -O3 -o valu_rate valu_rate.hip ; run on the GPU box.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef float v2 __attribute__((ext_vector_type(2)));

enum Kind { FMA, PK_FMA, ADD_U32, MIX_FMA_ADD, MIX_FMA_CVT, MUL_F32, EXP_F32, MIX_FMA_EXP, MIX_PK_ADD };
constexpr int kChains = 16;

template <Kind K>
__global__ __launch_bounds__(256) void chains(const float* __restrict__ in, unsigned long long* __restrict__ stamps,
                                              float* __restrict__ out, int iters) {
    const float a = in[threadIdx.x & 63], b = in[64 + (threadIdx.x & 63)];   // per-lane VGPR operands
    float x[kChains];
    unsigned int n[kChains];
#pragma unroll
    for (int c = 0; c < kChains; ++c) {
        x[c] = in[128 + c] + threadIdx.x * 1e-6f;
        n[c] = threadIdx.x + c;
    }
    const unsigned int k = (unsigned int)in[200];
    v2 p[kChains / 2];
#pragma unroll
    for (int c = 0; c < kChains / 2; ++c) p[c] = v2{x[2 * c], x[2 * c + 1]};
    const v2 a2 = v2{a, a}, b2 = v2{b, b};
    __syncthreads();
    unsigned long long t0 = 0, r0 = 0;
    if (threadIdx.x == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < kChains; ++c) {
            if constexpr (K == FMA) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x[c]) : "v"(a), "v"(b));
            if constexpr (K == MUL_F32) asm volatile("v_mul_f32 %0, %1, %0" : "+v"(x[c]) : "v"(a));
            if constexpr (K == ADD_U32) asm volatile("v_add_u32 %0, %1, %0" : "+v"(n[c]) : "v"(k));
            if constexpr (K == EXP_F32) asm volatile("v_exp_f32 %0, %0" : "+v"(x[c]));
            if constexpr (K == PK_FMA) {
                if (c < kChains / 2) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(p[c]) : "v"(a2), "v"(b2));
            }
            if constexpr (K == MIX_FMA_ADD) {   // 1:1 f32 fma and u32 add, alternating
                if (c & 1) asm volatile("v_add_u32 %0, %1, %0" : "+v"(n[c]) : "v"(k));
                else asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x[c]) : "v"(a), "v"(b));
            }
            if constexpr (K == MIX_FMA_CVT) {   // 1:1 f32 fma and f32 -> i32 convert, alternating
                if (c & 1) asm volatile("v_cvt_i32_f32 %0, %1" : "=v"(n[c]) : "v"(x[c - 1]));
                else asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x[c]) : "v"(a), "v"(b));
            }
            if constexpr (K == MIX_FMA_EXP) {   // 3:1 f32 fma and exp
                if ((c & 3) == 3) asm volatile("v_exp_f32 %0, %0" : "+v"(x[c]));
                else asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x[c]) : "v"(a), "v"(b));
            }
            if constexpr (K == MIX_PK_ADD) {    // 1:1 packed f32 fma and u32 add
                if (c & 1) asm volatile("v_add_u32 %0, %1, %0" : "+v"(n[c]) : "v"(k));
                else asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(p[c / 2]) : "v"(a2), "v"(b2));
            }
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
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <Kind K>
void run(const float* d_in, int wps, const char* name, int instr_per_iter) {
    const int blocks = 256 * wps;
    const int iters = 2048;
    unsigned long long* st;
    float* out;
    (void)hipMalloc(&st, sizeof(unsigned long long) * 2 * blocks);
    (void)hipMalloc(&out, sizeof(float) * blocks * 256);
    hipLaunchKernelGGL(chains<K>, dim3(blocks), dim3(256), 0, 0, d_in, st, out, iters);   // warm-up (clocks)
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
    std::vector<double> cyc(blocks), clk(blocks);
    for (int b = 0; b < blocks; ++b) {
        cyc[b] = (double)h[2 * b];
        clk[b] = h[2 * b + 1] ? (double)h[2 * b] / (double)h[2 * b + 1] * 0.1 : 0.0;   // GHz
    }
    std::sort(cyc.begin(), cyc.end());
    std::sort(clk.begin(), clk.end());
    const double per_wave = (double)iters * instr_per_iter;
    // whole launch: event time x the in-kernel clock over the wave-instructions each of the 1024 SIMDs issues
    const double per_simd = (double)blocks * 4.0 * per_wave / 1024.0;
    printf("%-26s waves/SIMD=%d  cycles/wave-instr/SIMD: launch %.2f, median block %.2f  (%.3f ms, clock %.2f GHz)\n",
           name, wps, ms * 1e-3 * clk[blocks / 2] * 1e9 / per_simd, cyc[blocks / 2] / (wps * per_wave), ms,
           clk[blocks / 2]);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipFree(st);
    (void)hipFree(out);
}

int main() {
    std::vector<float> h(256, 1.0f);
    for (int i = 0; i < 64; ++i) { h[i] = 0.9999f; h[64 + i] = 1e-4f; }
    h[200] = 3.0f;
    float* d_in;
    (void)hipMalloc(&d_in, sizeof(float) * 256);
    (void)hipMemcpy(d_in, h.data(), sizeof(float) * 256, hipMemcpyHostToDevice);
    for (int wps : {1, 2, 4, 8}) {
        run<FMA>(d_in, wps, "v_fma_f32 x16", kChains);
        run<MUL_F32>(d_in, wps, "v_mul_f32 x16", kChains);
        run<PK_FMA>(d_in, wps, "v_pk_fma_f32 x8", kChains / 2);
        run<ADD_U32>(d_in, wps, "v_add_u32 x16", kChains);
        run<EXP_F32>(d_in, wps, "v_exp_f32 x16", kChains);
        run<MIX_FMA_ADD>(d_in, wps, "8 fma + 8 add_u32", kChains);
        run<MIX_FMA_CVT>(d_in, wps, "8 fma + 8 cvt_i32", kChains);
        run<MIX_FMA_EXP>(d_in, wps, "12 fma + 4 exp", kChains);
        run<MIX_PK_ADD>(d_in, wps, "8 pk_fma + 8 add_u32", kChains);
    }
    (void)hipFree(d_in);
    return 0;
}
