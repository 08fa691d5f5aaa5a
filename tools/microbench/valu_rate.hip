// VALU issue-rate calibration on gfx950: N independent fma chains per lane, many waves per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 -o valu_rate valu_rate.hip ; run on the GPU box.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CHAINS, bool PACKED>
__global__ __launch_bounds__(256) void fma_chains(float* out, int iters, float a, float b) {
    float v[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) v[c] = threadIdx.x * 0.001f + c;
    typedef float v2 __attribute__((ext_vector_type(2)));
    for (int i = 0; i < iters; ++i) {
        if (PACKED) {
#pragma unroll
            for (int c = 0; c < CHAINS; c += 2) {
                v2 x = {v[c], v[c + 1]};
                x = __builtin_elementwise_fma(x, v2{a, a}, v2{b, b});
                v[c] = x.x;
                v[c + 1] = x.y;
            }
        } else {
#pragma unroll
            for (int c = 0; c < CHAINS; ++c) v[c] = __builtin_fmaf(v[c], a, b);
        }
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s += v[c];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int CHAINS, bool PACKED>
void run(int blocks, const char* name) {
    float* out;
    hipMalloc(&out, sizeof(float) * blocks * 256);
    const int iters = 4096;
    hipLaunchKernelGGL((fma_chains<CHAINS, PACKED>), dim3(blocks), dim3(256), 0, 0, out, iters, 0.999f, 0.001f);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((fma_chains<CHAINS, PACKED>), dim3(blocks), dim3(256), 0, 0, out, iters, 0.999f, 0.001f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= 5;
    const double instr = (double)blocks * 4 * iters * (PACKED ? CHAINS / 2 : CHAINS);   // wave-instructions
    const double per_simd = instr / 1024.0;                                              // 256 CUs x 4 SIMDs
    printf("%-28s blocks=%6d waves/SIMD=%5.1f  %.3f ms  wave-instr per SIMD per ns = %.3f  (cycles/instr @2.4GHz = %.2f)\n",
           name, blocks, blocks * 4 / 1024.0, ms, per_simd / (ms * 1e6), (ms * 1e6 * 2.4) / per_simd);
    hipFree(out);
}

int main() {
    for (int wps : {1, 2, 4, 8}) {
        const int blocks = 256 * wps;   // 4 waves per block -> wps waves per SIMD
        run<8, false>(blocks, "fma x8 chains");
        run<1, false>(blocks, "fma x1 chain (dependent)");
        run<8, true>(blocks, "pk_fma x8 chains");
    }
    return 0;
}
