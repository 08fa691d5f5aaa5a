// gather_rate.hip — cost of a scattered vector-memory load on gfx950, per wave instruction, as a
// function of the number of distinct 128-B lines it touches, the load width and the active lanes.
// This is the ceiling model for SSAOGeneration (26 bilinear depth taps per pixel, scattered lines).
//
// Each wave issues ITERS buffer loads. For load k, lane l reads line (base_k + l % L) of a window
// of WIN bytes, at byte (l / L) * width % 128 inside that line, so exactly L distinct lines are touched
// (L = 1..64; one scalar line base per load, so no VALU work per load). The window decides where the lines live: 16 KiB (L1-resident) or 2 MiB (L2-resident).
// Output: one line per configuration: ns per wave-load per CU and cycles at 2.4 GHz.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

constexpr int ITERS = 64;

template <int WIDTH>
__global__ __launch_bounds__(256) void gather(const float* __restrict__ buf, unsigned win_lines, int log2L, int half,
                                              float* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const unsigned wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
    __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)buf, 0, win_lines * 128u, 0x00020000);
    // per lane: line (lane mod L), byte (lane div L) * WIDTH inside it; per load: a scalar line base
    const int voff = (lane & ((1 << log2L) - 1)) * 128 + (((lane >> log2L) * WIDTH) & 127);
    const unsigned base_mask = win_lines / 2 - 1;
    float acc = 0.0f;
    unsigned h = wave * 2654435761u;
    if (!half || lane < 32) {
#pragma unroll 16
        for (int k = 0; k < ITERS; ++k) {
            h = h * 1664525u + 1013904223u;
            const int soff = (int)(((h >> 8) & base_mask) * 128u);
            if (WIDTH == 8) {
                auto v = __builtin_amdgcn_raw_buffer_load_b64(rsrc, voff, soff, 0);
                acc += __builtin_bit_cast(float, (unsigned)v[0]) + __builtin_bit_cast(float, (unsigned)v[1]);
            } else if (WIDTH == 16) {
                auto v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, soff, 0);
                acc += __builtin_bit_cast(float, (unsigned)v[0]) + __builtin_bit_cast(float, (unsigned)v[3]);
            } else {
                auto v = __builtin_amdgcn_raw_buffer_load_b32(rsrc, voff, soff, 0);
                acc += __builtin_bit_cast(float, v);
            }
        }
    }
    if (acc == 12345.0f) out[wave] = acc;   // keep the loads alive
}

int main(int argc, char** argv) {
    const int blocks = argc > 1 ? atoi(argv[1]) : 256 * 32;
    float* buf = nullptr;
    float* out = nullptr;
    const size_t max_bytes = 64u << 20;
    if (hipMalloc(&buf, max_bytes) != hipSuccess || hipMalloc(&out, (size_t)blocks * 4 * sizeof(float)) != hipSuccess) return 1;
    (void)hipMemset(buf, 0, max_bytes);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    printf("width_bytes,window_kib,lines_per_instr,active_lanes,ns_per_wave_load_per_cu,cycles_at_2p4ghz\n");
    const unsigned wins[2] = {16u << 10, 2u << 20};
    for (int width : {4, 8, 16})
        for (unsigned win : wins)
            for (int half : {0, 1})
                for (int lg = 0; lg <= 6; ++lg) {
                    const int L = 1 << lg;
                    if (half && L == 64) continue;
                    auto launch = [&]() {
                        const unsigned wl = win / 128u;
                        if (width == 8) gather<8><<<blocks, 256>>>(buf, wl, lg, half, out);
                        else if (width == 16) gather<16><<<blocks, 256>>>(buf, wl, lg, half, out);
                        else gather<4><<<blocks, 256>>>(buf, wl, lg, half, out);
                    };
                    launch();
                    (void)hipDeviceSynchronize();
                    (void)hipEventRecord(e0);
                    for (int r = 0; r < 5; ++r) launch();
                    (void)hipEventRecord(e1);
                    (void)hipEventSynchronize(e1);
                    float ms = 0.0f;
                    (void)hipEventElapsedTime(&ms, e0, e1);
                    const double wave_loads = 5.0 * blocks * 4.0 * ITERS;
                    const double ns = ms * 1e6 / (wave_loads / cus);
                    printf("%d,%u,%d,%d,%.3f,%.1f\n", width, win >> 10, L, half ? 32 : 64, ns, ns * 2.4);
                }
    (void)hipFree(buf);
    (void)hipFree(out);
    return 0;
}
