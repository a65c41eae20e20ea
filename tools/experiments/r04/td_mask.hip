// td_mask.hip — does the vector-memory data return (TA/TD) cost scale with the active lanes of
// a load, and with its width?  (round 4, u8 cross-lane sharing design)
//
// Each wave issues ITER global loads from a 16 KiB table that stays in L1, so the loop is
// bound by the address/data path (TA/TD), not by L2 or HBM.  Patterns of active lanes per load:
//   0 all 64 lanes, 1 even lanes (32), 2 lanes 0-31 (two whole quarter-waves idle),
//   3 lanes 0-15 (one quarter-wave), 4 every 4th lane (16, spread over all quarter-waves)
// and widths 4, 8, 16 B per lane.  Lane l reads 16 B at (l * 16 + it * 1024) mod 16 KiB: every
// wave-level load touches 8 consecutive 128-B lines when all lanes are active.
// Build: hipcc --offload-arch=gfx950 -O3 -o td_mask td_mask.hip ; run: ./td_mask  (prints JSON)
#include <hip/hip_runtime.h>

#include <cstdio>

typedef unsigned u4 __attribute__((ext_vector_type(4)));
typedef unsigned u2 __attribute__((ext_vector_type(2)));

template <int WIDTH, int PATTERN>
__global__ __launch_bounds__(256) void td_kernel(const unsigned *__restrict__ tab, unsigned *out, int iters)
{
    const unsigned lane = threadIdx.x & 63;
    bool on;
    switch (PATTERN) {
        case 0: on = true; break;
        case 1: on = (lane & 1) == 0; break;
        case 2: on = lane < 32; break;
        case 3: on = lane < 16; break;
        default: on = (lane & 3) == 0; break;
    }
    unsigned acc = 0;
    const char *base = reinterpret_cast<const char *>(tab);
    for (int it = 0; it < iters; ++it) {
        const unsigned off = (lane * 16 + (unsigned)it * 1024 + blockIdx.x * 64) & (16384 - 1);
        if (on) {
            if constexpr (WIDTH == 16) {
                const u4 v = *reinterpret_cast<const u4 *>(base + off);
                acc ^= v.x ^ v.y ^ v.z ^ v.w;
            } else if constexpr (WIDTH == 8) {
                const u2 v = *reinterpret_cast<const u2 *>(base + off);
                acc ^= v.x ^ v.y;
            } else {
                acc ^= *reinterpret_cast<const unsigned *>(base + off);
            }
        }
    }
    if (acc == 0x12345678u) out[blockIdx.x] = acc;  // keeps the loads
}

template <int WIDTH, int PATTERN>
float run(const unsigned *tab, unsigned *out, int iters)
{
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int blocks = 256 * 8;  // 8 workgroups of 4 waves per CU
    hipLaunchKernelGGL((td_kernel<WIDTH, PATTERN>), dim3(blocks), dim3(256), 0, 0, tab, out, iters);
    hipEventRecord(a);
    hipLaunchKernelGGL((td_kernel<WIDTH, PATTERN>), dim3(blocks), dim3(256), 0, 0, tab, out, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0.0f;
    hipEventElapsedTime(&ms, a, b);
    hipEventDestroy(a);
    hipEventDestroy(b);
    return ms;
}

int main()
{
    unsigned *tab = nullptr, *out = nullptr;
    hipMalloc(&tab, 16384);
    hipMalloc(&out, 1 << 20);
    hipMemset(tab, 1, 16384);
    const int iters = 4096;
    const double loads = 256.0 * 8 * 4 * iters;  // wave-level loads per launch
    std::printf("{\"iters\": %d, \"wave_loads\": %.0f, \"ns_per_wave_load_per_cu\": {\n", iters, loads);
    const char *pn[5] = {"all64", "even32", "lo32", "lo16", "every4th"};
    float t[3][5];
    t[0][0] = run<16, 0>(tab, out, iters); t[0][1] = run<16, 1>(tab, out, iters);
    t[0][2] = run<16, 2>(tab, out, iters); t[0][3] = run<16, 3>(tab, out, iters);
    t[0][4] = run<16, 4>(tab, out, iters);
    t[1][0] = run<8, 0>(tab, out, iters); t[1][1] = run<8, 1>(tab, out, iters);
    t[1][2] = run<8, 2>(tab, out, iters); t[1][3] = run<8, 3>(tab, out, iters);
    t[1][4] = run<8, 4>(tab, out, iters);
    t[2][0] = run<4, 0>(tab, out, iters); t[2][1] = run<4, 1>(tab, out, iters);
    t[2][2] = run<4, 2>(tab, out, iters); t[2][3] = run<4, 3>(tab, out, iters);
    t[2][4] = run<4, 4>(tab, out, iters);
    const int w[3] = {16, 8, 4};
    for (int i = 0; i < 3; ++i) {
        std::printf("  \"w%d\": {", w[i]);
        for (int p = 0; p < 5; ++p)
            std::printf("\"%s\": %.3f%s", pn[p], t[i][p] * 1e6 / (loads / 256.0), p < 4 ? ", " : "");
        std::printf("}%s\n", i < 2 ? "," : "");
    }
    std::printf("}}\n");
    hipFree(tab);
    hipFree(out);
    return 0;
}
