// td_mask.hip — what does a wave-level global load cost in the vector-memory path (TA/TD/TCP),
// as a function of its active lanes, its width and its address footprint?  (round 4: the u8
// cross-lane sharing design, and the meaning of TCP_TOTAL_CACHE_ACCESSES per load on C3)
//
// Each wave issues ITER global loads from a 16 KiB table that stays in L1, so the loop is
// bound by the address/data path, not by L2 or HBM.  Case = (width, lane stride, active lanes):
//   lane l reads WIDTH bytes at (l * STRIDE + it * 1024 + block * 64) mod 16 KiB;
//   active lanes: 0 all 64, 1 even lanes (32), 2 lanes 0-31 (two whole quarter-waves idle),
//   3 lanes 0-15 (one quarter-wave), 4 every 4th lane (16, spread over all quarter-waves).
// The cases run in the order printed, each launched twice (warm, timed): under rocprofv3 --pmc
// the timed launch of case k is dispatch 2k + 1 (tools/experiments/r04/td_pmc.py reads them).
// Build: hipcc --offload-arch=gfx950 -O3 -o td_mask td_mask.hip ; run: ./td_mask (prints JSON)
#include <hip/hip_runtime.h>

#include <cstdio>

typedef unsigned u4 __attribute__((ext_vector_type(4)));
typedef unsigned u2 __attribute__((ext_vector_type(2)));

template <int WIDTH, int STRIDE, int PATTERN>
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
        const unsigned off = (lane * STRIDE + (unsigned)it * 1024 + blockIdx.x * 64) & (16384 - 1);
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

constexpr int kBlocks = 256 * 8;  // 8 workgroups of 4 waves per CU
constexpr int kIters = 4096;

template <int WIDTH, int STRIDE, int PATTERN>
void run(const unsigned *tab, unsigned *out, const char *name, bool last)
{
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL((td_kernel<WIDTH, STRIDE, PATTERN>), dim3(kBlocks), dim3(256), 0, 0, tab, out, kIters);
    hipEventRecord(a);
    hipLaunchKernelGGL((td_kernel<WIDTH, STRIDE, PATTERN>), dim3(kBlocks), dim3(256), 0, 0, tab, out, kIters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0.0f;
    hipEventElapsedTime(&ms, a, b);
    hipEventDestroy(a);
    hipEventDestroy(b);
    const double wave_loads_per_cu = (double)kBlocks * 4 * kIters / 256.0;
    std::printf("  {\"case\": \"%s\", \"width\": %d, \"stride\": %d, \"pattern\": %d, "
                "\"ns_per_wave_load_per_cu\": %.4f}%s\n",
                name, WIDTH, STRIDE, PATTERN, ms * 1e6 / wave_loads_per_cu, last ? "" : ",");
}

int main()
{
    unsigned *tab = nullptr, *out = nullptr;
    hipMalloc(&tab, 16384);
    hipMalloc(&out, 1 << 20);
    hipMemset(tab, 1, 16384);
    std::printf("{\"iters\": %d, \"wave_loads\": %.0f, \"cases\": [\n", kIters, (double)kBlocks * 4 * kIters);
    // active-lane patterns (contiguous 16-B lanes: 8 lines per full wave)
    run<16, 16, 0>(tab, out, "w16 all64", false);
    run<16, 16, 1>(tab, out, "w16 even32", false);
    run<16, 16, 2>(tab, out, "w16 lo32", false);
    run<16, 16, 3>(tab, out, "w16 lo16", false);
    run<16, 16, 4>(tab, out, "w16 every4th", false);
    run<8, 16, 0>(tab, out, "w8 all64 (16-B stride)", false);
    run<8, 16, 1>(tab, out, "w8 even32", false);
    run<8, 16, 2>(tab, out, "w8 lo32", false);
    run<4, 16, 0>(tab, out, "w4 all64 (16-B stride)", false);
    // address footprint at full occupancy: how TCP counts accesses per wave-level load
    run<16, 0, 0>(tab, out, "w16 broadcast (1 address)", false);
    run<4, 4, 0>(tab, out, "w4 contiguous (256 B: 2 lines)", false);
    run<8, 8, 0>(tab, out, "w8 contiguous (512 B: 4 lines)", false);
    run<16, 32, 0>(tab, out, "w16 stride 32 (2 KiB: 16 lines)", false);
    run<16, 64, 0>(tab, out, "w16 stride 64 (4 KiB: 32 lines)", false);
    run<16, 128, 0>(tab, out, "w16 stride 128 (64 lines)", false);
    run<4, 128, 0>(tab, out, "w4 stride 128 (64 lines)", true);
    std::printf("]}\n");
    hipFree(tab);
    hipFree(out);
    return 0;
}
