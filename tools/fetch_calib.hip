// FETCH_SIZE calibration for the march's access pattern (MI355X_MICROARCH.md: on gfx950
// FETCH_SIZE reports 1/2 of the bytes of a wide coalesced streaming read; other patterns are
// uncalibrated).  Three kernels over a 4 GiB buffer, each reading a known number of bytes once:
//   stream     coalesced 16 B per lane                       known: 4 GiB
//   gather     16 B per lane, a wave's 64 lanes on 8 random 128-B lines, 8 lanes per line
//              (each line read once, whole)                 known: 4 GiB
//   half       as gather, 4 lanes per line: the first 64 B of each line only
//                                                            known: 2 GiB of requested bytes
// Run under rocprofv3 --pmc FETCH_SIZE (tools/fetch_calib.sh); prints the known bytes.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
            std::exit(1);                                                           \
        }                                                                           \
    } while (0)

constexpr size_t kLines = (size_t)1 << 25;  // 128-B lines: 4 GiB
constexpr size_t kSlots = kLines * 8;       // 16-B slots

__global__ __launch_bounds__(256) void stream_kernel(const float4 *__restrict__ a, float *out)
{
    float s = 0.0f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < kSlots;
         i += (size_t)gridDim.x * blockDim.x) {
        const float4 v = a[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 12345.678f) out[0] = s;  // keeps the loads; never true for the zero buffer
}

// lane l of a wave reads slot (l % LPL) of line perm[wave * (64 / LPL) + l / LPL]
template <int LPL>
__global__ __launch_bounds__(256) void gather_kernel(const float4 *__restrict__ a,
                                                     const uint32_t *__restrict__ perm,
                                                     float *out)
{
    constexpr int kLinesPerWave = 64 / LPL;
    const size_t waves = kLines / kLinesPerWave;
    const uint32_t lane = threadIdx.x & 63;
    float s = 0.0f;
    for (size_t w = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) / 64; w < waves;
         w += (size_t)gridDim.x * blockDim.x / 64) {
        const size_t line = perm[w * kLinesPerWave + lane / LPL];
        const float4 v = a[line * 8 + lane % LPL];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 12345.678f) out[0] = s;
}

int main()
{
    float4 *a = nullptr;
    uint32_t *perm = nullptr;
    float *out = nullptr;
    CK(hipMalloc(&a, kSlots * sizeof(float4)));
    CK(hipMemset(a, 0, kSlots * sizeof(float4)));
    CK(hipMalloc(&out, 4));
    std::vector<uint32_t> p(kLines);
    for (size_t i = 0; i < kLines; ++i) p[i] = (uint32_t)i;
    uint64_t x = 88172645463325252ull;
    for (size_t i = kLines - 1; i > 0; --i) {  // Fisher-Yates, xorshift64
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        std::swap(p[i], p[x % (i + 1)]);
    }
    CK(hipMalloc(&perm, kLines * 4));
    CK(hipMemcpy(perm, p.data(), kLines * 4, hipMemcpyHostToDevice));
    const dim3 grid(256 * 8 * 4), block(256);
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(stream_kernel, grid, block, 0, 0, a, out);
        hipLaunchKernelGGL(gather_kernel<8>, grid, block, 0, 0, a, perm, out);
        hipLaunchKernelGGL(gather_kernel<4>, grid, block, 0, 0, a, perm, out);
    }
    CK(hipDeviceSynchronize());
    std::printf("{\"stream_known_bytes\": %zu, \"gather_known_bytes\": %zu, "
                "\"half_requested_bytes\": %zu, \"perm_bytes\": %zu}\n",
                kSlots * 16, kLines * 128, kLines * 64, kLines * 4);
    (void)hipFree(a);
    (void)hipFree(perm);
    (void)hipFree(out);
    return 0;
}
