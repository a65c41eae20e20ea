// rsq_check — exhaustive GPU check of csrc/vr_exact_math.h against the library's correctly
// rounded sqrtf and division (the sequences hipcc emits under
// -fhip-fp32-correctly-rounded-divide-sqrt, which is what the march kernel runs outside the
// fast domain and what the CPU oracle's IEEE sqrtf / division compute).
//   sqrt_rn_normal(x) == sqrtf(x)     for every float x in [2^-96, 2^96]
//   rcp_rn_normal(s)  == 1.0f / s     for every float s in [2^-48, 2^48]
// Prints the counts checked and mismatched, and the first mismatches; exit status 0 iff none.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <cstring>

#include "../csrc/vr_exact_math.h"

__global__ void check_kernel(uint32_t lo_bits, uint32_t count, int which,
                             unsigned long long *bad, uint32_t *first)
{
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < count; i += stride) {
        const float x = __uint_as_float(lo_bits + i);
        float got, want;
        if (which == 0) {
            got = vr::sqrt_rn_normal(x);
            want = sqrtf(x);
        } else {
            got = vr::rcp_rn_normal(x);
            want = 1.0f / x;
        }
        if (__float_as_uint(got) != __float_as_uint(want)) {
            const unsigned long long n = atomicAdd(bad, 1ull);
            if (n < 4) first[n] = lo_bits + i;
        }
    }
}

static int run(const char *name, float lo, float hi, int which)
{
    uint32_t lo_bits, hi_bits;
    std::memcpy(&lo_bits, &lo, 4);
    std::memcpy(&hi_bits, &hi, 4);
    const uint32_t count = hi_bits - lo_bits + 1;
    unsigned long long *bad = nullptr;
    uint32_t *first = nullptr;
    if (hipMalloc(&bad, sizeof(*bad)) != hipSuccess || hipMalloc(&first, 4 * sizeof(*first)) != hipSuccess) {
        std::printf("hipMalloc failed\n");
        return 2;
    }
    hipMemset(bad, 0, sizeof(*bad));
    hipLaunchKernelGGL(check_kernel, dim3(4096), dim3(256), 0, 0, lo_bits, count, which, bad, first);
    unsigned long long nbad = 0;
    uint32_t f[4] = {0, 0, 0, 0};
    if (hipDeviceSynchronize() != hipSuccess) {
        std::printf("kernel failed\n");
        return 2;
    }
    hipMemcpy(&nbad, bad, sizeof(nbad), hipMemcpyDeviceToHost);
    hipMemcpy(f, first, sizeof(f), hipMemcpyDeviceToHost);
    std::printf("%s: %u floats in [%a, %a], mismatches %llu", name, count, lo, hi, nbad);
    for (unsigned long long k = 0; k < nbad && k < 4; ++k) {
        float v;
        std::memcpy(&v, &f[k], 4);
        std::printf(" %a", v);
    }
    std::printf("\n");
    hipFree(bad);
    hipFree(first);
    return nbad ? 1 : 0;
}

int main()
{
    int rc = run("sqrt_rn_normal", vr::kFastRsqLo, vr::kFastRsqHi, 0);
    rc |= run("rcp_rn_normal", 0x1p-48f, 0x1p48f, 1);
    return rc;
}
