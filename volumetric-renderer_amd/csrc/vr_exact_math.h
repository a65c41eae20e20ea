// vr_exact_math.h — IEEE-exact float operations for the shading extension, in fewer
// instructions than the library's general sequences (device code; shared by vr_kernels.hip and
// the exhaustive checker host/rsq_check.hip).
//
// The oracle (oracle/oracle.c, march_pixel) normalises the gradient with 1.0f / sqrtf(g2):
// one correctly rounded square root, then one correctly rounded division.  Built with
// -fhip-fp32-correctly-rounded-divide-sqrt, hipcc emits for these a 16-instruction sqrt
// (denormal scaling, v_sqrt_f32, a +-1 ulp residual correction, inf/zero/NaN select) and an
// 11-instruction division (div_scale x2, rcp, 4 fma, div_fmas, div_fixup).  On the domain
// g2 in [2^-96, 2^96] the scaling and the special-value select are dead, and the reciprocal
// of a normal s needs no scaling either, so:
//   sqrt : v_sqrt_f32, then the same residual correction (r = g2 - s' s for s' = s -+ 1 ulp);
//   1 / s: v_rcp_f32, then one Markstein step q' = q + q (1 - s q) with fmas.
// Both are checked against the library's correctly rounded sqrtf and 1.0f / x for EVERY float
// of their domains (host/rsq_check.hip, tests/test_gpu_exact_math.py): 0 mismatches is the
// condition for using them; outside the domain the library sequences run.
#pragma once

#include <hip/hip_runtime.h>

namespace vr {

constexpr float kFastRsqLo = 0x1p-96f, kFastRsqHi = 0x1p96f;

// sqrt(x) correctly rounded, for x in [kFastRsqLo, kFastRsqHi]
__device__ __forceinline__ float sqrt_rn_normal(float x)
{
    const float s = __builtin_amdgcn_sqrtf(x);
    const float dn = __uint_as_float(__float_as_uint(s) - 1u);
    const float up = __uint_as_float(__float_as_uint(s) + 1u);
    const float r_dn = __builtin_fmaf(-dn, s, x);
    const float r_up = __builtin_fmaf(-up, s, x);
    float t = r_dn <= 0.0f ? dn : s;
    t = r_up > 0.0f ? up : t;
    return t;
}

// 1 / s correctly rounded, for s = sqrt_rn_normal(x) (s in [2^-48, 2^48])
__device__ __forceinline__ float rcp_rn_normal(float s)
{
    const float q = __builtin_amdgcn_rcpf(s);
    const float e = __builtin_fmaf(-s, q, 1.0f);
    return __builtin_fmaf(e, q, q);
}

// 1.0f / sqrtf(x) with the oracle's two IEEE roundings
__device__ __forceinline__ float inv_sqrt_ieee(float x)
{
    if (x >= kFastRsqLo && x <= kFastRsqHi) return rcp_rn_normal(sqrt_rn_normal(x));
    return 1.0f / sqrtf(x);
}

}  // namespace vr
