// rt_sqrt.h — correctly rounded fp32 sqrt and reciprocal with short common
// paths (gfx950).
//
// HIP lowers sqrtf (correctly rounded, the reference's sqrtf) to 17 VALU ops:
// a scale-up of inputs below 2^-96, v_sqrt_f32, two fma residual checks that
// step the result one ulp down or up, the scale-down, and a class check that
// passes +-0 / +inf through (LLVM AMDGPU lowerFSQRTF32).  For inputs in
// [2^-96, FLT_MAX] the scaling and the class check are identities, so
// sqrt_cr runs only the v_sqrt_f32 + residual steps there — the same
// operations in the same order, hence bit-identical — and falls back to
// sqrtf for everything else (tiny, zero, negative, inf, NaN).  When every
// lane of a wave is in range the fallback block is skipped.
//
// 1.0f / x is lowered to the v_div_scale / v_rcp_f32 / Newton fma /
// v_div_fmas / v_div_fixup sequence (11 ops).  For |x| in [2^-60, 2^60]
// v_div_scale leaves both operands unscaled (no exponent gap near 96, no
// denormal numerator, reciprocal or quotient), v_div_fmas is a plain fma
// and v_div_fixup returns its input, so rcp_cr runs the remaining v_rcp_f32 +
// six fma (the numerator is 1, so the first quotient is the reciprocal
// itself) and falls back to 1.0f / x outside that range.
// tools/sqrt_exhaustive.hip checks sqrt_cr == sqrtf and rcp_cr == 1.0f / x
// over all 2^32 inputs.
#pragma once
#include <hip/hip_runtime.h>

// the in-range bodies (callers guarantee the range)
__device__ __forceinline__ float sqrt_core(float x) {  // x in [2^-96, FLT_MAX]
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sm = __int_as_float(__float_as_int(s) - 1);  // one ulp down
    const float sp = __int_as_float(__float_as_int(s) + 1);  // one ulp up
    const float rm = __builtin_fmaf(-sm, s, x);
    const float rp = __builtin_fmaf(-sp, s, x);
    const float r = rm <= 0.0f ? sm : s;
    return rp > 0.0f ? sp : r;
}

__device__ __forceinline__ float rcp_core(float x) {  // |x| in [2^-60, 2^60]
    float r = __builtin_amdgcn_rcpf(x);
    const float e0 = __builtin_fmaf(-x, r, 1.0f);
    r = __builtin_fmaf(e0, r, r);
    const float e1 = __builtin_fmaf(-x, r, 1.0f);
    const float q = __builtin_fmaf(e1, r, r);
    const float e2 = __builtin_fmaf(-x, q, 1.0f);
    return __builtin_fmaf(e2, r, q);
}

#ifdef RT_PLAIN_SQRT  // A/B builds: the compiler's full sequences
__device__ __forceinline__ float sqrt_cr(float x) { return sqrtf(x); }
__device__ __forceinline__ float rcp_cr(float x) { return 1.0f / x; }
__device__ __forceinline__ float inv_length_cr(float s) { return 1.0f / sqrtf(s); }
#else
__device__ __forceinline__ float sqrt_cr(float x) {
    if (x >= 0x1p-96f && x <= 0x1.fffffep+127f) return sqrt_core(x);
    return sqrtf(x);
}

__device__ __forceinline__ float rcp_cr(float x) {
    if (fabsf(x) >= 0x1p-60f && fabsf(x) <= 0x1p+60f) return rcp_core(x);
    return 1.0f / x;
}

// 1 / sqrt(s) as the reference's normalize computes it: RN(1 / RN(sqrt(s))).
// One range check covers both steps: s in [2^-96, 2^118] gives
// sqrt(s) in [2^-48, 2^59].
__device__ __forceinline__ float inv_length_cr(float s) {
    if (s >= 0x1p-96f && s <= 0x1p+118f) return rcp_core(sqrt_core(s));
    return 1.0f / sqrtf(s);
}
#endif
