// epilogue_fast.h -- branch-free statements of the dips epilogue for the
// batch kernels, each equal bit for bit to the specification in dips_math.h
// on the inputs the kernels feed it (checked exhaustively on the device by
// tools/altcheck.hip; profiles/r01_altcheck.txt):
//
//   recip_ge1(y)     == __fdiv_rn(1, y)        every f32 y in [1, 2^117)
//   exp_small(x)     == det_expf(x)            every f32 x in [-80, 80]
//   q_bits(x) & 0xFF == unorm_store(x)         every finite f32 x
//   sigmoid epilogue == visual_epilogue        every f32 diff in [-1, 1], k in {1, 2.5, 5, 7.3, 10, 160}
//
// The reference's f32 operation order is kept (no fused multiply-add where
// the specification rounds twice); the savings come from dropping branches
// and range checks that cannot trigger, Markstein's reciprocal without the
// v_div_scale/fixup scaffolding for y >= 1, one v_ldexp_f32 for the two-step
// 2^k scaling (exact while the result is normal: |x| <= 80), and the
// 2^23-offset add that rounds to an integer in the mantissa (no rint/cvt).
#pragma once

#include "dips_math.h"

namespace dips {

// |k| bound of the sigmoid scalar for which exp_small's argument stays in
// [-80, 80]: x = -k * diff / 2 with |diff| <= 1.
constexpr float kFastSigmoidMaxK = 160.0f;

// Correctly rounded 1/y for y >= 1 (Markstein: two Newton corrections of
// v_rcp_f32, each with one fused residual).
__device__ __forceinline__ float recip_ge1(float y) {
    const float r0 = __builtin_amdgcn_rcpf(y);
    const float e0 = __builtin_fmaf(-y, r0, 1.0f);
    const float r1 = __builtin_fmaf(r0, e0, r0);
    const float e1 = __builtin_fmaf(-y, r1, 1.0f);
    return __builtin_fmaf(e1, r1, r1);
}

// det_expf for |x| <= 80 (no special cases; same reduction and polynomial,
// the 2^k scaling as one exact ldexp).
__device__ __forceinline__ float exp_small(float x) {
    const float kf = rintf(x * 1.44269502162933349609375f);
    float r = x - kf * 0.693145751953125f;
    r = r - kf * 1.428606765330187045e-06f;
    float p = 1.3888889225e-3f;
    p = p * r + 8.3333337680e-3f;
    p = p * r + 4.1666667908e-2f;
    p = p * r + 1.6666667163e-1f;
    p = p * r + 0.5f;
    p = p * r + 1.0f;
    p = p * r + 1.0f;
    return __builtin_amdgcn_ldexpf(p, (int)kf);
}

// rgba8unorm store of a finite x: clamp(x * 255, 0, 255) rounded to an
// integer by adding 2^23 (RNE in the adder); the integer is the low byte of
// the returned bits.
__device__ __forceinline__ uint32_t q_bits(float x) {
    const float y = __builtin_amdgcn_fmed3f(x * 255.0f, 0.0f, 255.0f);
    return __float_as_uint(y + 8388608.0f);
}

// Pack the low bytes: gray (v, v, v, 255) or colour (r, g, b, 255) from the
// two quantised values hi / m (v_perm_b32 selector 0x0D = 0xFF).
__device__ __forceinline__ uint32_t pack_gray(uint32_t v) { return __builtin_amdgcn_perm(v, v, 0x0D000000u); }
__device__ __forceinline__ uint32_t pack_colour(uint32_t hi, uint32_t m, bool neg) {
    // neg: (hi, m, m) = hsl(0, s, 0.5); else (m, hi, m) = hsl(120, s, 0.5)
    return __builtin_amdgcn_perm(hi, m, neg ? 0x0D000004u : 0x0D000400u);
}

// RGBA texel (R, G, min(R, G), 255) of an epilogue-table entry R | G << 8
// (compat_batch_lut_kernel, alt_lut.h): visual_epilogue stores B = min(R, G)
// and A = 255 (compat_batch.hip).  The u16 halves of (R, G, R, FF) and
// (R, G, G, FF) are equal in the low half and (R | FF00, G | FF00) in the
// high one, so one packed u16 min finishes it.
__device__ __forceinline__ uint32_t lut_texel(uint32_t e) {
    typedef unsigned short us2 __attribute__((ext_vector_type(2)));
    const us2 x = __builtin_bit_cast(us2, __builtin_amdgcn_perm(e, e, 0x0D000100u));
    const us2 y = __builtin_bit_cast(us2, __builtin_amdgcn_perm(e, e, 0x0D010100u));
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(x, y));
}

// visual_epilogue(diff, FILT, k, COL) for finite diff in [-1, 1] and, with
// FILT = 0, |k| <= kFastSigmoidMaxK; kneg_half = -k / 2 (exact).
// FILT = 1 (inverse sigmoid) is not handled here.
template <int FILT, bool COL>
__device__ __forceinline__ uint32_t epilogue_fast(float diff, float kneg_half) {
    // map(): diff * 0.5 (exact); sigmoid: 1 / (1 + exp(-k * d)) - 0.5, where
    // -k * (diff * 0.5) == diff * (-k / 2) (one rounding either way)
    float d;
    if constexpr (FILT == 0) {
        d = recip_ge1(1.0f + exp_small(diff * kneg_half)) - 0.5f;
    } else {
        d = diff * 0.5f;
    }
    d = d * 5.0f;  // DIFF_SCALE / SENSITIVITY
    if constexpr (COL) {
        const float s = fabsf(d);
        const float m = 0.5f - s * 0.5f;  // l - chroma / 2 (chroma = s * 1)
        const float hi = s + m;           // chroma + m; x + m = m (x = chroma * 0 = 0)
        return pack_colour(q_bits(hi), q_bits(m), d < 0.0f);
    } else {
        return pack_gray(q_bits(0.5f - d));
    }
}

}  // namespace dips
