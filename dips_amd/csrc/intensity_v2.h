// intensity_v2.h -- conversion-free exact get_intensity for RGB8/RGBA8 vecs
// (shared by series_v2.hip and alt_kernels.hip).
//
// With J = max+min and E = P(max) + P(min), P(c) = the largest power of two
// <= c,
//     2 * get_intensity = u(max) + u(min) = RNE(J * 65793 * 2^-24 + E * 2^-31)
// exactly (u(c) = c/255 rounds UP to c*65793*2^-24 + 2^(msb(c)-31); checked
// exhaustively in tests/test_oracle.py and over all 2^24 RGB triples on the
// device by tools/i2check.hip).  J enters one v_fma_mix_f32 as J * 2^-9 (a
// normal f16) and E comes from the exponent field of the f16 value c * 2^-9
// (one packed f16 multiply + an AND).  Results live in the exactly scaled
// domain I2s = 2 * I * 2^22.
#pragma once

#include "series_common.h"

namespace dips {

typedef _Float16 h2 __attribute__((ext_vector_type(2)));

// 65793 * 2^7: J * 2^-9 (normal f16) times this is J * 65793 / 4.
constexpr float kI2Mul = 8421504.0f;
// I = I2s * 2^-23 (exact).
constexpr float kI2sToI = 1.0f / 8388608.0f;

// v_fma_mix_f32 on the low / high f16 halves of j and e (f32 multiplier k):
// one fused op, the f16 operands widened exactly.  (hipcc does not form it
// from fmaf((float)half, k, (float)half): it emits two v_cvt_f32_f16 and a
// v_pk_fma_f32.)  The f16 operands must be NORMAL numbers: with an f16
// denormal operand the gfx950 result is not the exact fused value
// (tools/i2check.hip), hence J enters as J * 2^-9.
__device__ __forceinline__ float fma_mix_lo(uint32_t j, float k, uint32_t e) {
    float r;
    asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1]" : "=v"(r) : "v"(j), "s"(k), "v"(e));
    return r;
}
__device__ __forceinline__ float fma_mix_hi(uint32_t j, float k, uint32_t e) {
    float r;
    asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[1,0,1] op_sel_hi:[1,0,1]" : "=v"(r) : "v"(j), "s"(k), "v"(e));
    return r;
}

// c * 2^-9 as normal f16s from the u16 pair read as f16 denormals
// (c * 2^-24) times 2^15 (exact).
__device__ __forceinline__ h2 norm_h2(h2 c) { return c * (h2){(_Float16)32768.0f, (_Float16)32768.0f}; }
// sign and exponent bits only: the largest power of two <= x (0 for 0)
__device__ __forceinline__ h2 pow2_floor_h2(h2 x) {
    return __builtin_bit_cast(h2, __builtin_bit_cast(uint32_t, x) & 0xFC00FC00u);
}

// Derived state of one vec (4 px): the scaled intensity pairs I2s
// (i[0] = pixels 0, 1; i[1] = pixels 2, 3).
struct St2 {
    f32x2 i[2];
};

// X32: the same intensities times 32 (I2s * 32 = I * 2^28): k * 32 is a
// free constant, E * 32 one packed f16 multiply per pixel pair (E * 2^-9 <=
// 0.5, so E * 2^-4 <= 16 stays exact), and the fused multiply-add rounds the
// exactly scaled sum -- a power-of-two scaling of the same f32 results.
template <int C, int CH, bool X32 = false>
__device__ __forceinline__ void derive_v2(const uint32_t (&d)[Fmt<C>::NDW], St2& s) {
    u16x2 r[2], g[2], b[2];
    pair_planes<C>(d, r, g, b);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        // max / min of the channels on the u16 planes read as f16 denormals
        // (c * 2^-24: same order as the bytes): one v_pk_maximum3_f16 and one
        // v_pk_minimum3_f16 per pixel pair
        h2 mx, mn;
        if constexpr (CH == 0) {
            const h2 rh = __builtin_bit_cast(h2, r[k]), gh = __builtin_bit_cast(h2, g[k]), bh = __builtin_bit_cast(h2, b[k]);
            mx = __builtin_elementwise_maximum(__builtin_elementwise_maximum(rh, gh), bh);
            mn = __builtin_elementwise_minimum(__builtin_elementwise_minimum(rh, gh), bh);
        } else {
            mx = mn = __builtin_bit_cast(h2, CH == 1 ? r[k] : (CH == 2 ? g[k] : b[k]));
        }
        const h2 xn = norm_h2(mx), nn = norm_h2(mn);
        const uint32_t jn = __builtin_bit_cast(uint32_t, xn + nn);  // J * 2^-9, exact
        h2 eh = pow2_floor_h2(xn) + pow2_floor_h2(nn);
        if constexpr (X32) eh = eh * (h2){(_Float16)32.0f, (_Float16)32.0f};
        const uint32_t e = __builtin_bit_cast(uint32_t, eh);
        constexpr float kmul = X32 ? kI2Mul * 32.0f : kI2Mul;
        s.i[k] = f32x2{fma_mix_lo(jn, kmul, e), fma_mix_hi(jn, kmul, e)};
    }
}

}  // namespace dips
