// dips_math.h -- scalar arithmetic shared by the HIP kernels of dips_amd.
//
// Every function here is the device-side statement of one piece of the
// reference's WGSL (RubenMovsesyan/DiPs, dips/src/gpu/shaders/*.wgsl).  The
// f32 operation order is part of the specification: the library is compiled
// with -ffp-contract=off so no FMA contraction changes a rounding.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dips {

// rgba8unorm texel load: c / 255 (dips_shader.wgsl:124,138,192,213).
// Correctly rounded f32 division (HIP's default; __fdiv_rn makes it explicit).
__device__ __forceinline__ float unorm_load(uint32_t c) {
    return __fdiv_rn((float)c, 255.0f);
}

// rgba8unorm texel store (dips_shader.wgsl:187,239): clamp to [0,1], *255,
// round half to even; NaN is stored as 0 (pinned).
__device__ __forceinline__ uint32_t unorm_store(float x) {
    if (!(x > 0.0f)) return 0u;
    if (x > 1.0f) x = 1.0f;
    return (uint32_t)rintf(x * 255.0f);
}

__device__ __forceinline__ float bits_f(uint32_t b) { return __uint_as_float(b); }
__device__ __forceinline__ float pow2i(int n) { return bits_f((uint32_t)(n + 127) << 23); }

// Deterministic f32 exp used for the sigmoid filter (dips_shader.wgsl:111).
// Cody-Waite reduction + degree-6 Horner polynomial; specification in
// DESIGN.md "f32 transcendental functions".
__device__ __forceinline__ float det_expf(float x) {
    if (x != x) return x;
    if (x > 88.72283935546875f) return __builtin_inff();
    if (x < -103.97208404541016f) return 0.0f;
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
    const int k = (int)kf;
    const int k1 = k / 2;
    p = p * pow2i(k1);
    p = p * pow2i(k - k1);
    return p;
}

// Deterministic f32 log used for the inverse sigmoid (dips_shader.wgsl:117).
__device__ __forceinline__ float det_logf(float x) {
    if (x != x || x < 0.0f) return __builtin_nanf("");
    if (x == 0.0f) return -__builtin_inff();
    if (x == __builtin_inff()) return __builtin_inff();
    uint32_t bits = __float_as_uint(x);
    int e = 0;
    if (bits < 0x00800000u) {
        x = x * 8388608.0f;
        bits = __float_as_uint(x);
        e = -23;
    }
    e += (int)(bits >> 23) - 127;
    float m = bits_f((bits & 0x007FFFFFu) | 0x3F800000u);
    if (m > 1.41421353816986083984375f) {
        m = m * 0.5f;
        e += 1;
    }
    const float f = m - 1.0f;
    const float s = __fdiv_rn(f, 2.0f + f);
    const float z = s * s;
    float t = 1.1111111194e-1f;
    t = t * z + 1.4285714924e-1f;
    t = t * z + 2.0000000298e-1f;
    t = t * z + 3.3333334327e-1f;
    t = t * z + 1.0f;
    const float lm = (2.0f * s) * t;
    const float ef = (float)e;
    return ef * 0.693145751953125f + (ef * 1.428606765330187045e-06f + lm);
}

// get_intensity (dips_shader.wgsl:64-82) of an RGB byte triple.
__device__ __forceinline__ float intensity_rgb(uint32_t r, uint32_t g, uint32_t b, uint32_t chroma) {
    const float fr = unorm_load(r), fg = unorm_load(g), fb = unorm_load(b);
    if (chroma == 1u) return fr;
    if (chroma == 2u) return fg;
    if (chroma == 3u) return fb;
    const float cmax = fmaxf(fmaxf(fr, fg), fb);
    const float cmin = fminf(fminf(fr, fg), fb);
    return (cmax + cmin) / 2.0f;
}

// Filter + sensitivity + colour epilogue of compute_main
// (dips_shader.wgsl:213-239; map :97-105, sigmoid :108-112,
// inv_sigmoid :114-118, diff_to_color :30-36, hsl_to_rgb :40-62).
// Returns packed RGBA8 (alpha 255).
__device__ __forceinline__ uint32_t visual_epilogue(float diff, uint32_t filter, float k,
                                                    bool colorize) {
    diff = diff * ((0.5f - -0.5f) / (1.0f - -1.0f));
    if (filter == 0u) {
        diff = __fdiv_rn(1.0f, 1.0f + det_expf(-k * diff)) - 0.5f;
    } else if (filter == 1u) {
        diff = __fdiv_rn(-det_logf(__fdiv_rn(1.0f, diff + 0.5f) - 1.0f), k);
    }
    diff *= 5.0f;
    float r, g, b;
    if (colorize) {
        // hsl_to_rgb(h, s, 0.5) with h = 0 (diff < 0) or 120: chroma = s,
        // x = chroma * 0, m = 0.5 - chroma / 2.
        const bool neg = diff < 0.0f;
        const float s = neg ? fabsf(diff) : diff;
        const float chroma = s * (1.0f - fabsf(2.0f * 0.5f - 1.0f));
        const float x = chroma * (1.0f - fabsf(0.0f - 1.0f));
        const float m = 0.5f - chroma / 2.0f;
        if (neg) { r = chroma + m; g = x + m; b = 0.0f + m; }
        else     { r = 0.0f + m; g = chroma + m; b = x + m; }
    } else {
        r = g = b = 0.5f - diff;
    }
    return unorm_store(r) | (unorm_store(g) << 8) | (unorm_store(b) << 16) | (255u << 24);
}

// Upper median of four (the 4-entry bubble sort of dips_shader.wgsl:196-211
// under naga's Restrict bounds policy is a full sort; element [2]).
__device__ __forceinline__ float upper_median4(float a, float b, float c, float d) {
    const float lo1 = fminf(a, b), hi1 = fmaxf(a, b);
    const float lo2 = fminf(c, d), hi2 = fmaxf(c, d);
    // The two middle elements of the sorted four are max(lo1,lo2) and
    // min(hi1,hi2); element [2] is the larger of them.
    return fmaxf(fmaxf(lo1, lo2), fminf(hi1, hi2));
}

// splitmix64 (synthetic frame generator).
__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

}  // namespace dips
