// series_common.h -- device helpers shared by the series kernels (gfx950):
// buffer descriptors and vec loads/stores, byte/pair-plane arithmetic, the
// exact unorm load, and the cross-lane reductions.
#pragma once

#include "dips_math.h"
#include "dips_kernels.h"

namespace dips {

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// gfx950 buffer-resource flags word (raw buffer, 32-bit format).
constexpr int kRsrcFlags = 0x00020000;
// cache policy of the streamed frame loads: nt (stream once).  Probe builds
// (round 2, profiles/r02_policy_energy.jsonl) overrode it to compare policies.
#ifndef DIPS_LOAD_AUX
#define DIPS_LOAD_AUX 2
#endif
constexpr int kAuxNT = DIPS_LOAD_AUX;

template <int C> struct Fmt;
template <> struct Fmt<3> { static constexpr int NDW = 3, PPV = 4, VB = 12; };
template <> struct Fmt<4> { static constexpr int NDW = 4, PPV = 4, VB = 16; };
template <> struct Fmt<1> { static constexpr int NDW = 4, PPV = 16, VB = 16; };

// Buffer descriptor of a wave-uniform byte range.  The inputs go through
// readfirstlane so the compiler can PROVE the descriptor uniform; otherwise
// it wraps every buffer op in a waterfall loop (cdna_hip_programming.md T20).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, uint32_t bytes) {
    const uint64_t a = (uint64_t)(uintptr_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    void* base = (void*)(uintptr_t)(((uint64_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(base, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), kRsrcFlags);
}

// Zero a.zero[0 .. a.zero_n) over the whole grid (the series the reduce
// kernel then adds into: stream order puts every atomic after this kernel; a
// separate fill launch costs ~4 us, 10 % of a 640x480 x 300-frame batch).
__device__ __forceinline__ void zero_series(const SeriesArgs& a) {
    if (a.zero == nullptr) return;
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < a.zero_n; j += stride) a.zero[j] = 0u;
}

template <int C, int AUX = kAuxNT>
__device__ __forceinline__ void load_vec(__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t (&v)[Fmt<C>::NDW]) {
    if constexpr (Fmt<C>::NDW == 3) {
        const u32x3 x = __builtin_amdgcn_raw_buffer_load_b96(r, off, 0, AUX);
        v[0] = x.x; v[1] = x.y; v[2] = x.z;
    } else {
        const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, AUX);
        v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
    }
}

template <int C, int AUX = kAuxNT>
__device__ __forceinline__ void store_vec(__amdgpu_buffer_rsrc_t r, uint32_t off, const uint32_t (&v)[Fmt<C>::NDW]) {
    if constexpr (Fmt<C>::NDW == 3) {
        u32x3 x; x.x = v[0]; x.y = v[1]; x.z = v[2];
        __builtin_amdgcn_raw_buffer_store_b96(x, r, off, 0, AUX);
    } else {
        u32x4 x; x.x = v[0]; x.y = v[1]; x.z = v[2]; x.w = v[3];
        __builtin_amdgcn_raw_buffer_store_b128(x, r, off, 0, AUX);
    }
}

__device__ __forceinline__ u16x2 as_u16x2(uint32_t x) { return __builtin_bit_cast(u16x2, x); }
__device__ __forceinline__ uint32_t as_u32(u16x2 x) { return __builtin_bit_cast(uint32_t, x); }

// |a - b| per byte of two packed dwords.
__device__ __forceinline__ uint32_t absdiff_bytes(uint32_t a, uint32_t b) {
    const u16x2 ae = as_u16x2(a & 0x00FF00FFu), be = as_u16x2(b & 0x00FF00FFu);
    const u16x2 ao = as_u16x2((a >> 8) & 0x00FF00FFu), bo = as_u16x2((b >> 8) & 0x00FF00FFu);
    const u16x2 de = __builtin_elementwise_max(ae, be) - __builtin_elementwise_min(ae, be);
    const u16x2 dd = __builtin_elementwise_max(ao, bo) - __builtin_elementwise_min(ao, bo);
    return as_u32(de) | (as_u32(dd) << 8);
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

// Exact rgba8unorm load without a division or a table: u(c) = c / 255
// correctly rounded equals fma(c, K_HI, c * K_LO) for every byte c, with
// K_HI + K_LO the double-float split of 1/255 (checked exhaustively in
// tests/test_oracle.py::test_unorm_fma_identity).  Two values per packed op.
constexpr float kUnormHi = 0x1.010102p-8f;
constexpr float kUnormLo = -0x1.fdfdfep-33f;

__device__ __forceinline__ f32x2 unorm2(f32x2 c) {
    const f32x2 hi = {kUnormHi, kUnormHi};
    const f32x2 lo = {kUnormLo, kUnormLo};
    return __builtin_elementwise_fma(c, hi, c * lo);
}

__device__ __forceinline__ f32x2 u16x2_to_f32x2(u16x2 v) {
    // byte values in the low byte of each half: v_cvt_f32_ubyte0 / ubyte2
    const uint32_t w = as_u32(v);
    return f32x2{(float)(w & 0xFFu), (float)((w >> 16) & 0xFFu)};
}

// Pair planes (two pixels per dword, one byte per u16 half) of one vec.
template <int C>
__device__ __forceinline__ void pair_planes(const uint32_t (&d)[Fmt<C>::NDW], u16x2 (&r)[2], u16x2 (&g)[2],
                                            u16x2 (&b)[2]) {
    if constexpr (C == 3) {
        // d0 = r0 g0 b0 r1 | d1 = g1 b1 r2 g2 | d2 = b2 r3 g3 b3 (byte 0 first)
        r[0] = as_u16x2(__builtin_amdgcn_perm(d[0], d[0], 0x0C030C00u));
        g[0] = as_u16x2(__builtin_amdgcn_perm(d[1], d[0], 0x0C040C01u));
        b[0] = as_u16x2(__builtin_amdgcn_perm(d[1], d[0], 0x0C050C02u));
        r[1] = as_u16x2(__builtin_amdgcn_perm(d[2], d[1], 0x0C050C02u));
        g[1] = as_u16x2(__builtin_amdgcn_perm(d[2], d[1], 0x0C060C03u));
        b[1] = as_u16x2(__builtin_amdgcn_perm(d[2], d[2], 0x0C030C00u));
    } else {
        // d_k = r g b a
        r[0] = as_u16x2(__builtin_amdgcn_perm(d[1], d[0], 0x0C040C00u));
        g[0] = as_u16x2(__builtin_amdgcn_perm(d[1], d[0], 0x0C050C01u));
        b[0] = as_u16x2(__builtin_amdgcn_perm(d[1], d[0], 0x0C060C02u));
        r[1] = as_u16x2(__builtin_amdgcn_perm(d[3], d[2], 0x0C040C00u));
        g[1] = as_u16x2(__builtin_amdgcn_perm(d[3], d[2], 0x0C050C01u));
        b[1] = as_u16x2(__builtin_amdgcn_perm(d[3], d[2], 0x0C060C02u));
    }
}

// ---------------------------------------------------------------------------
// Cross-lane reduction of several per-lane values at once, no LDS.
// N = 4 or 8 values.  The first steps exchange HALF of the values with the
// partner lane (xor 32 by v_permlane32_swap, xor 16 by v_permlane16_swap,
// xor 8 by DPP row_ror:8 when N = 8), so each lane ends up owning one value
// index; the remaining steps are plain DPP butterflies inside 8-lane groups.
// Value v's wave sum then sits in lane 8v (N = 8) or 16v (N = 4).  Compared
// with N separate butterflies this is ~1/3 of the instructions and the N
// chains overlap instead of running back to back.
// ---------------------------------------------------------------------------
#define DIPS_DPP(v, ctrl) ((uint32_t)__builtin_amdgcn_update_dpp(0, (int)(v), (ctrl), 0xF, 0xF, false))

__device__ __forceinline__ uint32_t swap32_sum(uint32_t a, uint32_t b) {
    const auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
    return r[0] + r[1];
}

__device__ __forceinline__ uint32_t swap16_sum(uint32_t a, uint32_t b) {
    const auto r = __builtin_amdgcn_permlane16_swap(a, b, false, false);
    return r[0] + r[1];
}

__device__ __forceinline__ uint32_t group8_sum(uint32_t y) {
    y += DIPS_DPP(y, 0xB1);   // quad_perm [1,0,3,2]  (xor 1)
    y += DIPS_DPP(y, 0x4E);   // quad_perm [2,3,0,1]  (xor 2)
    y += DIPS_DPP(y, 0x141);  // row_half_mirror      (xor 7 inside 8 lanes)
    return y;
}

// Sum over the 64 lanes of in[v]; on return lanes 8v .. 8v+7 hold value v's
// sum (every lane of that 8-lane group).
__device__ __forceinline__ uint32_t wave_sum8_lanes(const uint32_t (&in)[8], uint32_t lane) {
    uint32_t w[4], x[2];
#pragma unroll
    for (int k = 0; k < 4; ++k) w[k] = swap32_sum(in[k], in[4 + k]);  // lane owns 4*b5 + k
    x[0] = swap16_sum(w[0], w[2]);                                     // owns 4*b5 + 2*b4 + 0
    x[1] = swap16_sum(w[1], w[3]);                                     // owns 4*b5 + 2*b4 + 1
    const bool b3 = (lane & 8u) != 0;
    const uint32_t keep = b3 ? x[1] : x[0];
    const uint32_t send = b3 ? x[0] : x[1];
    return group8_sum(keep + DIPS_DPP(send, 0x128));                   // row_ror:8 (xor 8)
}

// Same for four values: lanes 16v .. 16v+15 hold value v's sum.
__device__ __forceinline__ uint32_t wave_sum4_lanes(const uint32_t (&in)[4]) {
    const uint32_t w0 = swap32_sum(in[0], in[2]);  // lane owns 2*b5 + 0
    const uint32_t w1 = swap32_sum(in[1], in[3]);  // lane owns 2*b5 + 1
    uint32_t y = swap16_sum(w0, w1);               // owns 2*b5 + b4
    y += DIPS_DPP(y, 0x128);                       // row_ror:8 (xor 8)
    return group8_sum(y);
}

// out[v] = sum over the 64 lanes of in[v] (wave-uniform results).
__device__ __forceinline__ void wave_sum8(const uint32_t (&in)[8], uint32_t (&out)[8], uint32_t lane) {
    const uint32_t y = wave_sum8_lanes(in, lane);
#pragma unroll
    for (int v = 0; v < 8; ++v) out[v] = (uint32_t)__builtin_amdgcn_readlane((int)y, 8 * v);
}

__device__ __forceinline__ void wave_sum4(const uint32_t (&in)[4], uint32_t (&out)[4]) {
    const uint32_t y = wave_sum4_lanes(in);
#pragma unroll
    for (int v = 0; v < 4; ++v) out[v] = (uint32_t)__builtin_amdgcn_readlane((int)y, 16 * v);
}

}  // namespace dips
