// window_net.h -- order statistic of a spatial window through a sorting
// network held in registers.
//
// The reference's spatial_median_filter bubble-sorts a zero-padded array of
// W^2 + 1 (dips) or W^2 (dips_alt) entries per pixel (dips_shader.wgsl:
// 150-169; dips_alt pre_compute_shader.wgsl:160-184), O(W^4) compares.  Only
// the (2h)^2 window values are non-zero; the kernels map the reference's
// index to a rank kk among those n = side^2 values (compat_kernels.hip
// window_select, alt_kernels.hip alt_window_select) and this header returns
// the kk-th smallest of them:
//
//   * the n values are read from the LDS tile into registers (constant
//     offsets: ds_read_b32 with immediate offsets);
//   * they are sorted by Batcher's odd-even merge network for the next power
//     of two P >= n, built at compile time, keeping only the comparators with
//     both ends below n (pads at the top positions would be +inf, and an
//     ascending comparator whose upper end holds +inf is a no-op, so the
//     dropped comparators never change anything);
//   * the rank kk is a template argument (one instantiation per window), so
//     the compiler drops every comparator that does not feed element kk.
//
// Intensities are +0.0 or positive finite floats, so their bit patterns
// order exactly like their values: a comparator is one v_min_u32 + one
// v_max_u32 and the selected value is returned bit for bit.  Equal values
// are interchangeable, so the result equals the reference's sorted element.
// Comparator counts for side = 2, 4, 6, 8, 10 (n = 4 .. 100): 5, 63, 268,
// 543, 1104 (vs n(n-1) = 9,900 compare-adds for a rank count at side 10).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <utility>

namespace dips {
namespace wnet {

constexpr int kMaxComparators = 1600;

template <int N>
struct Network {
    int count = 0;
    uint8_t lo[kMaxComparators] = {};
    uint8_t hi[kMaxComparators] = {};
    constexpr Network() {
        int p2 = 1;
        while (p2 < N) p2 <<= 1;
        // Batcher odd-even merge sort over p2 slots (Knuth 5.3.4, exercise 32)
        for (int p = 1; p < p2; p <<= 1) {
            for (int k = p; k >= 1; k >>= 1) {
                for (int j = k % p; j + k < p2; j += 2 * k) {
                    for (int i = 0; i < k && i + j + k < p2; ++i) {
                        const int a = i + j, b = i + j + k;
                        if (a / (2 * p) != b / (2 * p)) continue;
                        if (b >= N) continue;  // upper end is a +inf pad: no-op
                        lo[count] = (uint8_t)a;
                        hi[count] = (uint8_t)b;
                        ++count;
                    }
                }
            }
        }
    }
};

template <int N>
struct NetHolder {
    static constexpr Network<N> net{};
};

// Element types of the networks: u32 (f32 bit patterns, one window per
// value) and u16x2 (two quantised windows per value, v_pk_min/max_u16).
typedef unsigned short pk16 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t vmin(uint32_t a, uint32_t b) { return a < b ? a : b; }
__device__ __forceinline__ uint32_t vmax(uint32_t a, uint32_t b) { return a < b ? b : a; }
__device__ __forceinline__ pk16 vmin(pk16 a, pk16 b) { return __builtin_elementwise_min(a, b); }
__device__ __forceinline__ pk16 vmax(pk16 a, pk16 b) { return __builtin_elementwise_max(a, b); }
template <typename T> __device__ __forceinline__ T all_ones();
template <> __device__ __forceinline__ uint32_t all_ones<uint32_t>() { return 0xFFFFFFFFu; }
template <> __device__ __forceinline__ pk16 all_ones<pk16>() { return pk16{0xFFFF, 0xFFFF}; }

template <int A, int B, typename T>
__device__ __forceinline__ void cmpx(T* v) {
    const T a = v[A], b = v[B];
    v[A] = vmin(a, b);
    v[B] = vmax(a, b);
}

template <int N, typename T, size_t... I>
__device__ __forceinline__ void run_network(T* v, std::index_sequence<I...>) {
    (cmpx<NetHolder<N>::net.lo[I], NetHolder<N>::net.hi[I]>(v), ...);
}

// KK-th smallest (0-based) of tile[ty + r][tx + c], r, c in [0, SIDE).  KK is
// a compile-time constant, so after unrolling only the comparators that feed
// element KK survive (~19 % fewer at side 10) and no select is needed.
template <int SIDE, int KK, int LDS>
__device__ __forceinline__ float window_kth(const float (*tile)[LDS], int ty, int tx) {
    constexpr int n = SIDE * SIDE;
    static_assert(KK >= 0 && KK < n, "rank outside the window");
    static_assert(NetHolder<n>::net.count <= kMaxComparators, "network too large");
    uint32_t v[n];
#pragma unroll
    for (int r = 0; r < SIDE; ++r)
#pragma unroll
        for (int c = 0; c < SIDE; ++c) v[r * SIDE + c] = __float_as_uint(tile[ty + r][tx + c]);
    run_network<n>(v, std::make_index_sequence<NetHolder<n>::net.count>{});
    return __uint_as_float(v[KK]);
}

// The same order statistic for the two vertically adjacent windows at tile
// rows [ty, ty + SIDE) and [ty + 1, ty + SIDE + 1).  They share the
// SIDE - 1 middle rows (m = SIDE (SIDE - 1) values, sorted once); each adds
// one private row (SIDE values, sorted).  The KK-th smallest of a sorted S
// and a sorted row R is min over i of max(S[KK - i], R[i - 1]) (i values taken
// from R), so only S[KK - SIDE .. KK] is needed and the compiler keeps only
// the comparators feeding those.  Side 10: ~455 comparators per pixel
// instead of ~890.
template <int M, int R, int KK, typename T>
__device__ __forceinline__ T kth_of_two(const T* s, const T* r) {
    constexpr int lo = KK + 1 - M > 0 ? KK + 1 - M : 0;
    constexpr int hi = R < KK + 1 ? R : KK + 1;
    T best = all_ones<T>();
#pragma unroll
    for (int i = lo; i <= hi; ++i) {
        const int si = KK - i < 0 ? 0 : KK - i;
        const int ri = i - 1 < 0 ? 0 : i - 1;
        T term;
        if (i == 0)
            term = s[si];                            // nothing from R
        else if (KK - i < 0)
            term = r[ri];                            // all KK + 1 from R
        else
            term = vmax(s[si], r[ri]);
        best = vmin(term, best);
    }
    return best;
}

template <int SIDE, int KK, int LDS>
__device__ __forceinline__ void window_kth_pair(const float (*tile)[LDS], int ty, int tx, float& out0,
                                                float& out1) {
    constexpr int m = SIDE * (SIDE - 1);
    static_assert(KK >= 0 && KK < SIDE * SIDE, "rank outside the window");
    uint32_t s[m], r0[SIDE], r1[SIDE];
#pragma unroll
    for (int c = 0; c < SIDE; ++c) {
        r0[c] = __float_as_uint(tile[ty][tx + c]);
        r1[c] = __float_as_uint(tile[ty + SIDE][tx + c]);
    }
#pragma unroll
    for (int r = 0; r < SIDE - 1; ++r)
#pragma unroll
        for (int c = 0; c < SIDE; ++c) s[r * SIDE + c] = __float_as_uint(tile[ty + 1 + r][tx + c]);
    run_network<m>(s, std::make_index_sequence<NetHolder<m>::net.count>{});
    run_network<SIDE>(r0, std::make_index_sequence<NetHolder<SIDE>::net.count>{});
    run_network<SIDE>(r1, std::make_index_sequence<NetHolder<SIDE>::net.count>{});
    out0 = __uint_as_float(kth_of_two<m, SIDE, KK>(s, r0));
    out1 = __uint_as_float(kth_of_two<m, SIDE, KK>(s, r1));
}

// Four windows at once on quantised values: tile holds u8 values (one per
// u32), the windows at tile rows [ty, ty + SIDE) and [ty + 1, ty + SIDE + 1)
// for columns tx and tx + D share one pass of the same networks, column tx
// in the low and column tx + D in the high u16 half.  out0 / out1: the two
// rows' results, packed the same way.
template <int SIDE, int KK, int LDSW>
__device__ __forceinline__ void window_kth_quad(const uint32_t (*tile)[LDSW], int ty, int tx, int D, uint32_t& out0,
                                                uint32_t& out1) {
    constexpr int m = SIDE * (SIDE - 1);
    static_assert(KK >= 0 && KK < SIDE * SIDE, "rank outside the window");
    auto pk = [&](int r, int c) {
        return __builtin_bit_cast(pk16, tile[r][tx + c] | (tile[r][tx + D + c] << 16));
    };
    pk16 s[m], r0[SIDE], r1[SIDE];
#pragma unroll
    for (int c = 0; c < SIDE; ++c) {
        r0[c] = pk(ty, c);
        r1[c] = pk(ty + SIDE, c);
    }
#pragma unroll
    for (int r = 0; r < SIDE - 1; ++r)
#pragma unroll
        for (int c = 0; c < SIDE; ++c) s[r * SIDE + c] = pk(ty + 1 + r, c);
    run_network<m>(s, std::make_index_sequence<NetHolder<m>::net.count>{});
    run_network<SIDE>(r0, std::make_index_sequence<NetHolder<SIDE>::net.count>{});
    run_network<SIDE>(r1, std::make_index_sequence<NetHolder<SIDE>::net.count>{});
    out0 = __builtin_bit_cast(uint32_t, kth_of_two<m, SIDE, KK>(s, r0));
    out1 = __builtin_bit_cast(uint32_t, kth_of_two<m, SIDE, KK>(s, r1));
}

}  // namespace wnet
}  // namespace dips
