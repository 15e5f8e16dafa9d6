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
//   * element kk is picked with an unrolled select.
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

template <int A, int B>
__device__ __forceinline__ void cmpx(uint32_t* v) {
    const uint32_t a = v[A], b = v[B];
    v[A] = a < b ? a : b;
    v[B] = a < b ? b : a;
}

template <int N, size_t... I>
__device__ __forceinline__ void run_network(uint32_t* v, std::index_sequence<I...>) {
    (cmpx<NetHolder<N>::net.lo[I], NetHolder<N>::net.hi[I]>(v), ...);
}

// kk-th smallest (0-based) of tile[ty + r][tx + c], r, c in [0, SIDE).
template <int SIDE, int LDS>
__device__ __forceinline__ float window_kth(const float (*tile)[LDS], int ty, int tx, int kk) {
    constexpr int n = SIDE * SIDE;
    static_assert(NetHolder<n>::net.count <= kMaxComparators, "network too large");
    uint32_t v[n];
#pragma unroll
    for (int r = 0; r < SIDE; ++r)
#pragma unroll
        for (int c = 0; c < SIDE; ++c) v[r * SIDE + c] = __float_as_uint(tile[ty + r][tx + c]);
    run_network<n>(v, std::make_index_sequence<NetHolder<n>::net.count>{});
    uint32_t out = 0;
#pragma unroll
    for (int i = 0; i < n; ++i) out = i == kk ? v[i] : out;
    return __uint_as_float(out);
}

}  // namespace wnet
}  // namespace dips
