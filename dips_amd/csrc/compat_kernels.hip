// compat_kernels.hip -- the dips-compat ComputeState kernels on gfx950.
//
//   compat_precompute: pre_compute_main (pre_compute_shader.wgsl:92-132),
//                      the start texture S = q(upper median of the four
//                      spatially filtered first frames), run once.
//   compat_main:       compute_main (dips_shader.wgsl:172-240) for one frame:
//                      store the newest slot's filtered texel (quantised,
//                      A4), upper median of the four slots, diff against S,
//                      filter / sensitivity / colour epilogue, RGBA8 out.
//   compat_filter_frames: the spatial filter (W > 1) of one or many frames
//                      into gray ring texels, ahead of compat_main or the
//                      batch kernel.
//
// compat_precompute and compat_main cover 16x16 pixel tiles.  W = 1: one
// thread per pixel.  For a spatial window W > 1 compat_precompute stages the
// intensity of its (16 + 2h)^2 neighbourhood in LDS (out-of-frame texels are
// 0.0, dips_shader.wgsl:135-136) and each of its 16x8 threads selects the
// order statistic of two vertically adjacent windows through register
// sorting networks (window_net.h); compat_filter_frames does the same on
// quantised bytes, four windows per network pass (32x16 tiles).  Kernels are
// instantiated per window, so the W = 1 launches keep their small register
// budget.  The reference filters the newest slot in place while neighbours
// read it (a data race); here the filter reads the slot and
// writes a separate buffer (`raw`), which compat_main then stores.
#include "dips_math.h"
#include "dips_kernels.h"
#include "window_net.h"

namespace dips {

constexpr int kTile = 16;
constexpr int kMaxHalo = 5;                       // window <= 11
constexpr int kLds = kTile + 2 * kMaxHalo;        // 26

__device__ __forceinline__ float texel_intensity(const uint8_t* img, uint64_t p, uint32_t chroma) {
    const uint32_t v = *reinterpret_cast<const uint32_t*>(img + 4 * p);
    return intensity_rgb(v & 0xFFu, (v >> 8) & 0xFFu, (v >> 16) & 0xFFu, chroma);
}

// Stage the intensity neighbourhood of this workgroup's tile (NT threads).
template <int NT = kTile * kTile>
__device__ void stage_tile(float (*tile)[kLds], const uint8_t* img, uint32_t w, uint32_t h, int halo,
                           uint32_t chroma, uint32_t y0 = 0) {
    const int ox = (int)(blockIdx.x * kTile) - halo;
    const int oy = (int)(y0 + blockIdx.y * kTile) - halo;
    const int span = kTile + 2 * halo;
    for (int idx = threadIdx.y * kTile + threadIdx.x; idx < span * span; idx += NT) {
        const int ty = idx / span, tx = idx - ty * span;
        const int gx = ox + tx, gy = oy + ty;
        float v = 0.0f;
        if (gx >= 0 && gy >= 0 && gx < (int)w && gy < (int)h) v = texel_intensity(img, (uint64_t)gy * w + gx, chroma);
        tile[ty][tx] = v;
    }
}

// spatial_median_filter for W > 1 (dips_shader.wgsl:120-170): the sorted
// 121-entry array holds the (2h)^2 window values and zeros elsewhere; the
// bubble sort (j+1 clamped to 120 by naga's Restrict policy) sorts indices
// 0..min(W^2,120); the result is element min(W^2/2 + 1, 120).  All values are
// >= 0, so that element is 0 while it falls among the zeros, otherwise the
// (k - zeros)-th smallest window value.  window_rank is that rank among the
// (2h)^2 window values, or -1 when the result falls among the zeros (W = 3:
// k = 5 < 6 zeros, so W = 3 filters every texel to 0).
__host__ __device__ constexpr int window_rank(int window) {
    const int hw = window / 2;
    const int n = (2 * hw) * (2 * hw);
    const int ws2 = window * window;
    const int region = (ws2 < 120 ? ws2 : 120) + 1;
    const int zeros = region - n;
    const int k = ws2 / 2 + 1 > 120 ? 120 : ws2 / 2 + 1;
    return k < zeros ? -1 : k - zeros;
}

// tile[ty + j + hw][tx + i + hw] for i, j in [-hw, hw) -> rows/cols [ty, ty + SIDE).
// A thread filters the two pixels at tile rows ty, ty + 1 (window_kth_pair).
// Windows SIDE and SIDE + 1 share the side; each gets its own rank constant.
template <int SIDE>
__device__ __forceinline__ void window_select2(float (*tile)[kLds], int window, int ty, float& f0, float& f1) {
    constexpr int k0 = window_rank(SIDE), k1 = window_rank(SIDE + 1);
    f0 = f1 = 0.0f;
    if (window == SIDE) {
        if constexpr (k0 >= 0) wnet::window_kth_pair<SIDE, k0, kLds>(tile, ty, threadIdx.x, f0, f1);
    } else {
        if constexpr (k1 >= 0) wnet::window_kth_pair<SIDE, k1, kLds>(tile, ty, threadIdx.x, f0, f1);
    }
}

// SIDE = 2 * (window / 2): 0 for W = 1 (no neighbourhood, one pixel per
// thread, 16x16 threads), else the side of the sorted window (two vertically
// adjacent pixels per thread, 16x8 threads), so each launch carries only its
// own network's registers.
template <int SIDE>
constexpr int kRows = SIDE == 0 ? 1 : 2;

template <int SIDE>
__global__ __launch_bounds__(256) void compat_precompute_kernel(CompatArgs a) {
    constexpr int R = kRows<SIDE>;
    __shared__ float tile[kLds][kLds];
    const uint32_t x = blockIdx.x * kTile + threadIdx.x;
    const uint32_t yb = blockIdx.y * kTile + threadIdx.y * R;
    float m[R][4] = {};
    if constexpr (SIDE == 0) {
        const bool inside = x < a.width && yb < a.height;
        const uint64_t p = (uint64_t)yb * a.width + x;
#pragma unroll
        for (int k = 0; k < 4; ++k) m[0][k] = inside ? texel_intensity(a.slots[k], p, a.chroma) : 0.0f;
    } else if (window_rank(a.window) >= 0) {
        // one copy of the window network, run once per slot; results routed
        // into m[][] by an unrolled select (no dynamic register index)
#pragma unroll 1
        for (int k = 0; k < 4; ++k) {
            __syncthreads();
            stage_tile<kTile * kTile / R>(tile, a.slots[k], a.width, a.height, SIDE / 2, a.chroma);
            __syncthreads();
            float f0, f1;
            window_select2<SIDE>(tile, a.window, threadIdx.y * R, f0, f1);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                m[0][j] = j == k ? f0 : m[0][j];
                m[1][j] = j == k ? f1 : m[1][j];
            }
        }
    }
    // get_intensity(vec4(f, f, f, 1)) = f (pre_compute_shader.wgsl:105-108)
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t y = yb + r;
        if (x >= a.width || y >= a.height) continue;
        const uint64_t p = (uint64_t)y * a.width + x;
        const uint32_t s = unorm_store(upper_median4(m[r][0], m[r][1], m[r][2], m[r][3]));
        // start texture is gray RGBA8 (pre_compute_shader.wgsl:128-131)
        *reinterpret_cast<uint32_t*>(const_cast<uint8_t*>(a.start) + 4 * p) = s | (s << 8) | (s << 16) | (255u << 24);
    }
}

// compute_main's per-pixel tail once the newest slot's filtered intensity fi
// is known (dips_shader.wgsl:187-239).
// Slot store of compat_texel: kSlotQ stores the quantised filtered texel
// (compute_main, dips_shader.wgsl:187); the speculative dispatch of a deferred
// add_texture stores the frame's raw texel (kSlotRaw, W = 1) or nothing
// (kSlotNone, W > 1: the upload already put the raw frame there); the
// dispatch that claims it stores the gray texel afterwards.
constexpr int kSlotQ = 0, kSlotRaw = 1, kSlotNone = 2;

__device__ __forceinline__ uint32_t compat_texel(const CompatArgs& a, uint64_t p, float fi, int slot_mode = kSlotQ,
                                                 uint32_t raw = 0u) {
    // in-place store of the filtered newest slot, quantised (dips_shader.wgsl:187)
    const uint32_t qi = unorm_store(fi);
    if (slot_mode != kSlotNone)
        *reinterpret_cast<uint32_t*>(a.slots[a.newest] + 4 * p) =
            slot_mode == kSlotRaw ? raw : (qi | (qi << 8) | (qi << 16) | (255u << 24));
    float m[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        // the newest slot re-reads its own quantised gray texel (:192)
        m[i] = (uint32_t)i == a.newest ? intensity_rgb(qi, qi, qi, a.chroma) : texel_intensity(a.slots[i], p, a.chroma);
    }
    const float original = unorm_load(a.start[4 * p]);  // textureLoad(start_texture).r (:213)
    const float diff = original - upper_median4(m[0], m[1], m[2], m[3]);
    return visual_epilogue(diff, a.filter, a.sensitivity, a.colorize != 0u);
}

// compute_main for one frame once `raw` holds the newest slot's filter
// input: the frame itself (W = 1, vec4(I, I, I, 1), dips_shader.wgsl:123-126)
// or, for W > 1, its filtered ring texel from compat_filter_frames_kernel
// (gray q, whose intensity is u(q) under every chroma filter, so the store
// below writes q back).  One thread per pixel.
__global__ __launch_bounds__(256) void compat_main_kernel(CompatArgs a) {
    const uint32_t x = blockIdx.x * kTile + threadIdx.x;
    const uint32_t y = a.y0 + blockIdx.y * kTile + threadIdx.y;
    const uint32_t yend = a.y1 ? a.y1 : a.height;
    if (x >= a.width || y >= yend) return;
    const uint64_t p = (uint64_t)y * a.width + x;
    *reinterpret_cast<uint32_t*>(a.out + 4 * p) = compat_texel(a, p, texel_intensity(a.raw, p, a.chroma));
}

// The same with the frame read from, and the output written to, pinned HOST
// memory over PCIe (the per-frame call's zero-copy form: no DMA engine, the
// kernel's loads and stores move both directions at once).  System-scope
// accesses: the loads see what the host threads wrote before the launch and
// the stores reach host memory, bypassing the non-coherent cache levels.
// One thread per pixel over the rows' pixel range, so that a wave moves 256
// contiguous bytes each way.  (Four pixels per thread through 16-B
// system-coherent buffer loads / stores measured slower: 557-575 against
// 695-701 frames/s of 4K per-frame calls, profiles/r02_callback_direct_ab_vec.jsonl.)
//
// The output goes back as the RGBA8 texel (out_key 0) or as its key
// (out_key 1 / 2): every texel of visual_epilogue has A = 255, gray has
// R = G = B (COLORIZE off) and the two HSL cases have B = min(R, G)
// (dips_shader.wgsl:30-62, 231-239; q is monotonic), so one or two bytes per
// pixel carry it exactly and the copy-out threads rebuild the RGBA8 texel
// (host_stream.h expand_keys): 8.3 instead of 33.2 MB per 4K frame on the
// PCIe link that the frame's upload shares.
template <int SLOT_MODE>
__global__ __launch_bounds__(256) void compat_main_host_kernel(CompatArgs a) {
    const uint32_t yend = a.y1 ? a.y1 : a.height;
    const uint64_t p = (uint64_t)a.y0 * a.width + (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (p >= (uint64_t)yend * a.width) return;
    const uint32_t v = __hip_atomic_load(reinterpret_cast<const uint32_t*>(a.raw + 4 * p), __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_SYSTEM);
    const float fi = intensity_rgb(v & 0xFFu, (v >> 8) & 0xFFu, (v >> 16) & 0xFFu, a.chroma);
    const uint32_t texel = compat_texel(a, p, fi, SLOT_MODE, v);
    if (a.out_key == 1u)
        __hip_atomic_store(a.out + p, (uint8_t)texel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else if (a.out_key == 2u)
        __hip_atomic_store(reinterpret_cast<uint16_t*>(a.out + 2 * p), (uint16_t)texel, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    else
        __hip_atomic_store(reinterpret_cast<uint32_t*>(a.out + 4 * p), texel, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}

// The same from the packed input (in_key 1 / 2, pack_frame): a pixel is its
// chroma channel v, or its (max, min) of R, G, B, which is all get_intensity
// reads (dips_shader.wgsl:64-82): the intensity of (max, min, min) equals the
// pixel's under chroma None, of (v, v, v) the pixel's under chroma R/G/B.  A
// raw ring slot (kSlotRaw) receives that texel, whose intensity -- the only
// thing the ring's readers take from it -- is the frame's.  G = 4 / IN
// pixels per thread, one 4-byte system-scope load (a wave reads 256
// contiguous bytes, the one-pixel-per-thread kernel's shape, which measured
// best); their keys in one store.  Groups at absolute pixel indices
// multiple of G, so loads and stores are naturally aligned; a group cut by
// the rows' ends does its pixels one by one.
template <int IN>
__device__ __forceinline__ uint32_t packed_texel_in(uint32_t w, int g, uint32_t& mx) {
    if constexpr (IN == 2) {
        mx = (w >> (16 * g)) & 0xFFu;
        const uint32_t mn = (w >> (16 * g + 8)) & 0xFFu;
        return mx | (mn << 8) | (mn << 16) | 0xFF000000u;
    } else {
        mx = (w >> (8 * g)) & 0xFFu;
        return mx * 0x010101u | 0xFF000000u;
    }
}

template <int SLOT_MODE, int IN>
__global__ __launch_bounds__(256) void compat_main_host_packed_kernel(CompatArgs a) {
    constexpr int G = 4 / IN;
    const uint32_t yend = a.y1 ? a.y1 : a.height;
    const uint64_t p0 = (uint64_t)a.y0 * a.width, p1 = (uint64_t)yend * a.width;
    const uint64_t q = (p0 / G) * G + (uint64_t)G * ((uint64_t)blockIdx.x * 256u + threadIdx.x);
    if (q >= p1) return;
    const uint32_t kb = a.out_key;  // 1 or 2 key bytes per pixel
    if (q >= p0 && q + G <= p1) {
        const uint32_t w = __hip_atomic_load(reinterpret_cast<const uint32_t*>(a.raw + IN * q), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_SYSTEM);
        uint64_t keys = 0;
#pragma unroll
        for (int g = 0; g < G; ++g) {
            uint32_t mx;
            const uint32_t raw = packed_texel_in<IN>(w, g, mx);
            const float fi = intensity_rgb(raw & 0xFFu, (raw >> 8) & 0xFFu, (raw >> 16) & 0xFFu, a.chroma);
            const uint32_t t = compat_texel(a, q + (uint64_t)g, fi, SLOT_MODE, raw);
            keys |= (uint64_t)(kb == 1u ? (t & 0xFFu) : (t & 0xFFFFu)) << (8 * kb * g);
        }
        if (kb * G == 2)
            __hip_atomic_store(reinterpret_cast<uint16_t*>(a.out + q), (uint16_t)keys, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        else if (kb * G == 4)
            __hip_atomic_store(reinterpret_cast<uint32_t*>(a.out + kb * q), (uint32_t)keys, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        else
            __hip_atomic_store(reinterpret_cast<uint64_t*>(a.out + 2 * q), keys, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        return;
    }
    for (int g = 0; g < G; ++g) {
        const uint64_t p = q + (uint64_t)g;
        if (p < p0 || p >= p1) continue;
        uint32_t w;
        if constexpr (IN == 2)
            w = __hip_atomic_load(reinterpret_cast<const uint16_t*>(a.raw + 2 * p), __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_SYSTEM);
        else
            w = __hip_atomic_load(a.raw + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        uint32_t mx;
        const uint32_t raw = packed_texel_in<IN>(w, 0, mx);
        const float fi = intensity_rgb(raw & 0xFFu, (raw >> 8) & 0xFFu, (raw >> 16) & 0xFFu, a.chroma);
        const uint32_t t = compat_texel(a, p, fi, SLOT_MODE, raw);
        if (kb == 1u)
            __hip_atomic_store(a.out + p, (uint8_t)t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        else
            __hip_atomic_store(reinterpret_cast<uint16_t*>(a.out + 2 * p), (uint16_t)t, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// A ring slot as frame_callback leaves it for a W = 1 frame: the gray texel
// q(get_intensity(frame)) (dips_shader.wgsl:123-126, 187) -- the state
// compat_main writes in place, rebuilt from a raw frame for resume.
__global__ __launch_bounds__(256) void compat_gray_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                         uint64_t n_px, uint32_t chroma) {
    const uint64_t p = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (p >= n_px) return;
    const uint32_t q = unorm_store(texel_intensity(src, p, chroma));
    *reinterpret_cast<uint32_t*>(dst + 4 * p) = q | (q << 8) | (q << 16) | (255u << 24);
}

// The same in place: a ring slot holding a raw frame becomes the gray texel
// compute_main stores (the dispatch that claims a speculative one).
__global__ __launch_bounds__(256) void compat_quantise_slot_kernel(uint8_t* slot, uint64_t n_px, uint32_t chroma) {
    const uint64_t p = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (p >= n_px) return;
    const uint32_t q = unorm_store(texel_intensity(slot, p, chroma));
    *reinterpret_cast<uint32_t*>(slot + 4 * p) = q | (q << 8) | (q << 16) | (255u << 24);
}

hipError_t launch_compat_quantise_slot(uint8_t* slot, uint64_t n_px, uint32_t chroma, hipStream_t s) {
    if (n_px == 0) return hipSuccess;
    if (!fits_grid256(n_px)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(compat_quantise_slot_kernel, dim3((uint32_t)((n_px + 255) / 256)), dim3(256), 0, s, slot, n_px,
                       chroma);
    return hipGetLastError();
}

hipError_t launch_compat_gray(const uint8_t* src, uint8_t* dst, uint64_t n_px, uint32_t chroma, hipStream_t s) {
    if (n_px == 0) return hipSuccess;
    if (!fits_grid256(n_px)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(compat_gray_kernel, dim3((uint32_t)((n_px + 255) / 256)), dim3(256), 0, s, src, dst, n_px, chroma);
    return hipGetLastError();
}

// The ring texel of compute_main for a whole batch of frames (W > 1, steady
// state): gray q(filtered intensity), the value compat_main stores into the
// newest slot (dips_shader.wgsl:187).  q is non-decreasing, so q of the k-th
// smallest intensity is the k-th smallest q: the tile holds q(I) and the
// networks run on bytes, two windows per instruction (u16x2 halves,
// window_kth_quad).  A workgroup covers 32x16 pixels; each thread filters
// columns tx and tx + 16 of rows 2ty and 2ty + 1.  blockIdx.z = frame.
constexpr int kFilterW = 32;

template <int WIN>
__global__ __launch_bounds__(128) void compat_filter_frames_kernel(const uint8_t* __restrict__ frames,
                                                                   uint8_t* __restrict__ dst, uint32_t w, uint32_t h,
                                                                   uint32_t chroma) {
    constexpr int SIDE = 2 * (WIN / 2), KK = window_rank(WIN);
    constexpr int LW = kFilterW + SIDE, LH = kTile + SIDE;
    __shared__ uint32_t tile[LH][LW];
    const uint64_t fo = (uint64_t)blockIdx.z * w * h * 4u;
    const uint32_t tx = threadIdx.x, ty = threadIdx.y;
    uint32_t o0 = 0, o1 = 0;  // q of rows 2ty, 2ty + 1; column tx low, tx + 16 high
    if constexpr (KK >= 0) {
        const int ox = (int)(blockIdx.x * kFilterW) - SIDE / 2;
        const int oy = (int)(blockIdx.y * kTile) - SIDE / 2;
        for (int idx = ty * kTile + tx; idx < LH * LW; idx += kTile * kTile / 2) {
            const int r = idx / LW, c = idx - r * LW;
            const int gx = ox + c, gy = oy + r;
            uint32_t q = 0;  // out-of-frame texels are 0.0 (dips_shader.wgsl:135-136)
            if (gx >= 0 && gy >= 0 && gx < (int)w && gy < (int)h)
                q = unorm_store(texel_intensity(frames + fo, (uint64_t)gy * w + gx, chroma));
            tile[r][c] = q;
        }
        __syncthreads();
        wnet::window_kth_quad<SIDE, KK, LW>(tile, 2 * ty, tx, kTile, o0, o1);
    }
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const uint32_t y = blockIdx.y * kTile + 2 * ty + r;
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const uint32_t x = blockIdx.x * kFilterW + tx + c * kTile;
            if (x >= w || y >= h) continue;
            const uint32_t q = ((r ? o1 : o0) >> (16 * c)) & 0xFFu;
            *reinterpret_cast<uint32_t*>(dst + fo + 4 * ((uint64_t)y * w + x)) = q | (q << 8) | (q << 16) | (255u << 24);
        }
    }
}

hipError_t launch_compat_filter_frames(const uint8_t* frames, uint8_t* dst, uint32_t width, uint32_t height,
                                       uint32_t n, int32_t window, uint32_t chroma, hipStream_t s) {
    if (n == 0) return hipSuccess;
    if (n > 65535u) return hipErrorInvalidValue;
    dim3 grid((width + kFilterW - 1) / kFilterW, (height + kTile - 1) / kTile, n);
    switch (window) {
#define DIPS_WIN(W)                                                                                                \
    case W:                                                                                                        \
        hipLaunchKernelGGL(compat_filter_frames_kernel<W>, grid, dim3(kTile, kTile / 2), 0, s, frames, dst, width, \
                           height, chroma);                                                                        \
        break;
        DIPS_WIN(2) DIPS_WIN(3) DIPS_WIN(4) DIPS_WIN(5) DIPS_WIN(6) DIPS_WIN(7) DIPS_WIN(8) DIPS_WIN(9) DIPS_WIN(10)
        DIPS_WIN(11)
#undef DIPS_WIN
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_compat_precompute(const CompatArgs& a, hipStream_t s) {
    dim3 grid((a.width + kTile - 1) / kTile, (a.height + kTile - 1) / kTile);
    switch (a.window / 2) {
#define DIPS_SIDE(H) \
    case H: hipLaunchKernelGGL(compat_precompute_kernel<2 * H>, grid, dim3(kTile, kTile / kRows<2 * H>), 0, s, a); break;
        DIPS_SIDE(0) DIPS_SIDE(1) DIPS_SIDE(2) DIPS_SIDE(3) DIPS_SIDE(4) DIPS_SIDE(5)
#undef DIPS_SIDE
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_compat_main(const CompatArgs& a, hipStream_t s) {
    const uint32_t yend = a.y1 ? a.y1 : a.height;
    if (a.y0 >= yend || yend > a.height) return hipErrorInvalidValue;
    dim3 grid((a.width + kTile - 1) / kTile, (yend - a.y0 + kTile - 1) / kTile);
    hipLaunchKernelGGL(compat_main_kernel, grid, dim3(kTile, kTile), 0, s, a);
    return hipGetLastError();
}

// Copies between pinned host memory (device-visible pointer) and HBM by a
// kernel instead of a DMA engine (the host-fed pipelines, host_stream.h):
// system-scope accesses on the host side, one word per thread.
template <typename T>
__global__ __launch_bounds__(256) void copy_from_host_kernel(const T* src, T* __restrict__ dst, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    dst[i] = __hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <typename T>
__global__ __launch_bounds__(256) void copy_to_host_kernel(const T* __restrict__ src, T* dst, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    __hip_atomic_store(dst + i, src[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <bool TO_HOST>
static hipError_t launch_host_copy(const uint8_t* src, uint8_t* dst, uint64_t bytes, hipStream_t s) {
    if (bytes == 0) return hipSuccess;
    const bool w8 = bytes % 8u == 0 && ((uintptr_t)src & 7u) == 0 && ((uintptr_t)dst & 7u) == 0;
    if (!w8 && (bytes % 4u != 0 || ((uintptr_t)src & 3u) != 0 || ((uintptr_t)dst & 3u) != 0))
        return hipErrorInvalidValue;
    const uint64_t n = w8 ? bytes / 8u : bytes / 4u;
    if (!fits_grid256(n)) return hipErrorInvalidValue;
    const dim3 grid((uint32_t)((n + 255) / 256));
    if (w8) {
        auto* a = reinterpret_cast<const uint64_t*>(src);
        auto* b = reinterpret_cast<uint64_t*>(dst);
        if (TO_HOST) hipLaunchKernelGGL(copy_to_host_kernel<uint64_t>, grid, dim3(256), 0, s, a, b, n);
        else hipLaunchKernelGGL(copy_from_host_kernel<uint64_t>, grid, dim3(256), 0, s, a, b, n);
    } else {
        auto* a = reinterpret_cast<const uint32_t*>(src);
        auto* b = reinterpret_cast<uint32_t*>(dst);
        if (TO_HOST) hipLaunchKernelGGL(copy_to_host_kernel<uint32_t>, grid, dim3(256), 0, s, a, b, n);
        else hipLaunchKernelGGL(copy_from_host_kernel<uint32_t>, grid, dim3(256), 0, s, a, b, n);
    }
    return hipGetLastError();
}

hipError_t launch_copy_from_host(const uint8_t* src, uint8_t* dst, uint64_t bytes, hipStream_t s) {
    return launch_host_copy<false>(src, dst, bytes, s);
}

hipError_t launch_copy_to_host(const uint8_t* src, uint8_t* dst, uint64_t bytes, hipStream_t s) {
    return launch_host_copy<true>(src, dst, bytes, s);
}

template <int IN>
static hipError_t launch_packed_in(const CompatArgs& a, dim3 grid, hipStream_t s, int slot_mode) {
    void (*k)(CompatArgs) = nullptr;
    switch (slot_mode) {
        case kSlotQ: k = compat_main_host_packed_kernel<kSlotQ, IN>; break;
        case kSlotRaw: k = compat_main_host_packed_kernel<kSlotRaw, IN>; break;
        case kSlotNone: k = compat_main_host_packed_kernel<kSlotNone, IN>; break;
        default: return hipErrorInvalidValue;
    }
    hipLaunchKernelGGL(k, grid, dim3(256), 0, s, a);
    return hipGetLastError();
}

static hipError_t launch_packed(const CompatArgs& a, dim3 grid, hipStream_t s, int slot_mode) {
    if (a.in_key == 2u) return launch_packed_in<2>(a, grid, s, slot_mode);
    if (a.in_key == 1u) return launch_packed_in<1>(a, grid, s, slot_mode);
    return hipErrorInvalidValue;
}

hipError_t launch_compat_main_host(const CompatArgs& a, hipStream_t s, int slot_mode) {
    const uint32_t yend = a.y1 ? a.y1 : a.height;
    if (a.y0 >= yend || yend > a.height) return hipErrorInvalidValue;
    const uint64_t n_px = (uint64_t)(yend - a.y0) * a.width;
    if (!fits_grid256(n_px)) return hipErrorInvalidValue;
    if (a.out_key != 0u && a.in_key != 0u) {
        const uint32_t G = 4u / a.in_key;
        const uint64_t p0 = (uint64_t)a.y0 * a.width, p1 = (uint64_t)yend * a.width;
        const uint64_t groups = (p1 + G - 1) / G - p0 / G;
        const dim3 gp((uint32_t)((groups + 255) / 256));
        return launch_packed(a, gp, s, slot_mode);
    }
    const dim3 grid((uint32_t)((n_px + 255) / 256));
    switch (slot_mode) {
        case kSlotQ: hipLaunchKernelGGL(compat_main_host_kernel<kSlotQ>, grid, dim3(256), 0, s, a); break;
        case kSlotRaw: hipLaunchKernelGGL(compat_main_host_kernel<kSlotRaw>, grid, dim3(256), 0, s, a); break;
        case kSlotNone: hipLaunchKernelGGL(compat_main_host_kernel<kSlotNone>, grid, dim3(256), 0, s, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace dips
