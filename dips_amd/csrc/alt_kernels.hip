// alt_kernels.hip -- the dips_alt operator (DiPsCompute) on gfx950, SURVEY.md
// s8f next-4: a snapshot reference, an N-slot temporal "median" and the
// DIFF_SCALE epilogue (dips_alt/src/dips_compute/shaders/pre_compute_shader.wgsl,
// host side dips_alt/src/dips_compute/mod.rs:498-646, driver loop
// dips_alt/src/lib.rs:588-683).
//
//   alt_frame_kernel<N>   one send_frame dispatch (pre_compute_main :188-263)
//                         for any N = num_textures in 1..16 and any spatial
//                         window; W > 1 stages the intensity neighbourhood of
//                         the 16x16 tile in LDS and sorts the windows of two
//                         vertically adjacent pixels per thread in registers
//                         (window_net.h).
//   alt_batch_kernel      a whole run of HBM-resident frames for N = 2, W = 1,
//                         the configuration dips_alt runs (FRAME_COUNT = 2,
//                         lib.rs:36; window_size 1, mod.rs:176-186).  A wave
//                         owns a tile of pixels and walks a range of frames;
//                         the previous frame's intensities and the snapshot
//                         stay in registers, so a frame costs its 4 B/px read
//                         plus the 4 B/px output write and nothing else.
//
// Numerics: the temporal sort of n values in a zero-filled 16-entry array,
// element [n/2] (:212-227, :232, :238), is sorted(v + {0})[n/2] for n < 16
// (one trailing zero inside the sorted range) and sorted(v)[8] for n = 16
// (index 16 clamped to 15 by naga's Restrict policy).  Intensities are >= 0,
// so for n = 2 it is min(v0, v1) and for n = 1 it is 0.
#include "alt_lut.h"
#include "epilogue_fast.h"
#include "intensity_v2.h"
#include "window_net.h"

#include <cstdlib>

namespace dips {

namespace {

constexpr int kTile = 16;
constexpr int kMaxHalo = 5;                 // window <= 11
constexpr int kLds = kTile + 2 * kMaxHalo;  // 26

__device__ __forceinline__ float alt_texel_intensity(const uint8_t* img, uint64_t p, uint32_t chroma) {
    const uint32_t v = *reinterpret_cast<const uint32_t*>(img + 4 * p);
    return intensity_rgb(v & 0xFFu, (v >> 8) & 0xFFu, (v >> 16) & 0xFFu, chroma);
}

// Intensities of this workgroup's tile plus a halo of `halo` texels; texels
// outside the frame are 0.0 (pre_compute_shader.wgsl:148-150).
template <int NT = kTile * kTile>
__device__ void alt_stage_tile(float (*tile)[kLds], const uint8_t* img, uint32_t w, uint32_t h, int halo,
                               uint32_t chroma, uint32_t y0) {
    const int ox = (int)(blockIdx.x * kTile) - halo;
    const int oy = (int)(y0 + blockIdx.y * kTile) - halo;
    const int span = kTile + 2 * halo;
    for (int idx = threadIdx.y * kTile + threadIdx.x; idx < span * span; idx += NT) {
        const int ty = idx / span, tx = idx - ty * span;
        const int gx = ox + tx, gy = oy + ty;
        float v = 0.0f;
        if (gx >= 0 && gy >= 0 && gx < (int)w && gy < (int)h) v = alt_texel_intensity(img, (uint64_t)gy * w + gx, chroma);
        tile[ty][tx] = v;
    }
}

// dips_alt spatial_median_filter for W > 1 (:141-184): the W^2-entry sort
// holds the (2h)^2 window values (offsets [-h, h) on both axes) and
// W^2 - (2h)^2 zeros; the result is element W^2/2 + 1.  All values are >= 0,
// so that element is 0 while it falls among the zeros, otherwise the
// (k - zeros)-th smallest window value.
__host__ __device__ constexpr int alt_window_rank(int window) {
    const int hw = window / 2;
    const int n = (2 * hw) * (2 * hw);
    const int ws2 = window * window;
    const int zeros = ws2 - n;
    const int k = ws2 / 2 + 1;
    return k < zeros ? -1 : k - zeros;
}

// The filtered intensities of the two vertically adjacent pixels at tile
// rows ty, ty + 1 (window_net.h window_kth_pair).
template <int SIDE>
__device__ __forceinline__ void alt_window_select2(float (*tile)[kLds], int window, int ty, float& f0, float& f1) {
    constexpr int k0 = alt_window_rank(SIDE), k1 = alt_window_rank(SIDE + 1);
    f0 = f1 = 0.0f;
    if (window == SIDE) {
        if constexpr (k0 >= 0) wnet::window_kth_pair<SIDE, k0, kLds>(tile, ty, threadIdx.x, f0, f1);
    } else {
        if constexpr (k1 >= 0) wnet::window_kth_pair<SIDE, k1, kLds>(tile, ty, threadIdx.x, f0, f1);
    }
}

// Element [n/2] of the sorted zero-padded temporal array (see file comment).
template <int N>
__device__ __forceinline__ float alt_temporal(const float (&v)[N]) {
    if constexpr (N == 1) {
        return 0.0f;
    } else if constexpr (N == 2) {
        return fminf(v[0], v[1]);
    } else {
        constexpr int kk = N == kAltMaxTextures ? N / 2 : N / 2 - 1;  // rank among v
        float r = 0.0f;
#pragma unroll
        for (int c = 0; c < N; ++c) {
            int rank = 0;
#pragma unroll
            for (int j = 0; j < N; ++j) rank += (v[j] < v[c] || (v[j] == v[c] && j < c)) ? 1 : 0;
            r = rank == kk ? v[c] : r;
        }
        return r;
    }
}

__device__ __forceinline__ uint32_t gray_rgba(uint32_t s) { return s | (s << 8) | (s << 16) | (255u << 24); }

// send_frame's per-pixel tail once the N slot intensities are known
// (:228-261).
template <int N>
__device__ __forceinline__ uint32_t alt_texel(const AltArgs& a, uint64_t p, const float (&v)[N]) {
    const float med = alt_temporal<N>(v);
    uint32_t o;
    if (a.snapshot) {
        // snapshot == 1: store the intensity into the snapshot and the output
        // texture (:231-235)
        const uint32_t s = unorm_store(med);
        a.snap[p] = (uint8_t)s;
        o = gray_rgba(s);
    } else {
        // textureLoad(snapshot_texture).r - median, then map / filter /
        // DIFF_SCALE / colour (:237-261)
        o = visual_epilogue(unorm_load(a.snap[p]) - med, a.filter, a.scalar, a.colorize != 0u);
    }
    return o;
}

template <int N>
__device__ __forceinline__ void alt_finish(const AltArgs& a, uint64_t p, const float (&v)[N]) {
    *reinterpret_cast<uint32_t*>(a.out + 4 * p) = alt_texel<N>(a, p, v);
}

// SIDE = 2 * (window / 2): 0 for W = 1 (one pixel per thread, 16x16
// threads), else two vertically adjacent pixels per thread (16x8 threads).
template <int SIDE>
constexpr int kAltRows = SIDE == 0 ? 1 : 2;

template <int N, int SIDE>
__global__ __launch_bounds__(256) void alt_frame_kernel(AltArgs a) {
    constexpr int R = kAltRows<SIDE>;
    __shared__ float tile[kLds][kLds];
    const uint32_t x = blockIdx.x * kTile + threadIdx.x;
    const uint32_t yb = a.y0 + blockIdx.y * kTile + threadIdx.y * R;
    const uint32_t yend = a.y1 ? a.y1 : a.height;
    float v[R][N] = {};
    // median_array[k] = spatial_median_filter(coords, dims, k)
    // (the generated array, dynamic_texture_array.rs:67-69)
    if constexpr (SIDE == 0) {
        if (x >= a.width || yb >= yend) return;
        const uint64_t p = (uint64_t)yb * a.width + x;
#pragma unroll
        for (int k = 0; k < N; ++k) v[0][k] = alt_texel_intensity(a.slots[k], p, a.chroma);
    } else {
        // one copy of the window network, run once per slot; the results are
        // routed into v[][] by an unrolled select (no dynamic register index)
#pragma unroll 1
        for (int k = 0; k < N; ++k) {
            __syncthreads();
            alt_stage_tile<kTile * kTile / R>(tile, a.slots[k], a.width, a.height, SIDE / 2, a.chroma, a.y0);
            __syncthreads();
            float f0, f1;
            alt_window_select2<SIDE>(tile, a.window, threadIdx.y * R, f0, f1);
#pragma unroll
            for (int j = 0; j < N; ++j) {
                v[0][j] = j == k ? f0 : v[0][j];
                v[1][j] = j == k ? f1 : v[1][j];
            }
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t y = yb + r;
        if (x < a.width && y < yend) alt_finish<N>(a, (uint64_t)y * a.width + x, v[r]);
    }
}

// send_frame for W = 1 in the per-frame call's zero-copy form: the new frame
// is read from pinned HOST memory (`in`) over PCIe, written into its ring
// slot (queue.write_texture, dips_alt/src/dips_compute/mod.rs:498-646) and
// used as that slot's texel; the output goes straight to pinned host memory
// (a.out).  System-scope accesses (see compat_main_host_kernel).  One thread
// per pixel over the rows' pixel range.
template <int N>
__global__ __launch_bounds__(256) void alt_frame_host_kernel(AltArgs a, const uint8_t* in, uint8_t* newest_slot,
                                                             uint32_t newest) {
    const uint32_t yend = a.y1 ? a.y1 : a.height;
    const uint64_t p = (uint64_t)a.y0 * a.width + (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (p >= (uint64_t)yend * a.width) return;
    const uint32_t raw =
        __hip_atomic_load(reinterpret_cast<const uint32_t*>(in + 4 * p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    *reinterpret_cast<uint32_t*>(newest_slot + 4 * p) = raw;
    float v[N];
#pragma unroll
    for (int k = 0; k < N; ++k)
        v[k] = (uint32_t)k == newest ? intensity_rgb(raw & 0xFFu, (raw >> 8) & 0xFFu, (raw >> 16) & 0xFFu, a.chroma)
                                     : alt_texel_intensity(a.slots[k], p, a.chroma);
    __hip_atomic_store(reinterpret_cast<uint32_t*>(a.out + 4 * p), alt_texel<N>(a, p, v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---------------------------------------------------------------------------
// Batch kernel (N = 2, W = 1, RGBA8)
// ---------------------------------------------------------------------------

template <int U>
struct AltTile {
    uint32_t voff[U];  // byte offset of the lane's vec u inside a frame
};

// I2s of a vec's four pixels: from RGBA8 bytes (CH = chroma filter 0..3), or
// CH = kAltPrefiltered: the vec already holds the four spatially filtered
// intensities as f32 I2s (alt_filter_frames_kernel, W > 1).
constexpr int kAltPrefiltered = -1;
template <int CH>
__device__ __forceinline__ void alt_derive(const uint32_t (&d)[4], St2& s) {
    if constexpr (CH == kAltPrefiltered) {
        s.i[0] = f32x2{__uint_as_float(d[0]), __uint_as_float(d[1])};
        s.i[1] = f32x2{__uint_as_float(d[2]), __uint_as_float(d[3])};
    } else {
        derive_v2<4, CH>(d, s);
    }
}

template <int CH, int U>
__device__ __forceinline__ void alt_intensity(const uint8_t* frame, uint32_t fb, const AltTile<U>& tl,
                                              f32x2 (&dst)[U][2]) {
    const __amdgpu_buffer_rsrc_t r = make_rsrc(frame, fb);
#pragma unroll
    for (int u = 0; u < U; ++u) {
        uint32_t d[4];
        load_vec<4>(r, tl.voff[u], d);
        St2 s;
        alt_derive<CH>(d, s);
        dst[u][0] = s.i[0];
        dst[u][1] = s.i[1];
    }
}

// exact u(c) = c / 255 without a division (series_common.h, exhaustively checked)
__device__ __forceinline__ float unorm_fma(uint32_t c) {
    const float f = (float)c;
    return __builtin_fmaf(f, kUnormHi, f * kUnormLo);
}

// The epilogue texel of diff from the LDS copy of the table (alt_lut.h):
// level 1 by the cluster rint(510 * diff), level 2 by the cluster's shifted
// diff bits.  diff must be one of the table's values (it is: u(S) - I).
__device__ __forceinline__ uint32_t alt_lut_texel(const uint32_t* l1, const uint16_t* l2, float diff) {
    const float t = __builtin_fmaf(diff, 510.0f, kAltLutRound);
    const uint32_t a1 = (__float_as_uint(t) << 3) - kAltLutL1Bias;
    const uint2 e = *reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(l1) + a1);
    const uint32_t a2 = ((__float_as_uint(diff) >> e.y) << 1) + e.x;
    return lut_texel(*reinterpret_cast<const uint16_t*>(reinterpret_cast<const char*>(l2) + a2));
}

// FAST: the branch-free epilogue of epilogue_fast.h (sigmoid with |k| <= 160,
// or no filter); otherwise the specification's visual_epilogue.  LUT: the
// epilogue table of alt_lut.h in LDS instead (FILT / COL / FAST unused).
// U vecs per lane; D frames of loads in flight per wave (D - 1 ahead).
template <int CH, int FILT, int COL, bool FAST, int U, bool LUT = false, int D = 2>
__global__ __launch_bounds__(256) void alt_batch_kernel(AltBatchArgs a) {
    __shared__ uint32_t lut1[LUT ? 2 * kAltLutClusters : 2];
    __shared__ uint16_t lut2[LUT ? kAltLutL2Max : 2];
    if constexpr (LUT) {
        // every wave of the group helps fill the table, then waits for it
        for (uint32_t i = threadIdx.x; i < 2u * kAltLutClusters; i += 256u) lut1[i] = a.lut_l1[i];
        const uint32_t* src = reinterpret_cast<const uint32_t*>(a.lut_l2);
        uint32_t* dst = reinterpret_cast<uint32_t*>(lut2);
        for (uint32_t i = threadIdx.x; i < (uint32_t)kAltLutL2Max / 2u; i += 256u) dst[i] = src[i];
        __syncthreads();
    }
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t item = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
    if (item >= a.n_tiles * a.n_chunks) return;
    const uint32_t c = item / a.n_tiles;
    const uint32_t tile = item - c * a.n_tiles;
    const uint32_t t0 = c * a.chunk;
    const uint32_t t1 = min(t0 + a.chunk, a.n_frames);
    const uint32_t fb = a.frame_bytes;
    AltTile<U> tl;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        // vecs past the frame end read as 0 and their stores are dropped
        // (buffer range checking), so a ragged last tile needs no branch
        const uint32_t vec = (tile * U + (uint32_t)u) * 64u + lane;
        tl.voff[u] = vec < a.n_vec ? vec * 16u : 0x80000000u;
    }

    // intensities of the previous frame (slot (g+1) mod 2 holds it)
    f32x2 prev[U][2];
    alt_intensity<CH, U>(t0 == 0 ? a.prev0 : a.frames + (uint64_t)(t0 - 1) * fb, fb, tl, prev);

    // snapshot bytes in force at t0: the batch's last snapshot before t0,
    // recomputed from its two frames, or the snapshot texture
    uint32_t snapb[U];
    const int32_t s = a.chunk_snap[c];
    if (s < 0) {
        const __amdgpu_buffer_rsrc_t rs = make_rsrc(a.snap_in, a.n_vec * 4u);
#pragma unroll
        for (int u = 0; u < U; ++u) snapb[u] = __builtin_amdgcn_raw_buffer_load_b32(rs, tl.voff[u] >> 2, 0, 0);
    } else {
        f32x2 is[U][2], ip[U][2];
        alt_intensity<CH, U>(a.frames + (uint64_t)s * fb, fb, tl, is);
        alt_intensity<CH, U>(s == 0 ? a.prev0 : a.frames + (uint64_t)(s - 1) * fb, fb, tl, ip);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            uint32_t b = 0;
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const f32x2 m = __builtin_elementwise_min(is[u][k], ip[u][k]) * (f32x2){kI2sToI, kI2sToI};
                b |= unorm_store(m.x) << (16 * k);
                b |= unorm_store(m.y) << (16 * k + 8);
            }
            snapb[u] = b;
        }
    }
    float snapf[U][4];
    auto unpack_snap = [&]() {
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int q = 0; q < 4; ++q) snapf[u][q] = unorm_fma((snapb[u] >> (8 * q)) & 0xFFu);
    };
    unpack_snap();

    auto load_frame = [&](uint32_t t, uint32_t (&d)[U][4]) {
        const __amdgpu_buffer_rsrc_t r = make_rsrc(a.frames + (uint64_t)t * fb, fb);
#pragma unroll
        for (int u = 0; u < U; ++u) load_vec<4>(r, tl.voff[u], d[u]);
    };

    auto process = [&](uint32_t t, const uint32_t (&d)[U][4]) {
        const bool snap_now = a.flags[t] != 0;  // wave-uniform (scalar load)
        const __amdgpu_buffer_rsrc_t ro = make_rsrc(a.out + (uint64_t)t * fb, fb);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            St2 n;
            alt_derive<CH>(d[u], n);
            float med[4];
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const f32x2 m = __builtin_elementwise_min(n.i[k], prev[u][k]) * (f32x2){kI2sToI, kI2sToI};
                med[2 * k] = m.x;
                med[2 * k + 1] = m.y;
                prev[u][k] = n.i[k];
            }
            uint32_t o[4];
            if (snap_now) {
                uint32_t b = 0;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const uint32_t sq = unorm_store(med[q]);
                    b |= sq << (8 * q);
                    o[q] = gray_rgba(sq);
                }
                snapb[u] = b;
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    if constexpr (LUT)
                        o[q] = alt_lut_texel(lut1, lut2, snapf[u][q] - med[q]);
                    else if constexpr (FAST)
                        o[q] = epilogue_fast<FILT, COL != 0>(snapf[u][q] - med[q], a.kneg_half);
                    else
                        o[q] = visual_epilogue(snapf[u][q] - med[q], (uint32_t)FILT, a.scalar, COL != 0);
                }
            }
            store_vec<4>(ro, tl.voff[u], o);
        }
        if (snap_now) unpack_snap();
    };

    // D frames in flight per wave: frames t+1 .. t+D-1 load while t is processed
    uint32_t buf[D][U][4];
    uint32_t t = t0;
#pragma unroll
    for (int j = 0; j < D - 1; ++j)
        if (t0 + (uint32_t)j < t1) load_frame(t0 + (uint32_t)j, buf[j]);
    bool more = true;
    while (more) {
#pragma unroll
        for (int j = 0; j < D; ++j) {
            if (more) {
                // the slot processed one step ago takes frame t + D - 1
                if (t + D - 1 < t1) load_frame(t + D - 1, buf[(j + D - 1) % D]);
                process(t, buf[j]);
                more = ++t < t1;
            }
        }
    }

    if (a.last_snap >= (int32_t)t0 && a.last_snap < (int32_t)t1) {
        const __amdgpu_buffer_rsrc_t rs = make_rsrc(a.snap_out, a.n_vec * 4u);
#pragma unroll
        for (int u = 0; u < U; ++u) __builtin_amdgcn_raw_buffer_store_b32(snapb[u], rs, tl.voff[u] >> 2, 0, 0);
    }
}

template <int N>
hipError_t launch_frame_n(const AltArgs& a, hipStream_t s) {
    const uint32_t yend = a.y1 ? a.y1 : a.height;
    if (a.y0 >= yend || yend > a.height) return hipErrorInvalidValue;
    dim3 grid((a.width + kTile - 1) / kTile, (yend - a.y0 + kTile - 1) / kTile);
    switch (a.window / 2) {
#define DIPS_SIDE(H) \
    case H: hipLaunchKernelGGL((alt_frame_kernel<N, 2 * H>), grid, dim3(kTile, kTile / kAltRows<2 * H>), 0, s, a); break;
        DIPS_SIDE(0) DIPS_SIDE(1) DIPS_SIDE(2) DIPS_SIDE(3) DIPS_SIDE(4) DIPS_SIDE(5)
#undef DIPS_SIDE
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// The spatially filtered intensity of every pixel of n frames (dips_alt
// spatial_median_filter, W > 1, pre_compute_shader.wgsl:134-186) as f32 I2s
// = I * 2^23 (exact), laid out like the RGBA8 frame (4 B/px), for the
// prefiltered batch kernel.  The temporal min and the epilogue act on these
// f32 values, so unlike the dips ring (compat_filter_frames_kernel) they are
// not quantised.  blockIdx.z = frame.
template <int WIN>
__global__ __launch_bounds__(128) void alt_filter_frames_kernel(const uint8_t* __restrict__ frames,
                                                                float* __restrict__ dst, uint32_t w, uint32_t h,
                                                                uint32_t chroma) {
    constexpr int SIDE = 2 * (WIN / 2), KK = alt_window_rank(WIN);
    __shared__ float tile[kLds][kLds];
    const uint64_t po = (uint64_t)blockIdx.z * w * h;
    float f0 = 0.0f, f1 = 0.0f;
    if constexpr (KK >= 0) {
        alt_stage_tile<kTile * kTile / 2>(tile, frames + 4 * po, w, h, SIDE / 2, chroma, 0);
        __syncthreads();
        wnet::window_kth_pair<SIDE, KK, kLds>(tile, 2 * threadIdx.y, threadIdx.x, f0, f1);
    }
    const uint32_t x = blockIdx.x * kTile + threadIdx.x;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const uint32_t y = blockIdx.y * kTile + 2 * threadIdx.y + r;
        if (x < w && y < h) dst[po + (uint64_t)y * w + x] = (r ? f1 : f0) * 8388608.0f;
    }
}

template <int CH, int FILT, bool FAST>
const void* batch_ptr_fc(bool colorize) {
    return colorize ? reinterpret_cast<const void*>(&alt_batch_kernel<CH, FILT, 1, FAST, kUnrollAlt>)
                    : reinterpret_cast<const void*>(&alt_batch_kernel<CH, FILT, 0, FAST, kUnrollAlt>);
}

template <int CH>
const void* batch_ptr_c(int filter, bool colorize, bool fast) {
    switch (filter) {
        case 0: return fast ? batch_ptr_fc<CH, 0, true>(colorize) : batch_ptr_fc<CH, 0, false>(colorize);
        case 1: return batch_ptr_fc<CH, 1, false>(colorize);
        default: return batch_ptr_fc<CH, 255, true>(colorize);  // any other code: identity (:249)
    }
}

__global__ __launch_bounds__(256) void alt_lut_fill_kernel(uint16_t* __restrict__ l2, const float* __restrict__ diffs,
                                                           const uint16_t* __restrict__ slots, uint32_t n,
                                                           uint32_t filter, float k, uint32_t colorize) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i < n) l2[slots[i]] = (uint16_t)(visual_epilogue(diffs[i], filter, k, colorize != 0u) & 0xFFFFu);
}

// Exhaustive check of the table for the current properties: every snapshot
// byte S and every byte pair (max, min) -- all intensities of every chroma
// mode and of the prefiltered path -- through alt_lut_texel against the
// specification's texel.  blockIdx.y = S.
__global__ __launch_bounds__(256) void alt_lut_check_kernel(const uint32_t* __restrict__ l1,
                                                            const uint16_t* __restrict__ l2, uint32_t filter, float k,
                                                            uint32_t colorize, unsigned long long* __restrict__ bad) {
    const uint32_t p = blockIdx.x * 256u + threadIdx.x;  // mx * 256 + mn
    const uint32_t mx = p >> 8, mn = p & 0xFFu;
    if (mn > mx) return;
    const float diff = unorm_load(blockIdx.y) - intensity_rgb(mx, mn, mn, 0u);
    const uint32_t want = visual_epilogue(diff, filter, k, colorize != 0u);
    if (alt_lut_texel(l1, l2, diff) != want) atomicAdd(bad, 1ull);
}

}  // namespace

hipError_t launch_alt_lut_check(const uint32_t* l1, const uint16_t* l2, uint32_t filter, float k, bool colorize,
                                unsigned long long* bad, hipStream_t s) {
    hipLaunchKernelGGL(alt_lut_check_kernel, dim3(256, 256), dim3(256), 0, s, l1, l2, filter, k, colorize ? 1u : 0u,
                       bad);
    return hipGetLastError();
}

template <int U, int D>
static const void* alt_lut_ptr(int chroma) {
    switch (chroma) {
#define DIPS_ALT_LUT_CH(C) \
    case C: return reinterpret_cast<const void*>(&alt_batch_kernel<C, 0, 0, true, U, true, D>);
        DIPS_ALT_LUT_CH(0) DIPS_ALT_LUT_CH(1) DIPS_ALT_LUT_CH(2) DIPS_ALT_LUT_CH(3) DIPS_ALT_LUT_CH(kAltPrefiltered)
#undef DIPS_ALT_LUT_CH
        default: return nullptr;
    }
}

const void* alt_batch_lut_kernel_ptr(int chroma) { return alt_lut_ptr<kUnrollAltLut, kDepthAltLut>(chroma); }

hipError_t launch_alt_batch_lut(const AltBatchArgs& a, int chroma, uint32_t blocks, hipStream_t s) {
    const void* k = alt_batch_lut_kernel_ptr(chroma);
    if (!k || blocks == 0 || !a.lut_l1 || !a.lut_l2) return hipErrorInvalidValue;
    AltBatchArgs args = a;
    void* params[] = {&args};
    return hipLaunchKernel(k, dim3(blocks), dim3(256), params, 0, s);
}

hipError_t launch_alt_lut_fill(uint16_t* lut_l2, const float* diffs, const uint16_t* slots, uint32_t n,
                               uint32_t filter, float k, bool colorize, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(alt_lut_fill_kernel, dim3((n + 255u) / 256u), dim3(256), 0, s, lut_l2, diffs, slots, n, filter,
                       k, colorize ? 1u : 0u);
    return hipGetLastError();
}

template <int N>
hipError_t launch_frame_host_n(const AltArgs& a, const uint8_t* in, uint8_t* newest_slot, uint32_t newest,
                               hipStream_t s) {
    const uint32_t yend = a.y1 ? a.y1 : a.height;
    if (a.y0 >= yend || yend > a.height || a.window > 1 || newest >= (uint32_t)N) return hipErrorInvalidValue;
    const uint64_t n_px = (uint64_t)(yend - a.y0) * a.width;
    if (!fits_grid256(n_px)) return hipErrorInvalidValue;
    hipLaunchKernelGGL((alt_frame_host_kernel<N>), dim3((uint32_t)((n_px + 255) / 256)), dim3(256), 0, s, a, in,
                       newest_slot, newest);
    return hipGetLastError();
}

hipError_t launch_alt_frame_host(const AltArgs& a, const uint8_t* in, uint8_t* newest_slot, uint32_t newest,
                                 hipStream_t s) {
    switch (a.n_tex) {
#define DIPS_ALT_N(NV) \
    case NV: return launch_frame_host_n<NV>(a, in, newest_slot, newest, s);
        DIPS_ALT_N(1) DIPS_ALT_N(2) DIPS_ALT_N(3) DIPS_ALT_N(4) DIPS_ALT_N(5) DIPS_ALT_N(6) DIPS_ALT_N(7)
        DIPS_ALT_N(8) DIPS_ALT_N(9) DIPS_ALT_N(10) DIPS_ALT_N(11) DIPS_ALT_N(12) DIPS_ALT_N(13)
        DIPS_ALT_N(14) DIPS_ALT_N(15) DIPS_ALT_N(16)
#undef DIPS_ALT_N
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_alt_frame(const AltArgs& a, hipStream_t s) {
    switch (a.n_tex) {
#define DIPS_ALT_N(NV) \
    case NV: return launch_frame_n<NV>(a, s);
        DIPS_ALT_N(1) DIPS_ALT_N(2) DIPS_ALT_N(3) DIPS_ALT_N(4) DIPS_ALT_N(5) DIPS_ALT_N(6) DIPS_ALT_N(7)
        DIPS_ALT_N(8) DIPS_ALT_N(9) DIPS_ALT_N(10) DIPS_ALT_N(11) DIPS_ALT_N(12) DIPS_ALT_N(13)
        DIPS_ALT_N(14) DIPS_ALT_N(15) DIPS_ALT_N(16)
#undef DIPS_ALT_N
        default: return hipErrorInvalidValue;
    }
}

const void* alt_batch_kernel_ptr(int chroma, int filter, bool colorize, bool fast) {
    switch (chroma) {
        case 0: return batch_ptr_c<0>(filter, colorize, fast);
        case 1: return batch_ptr_c<1>(filter, colorize, fast);
        case 2: return batch_ptr_c<2>(filter, colorize, fast);
        case 3: return batch_ptr_c<3>(filter, colorize, fast);
        case kAltPrefiltered: return batch_ptr_c<kAltPrefiltered>(filter, colorize, fast);
        default: return nullptr;
    }
}

hipError_t launch_alt_batch(const AltBatchArgs& a, int chroma, int filter, bool colorize, bool fast, uint32_t blocks,
                            hipStream_t s) {
    const void* k = alt_batch_kernel_ptr(chroma, filter, colorize, fast);
    if (!k || blocks == 0) return hipErrorInvalidValue;
    AltBatchArgs args = a;
    void* params[] = {&args};
    return hipLaunchKernel(k, dim3(blocks), dim3(256), params, 0, s);
}

hipError_t launch_alt_filter_frames(const uint8_t* frames, float* dst, uint32_t width, uint32_t height, uint32_t n,
                                   int32_t window, uint32_t chroma, hipStream_t s) {
    if (n == 0) return hipSuccess;
    if (n > 65535u) return hipErrorInvalidValue;
    dim3 grid((width + kTile - 1) / kTile, (height + kTile - 1) / kTile, n);
    switch (window) {
#define DIPS_WIN(W)                                                                                             \
    case W:                                                                                                     \
        hipLaunchKernelGGL(alt_filter_frames_kernel<W>, grid, dim3(kTile, kTile / 2), 0, s, frames, dst, width, \
                           height, chroma);                                                                     \
        break;
        DIPS_WIN(2) DIPS_WIN(3) DIPS_WIN(4) DIPS_WIN(5) DIPS_WIN(6) DIPS_WIN(7) DIPS_WIN(8) DIPS_WIN(9) DIPS_WIN(10)
        DIPS_WIN(11)
#undef DIPS_WIN
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// Ring-slot refresh after a batch (write_texture, dips_alt mod.rs:510-521):
// up to two frame copies in one launch on the compute stream.  A
// device-to-device hipMemcpyAsync is an SDMA job, queued on the same copy
// engines as the pipelined PCIe feed; as a kernel it takes a few microseconds
// of HBM time instead.
__global__ __launch_bounds__(256) void copy_frames_kernel(CopyFramesArgs a) {
    const uint32_t j = blockIdx.y;
    const uint4* __restrict__ src = reinterpret_cast<const uint4*>(a.src[j]);
    uint4* __restrict__ dst = reinterpret_cast<uint4*>(a.dst[j]);
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < a.n16; i += (uint64_t)gridDim.x * 256u)
        dst[i] = src[i];
}

hipError_t launch_copy_frames(const CopyFramesArgs& a, uint32_t count, hipStream_t s) {
    if (count == 0) return hipSuccess;
    if (count > 2) return hipErrorInvalidValue;
    const uint64_t want = (a.n16 + 255u) / 256u;
    const uint32_t bx = (uint32_t)(want < 2048u ? (want == 0 ? 1u : want) : 2048u);
    hipLaunchKernelGGL(copy_frames_kernel, dim3(bx, count), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace dips
