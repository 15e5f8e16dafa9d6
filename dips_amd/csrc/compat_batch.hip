// compat_batch.hip -- the dips ComputeState (frame_callback) over a batch of
// HBM-resident frames, W = 1, in steady state.
//
// From the 8th frame on (global index t >= 7) every slot of the temporal
// ring holds a frame that went through the in-place filter of compute_main
// (dips_shader.wgsl:123-126, 187): the gray texel q(I(F)).  The dispatch of
// frame t then reads the four slots {q_t, q_t-1, q_t-2, q_t-3} as u(q)
// (:192), and u() is increasing, so the upper median of the four intensities
// is u(upper median of the four bytes).  The per-pixel state is three bytes
// (the previous frames' q) plus the start-texture byte S, and the output is
// the epilogue of u(S) - u(m) (:213-239).  A wave owns a tile of 512 pixels
// and walks a chunk of frames with that state in registers (byte pairs as
// u16x2 planes, so the 4-way median is six packed u16 min/max per pixel
// pair); a chunk start rebuilds it from the three preceding frames (HBM) or,
// for the first chunk, from the ring slots.  The last chunk leaves the last
// four frames in the ring slots as gray texels, as the per-frame path would.
// Frames t < 7 (start texture, the unquantised F1..F3) go through the
// per-frame kernels (compat_kernels.hip); dips_abi.hip splits the batch.
#include "epilogue_fast.h"
#include "intensity_v2.h"

#include <cstdlib>

namespace dips {

namespace {

// exact u(c) for the two bytes of a u16x2 plane (low byte of each half)
__device__ __forceinline__ f32x2 unorm_plane(uint32_t p) {
    return unorm2(u16x2_to_f32x2(as_u16x2(p)));  // v_cvt_f32_ubyte0 / ubyte2
}

// gray RGBA texels (q, q, q, 255) of the two bytes of a plane
__device__ __forceinline__ void gray_pair(uint32_t p, uint32_t& lo, uint32_t& hi) {
    lo = __builtin_amdgcn_perm(p, p, 0x0D000000u);
    hi = __builtin_amdgcn_perm(p, p, 0x0D020202u);
}

// q(I) of a vec's four pixels as two u16x2 planes, from I2s = I * 2^23:
// I * 255 = I2s * (255 * 2^-23) (one rounding either way); I in [0, 1], so
// no clamp; + 2^23 rounds half-to-even into the mantissa's low byte.
__device__ __forceinline__ void quantise_planes(const St2& s, uint32_t (&q)[2]) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const uint32_t a = __float_as_uint(s.i[k].x * (255.0f / 8388608.0f) + 8388608.0f);
        const uint32_t b = __float_as_uint(s.i[k].y * (255.0f / 8388608.0f) + 8388608.0f);
        q[k] = __builtin_amdgcn_perm(b, a, 0x0C040C00u);
    }
}

// R bytes of a vec of four RGBA texels as two u16x2 planes
__device__ __forceinline__ void r_planes(const uint32_t (&d)[4], uint32_t (&q)[2]) {
    q[0] = __builtin_amdgcn_perm(d[1], d[0], 0x0C040C00u);
    q[1] = __builtin_amdgcn_perm(d[3], d[2], 0x0C040C00u);
}

__device__ __forceinline__ u16x2 umax(u16x2 a, u16x2 b) { return __builtin_elementwise_max(a, b); }
__device__ __forceinline__ u16x2 umin(u16x2 a, u16x2 b) { return __builtin_elementwise_min(a, b); }

// element [2] of the sorted four (upper median), per u16 lane
__device__ __forceinline__ uint32_t upper4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    const u16x2 A = as_u16x2(a), B = as_u16x2(b), C = as_u16x2(c), D = as_u16x2(d);
    return as_u32(umax(umax(umin(A, B), umin(C, D)), umin(umax(A, B), umax(C, D))));
}

template <int CH, int FILT, int COL, bool FAST, int U>
__global__ __launch_bounds__(256) void compat_batch_kernel(CompatBatchArgs a) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t item = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
    if (item >= a.n_tiles * a.n_chunks) return;
    const uint32_t c = item / a.n_tiles;
    const uint32_t tile = item - c * a.n_tiles;
    const uint32_t t0 = c * a.chunk;
    const uint32_t t1 = min(t0 + a.chunk, a.n_frames);
    const uint32_t fb = a.frame_bytes;
    uint32_t voff[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t vec = (tile * U + (uint32_t)u) * 64u + lane;
        voff[u] = vec < a.n_vec ? vec * 16u : 0x80000000u;  // out of range: loads 0, stores dropped
    }

    // u(S) of the start texture (textureLoad(start_texture).r, :213)
    f32x2 us[U][2];
    {
        const __amdgpu_buffer_rsrc_t r = make_rsrc(a.start, fb);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            uint32_t d[4], p[2];
            load_vec<4>(r, voff[u], d);
            r_planes(d, p);
            us[u][0] = unorm_plane(p[0]);
            us[u][1] = unorm_plane(p[1]);
        }
    }
    // q of the three frames before t0: ring slots (first chunk) or frames
    uint32_t q1[U][2], q2[U][2], q3[U][2];
    auto prev_q = [&](int j, uint32_t (&dst)[U][2]) {
        if (c == 0) {
            const __amdgpu_buffer_rsrc_t r = make_rsrc(a.pre[j], fb);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                uint32_t d[4];
                load_vec<4>(r, voff[u], d);
                r_planes(d, dst[u]);
            }
        } else {
            const __amdgpu_buffer_rsrc_t r = make_rsrc(a.frames + (uint64_t)(t0 - 1 - j) * fb, fb);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                uint32_t d[4];
                load_vec<4>(r, voff[u], d);
                St2 s;
                derive_v2<4, CH>(d, s);
                quantise_planes(s, dst[u]);
            }
        }
    };
    prev_q(0, q1);
    prev_q(1, q2);
    prev_q(2, q3);

    auto load_frame = [&](uint32_t t, uint32_t (&d)[U][4]) {
        const __amdgpu_buffer_rsrc_t r = make_rsrc(a.frames + (uint64_t)t * fb, fb);
#pragma unroll
        for (int u = 0; u < U; ++u) load_vec<4>(r, voff[u], d[u]);
    };
    auto process = [&](uint32_t t, const uint32_t (&d)[U][4]) {
        const __amdgpu_buffer_rsrc_t ro = make_rsrc(a.out + (uint64_t)t * fb, fb);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            St2 s;
            derive_v2<4, CH>(d[u], s);
            uint32_t q0[2];
            quantise_planes(s, q0);
            uint32_t o[4];
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const uint32_t m = upper4(q0[k], q1[u][k], q2[u][k], q3[u][k]);
                const f32x2 diff = us[u][k] - unorm_plane(m);
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const float df = h ? diff.y : diff.x;
                    if constexpr (FAST)
                        o[2 * k + h] = epilogue_fast<FILT, COL != 0>(df, a.kneg_half);
                    else
                        o[2 * k + h] = visual_epilogue(df, (uint32_t)FILT, a.k, COL != 0);
                }
                q3[u][k] = q2[u][k];
                q2[u][k] = q1[u][k];
                q1[u][k] = q0[k];
            }
            store_vec<4>(ro, voff[u], o);
        }
    };

    constexpr int D = 2;  // frames of loads in flight
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

    if (c + 1 == a.n_chunks) {
        // the ring slots of the last four frames hold their gray texels
        // (post[0] = frame n-1 ... post[3] = frame n-4; null = not in the batch)
        // frame n-4 left the register state; its q is rebuilt from HBM
        uint32_t q4[U][2];
        if (a.post[3] != nullptr) {
            const __amdgpu_buffer_rsrc_t r = make_rsrc(a.frames + (uint64_t)(a.n_frames - 4) * fb, fb);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                uint32_t d[4];
                load_vec<4>(r, voff[u], d);
                St2 s;
                derive_v2<4, CH>(d, s);
                quantise_planes(s, q4[u]);
            }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (a.post[j] == nullptr) continue;
            const __amdgpu_buffer_rsrc_t r = make_rsrc(a.post[j], fb);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t(&p)[2] = j == 0 ? q1[u] : (j == 1 ? q2[u] : (j == 2 ? q3[u] : q4[u]));
                uint32_t o[4];
                gray_pair(p[0], o[0], o[1]);
                gray_pair(p[1], o[2], o[3]);
                store_vec<4>(r, voff[u], o);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// The epilogue as a table.  In steady state (t >= 7, W = 1) the output texel
// of compute_main is a function of two bytes only: the start-texture byte S
// and the upper-median byte m (diff = u(S) - u(m), :192, :213; everything
// after is a pure function of diff and the properties).  compat_lut_kernel
// evaluates the specification (dips_math.h visual_epilogue) once per (S, m)
// and keeps R | G << 8; B and A follow: A = 255, and B = m' = min(R, G)
// because the colour branch stores (chroma + m', m', m') or (m', chroma + m',
// m') with chroma >= 0, q() is monotone and NaN stores as 0 (so NaN channels
// never exceed m'), and the gray branch stores R = G = B.  The batch kernel keeps the 128 KiB table
// in LDS (one 1024-thread workgroup per CU) and replaces the per-pixel
// filter / sigmoid / colour arithmetic with one ds_read_u16 per pixel, for
// every filter, sensitivity and colour setting alike.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void compat_lut_kernel(uint16_t* __restrict__ lut, uint32_t filter, float k,
                                                         uint32_t colorize) {
    const uint32_t idx = blockIdx.x * 256u + threadIdx.x;  // S * 256 + m
    const float diff = unorm_load(idx >> 8) - unorm_load(idx & 0xFFu);
    lut[idx] = (uint16_t)(visual_epilogue(diff, filter, k, colorize != 0u) & 0xFFFFu);
}

constexpr int kLutWaves = (int)kCompatLutWaves;

// U vecs per lane, D frames of loads in flight (D - 1 ahead of the one
// being processed)
template <int CH, int U, int D>
__global__ __launch_bounds__(64 * kLutWaves) void compat_batch_lut_kernel(CompatBatchArgs a) {
    __shared__ uint32_t lds[32768];  // 65536 u16 entries (128 KiB)
    {
        const u32x4* src = reinterpret_cast<const u32x4*>(a.lut);
        u32x4* dst = reinterpret_cast<u32x4*>(lds);
        for (uint32_t i = threadIdx.x; i < 8192u; i += 64u * kLutWaves) dst[i] = src[i];
    }
    __syncthreads();
    const uint16_t* tab = reinterpret_cast<const uint16_t*>(lds);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t item = __builtin_amdgcn_readfirstlane(blockIdx.x * (uint32_t)kLutWaves + (threadIdx.x >> 6));
    if (item >= a.n_tiles * a.n_chunks) return;
    const uint32_t c = item / a.n_tiles;
    const uint32_t tile = item - c * a.n_tiles;
    const uint32_t t0 = c * a.chunk;
    const uint32_t t1 = min(t0 + a.chunk, a.n_frames);
    const uint32_t fb = a.frame_bytes;
    uint32_t voff[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t vec = (tile * U + (uint32_t)u) * 64u + lane;
        voff[u] = vec < a.n_vec ? vec * 16u : 0x80000000u;  // out of range: loads 0, stores dropped
    }

    // S << 8 of the start texture's R bytes, as u16x2 planes: S * 256 + m is
    // then one OR per pixel pair
    uint32_t s8[U][2];
    {
        const __amdgpu_buffer_rsrc_t r = make_rsrc(a.start, fb);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            uint32_t d[4], p[2];
            load_vec<4>(r, voff[u], d);
            r_planes(d, p);
            s8[u][0] = p[0] << 8;
            s8[u][1] = p[1] << 8;
        }
    }
    uint32_t q1[U][2], q2[U][2], q3[U][2];
    auto prev_q = [&](int j, uint32_t (&dst)[U][2]) {
        if (c == 0) {
            const __amdgpu_buffer_rsrc_t r = make_rsrc(a.pre[j], fb);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                uint32_t d[4];
                load_vec<4>(r, voff[u], d);
                r_planes(d, dst[u]);
            }
        } else {
            const __amdgpu_buffer_rsrc_t r = make_rsrc(a.frames + (uint64_t)(t0 - 1 - j) * fb, fb);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                uint32_t d[4];
                load_vec<4>(r, voff[u], d);
                St2 s;
                derive_v2<4, CH>(d, s);
                quantise_planes(s, dst[u]);
            }
        }
    };
    prev_q(0, q1);
    prev_q(1, q2);
    prev_q(2, q3);

    auto load_frame = [&](uint32_t t, uint32_t (&d)[U][4]) {
        const __amdgpu_buffer_rsrc_t r = make_rsrc(a.frames + (uint64_t)t * fb, fb);
#pragma unroll
        for (int u = 0; u < U; ++u) load_vec<4>(r, voff[u], d[u]);
    };
    auto process = [&](uint32_t t, const uint32_t (&d)[U][4]) {
        const __amdgpu_buffer_rsrc_t ro = make_rsrc(a.out + (uint64_t)t * fb, fb);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            St2 s;
            derive_v2<4, CH>(d[u], s);
            uint32_t q0[2];
            quantise_planes(s, q0);
            uint32_t o[4];
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const uint32_t x = s8[u][k] | upper4(q0[k], q1[u][k], q2[u][k], q3[u][k]);
                o[2 * k] = lut_texel(tab[x & 0xFFFFu]);
                o[2 * k + 1] = lut_texel(tab[x >> 16]);
                q3[u][k] = q2[u][k];
                q2[u][k] = q1[u][k];
                q1[u][k] = q0[k];
            }
            store_vec<4>(ro, voff[u], o);
        }
    };

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

    if (c + 1 == a.n_chunks) {
        uint32_t q4[U][2];
        if (a.post[3] != nullptr) {
            const __amdgpu_buffer_rsrc_t r = make_rsrc(a.frames + (uint64_t)(a.n_frames - 4) * fb, fb);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                uint32_t d[4];
                load_vec<4>(r, voff[u], d);
                St2 s;
                derive_v2<4, CH>(d, s);
                quantise_planes(s, q4[u]);
            }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (a.post[j] == nullptr) continue;
            const __amdgpu_buffer_rsrc_t r = make_rsrc(a.post[j], fb);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t(&p)[2] = j == 0 ? q1[u] : (j == 1 ? q2[u] : (j == 2 ? q3[u] : q4[u]));
                uint32_t o[4];
                gray_pair(p[0], o[0], o[1]);
                gray_pair(p[1], o[2], o[3]);
                store_vec<4>(r, voff[u], o);
            }
        }
    }
}

template <int CH, int FILT, bool FAST>
const void* cb_ptr_fc(bool colorize) {
    return colorize ? reinterpret_cast<const void*>(&compat_batch_kernel<CH, FILT, 1, FAST, kUnrollCompatBatch>)
                    : reinterpret_cast<const void*>(&compat_batch_kernel<CH, FILT, 0, FAST, kUnrollCompatBatch>);
}

template <int CH>
const void* cb_ptr_c(int filter, bool colorize, bool fast) {
    switch (filter) {
        case 0: return fast ? cb_ptr_fc<CH, 0, true>(colorize) : cb_ptr_fc<CH, 0, false>(colorize);
        case 1: return cb_ptr_fc<CH, 1, false>(colorize);
        default: return cb_ptr_fc<CH, 255, true>(colorize);  // DiPsFilter::Unfiltered and any other code
    }
}

}  // namespace

const void* compat_batch_kernel_ptr(int chroma, int filter, bool colorize, bool fast) {
    switch (chroma) {
        case 0: return cb_ptr_c<0>(filter, colorize, fast);
        case 1: return cb_ptr_c<1>(filter, colorize, fast);
        case 2: return cb_ptr_c<2>(filter, colorize, fast);
        case 3: return cb_ptr_c<3>(filter, colorize, fast);
        default: return nullptr;
    }
}

template <int U, int D>
static const void* cbl_ptr(int chroma) {
    switch (chroma) {
        case 0: return reinterpret_cast<const void*>(&compat_batch_lut_kernel<0, U, D>);
        case 1: return reinterpret_cast<const void*>(&compat_batch_lut_kernel<1, U, D>);
        case 2: return reinterpret_cast<const void*>(&compat_batch_lut_kernel<2, U, D>);
        case 3: return reinterpret_cast<const void*>(&compat_batch_lut_kernel<3, U, D>);
        default: return nullptr;
    }
}

const void* compat_batch_lut_kernel_ptr(int chroma) { return cbl_ptr<kUnrollCompatLut, kDepthCompatLut>(chroma); }

hipError_t launch_compat_lut(uint16_t* lut, uint32_t filter, float k, bool colorize, hipStream_t s) {
    hipLaunchKernelGGL(compat_lut_kernel, dim3(256), dim3(256), 0, s, lut, filter, k, colorize ? 1u : 0u);
    return hipGetLastError();
}

hipError_t launch_compat_batch_lut(const CompatBatchArgs& a, int chroma, uint32_t blocks, hipStream_t s) {
    const void* k = compat_batch_lut_kernel_ptr(chroma);
    if (!k || blocks == 0 || !a.lut) return hipErrorInvalidValue;
    CompatBatchArgs args = a;
    void* params[] = {&args};
    return hipLaunchKernel(k, dim3(blocks), dim3(64 * kLutWaves), params, 0, s);
}

hipError_t launch_compat_batch(const CompatBatchArgs& a, int chroma, int filter, bool colorize, bool fast,
                               uint32_t blocks, hipStream_t s) {
    const void* k = compat_batch_kernel_ptr(chroma, filter, colorize, fast);
    if (!k || blocks == 0) return hipErrorInvalidValue;
    CompatBatchArgs args = a;
    void* params[] = {&args};
    return hipLaunchKernel(k, dim3(blocks), dim3(256), params, 0, s);
}

}  // namespace dips
