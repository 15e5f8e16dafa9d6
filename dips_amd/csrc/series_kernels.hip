// series_kernels.hip -- the hot path: per-frame difference series on gfx950.
//
// What it computes (north star; reference semantics dips_shader.wgsl:64-82
// for the intensity, README.md:7-11 for the two modes): for every frame F_t
// of a batch and its reference R (frame 0 / a given frame for 'overall', the
// previous frame for 'per-frame'), one dips_series_entry {SAD, SJ, count,
// SI_fixed} and optionally the byte map |F_t - R|.
//
// Layout and schedule (DESIGN.md "series_fast"):
//  * a frame is a flat byte array; one lane owns a "vec" of whole pixels,
//    RGB8 12 B = 4 px, RGBA8 16 B = 4 px, GRAY8 16 B = 16 px, loaded with one
//    buffer_load_dwordx3/x4 (nt) so a wave-instruction reads 768 B / 1 KiB
//    of contiguous HBM;
//  * a tile = 64 lanes x U vecs, fixed for the whole frame batch; the
//    reference's derived state (bytes, J pairs, f32 intensity) for the tile
//    stays in VGPRs, so every frame byte is read from HBM exactly once;
//  * the (tile, frame) space is split into one contiguous range per resident
//    wave (persistent grid, perfectly balanced); a wave walks frames of one
//    tile with the next frame's loads in flight while it reduces the current;
//  * per (tile, frame) the wave reduces in registers/DPP and lane 0 writes one
//    16-byte partial record; series_reduce sums the records per frame with
//    64-bit integer atomics (order-independent, hence bit-reproducible).
#include "dips_math.h"
#include "dips_kernels.h"

namespace dips {

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// gfx950 buffer-resource flags word (raw buffer, 32-bit format).
constexpr int kRsrcFlags = 0x00020000;
// cache policy of the streamed frame loads: nt (stream once).
constexpr int kAuxNT = 2;

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

template <int C>
__device__ __forceinline__ void load_vec(__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t (&v)[Fmt<C>::NDW]) {
    if constexpr (Fmt<C>::NDW == 3) {
        const u32x3 x = __builtin_amdgcn_raw_buffer_load_b96(r, off, 0, kAuxNT);
        v[0] = x.x; v[1] = x.y; v[2] = x.z;
    } else {
        const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kAuxNT);
        v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
    }
}

template <int C>
__device__ __forceinline__ void store_vec(__amdgpu_buffer_rsrc_t r, uint32_t off, const uint32_t (&v)[Fmt<C>::NDW]) {
    if constexpr (Fmt<C>::NDW == 3) {
        u32x3 x; x.x = v[0]; x.y = v[1]; x.z = v[2];
        __builtin_amdgcn_raw_buffer_store_b96(x, r, off, 0, kAuxNT);
    } else {
        u32x4 x; x.x = v[0]; x.y = v[1]; x.z = v[2]; x.w = v[3];
        __builtin_amdgcn_raw_buffer_store_b128(x, r, off, 0, kAuxNT);
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

// Derived state of 4 RGB(A) pixels: J = max+min as two u16 pairs and the
// doubled intensity I2 = u(max) + u(min) (= 2 * get_intensity, exact).
struct Px4 {
    uint32_t j[2];
    float i2[4];
};

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

template <int C, int CH>
__device__ __forceinline__ void derive_px4(const uint32_t (&d)[Fmt<C>::NDW], const float* lut, Px4& s) {
    u16x2 r[2], g[2], b[2];
    pair_planes<C>(d, r, g, b);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        u16x2 mx, mn;
        if constexpr (CH == 0) {
            mx = __builtin_elementwise_max(__builtin_elementwise_max(r[k], g[k]), b[k]);
            mn = __builtin_elementwise_min(__builtin_elementwise_min(r[k], g[k]), b[k]);
        } else if constexpr (CH == 1) {
            mx = mn = r[k];
        } else if constexpr (CH == 2) {
            mx = mn = g[k];
        } else {
            mx = mn = b[k];
        }
        s.j[k] = as_u32(mx + mn);
        s.i2[2 * k + 0] = lut[mx.x] + lut[mn.x];
        s.i2[2 * k + 1] = lut[mx.y] + lut[mn.y];
    }
}

template <int C> struct RefState;
template <> struct RefState<3> { uint32_t b[3]; Px4 px; };
template <> struct RefState<4> { uint32_t b[4]; Px4 px; };
template <> struct RefState<1> { uint32_t b[4]; float i[16]; };

struct Acc {
    uint32_t sad, sj, cnt;
    double si;
};

template <int C, int CH>
__device__ __forceinline__ void derive_ref(const uint32_t (&d)[Fmt<C>::NDW], const float* lut, RefState<C>& s) {
#pragma unroll
    for (int k = 0; k < Fmt<C>::NDW; ++k) s.b[k] = d[k];
    if constexpr (C == 1) {
#pragma unroll
        for (int k = 0; k < 16; ++k) s.i[k] = lut[(d[k >> 2] >> (8 * (k & 3))) & 0xFFu];
    } else {
        derive_px4<C, CH>(d, lut, s.px);
    }
}

// Accumulate one vec of the current frame against the reference state; in
// per-frame mode the state then becomes the current frame's.
template <int C, int CH, bool PF, bool MAP>
__device__ __forceinline__ void process_vec(RefState<C>& ref, const uint32_t (&f)[Fmt<C>::NDW], const float* lut,
                                            float thr, Acc& acc, uint32_t (&map)[Fmt<C>::NDW]) {
#pragma unroll
    for (int k = 0; k < Fmt<C>::NDW; ++k) {
        acc.sad = __builtin_amdgcn_sad_u8(f[k], ref.b[k], acc.sad);
        if constexpr (MAP) map[k] = absdiff_bytes(f[k], ref.b[k]);
    }
    if constexpr (C == 1) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const float cur = lut[(f[k >> 2] >> (8 * (k & 3))) & 0xFFu];
            const float a = fabsf(cur - ref.i[k]);
            const bool sel = a > thr;
            acc.cnt += sel ? 1u : 0u;
            acc.si += (double)(sel ? a : 0.0f);
            if constexpr (PF) ref.i[k] = cur;
        }
    } else {
        Px4 cur;
        derive_px4<C, CH>(f, lut, cur);
        acc.sj = __builtin_amdgcn_sad_u16(cur.j[0], ref.px.j[0], acc.sj);
        acc.sj = __builtin_amdgcn_sad_u16(cur.j[1], ref.px.j[1], acc.sj);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float a = fabsf(cur.i2[k] - ref.px.i2[k]);
            const bool sel = a > thr;
            acc.cnt += sel ? 1u : 0u;
            acc.si += (double)(sel ? a : 0.0f);
        }
        if constexpr (PF) ref.px = cur;
    }
    if constexpr (PF) {
#pragma unroll
        for (int k = 0; k < Fmt<C>::NDW; ++k) ref.b[k] = f[k];
    }
}

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

template <int C, int CH, int U, bool PF, bool MAP>
__global__ __launch_bounds__(256) void series_fast_kernel(SeriesArgs a) {
    using F = Fmt<C>;
    __shared__ float lut[256];
    lut[threadIdx.x] = unorm_load(threadIdx.x);
    __syncthreads();

    const uint32_t lane = threadIdx.x & 63u;
    // wave id through readfirstlane: every loop bound and address below is
    // then provably wave-uniform (scalar registers, no waterfall loops).
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
    if (wave >= a.n_waves) return;
    const uint32_t fb = a.frame_bytes;
    // Doubled-intensity units for RGB(A) (I2 = 2I), plain intensity for gray.
    constexpr double kFixScale = (C == 1) ? 4294967296.0 : 2147483648.0;

    uint64_t i = (uint64_t)wave * a.items / a.n_waves;
    const uint64_t iend = (uint64_t)(wave + 1) * a.items / a.n_waves;
    while (i < iend) {
        const uint32_t tile = (uint32_t)(i / a.n_frames);
        uint32_t t = (uint32_t)(i - (uint64_t)tile * a.n_frames);
        const uint64_t remaining = iend - i;
        const uint32_t tend = (uint32_t)((uint64_t)a.n_frames < t + remaining ? (uint64_t)a.n_frames : t + remaining);
        i += tend - t;

        uint32_t voff[U];
#pragma unroll
        for (int u = 0; u < U; ++u) voff[u] = ((tile * U + u) * 64u + lane) * (uint32_t)F::VB;

        // Reference state of this tile.
        const uint8_t* rp = PF ? (t == 0 ? a.ref0 : a.frames + (uint64_t)(t - 1) * fb) : a.ref0;
        RefState<C> ref[U];
        {
            const __amdgpu_buffer_rsrc_t rr = make_rsrc(rp, fb);
            uint32_t d[U][F::NDW];
#pragma unroll
            for (int u = 0; u < U; ++u) load_vec<C>(rr, voff[u], d[u]);
#pragma unroll
            for (int u = 0; u < U; ++u) derive_ref<C, CH>(d[u], lut, ref[u]);
        }

        uint32_t cur[U][F::NDW];
        {
            const __amdgpu_buffer_rsrc_t rf = make_rsrc(a.frames + (uint64_t)t * fb, fb);
#pragma unroll
            for (int u = 0; u < U; ++u) load_vec<C>(rf, voff[u], cur[u]);
        }
        for (; t < tend; ++t) {
            uint32_t nxt[U][F::NDW];
            if (t + 1 < tend) {
                const __amdgpu_buffer_rsrc_t rn = make_rsrc(a.frames + (uint64_t)(t + 1) * fb, fb);
#pragma unroll
                for (int u = 0; u < U; ++u) load_vec<C>(rn, voff[u], nxt[u]);
            }
            Acc acc{0u, 0u, 0u, 0.0};
            uint32_t map[U][F::NDW];
#pragma unroll
            for (int u = 0; u < U; ++u) process_vec<C, CH, PF, MAP>(ref[u], cur[u], lut, a.thr, acc, map[u]);
            if constexpr (MAP) {
                const __amdgpu_buffer_rsrc_t rm = make_rsrc(a.dmap + (uint64_t)t * fb, fb);
#pragma unroll
                for (int u = 0; u < U; ++u) store_vec<C>(rm, voff[u], map[u]);
            }
            uint32_t sad = wave_sum_u32(acc.sad);
            uint32_t sj = (C == 1) ? 0u : wave_sum_u32(acc.sj);
            uint32_t cnt = wave_sum_u32(acc.cnt);
            double si = wave_sum_f64(acc.si);
            if (lane == 0) {
                if constexpr (C == 1) sj = 2u * sad;
                const uint64_t sif = (uint64_t)(si * kFixScale);
                u32x4 rec;
                rec.x = sad;
                rec.y = sj;
                const uint64_t hi = sif | ((uint64_t)cnt << 48);
                rec.z = (uint32_t)hi;
                rec.w = (uint32_t)(hi >> 32);
                *reinterpret_cast<u32x4*>(a.partials + 2 * ((uint64_t)tile * a.n_frames + t)) = rec;
            }
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int k = 0; k < F::NDW; ++k) cur[u][k] = nxt[u][k];
        }
    }
}

// Sum the 16-byte partial records of `tiles_per_thread` tiles for one frame
// and add them to the series with 64-bit integer atomics.
__global__ __launch_bounds__(256) void series_reduce_kernel(const uint64_t* __restrict__ partials, uint32_t n_frames,
                                                            uint32_t n_tiles, uint32_t tiles_per_block,
                                                            dips_series_entry* __restrict__ series) {
    const uint32_t t = blockIdx.x * 256u + threadIdx.x;
    if (t >= n_frames) return;
    const uint32_t tile0 = blockIdx.y * tiles_per_block;
    const uint32_t tile1 = min(n_tiles, tile0 + tiles_per_block);
    uint64_t sad = 0, sj = 0, cnt = 0, sif = 0;
    for (uint32_t tile = tile0; tile < tile1; ++tile) {
        const u32x4 rec = *reinterpret_cast<const u32x4*>(partials + 2 * ((uint64_t)tile * n_frames + t));
        sad += rec.x;
        sj += rec.y;
        const uint64_t hi = ((uint64_t)rec.w << 32) | rec.z;
        cnt += hi >> 48;
        sif += hi & 0x0000FFFFFFFFFFFFull;
    }
    atomicAdd(reinterpret_cast<unsigned long long*>(&series[t].sad), (unsigned long long)sad);
    atomicAdd(reinterpret_cast<unsigned long long*>(&series[t].sj), (unsigned long long)sj);
    atomicAdd(reinterpret_cast<unsigned long long*>(&series[t].count), (unsigned long long)cnt);
    atomicAdd(reinterpret_cast<unsigned long long*>(&series[t].si_fixed), (unsigned long long)sif);
}

// Generic path: any frame shape and alignment.  One thread per pixel, the
// intensity computed in the reference's own form ((cmax+cmin)/2.0,
// dips_shader.wgsl:73-81) rather than the fast kernel's I2 pairs, so the two
// kernels cross-check each other.
template <int C>
__global__ __launch_bounds__(256) void series_generic_kernel(GenericArgs a) {
    __shared__ uint64_t red[4][4];
    const uint32_t t = blockIdx.x / a.blocks_per_frame;
    const uint64_t p = (uint64_t)(blockIdx.x - t * a.blocks_per_frame) * 256u + threadIdx.x;
    const uint64_t fb = a.frame_bytes;
    const uint8_t* F = a.frames + (uint64_t)t * fb;
    const uint8_t* R = a.mode == 1u ? (t == 0 ? a.ref0 : a.frames + (uint64_t)(t - 1) * fb) : a.ref0;
    uint64_t sad = 0, sj = 0, cnt = 0, sif = 0;
    if (p < a.n_px) {
        uint32_t fv[4] = {0, 0, 0, 0}, rv[4] = {0, 0, 0, 0};
#pragma unroll
        for (int c = 0; c < C; ++c) {
            fv[c] = F[p * C + c];
            rv[c] = R[p * C + c];
            const uint32_t d = fv[c] > rv[c] ? fv[c] - rv[c] : rv[c] - fv[c];
            sad += d;
            if (a.dmap) a.dmap[(uint64_t)t * fb + p * C + c] = (uint8_t)d;
        }
        if constexpr (C == 1) {
            fv[1] = fv[2] = fv[0];
            rv[1] = rv[2] = rv[0];
        }
        const float If = intensity_rgb(fv[0], fv[1], fv[2], a.chroma);
        const float Ir = intensity_rgb(rv[0], rv[1], rv[2], a.chroma);
        uint32_t jf, jr;
        if (a.chroma >= 1u && a.chroma <= 3u) {
            jf = 2u * fv[a.chroma - 1u];
            jr = 2u * rv[a.chroma - 1u];
        } else {
            jf = max(max(fv[0], fv[1]), fv[2]) + min(min(fv[0], fv[1]), fv[2]);
            jr = max(max(rv[0], rv[1]), rv[2]) + min(min(rv[0], rv[1]), rv[2]);
        }
        sj = jf > jr ? jf - jr : jr - jf;
        const float dI = fabsf(If - Ir);
        if (dI > a.tau) {
            cnt = 1;
            sif = (uint64_t)((double)dI * 4294967296.0);
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        sad += __shfl_xor(sad, o, 64);
        sj += __shfl_xor(sj, o, 64);
        cnt += __shfl_xor(cnt, o, 64);
        sif += __shfl_xor(sif, o, 64);
    }
    const uint32_t w = threadIdx.x >> 6;
    if ((threadIdx.x & 63u) == 0) {
        red[w][0] = sad;
        red[w][1] = sj;
        red[w][2] = cnt;
        red[w][3] = sif;
    }
    __syncthreads();
    if (threadIdx.x < 4) {
        const uint64_t v = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
        atomicAdd(reinterpret_cast<unsigned long long*>(&a.series[t]) + threadIdx.x, (unsigned long long)v);
    }
}

// Synthetic frames: F_t[y,x,c] = clamp(base + blob_t + noise, 0, 255)
// (bit-identical to oracle/dips_oracle.c dips_oracle_synth).
__global__ __launch_bounds__(256) void synth_kernel(SynthArgs a) {
    const uint64_t stride = (uint64_t)gridDim.x * 256u;
    const uint64_t n_chunks = (a.total_bytes + 15u) / 16u;
    for (uint64_t g = (uint64_t)blockIdx.x * 256u + threadIdx.x; g < n_chunks; g += stride) {
        const uint64_t base = g * 16u;
        uint64_t tl = base / a.frame_bytes;
        uint64_t off = base - tl * a.frame_bytes;
        uint64_t pix = off / a.channels;
        uint32_t c = (uint32_t)(off - pix * a.channels);
        uint32_t y = (uint32_t)(pix / a.width);
        uint32_t x = (uint32_t)(pix - (uint64_t)y * a.width);
        uint64_t t = a.t0 + tl;
        uint64_t fkey = splitmix64(a.seed + t);
        int64_t cx = (int64_t)(((uint64_t)(a.width / 4u) + 4u * t) % a.width);
        const int64_t cy = a.height / 2u;
        const int64_t rad2 = (int64_t)a.radius * a.radius;
        uint32_t w[4] = {0, 0, 0, 0};
        const int nb = (int)((a.total_bytes - base) < 16u ? (a.total_bytes - base) : 16u);
        for (int k = 0; k < nb; ++k) {
            const uint64_t idx = ((uint64_t)y * a.width + x) * a.channels + c;
            const int64_t dx = (int64_t)x - cx, dy = (int64_t)y - cy;
            const int blob = (dx * dx + dy * dy <= rad2) ? 64 : 0;
            const int bse = (int)(splitmix64(a.seed ^ idx) & 0xFFu);
            const uint64_t h = splitmix64(fkey ^ idx);
            const int noise = (int)(((h >> 32) * 9u) >> 32) - 4;
            int v = bse + blob + noise;
            v = v < 0 ? 0 : (v > 255 ? 255 : v);
            w[k >> 2] |= (uint32_t)v << (8 * (k & 3));
            // advance (c, x, y, frame)
            if (++c == a.channels) {
                c = 0;
                if (++x == a.width) {
                    x = 0;
                    if (++y == a.height) {
                        y = 0;
                        ++t;
                        fkey = splitmix64(a.seed + t);
                        cx = (int64_t)(((uint64_t)(a.width / 4u) + 4u * t) % a.width);
                    }
                }
            }
        }
        uint8_t* dst = a.dst + base;
        if (nb == 16 && ((uintptr_t)dst & 15u) == 0) {
            u32x4 v4;
            v4.x = w[0]; v4.y = w[1]; v4.z = w[2]; v4.w = w[3];
            __builtin_nontemporal_store(v4, reinterpret_cast<u32x4*>(dst));
        } else {
            for (int k = 0; k < nb; ++k) dst[k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
        }
    }
}

// ---------------------------------------------------------------------------
// Host-side launchers (instantiation table)
// ---------------------------------------------------------------------------

template <int C, int CH, int U, bool PF, bool MAP>
static const void* fast_ptr() {
    return reinterpret_cast<const void*>(&series_fast_kernel<C, CH, U, PF, MAP>);
}

template <int C, int U>
static const void* pick_fast_u(int chroma, bool pf, bool map) {
    if constexpr (C == 1) {
        (void)chroma;
        return pf ? (map ? fast_ptr<C, 0, U, true, true>() : fast_ptr<C, 0, U, true, false>())
                  : (map ? fast_ptr<C, 0, U, false, true>() : fast_ptr<C, 0, U, false, false>());
    } else {
#define DIPS_PICK_CH(CHV)                                                                      \
    case CHV:                                                                                  \
        return pf ? (map ? fast_ptr<C, CHV, U, true, true>() : fast_ptr<C, CHV, U, true, false>()) \
                  : (map ? fast_ptr<C, CHV, U, false, true>() : fast_ptr<C, CHV, U, false, false>());
        switch (chroma) {
            DIPS_PICK_CH(0)
            DIPS_PICK_CH(1)
            DIPS_PICK_CH(2)
            DIPS_PICK_CH(3)
            default: return nullptr;
        }
#undef DIPS_PICK_CH
    }
}

int fast_unroll(int channels) { return channels == 1 ? kUnrollGray : kUnrollRGB; }

const void* series_fast_kernel_ptr(int channels, int chroma, bool per_frame, bool map) {
    switch (channels) {
        case 1: return pick_fast_u<1, kUnrollGray>(chroma, per_frame, map);
        case 3: return pick_fast_u<3, kUnrollRGB>(chroma, per_frame, map);
        case 4: return pick_fast_u<4, kUnrollRGB>(chroma, per_frame, map);
        default: return nullptr;
    }
}

int pixels_per_vec(int channels) { return channels == 1 ? 16 : 4; }

hipError_t launch_series_fast(const SeriesArgs& a, int channels, int chroma, bool per_frame, bool map,
                              uint32_t blocks, hipStream_t s) {
    const void* k = series_fast_kernel_ptr(channels, chroma, per_frame, map);
    if (!k) return hipErrorInvalidValue;
    SeriesArgs args = a;
    void* params[] = {&args};
    return hipLaunchKernel(k, dim3(blocks), dim3(256), params, 0, s);
}

hipError_t launch_series_reduce(const uint64_t* partials, uint32_t n_frames, uint32_t n_tiles,
                                dips_series_entry* series, hipStream_t s) {
    const uint32_t tpb = 64;
    dim3 grid((n_frames + 255u) / 256u, (n_tiles + tpb - 1u) / tpb);
    hipLaunchKernelGGL(series_reduce_kernel, grid, dim3(256), 0, s, partials, n_frames, n_tiles, tpb, series);
    return hipGetLastError();
}

hipError_t launch_series_generic(const GenericArgs& a, int channels, hipStream_t s) {
    const uint64_t blocks = (uint64_t)a.blocks_per_frame * a.n_frames;
    switch (channels) {
        case 1: hipLaunchKernelGGL(series_generic_kernel<1>, dim3((uint32_t)blocks), dim3(256), 0, s, a); break;
        case 3: hipLaunchKernelGGL(series_generic_kernel<3>, dim3((uint32_t)blocks), dim3(256), 0, s, a); break;
        case 4: hipLaunchKernelGGL(series_generic_kernel<4>, dim3((uint32_t)blocks), dim3(256), 0, s, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_synth(const SynthArgs& a, hipStream_t s) {
    const uint64_t n_chunks = (a.total_bytes + 15u) / 16u;
    uint64_t blocks = (n_chunks + 255u) / 256u;
    if (blocks > 8192u) blocks = 8192u;
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(synth_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace dips
