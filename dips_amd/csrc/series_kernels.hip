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
#include "series_common.h"

namespace dips {

// Derived state of 4 RGB(A) pixels: J = max+min as two u16 pairs and the
// doubled intensity I2 = u(max) + u(min) (= 2 * get_intensity, exact), as
// two f32 pairs.
struct Px4 {
    uint32_t j[2];
    f32x2 i2[2];
};

// Placeholder kept in the signatures of the per-vec helpers; the exact
// arithmetic u() needs no table (an LDS table measured slower on gfx950).
struct Lut {
    const float* p;
    uint32_t lb;  // lane & 31
};

__device__ __forceinline__ f32x2 unorm_pair(u16x2 v, Lut) { return unorm2(u16x2_to_f32x2(v)); }

template <int C, int CH>
__device__ __forceinline__ void derive_px4(const uint32_t (&d)[Fmt<C>::NDW], Px4& s, Lut lut) {
    u16x2 r[2], g[2], b[2];
    pair_planes<C>(d, r, g, b);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        if constexpr (CH == 0) {
            const u16x2 mx = __builtin_elementwise_max(__builtin_elementwise_max(r[k], g[k]), b[k]);
            const u16x2 mn = __builtin_elementwise_min(__builtin_elementwise_min(r[k], g[k]), b[k]);
            s.j[k] = as_u32(mx + mn);
            s.i2[k] = unorm_pair(mx, lut) + unorm_pair(mn, lut);
        } else {
            const u16x2 ch = CH == 1 ? r[k] : (CH == 2 ? g[k] : b[k]);
            s.j[k] = as_u32(ch + ch);
            const f32x2 uc = unorm_pair(ch, lut);
            s.i2[k] = uc + uc;
        }
    }
}

template <int C> struct RefState;
template <> struct RefState<3> { uint32_t b[3]; Px4 px; };
template <> struct RefState<4> { uint32_t b[4]; Px4 px; };
template <> struct RefState<1> { uint32_t b[4]; f32x2 i[8]; };

// Per-lane accumulators.  Each selected dI is an f32 multiple of 2^-31
// (RGB, I2 units) or 2^-32 (gray) in [0, 2], so a per-lane f64 sum of up to
// 32 of them is EXACT (< 2^6 with 2^-32 granularity: 38 bits < 53).  The
// pixel count is wave-wide: the popcount of each compare mask on the scalar
// unit (measured: an LDS table for u() and a per-lane count in VALU are both
// slower; an f32 hi/lo split of dI is exact too but costs more VALU).
struct Acc {
    uint32_t sad, sj;  // per lane
    uint32_t cnt;      // wave-wide
    double si;         // per lane
};

__device__ __forceinline__ void acc_intensity(Acc& acc, f32x2 cur, f32x2 ref, float thr) {
    const f32x2 d = cur - ref;
    const float a0 = fabsf(d.x), a1 = fabsf(d.y);
    const bool s0 = a0 > thr, s1 = a1 > thr;
    acc.cnt += (uint32_t)__builtin_popcountll(__ballot(s0)) + (uint32_t)__builtin_popcountll(__ballot(s1));
    acc.si += (double)(s0 ? a0 : 0.0f) + (double)(s1 ? a1 : 0.0f);
}

template <int C, int CH>
__device__ __forceinline__ void derive_ref(const uint32_t (&d)[Fmt<C>::NDW], RefState<C>& s, Lut lut) {
#pragma unroll
    for (int k = 0; k < Fmt<C>::NDW; ++k) s.b[k] = d[k];
    if constexpr (C == 1) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t w = d[k >> 1] >> (16 * (k & 1));
            s.i[k] = unorm2(f32x2{(float)(w & 0xFFu), (float)((w >> 8) & 0xFFu)});
        }
    } else {
        derive_px4<C, CH>(d, s.px, lut);
    }
}

// Accumulate one vec of the current frame against the reference state `ref`;
// in per-frame mode the current frame's state is written to `next` (the
// caller ping-pongs two state arrays, so no register copies are needed).
template <int C, int CH, bool PF, bool MAP>
__device__ __forceinline__ void process_vec(const RefState<C>& ref, RefState<C>& next, const uint32_t (&f)[Fmt<C>::NDW],
                                            float thr, Acc& acc, uint32_t (&map)[Fmt<C>::NDW], Lut lut) {
#pragma unroll
    for (int k = 0; k < Fmt<C>::NDW; ++k) {
        acc.sad = __builtin_amdgcn_sad_u8(f[k], ref.b[k], acc.sad);
        if constexpr (MAP) map[k] = absdiff_bytes(f[k], ref.b[k]);
    }
    if constexpr (C == 1) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t w = f[k >> 1] >> (16 * (k & 1));
            const f32x2 cur = unorm2(f32x2{(float)(w & 0xFFu), (float)((w >> 8) & 0xFFu)});
            acc_intensity(acc, cur, ref.i[k], thr);
            if constexpr (PF) next.i[k] = cur;
        }
    } else {
        Px4 cur;
        derive_px4<C, CH>(f, cur, lut);
        acc.sj = __builtin_amdgcn_sad_u16(cur.j[0], ref.px.j[0], acc.sj);
        acc.sj = __builtin_amdgcn_sad_u16(cur.j[1], ref.px.j[1], acc.sj);
        acc_intensity(acc, cur.i2[0], ref.px.i2[0], thr);
        acc_intensity(acc, cur.i2[1], ref.px.i2[1], thr);
        if constexpr (PF) next.px = cur;
    }
    if constexpr (PF) {
#pragma unroll
        for (int k = 0; k < Fmt<C>::NDW; ++k) next.b[k] = f[k];
    }
}

// Accumulate one frame of one tile into four per-lane reduction values
//   RGB(A): {SAD, SJ + count << 20, H, L};  gray: {SAD + count << 20, H, L, 0}
// (H, L: the exact fixed-point split of the intensity sum, see Acc).  The
// count rides in bits 20.. because both wave sums stay below 2^20 for the
// tile sizes used here (1024 RGB / 2048 gray pixels per wave and frame).
template <int C, int CH, int U, bool PF, bool MAP>
__device__ __forceinline__ void frame_accumulate(const SeriesArgs& a, const RefState<C> (&ref)[U],
                                                 RefState<C> (&next)[U], const uint32_t (&cur)[U][Fmt<C>::NDW],
                                                 const uint32_t (&voff)[U], uint32_t t, uint32_t* vals, Lut lut) {
    using F = Fmt<C>;
    constexpr int kScaleBits = (C == 1) ? 32 : 31;
    Acc acc{};
    uint32_t map[U][F::NDW];
#pragma unroll
    for (int u = 0; u < U; ++u) process_vec<C, CH, PF, MAP>(ref[u], next[u], cur[u], a.thr, acc, map[u], lut);
    if constexpr (MAP) {
        const __amdgpu_buffer_rsrc_t rm = make_rsrc(a.dmap + (uint64_t)t * a.frame_bytes, a.vec_bytes);
#pragma unroll
        for (int u = 0; u < U; ++u) store_vec<C>(rm, voff[u], map[u]);
    }
    // the wave-wide count enters the lane sum through lane 0 only
    acc.cnt = (threadIdx.x & 63u) == 0u ? acc.cnt : 0u;
    // exact per-lane fixed point, split so both halves sum in u32 over the
    // wave: H = whole units of 2^-16, L = the remainder in 2^-kScaleBits
    const double q = acc.si * 65536.0;
    const uint32_t hfix = (uint32_t)q;  // trunc
    const int32_t lfix = (int32_t)((q - (double)hfix) * (double)(1ull << (kScaleBits - 16)));
    if constexpr (C == 1) {
        vals[0] = acc.sad + (acc.cnt << 20);
        vals[1] = hfix;
        vals[2] = (uint32_t)lfix;
        vals[3] = 0u;
    } else {
        vals[0] = acc.sad;
        vals[1] = acc.sj + (acc.cnt << 20);
        vals[2] = hfix;
        vals[3] = (uint32_t)lfix;
    }
}

// Partial record of one (tile, frame): the four raw wave sums (decoded by
// series_reduce_kernel, see decode_record); written by lane 0 only, branch
// free: the other lanes' offsets fall outside the descriptor's range and the
// hardware drops them.
template <int C>
__device__ __forceinline__ void write_record(__amdgpu_buffer_rsrc_t rpart, uint32_t t, uint32_t lane,
                                             const uint32_t* s) {
    u32x4 rec;
    rec.x = s[0];
    rec.y = s[1];
    rec.z = s[2];
    rec.w = s[3];
    __builtin_amdgcn_raw_buffer_store_b128(rec, rpart, lane == 0 ? t * 16u : 0x80000000u, 0, 0);
}

// D = frames of loads kept in flight per wave (register ring of D frames);
// frames are processed in pairs whose eight reduction values share one
// wave_sum8.
#ifndef DIPS_MIN_WAVES_PER_SIMD
#define DIPS_MIN_WAVES_PER_SIMD 1
#endif
template <int C, int CH, int U, int D, bool PF, bool MAP>
__global__ __launch_bounds__(256, DIPS_MIN_WAVES_PER_SIMD) void series_fast_kernel(SeriesArgs a) {
    static_assert(D % 2 == 0, "frames are processed in pairs: D must be even");
    using F = Fmt<C>;
    const uint32_t lane = threadIdx.x & 63u;
    const Lut lut{nullptr, lane & 31u};
    // wave id through readfirstlane: every loop bound and address below is
    // then provably wave-uniform (scalar registers, no waterfall loops).
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
    if (wave >= a.n_waves) return;
    const uint32_t fb = a.frame_bytes, vb = a.vec_bytes;

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

        // Reference state of this tile (ping-pong pair in per-frame mode:
        // even frames read sa and write sb, odd frames the reverse).
        const uint8_t* rp = PF ? (t == 0 ? a.ref0 : a.frames + (uint64_t)(t - 1) * fb) : a.ref0;
        RefState<C> sa[U], sb[U];
        {
            const __amdgpu_buffer_rsrc_t rr = make_rsrc(rp, vb);
            uint32_t d[U][F::NDW];
#pragma unroll
            for (int u = 0; u < U; ++u) load_vec<C>(rr, voff[u], d[u]);
#pragma unroll
            for (int u = 0; u < U; ++u) derive_ref<C, CH>(d[u], sa[u], lut);
        }
        const __amdgpu_buffer_rsrc_t rpart = make_rsrc(a.partials + 2 * (uint64_t)tile * a.n_frames, a.n_frames * 16u);
#ifdef DIPS_PROBE_SAMEFRAME
        // probe build only: every frame load re-reads the segment's first
        // frame (L2/MALL hits) -- the kernel's compute-only time
        const uint32_t tlast = t;
#else
        const uint32_t tlast = tend - 1;
#endif

        // Ring of D frames in flight; loads past the segment are clamped to
        // its last frame (one redundant frame per segment, no branches).
        uint32_t buf[D][U][F::NDW];
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const uint32_t tl = min(t + (uint32_t)d, tlast);
            const __amdgpu_buffer_rsrc_t rf = make_rsrc(a.frames + (uint64_t)tl * fb, vb);
#pragma unroll
            for (int u = 0; u < U; ++u) load_vec<C>(rf, voff[u], buf[d][u]);
        }
        // Steady state: D frames per iteration, straight-line code.
        for (; t + D <= tend; t += D) {
#pragma unroll
            for (int d = 0; d < D; d += 2) {
                uint32_t v[8], sum[8];
                frame_accumulate<C, CH, U, PF, MAP>(a, sa, sb, buf[d], voff, t + d, v, lut);
                // keep the refill of buf[d] behind its last use: hoisting it
                // would cost a register copy of the whole buffer
                __builtin_amdgcn_sched_barrier(0);
                {
                    const uint32_t tl = min(t + (uint32_t)(d + D), tlast);
                    const __amdgpu_buffer_rsrc_t rn = make_rsrc(a.frames + (uint64_t)tl * fb, vb);
#pragma unroll
                    for (int u = 0; u < U; ++u) load_vec<C>(rn, voff[u], buf[d][u]);
                }
                if constexpr (PF) frame_accumulate<C, CH, U, PF, MAP>(a, sb, sa, buf[d + 1], voff, t + d + 1, v + 4, lut);
                else frame_accumulate<C, CH, U, PF, MAP>(a, sa, sb, buf[d + 1], voff, t + d + 1, v + 4, lut);
                __builtin_amdgcn_sched_barrier(0);
                {
                    const uint32_t tl = min(t + (uint32_t)(d + 1 + D), tlast);
                    const __amdgpu_buffer_rsrc_t rn = make_rsrc(a.frames + (uint64_t)tl * fb, vb);
#pragma unroll
                    for (int u = 0; u < U; ++u) load_vec<C>(rn, voff[u], buf[d + 1][u]);
                }
                wave_sum8(v, sum, lane);
                write_record<C>(rpart, t + d, lane, sum);
                write_record<C>(rpart, t + d + 1, lane, sum + 4);
            }
        }
        // Tail (< D frames): already in buf[0 .. tend - t - 1].  State parity
        // is even here (D is even), so frame t + d reads sa when d is even.
#pragma unroll
        for (int d = 0; d < D - 1; ++d) {
            if (t + d < tend) {
                uint32_t v[4], sum[4];
                if (PF && (d & 1)) frame_accumulate<C, CH, U, PF, MAP>(a, sb, sa, buf[d], voff, t + d, v, lut);
                else frame_accumulate<C, CH, U, PF, MAP>(a, sa, sb, buf[d], voff, t + d, v, lut);
                wave_sum4(v, sum);
                write_record<C>(rpart, t + d, lane, sum);
            }
        }
    }
}

// Sum the 16-byte partial records of `tiles_per_block` tiles for one frame
// and add them to the series with 64-bit integer atomics.  A record holds the
// four wave sums of one (tile, frame):
//   RGB(A): {SAD, SJ + count << 20, H, L}     SI_fixed = H << 15 + L
//   gray:   {SAD + count << 20, H, L, 0}      SI_fixed = H << 16 + L, SJ = 2 SAD
//   gray table kernel: {SAD, sum d, sum corr, count}
//                                             SI_fixed = 2 (8421504 sum d + sum corr), SJ = 2 SAD
// (H, L: the split of the exact per-lane fixed-point intensity sum).
struct ReduceAcc {
    uint64_t sad = 0, sj = 0, cnt = 0, h = 0;
    int64_t l = 0;
};

template <uint32_t LAYOUT>
__device__ __forceinline__ void reduce_add(ReduceAcc& s, const u32x4 rec) {
    if constexpr (LAYOUT == 2u) {
        s.sad += rec.x;
        s.h += rec.y;  // sum d
        s.l += rec.z;  // sum corr
        s.cnt += rec.w;
    } else if constexpr (LAYOUT == 1u) {
        s.sad += rec.x & 0xFFFFFu;
        s.cnt += rec.x >> 20;
        s.h += rec.y;
        s.l += (int64_t)(int32_t)rec.z;
    } else {
        s.sad += rec.x;
        s.sj += rec.y & 0xFFFFFu;
        s.cnt += rec.y >> 20;
        s.h += rec.z;
        s.l += (int64_t)(int32_t)rec.w;
    }
}

// Records of tiles tile0 .. tile1-1 for frame t: eight independent loads in
// flight per thread (a rolled loop with the layout test inside kept one and
// ran latency-bound); each record is read once, hence non-temporal.
template <uint32_t LAYOUT>
__device__ __forceinline__ void reduce_tiles(ReduceAcc& s, const uint64_t* __restrict__ partials, uint32_t n_frames,
                                             uint32_t t, uint32_t tile0, uint32_t tile1) {
    const u32x4* p = reinterpret_cast<const u32x4*>(partials) + ((uint64_t)tile0 * n_frames + t);
    uint32_t tile = tile0;
    for (; tile + 8u <= tile1; tile += 8u, p += 8u * (uint64_t)n_frames) {
        u32x4 rec[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) rec[k] = __builtin_nontemporal_load(p + (uint64_t)k * n_frames);
#pragma unroll
        for (int k = 0; k < 8; ++k) reduce_add<LAYOUT>(s, rec[k]);
    }
    for (; tile < tile1; ++tile, p += n_frames) reduce_add<LAYOUT>(s, __builtin_nontemporal_load(p));
}

__global__ __launch_bounds__(256) void series_reduce_kernel(const uint64_t* __restrict__ partials, uint32_t n_frames,
                                                            uint32_t n_tiles, uint32_t tiles_per_block, uint32_t layout,
                                                            dips_series_entry* __restrict__ series) {
    const uint32_t t = blockIdx.x * 256u + threadIdx.x;
    if (t >= n_frames) return;
    const uint32_t tile0 = blockIdx.y * tiles_per_block;
    const uint32_t tile1 = min(n_tiles, tile0 + tiles_per_block);
    ReduceAcc s;
    if (layout == 2u)
        reduce_tiles<2u>(s, partials, n_frames, t, tile0, tile1);
    else if (layout == 1u)
        reduce_tiles<1u>(s, partials, n_frames, t, tile0, tile1);
    else
        reduce_tiles<0u>(s, partials, n_frames, t, tile0, tile1);
    const uint64_t sad = s.sad, cnt = s.cnt, h = s.h;
    const int64_t l = s.l;
    const uint64_t sj = (layout == 1u || layout == 2u) ? 2u * sad : s.sj;
    const uint64_t sif =
        layout == 2u ? 2u * (8421504u * h + (uint64_t)l) : (h << (layout == 1u ? 16 : 15)) + (uint64_t)l;
    atomicAdd(reinterpret_cast<unsigned long long*>(&series[t].sad), (unsigned long long)sad);
    atomicAdd(reinterpret_cast<unsigned long long*>(&series[t].sj), (unsigned long long)sj);
    atomicAdd(reinterpret_cast<unsigned long long*>(&series[t].count), (unsigned long long)cnt);
    atomicAdd(reinterpret_cast<unsigned long long*>(&series[t].si_fixed), (unsigned long long)sif);
}

// Read-only stream of `n16` 16-byte words (non-temporal loads, 4 in flight
// per lane, grid-stride): the measured read ceiling the series kernel is
// compared with ("% of a measured read-only-stream ceiling").
// The XOR keeps the loads alive; `out` is written only on a magic value.
__global__ __launch_bounds__(256) void read_ceiling_kernel(const u32x4* __restrict__ p, uint64_t n16,
                                                           uint32_t* __restrict__ out) {
    constexpr int kUnr = 4;
    uint32_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * 256u * kUnr;
    for (uint64_t i = (uint64_t)blockIdx.x * 256u * kUnr + threadIdx.x; i < n16; i += stride) {
        u32x4 v[kUnr];
#pragma unroll
        for (int u = 0; u < kUnr; ++u) {
            const uint64_t j = i + (uint64_t)u * 256u;
            v[u] = j < n16 ? __builtin_nontemporal_load(p + j) : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < kUnr; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    if (acc == 0x9E3779B9u) out[0] = acc;
}

// Read-only walk with the series kernels' access shape: the persistent
// (tile, frame) item schedule of series_v2_kernel -- one contiguous range per
// wave, or with a.part_frames = L > 0 the part-major schedule (items (part,
// tile) with stride n_waves, as series_v2_body) -- a wave's 64 lanes x U vecs
// of VB bytes per frame, two frames of loads in flight, no compute.  Its rate
// is the ceiling of that shape (profiles/r02_read_walk_probe.jsonl).
template <int VB, int U>
__global__ __launch_bounds__(256) void read_walk_kernel(SeriesArgs a, uint32_t* __restrict__ out) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
    if (wave >= a.n_waves) return;
    uint64_t i = (uint64_t)wave * a.items / a.n_waves;
    const uint64_t iend = (uint64_t)(wave + 1) * a.items / a.n_waves;
    const bool parts = a.part_frames != 0u;
    const uint32_t plen = parts ? a.part_frames : 1u;
    const uint64_t pitems = parts ? (uint64_t)((a.n_frames + plen - 1) / plen) * a.n_tiles : 0u;
    uint64_t it = wave;
    uint32_t acc = 0;
    while (true) {
        uint32_t tile, t, tend;
        if (!parts) {
            if (i >= iend) break;
            tile = (uint32_t)(i / a.n_frames);
            t = (uint32_t)(i - (uint64_t)tile * a.n_frames);
            const uint64_t rem = iend - i;
            tend = (uint32_t)((uint64_t)a.n_frames < t + rem ? (uint64_t)a.n_frames : t + rem);
            i += tend - t;
        } else {
            if (it >= pitems) break;
            const uint32_t part = (uint32_t)(it / a.n_tiles);
            tile = (uint32_t)(it - (uint64_t)part * a.n_tiles);
            t = part * plen;
            tend = min(a.n_frames, t + plen);
            it += a.n_waves;
        }
        const uint32_t voff = (tile * (uint32_t)U * 64u + lane) * (uint32_t)VB;
        for (; t < tend; t += 2) {
            const uint32_t t1 = t + 1 < tend ? t + 1 : t;
            const __amdgpu_buffer_rsrc_t r0 = make_rsrc(a.frames + (uint64_t)t * a.frame_bytes, a.vec_bytes);
            const __amdgpu_buffer_rsrc_t r1 = make_rsrc(a.frames + (uint64_t)t1 * a.frame_bytes, a.vec_bytes);
            uint32_t x = 0;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if constexpr (VB == 12) {
                    const u32x3 p0 = __builtin_amdgcn_raw_buffer_load_b96(r0, voff + u * 64 * VB, 0, kAuxNT);
                    const u32x3 p1 = __builtin_amdgcn_raw_buffer_load_b96(r1, voff + u * 64 * VB, 0, kAuxNT);
                    x ^= p0.x ^ p0.y ^ p0.z ^ p1.x ^ p1.y ^ p1.z;
                } else {
                    const u32x4 p0 = __builtin_amdgcn_raw_buffer_load_b128(r0, voff + u * 64 * VB, 0, kAuxNT);
                    const u32x4 p1 = __builtin_amdgcn_raw_buffer_load_b128(r1, voff + u * 64 * VB, 0, kAuxNT);
                    x ^= p0.x ^ p0.y ^ p0.z ^ p0.w ^ p1.x ^ p1.y ^ p1.z ^ p1.w;
                }
            }
            acc ^= x;
        }
    }
    if (acc == 0x9E3779B9u) out[0] = acc;
}

hipError_t launch_read_walk(const SeriesArgs& a, int vec_bytes, uint32_t blocks, uint32_t* out, hipStream_t s) {
    switch (vec_bytes) {
        case 12: hipLaunchKernelGGL((read_walk_kernel<12, kUnrollV2Rgb>), dim3(blocks), dim3(256), 0, s, a, out); break;
        case 16: hipLaunchKernelGGL((read_walk_kernel<16, kUnrollV2>), dim3(blocks), dim3(256), 0, s, a, out); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_read_ceiling(const uint8_t* p, uint64_t bytes, uint32_t* out, hipStream_t s) {
    if (((uintptr_t)p & 15u) != 0) return hipErrorInvalidValue;
    const uint64_t n16 = bytes / 16u;
    if (n16 == 0) return hipSuccess;
    hipLaunchKernelGGL(read_ceiling_kernel, dim3(1024), dim3(256), 0, s, reinterpret_cast<const u32x4*>(p), n16, out);
    return hipGetLastError();
}

template <int C>
__device__ __forceinline__ void generic_segment(const GenericArgs& a, uint64_t seg, uint64_t (&red)[4][4]) {
    const uint32_t t = (uint32_t)(seg / a.blocks_per_frame);
    const uint64_t p = a.px0 + (seg - (uint64_t)t * a.blocks_per_frame) * 256u + threadIdx.x;
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
    __syncthreads();  // red is reused by the next segment
}

// Generic path: any frame shape and alignment.  One thread per pixel, the
// intensity computed in the reference's own form ((cmax+cmin)/2.0,
// dips_shader.wgsl:73-81) rather than the fast kernel's I2 pairs, so the two
// kernels cross-check each other.  Each workgroup walks 256-pixel segments
// with a stride of the grid: a dispatch's grid is at most 2^32 work-items,
// which two GRAY8 frames of 2^31 pixels already exceed
// (tests/test_gpu_max_frames.py; the launch then ran only the grid size
// modulo 2^32).
template <int C>
__global__ __launch_bounds__(256) void series_generic_kernel(GenericArgs a) {
    __shared__ uint64_t red[4][4];
    const uint64_t n_seg = (uint64_t)a.blocks_per_frame * a.n_frames;
    for (uint64_t seg = blockIdx.x; seg < n_seg; seg += gridDim.x) {
        generic_segment<C>(a, seg, red);
    }
}

// Synthetic frames: F_t[y,x,c] = clamp(base + blob_t + noise, 0, 255)
// (bit-identical to the CPU generator of the test oracle,
// checked by tests/test_gpu_series.py::test_synth_device_bit_exact).
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
    return reinterpret_cast<const void*>(&series_fast_kernel<C, CH, U, (C == 1 ? kDepthGray : kDepthRGB), PF, MAP>);
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

// RGB8 / RGBA8 run series_v2_kernel (series_v2.hip); GRAY8 the kernel above.
int fast_unroll(int channels) { return channels == 1 ? kUnrollGray : (channels == 3 ? kUnrollV2Rgb : kUnrollV2); }

const void* series_fast_kernel_ptr(int channels, int chroma, bool per_frame, bool map, bool align, int isi) {
    switch (channels) {
        case 1: return pick_fast_u<1, kUnrollGray>(chroma, per_frame, map);
        case 3:
        case 4: return series_v2_kernel_ptr(channels, chroma, per_frame, map, align, isi);
        default: return nullptr;
    }
}

// gray: dI > tau on the f32 intensity; RGB(A) v2: |dI2s| > tau * 2^23 with
// I2s = 2 I * 2^22 (exact power-of-two scalings of the reference comparison)
// (integer-sum form, isi: intensities x32, series_v2.hip ISI)
float series_threshold(int channels, float tau, int isi) {
    return channels == 1 ? tau : tau * (isi != 0 ? 268435456.0f : 8388608.0f);
}

int pixels_per_vec(int channels) { return channels == 1 ? 16 : 4; }

hipError_t launch_series_fast(const SeriesArgs& a, int channels, int chroma, bool per_frame, bool map,
                              uint32_t blocks, hipStream_t s, bool align, int isi) {
    const void* k = series_fast_kernel_ptr(channels, chroma, per_frame, map, align, isi);
    if (!k) return hipErrorInvalidValue;
    SeriesArgs args = a;
    void* params[] = {&args};
    return hipLaunchKernel(k, dim3(blocks), dim3(256), params, 0, s);
}

hipError_t launch_series_reduce(const uint64_t* partials, uint32_t n_frames, uint32_t n_tiles, int layout,
                                dips_series_entry* series, hipStream_t s) {
    // 64 tiles per thread (eight rounds of eight loads) when that still
    // gives >= 2048 groups (4K: 20 x 127), else down to 8 (one round): small
    // batches are latency-bound here (640x480 x 300 frames: 4 groups, 6 us)
    const uint32_t gx = (n_frames + 255u) / 256u;
    uint32_t tpb = 64;
    while (tpb > 8u && (uint64_t)gx * ((n_tiles + tpb - 1u) / tpb) < 2048u && n_tiles / (tpb >> 1) < 65535u) tpb >>= 1;
    dim3 grid(gx, (n_tiles + tpb - 1u) / tpb);
    hipLaunchKernelGGL(series_reduce_kernel, grid, dim3(256), 0, s, partials, n_frames, n_tiles, tpb, (uint32_t)layout,
                       series);
    return hipGetLastError();
}

hipError_t launch_series_generic(const GenericArgs& a, int channels, hipStream_t s) {
    // one workgroup per 256-pixel segment up to 4 M of them (every batch below
    // that launches as before); past it the workgroups loop over segments
    const uint64_t n_seg = (uint64_t)a.blocks_per_frame * a.n_frames;
    const uint64_t blocks = n_seg < (1ull << 22) ? n_seg : (1ull << 22);
    if (blocks == 0) return hipSuccess;
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
