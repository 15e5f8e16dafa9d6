// series_gray.hip -- the GRAY8 series kernel with the per-pixel statistics
// as a table (series_gray_lut_kernel).
//
// For one gray byte pair (a = the frame's, b = the reference's) everything
// the series needs is a function of (a, b) alone: with u(c) = c / 255
// correctly rounded, dI = |RN(u(a) - u(b))| (dips_shader.wgsl:64-82 with
// the three channels equal), the pixel is counted when dI > tau, and its
// contribution to SI_fixed = sum dI * 2^32 is 2 V with V = dI * 2^31, an
// integer.  Exhaustively over all 65,536 pairs (tests/test_oracle.py::
// test_gray_si_decomposition):
//     V = 8421504 * d + corr,   d = |a - b|,   corr in {0, 1, 2, 4, ..., 128}
// (u(c) * 2^31 = 8421504 c + P(c) exactly, 8421504 = 65793 * 2^7 and P(c)
// the largest power of two <= c, series_v2.hip; the f32 rounding of the
// difference leaves a non-negative power-of-two remainder).  So per selected pixel the
// kernel needs d and corr, each one byte, and per frame
//     SI_fixed = 2 (8421504 * sum d + sum corr),   count = #selected.
// gray_lut_kernel writes, for the current tau, a u16 table of the entries
//     e(a, b) = selected ? d | corr << 8 : 0,
// and the series kernel keeps it (128 KiB) in LDS, one 1024-thread group per
// CU.  Per pixel pair one v_perm_b32 builds the two indices, two ds_read_u16
// fetch the entries, one v_perm_b32 puts both in one register, and three
// SADs (bytes, u16 halves, u16 halves minus 1) yield sum d, sum corr and the
// count exactly.  No f32, no f64: the exact f32 arithmetic of the reference
// is folded into the table.  SAD is the byte SAD and SJ = 2 SAD.  Two table
// layouts (keyed by (a, b) -- layout 2 -- or by (a ^ b, a) with a band clamp
// -- layout 5), chosen per workgroup from the content it walks (layout 4,
// series_gray_lut_kernel below).
//
// Records: {SAD, sum d, sum corr, count} per (tile, frame); series_reduce
// (mode 2) forms SI_fixed = 2 (8421504 sum d + sum corr) in 64 bits.
#include "series_common.h"

#include <type_traits>

namespace dips {

constexpr uint32_t kGrayV = 8421504u;          // V = kGrayV * d + corr

// Layout 2 stores the entry of (a, b) at u16 index a * 256 + (b ^ sw(a)),
// sw(a) = (a << 2) & 0x3C.  A ds_read_u16's bank is (byte address / 4) mod
// 32 = bits 1-5 of the stored b; unswizzled that is b alone, and where the
// reference is smooth (b within a few levels across the 32 lanes of a half)
// the lanes pile onto 2-4 banks: 4K gray8 with flat +-3 noise ran at 39 %
// of 8 TB/s against 65 % on the bench's random-base frames
// (profiles/r02_content_rate.jsonl).  XOR-ing the low
// four bits of a into bank bits 2-5 spreads such boxes of (a, b) over the
// banks (bank-conflict simulation: flat +-3 12.2 -> 3.9 LDS cycles per
// read, random unchanged at 7.1) and costs two VALU per four pixels (the
// reference dword is swizzled once before the index perms).
constexpr uint32_t kGraySwizzle = 0x3Cu;

// Layout 5: the entry of (a, b) at u16 index x * 256 + a, x = a ^ b.  Rows
// x < 2^m hold only pairs with |a - b| < 2^m; when every one of them is below
// the threshold (2^m - 1 <= the largest |a - b| that is never selected for
// tau), all their entries are 0, and the kernel clamps every index below
// K = 256 * 2^m - 1 up to K (one v_pk_max_u16 per pixel pair): all those
// lanes read the one entry K, an LDS broadcast instead of a random gather.
// Consecutive video frames put most pixels there -- the bench's synthetic
// clips (+-4 noise per frame) ~63 % at tau = 8/255, flat content nearly all.
// m comes from the band word the table kernel leaves after the table (256 -
// the first row holding a selected pair), so the clamp is exact by
// construction for any tau.  (An earlier layout 3 also swizzled the column
// against bank conflicts; layout 5 without it measured faster on the bench
// content, profiles/r04/d/gray_layout_ab.jsonl.)
constexpr uint32_t kGrayBandOffset = 131072u;  // byte offset of the band word (after the table)

// The tables for threshold tau (65,536 spec evaluations), 131,072 bytes:
// layout 2 -- one u16 table, entry d | corr << 8 at byte 2 idx (swizzled);
// layout 5 -- the same entries keyed by (x = a ^ b, a) (see kGrayBandOffset),
// plus the band word: max over the rows x holding a selected pair of 256 - x
// (0 when none is), which the caller zeroes before the launch.  One block per
// row x in layout 5.
__global__ __launch_bounds__(256) void gray_lut_kernel(uint8_t* __restrict__ tab, float tau, uint32_t layout) {
    const uint32_t idx = blockIdx.x * 256u + threadIdx.x;
    uint32_t a = idx >> 8, b = idx & 0xFFu;
    if (layout == 5u) {
        const uint32_t x = idx >> 8;
        a = idx & 0xFFu;
        b = a ^ x;
    }
    const float di = fabsf(unorm_load(a) - unorm_load(b));
    const bool sel = di > tau;
    const uint64_t v = (uint64_t)((double)di * 2147483648.0);  // exact: di is a multiple of 2^-31
    const uint32_t d = a > b ? a - b : b - a;
    const uint32_t corr = (uint32_t)(v - (uint64_t)kGrayV * d);  // in [0, 128] (exhaustive test)
    const uint16_t e = sel ? (uint16_t)(d | corr << 8) : (uint16_t)0;
    if (layout == 5u) {
        reinterpret_cast<uint16_t*>(tab)[idx] = e;
        if (__syncthreads_or(sel) && threadIdx.x == 0u)
            atomicMax(reinterpret_cast<uint32_t*>(tab + kGrayBandOffset), 256u - blockIdx.x);
    } else {
        const uint32_t pos = (a << 8) | (b ^ ((a << 2) & kGraySwizzle));
        reinterpret_cast<uint16_t*>(tab)[pos] = e;
    }
}

namespace {

constexpr int kGrayWaves = 16;  // waves per workgroup (one group per CU holds the table)

// Records of frames t, t+1 from their 8 reduced values (lanes 8v hold v);
// the wave-wide counts go into value 3 (lanes 24 and 56).
__device__ __forceinline__ void gstore_pair(__amdgpu_buffer_rsrc_t rpart, uint32_t t, uint32_t rec_off8, uint32_t lane,
                                            uint32_t y, uint32_t cnt0, uint32_t cnt1) {
    const uint32_t add = lane == 24u ? cnt0 : (lane == 56u ? cnt1 : 0u);
    __builtin_amdgcn_raw_buffer_store_b32(y + add, rpart, rec_off8, t * 16u, 0);
}

__device__ __forceinline__ void gstore_one(__amdgpu_buffer_rsrc_t rpart, uint32_t t, uint32_t rec_off4, uint32_t lane,
                                           uint32_t y, uint32_t cnt) {
    const uint32_t add = lane == 48u ? cnt : 0u;
    __builtin_amdgcn_raw_buffer_store_b32(y + add, rpart, rec_off4, t * 16u, 0);
}

// One frame of one tile against the reference bytes rb: the 4 per-lane
// values {SAD, sum d, sum corr, count}.
// LAYOUT 5: kk = the band clamp K in both u16 halves.
template <int U, bool MAP, int LAYOUT>
__device__ __forceinline__ void gray_frame(const SeriesArgs& a, const uint8_t* lds, const uint32_t (&rb)[U][4],
                                           const uint32_t (&cur)[U][4], uint32_t kk, uint32_t voff, uint32_t t,
                                           uint32_t* vals, uint32_t& cnt) {
    static_assert(LAYOUT == 2 || LAYOUT == 5, "table layouts 2 and 5");
    uint32_t sad = 0, acc = 0, accd = 0, accc = 0;
    uint32_t map[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t f = cur[u][k], r = rb[u][k];
            sad = __builtin_amdgcn_sad_u8(f, r, sad);
            if constexpr (MAP) map[u][k] = absdiff_bytes(f, r);
            // table indices of pixels (0, 2) and (1, 3) as u16 pairs, per byte
            // of the dword at once: layout 2 f_i * 256 + (r_i ^ sw(f_i));
            // layout 5 x_i * 256 + f_i, x_i = f_i ^ r_i, the indices below
            // the band clamp raised to it
            uint32_t i02, i13;
            if constexpr (LAYOUT == 5) {
                const uint32_t x = f ^ r;
                i02 = as_u32(__builtin_elementwise_max(as_u16x2(__builtin_amdgcn_perm(x, f, 0x06020400u)),
                                                       as_u16x2(kk)));
                i13 = as_u32(__builtin_elementwise_max(as_u16x2(__builtin_amdgcn_perm(x, f, 0x07030501u)),
                                                       as_u16x2(kk)));
            } else {
                const uint32_t rs = r ^ ((f << 2) & (kGraySwizzle * 0x01010101u));
                i02 = __builtin_amdgcn_perm(f, rs, 0x06020400u);
                i13 = __builtin_amdgcn_perm(f, rs, 0x07030501u);
            }
            {
                // one u16 entry e = d | corr << 8 per pixel (0: not selected,
                // else d >= 1), two pixels' entries in one register.  Three
                // SAD sums per pixel pair carry everything:
                //   sb = sum of bytes         = sum d + sum corr
                //   s0 = sum e                = sum d + 256 sum corr
                //   s1 = sum |e - 1|          = s0 + n - 2 count
                // (n = pixels summed; |0 - 1| = 1 for an unselected pixel)
                const uint16_t* t16 = reinterpret_cast<const uint16_t*>(lds);
                const uint32_t r02 = __builtin_amdgcn_perm((uint32_t)t16[i02 >> 16], (uint32_t)t16[i02 & 0xFFFFu],
                                                           0x05040100u);
                const uint32_t r13 = __builtin_amdgcn_perm((uint32_t)t16[i13 >> 16], (uint32_t)t16[i13 & 0xFFFFu],
                                                           0x05040100u);
                accc = __builtin_amdgcn_sad_u8(r02, 0u, accc);
                accc = __builtin_amdgcn_sad_u8(r13, 0u, accc);
                accd = __builtin_amdgcn_sad_u16(r02, 0u, accd);
                accd = __builtin_amdgcn_sad_u16(r13, 0u, accd);
                acc = __builtin_amdgcn_sad_u16(r02, 0x00010001u, acc);
                acc = __builtin_amdgcn_sad_u16(r13, 0x00010001u, acc);
            }
        }
    }
    // sb = accc, s0 = accd, s1 = acc (all < 2^22 for 64 px per lane):
    // sum corr = (s0 - sb) / 255, sum d = sb - sum corr,
    // count = (s0 + n - s1) / 2
    constexpr uint32_t n = (uint32_t)U * 16u;
    const uint32_t sc = (accd - accc) / 255u;
    const uint32_t sd = accc - sc;
    const uint32_t c = (accd + n - acc) >> 1;
    acc = sd | (sc << 16);  // sum d < 2^15, sum corr < 2^14
    if constexpr (MAP) {
        const __amdgpu_buffer_rsrc_t rm = make_rsrc(a.dmap + (uint64_t)t * a.frame_bytes, a.vec_bytes);
#pragma unroll
        for (int u = 0; u < U; ++u) store_vec<1>(rm, voff + (uint32_t)(u * 64 * 16), map[u]);
    }
    vals[0] = sad;
    vals[1] = acc & 0xFFFFu;
    vals[2] = acc >> 16;
    vals[3] = c;  // per-lane count, summed with the other values
    cnt = 0u;
}

// The item walk of the table kernel over its table in LDS (`lds`; `lut` =
// the table's global copy, whose band word layout 5 reads).
template <int U, bool PF, bool MAP, int LAYOUT, int GW>
__device__ __forceinline__ void gray_walk(const SeriesArgs& a, const uint8_t* lds, const uint8_t* lut) {
    static_assert(U * 64 * 16 <= 4096, "vec offsets must fit the 12-bit immediate");
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * (uint32_t)GW + (threadIdx.x >> 6));
    if (wave >= a.n_waves) return;
    const uint32_t fb = a.frame_bytes, vb = a.vec_bytes;
    const uint32_t rec_off8 = (lane & 7u) == 0u ? (lane >> 5) * 16u + ((lane >> 3) & 3u) * 4u : 0x80000000u;
    const uint32_t rec_off4 = (lane & 15u) == 0u ? (lane >> 4) * 4u : 0x80000000u;
    uint32_t kk = 0u;
    if constexpr (LAYOUT == 5) {
        // the band clamp from the word after the table: rows x < 2^m hold no
        // selected pair, m = floor(log2(the first row that does)), K = 256 * 2^m - 1
        const uint32_t w = *reinterpret_cast<const uint32_t*>(lut + kGrayBandOffset);
        const uint32_t first = 256u - min(w, 255u);  // 1 .. 256 (row 0, a == b, is never selected)
        const uint32_t kc = (256u << (31u - __builtin_clz(first))) - 1u;
        kk = kc | (kc << 16);
    }

    // one contiguous (tile, frame) range per wave, or (a.part_frames = L > 0)
    // the part-major schedule of series_v2.hip: items (part, tile) dealt with
    // stride n_waves, concurrent waves on adjacent tiles of the same frames
    uint64_t i = (uint64_t)wave * a.items / a.n_waves;
    const uint64_t iend = (uint64_t)(wave + 1) * a.items / a.n_waves;
    const bool parts = PF && a.part_frames != 0u;  // wave-uniform; per-frame batches only
    const uint32_t plen = parts ? a.part_frames : 1u;
    const uint64_t pitems = parts ? (uint64_t)((a.n_frames + plen - 1) / plen) * a.n_tiles : 0u;
    uint64_t it = wave;
    while (true) {
        uint32_t tile, t0, tend;
        if (!parts) {
            if (i >= iend) break;
            tile = (uint32_t)(i / a.n_frames);
            t0 = (uint32_t)(i - (uint64_t)tile * a.n_frames);
            const uint64_t remaining = iend - i;
            tend = (uint32_t)((uint64_t)a.n_frames < t0 + remaining ? (uint64_t)a.n_frames : t0 + remaining);
            i += tend - t0;
        } else {
            if (it >= pitems) break;
            const uint32_t part = (uint32_t)(it / a.n_tiles);
            tile = (uint32_t)(it - (uint64_t)part * a.n_tiles);
            t0 = part * plen;
            tend = min(a.n_frames, t0 + plen);
            it += a.n_waves;
        }
        const uint32_t n = tend - t0;
        const uint32_t tlast = tend - 1;
        const uint32_t voff = (tile * U * 64u + lane) * 16u;
        const __amdgpu_buffer_rsrc_t rpart =
            make_rsrc(a.partials + 2 * (uint64_t)tile * a.n_frames, a.n_frames * 16u);

        auto load_frame = [&](uint32_t tf, uint32_t (&dst)[U][4]) {
            const __amdgpu_buffer_rsrc_t r = make_rsrc(a.frames + (uint64_t)min(tf, tlast) * fb, vb);
#pragma unroll
            for (int u = 0; u < U; ++u) load_vec<1>(r, voff + (uint32_t)(u * 64 * 16), dst[u]);
        };

        // ring as in series_v2_kernel: PF -- frame k of the segment in slot
        // (k+1)&3, its reference in slot k&3; overall -- frame k in slot k&3
        uint32_t buf[4][U][4];
        uint32_t rb[U][4];
        {
            const uint8_t* rp = PF ? (t0 == 0 ? a.ref0 : a.frames + (uint64_t)(t0 - 1) * fb) : a.ref0;
            const __amdgpu_buffer_rsrc_t rr = make_rsrc(rp, vb);
            uint32_t (&dref)[U][4] = PF ? buf[0] : rb;
#pragma unroll
            for (int u = 0; u < U; ++u) load_vec<1>(rr, voff + (uint32_t)(u * 64 * 16), dref[u]);
            if constexpr (PF) {
                load_frame(t0, buf[1]);
                load_frame(t0 + 1, buf[2]);
                load_frame(t0 + 2, buf[3]);
            } else {
                load_frame(t0, buf[0]);
                load_frame(t0 + 1, buf[1]);
                load_frame(t0 + 2, buf[2]);
                load_frame(t0 + 3, buf[3]);
            }
        }

        uint32_t k = 0;
        for (; k + 4 <= n; k += 4) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                uint32_t v[8], c0, c1;
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const int j = 2 * h + q;
                    const uint32_t tf = t0 + k + (uint32_t)j;
                    if constexpr (PF) {
                        gray_frame<U, MAP, LAYOUT>(a, lds, buf[j], buf[(j + 1) & 3], kk, voff, tf, v + 4 * q,
                                                   q ? c1 : c0);
                        __builtin_amdgcn_sched_barrier(0);
                        load_frame(tf + 3, buf[j]);
                    } else {
                        gray_frame<U, MAP, LAYOUT>(a, lds, rb, buf[j], kk, voff, tf, v + 4 * q, q ? c1 : c0);
                        __builtin_amdgcn_sched_barrier(0);
                        load_frame(tf + 4, buf[j]);
                    }
                }
                const uint32_t y = wave_sum8_lanes(v, lane);
                gstore_pair(rpart, t0 + k + 2 * h, rec_off8, lane, y, c0, c1);
            }
        }
        // tail: up to 3 frames (written out: with the part-major schedule
        // hipcc no longer unrolls a loop here, and a rolled one would index
        // the register ring at run time)
        auto tail = [&](auto jc) {
            constexpr int j = decltype(jc)::value;
            if (k + (uint32_t)j < n) {
                uint32_t v[4], c;
                const uint32_t tf = t0 + k + (uint32_t)j;
                if constexpr (PF)
                    gray_frame<U, MAP, LAYOUT>(a, lds, buf[j], buf[j + 1], kk, voff, tf, v, c);
                else
                    gray_frame<U, MAP, LAYOUT>(a, lds, rb, buf[j], kk, voff, tf, v, c);
                const uint32_t y = wave_sum4_lanes(v);
                gstore_one(rpart, tf, rec_off4, lane, y, c);
            }
        };
        tail(std::integral_constant<int, 0>{});
        tail(std::integral_constant<int, 1>{});
        tail(std::integral_constant<int, 2>{});
    }
}

// LAYOUT 4 (auto, the default): layout 5 or 2 per workgroup from a sample of
// its own items (gray_sample) -- the table of the chosen layout is the one
// copied into LDS (a.lut: layout 5's table + band word, then layout 2's at
// kGrayLutAllocBytes).  Layout 5 (keyed by (a ^ b, a), band clamp, no bank
// swizzle) turns the lookups of band pixels into broadcasts, and its other
// lookups spread over the banks as the frame bytes a do: well when a wave's
// 64 lanes see many levels, badly when they see a handful (flat content:
// 16-way conflicts).  Layout 2 (keyed by (a, b), swizzled) has no broadcasts
// but few conflicts on such narrow content.  So: layout 5 when the band holds
// >= probe_min / 1024 of the sampled pixels and either nearly all of them
// (probe_hi / 1024) or the waves' bytes spread over >= probe_spread levels on
// average, else layout 2 (measured over five contents,
// profiles/r04/d/).  Until round 4's last pass a separate probe kernel took
// one sample per launch; sampling inside the kernel drops that launch and its
// fill (11-12 us of a 640x480 x 300-frame batch, profiles/r04/small/) and
// lets each workgroup follow the content of the tiles it walks.

// One wave's sample: the first 64-vec row of its first item's tile (a frame
// and its reference, as gray_walk will read them), band pixels below layout 5's clamp
// (x = a ^ b < 2^m), the spread max - min of the frame bytes, pixels counted.
template <int U, bool PF>
__device__ __forceinline__ void gray_sample(const SeriesArgs& a, uint32_t wave, uint32_t lane, const uint8_t* lut5,
                                            uint32_t& band, uint32_t& spread, uint32_t& px) {
    band = 0u;
    spread = 0u;
    px = 0u;
    if (wave >= a.n_waves) return;
    uint32_t tile, t0;
    if (PF && a.part_frames != 0u) {  // item `wave` of the part-major order
        const uint32_t part = wave / a.n_tiles;
        tile = wave - part * a.n_tiles;
        t0 = part * a.part_frames;
    } else {
        const uint64_t i = (uint64_t)wave * a.items / a.n_waves;
        tile = (uint32_t)(i / a.n_frames);
        t0 = (uint32_t)(i - (uint64_t)tile * a.n_frames);
    }
    // the item's second frame when it has one: its first can be the batch's
    // frame 0, which a caller often passes as its own reference too (an
    // identical pair, all band: the flat-content rate fell to 52 % when half
    // the workgroups sampled that pair)
    const uint32_t ts = min(t0 + 1u, a.n_frames - 1u);
    const uint8_t* f = a.frames + (uint64_t)ts * a.frame_bytes;
    const uint8_t* r = PF ? (ts == 0 ? a.ref0 : f - a.frame_bytes) : a.ref0;
    const uint32_t w = *reinterpret_cast<const uint32_t*>(lut5 + kGrayBandOffset);
    const uint32_t first = 256u - min(w, 255u);
    const uint32_t lim = 1u << (31u - __builtin_clz(first));  // 2^m
    const uint32_t off = (tile * U * 64u + lane) * 16u;
    uint32_t c = 0u, mx = 0u, mn = 255u, n = 0u;
    if (off < a.vec_bytes) {
        const __amdgpu_buffer_rsrc_t rf = make_rsrc(f, a.vec_bytes), rr = make_rsrc(r, a.vec_bytes);
        const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rf, off, 0, 0);
        const u32x4 y = __builtin_amdgcn_raw_buffer_load_b128(rr, off, 0, 0);
        const uint32_t fa[4] = {x.x, x.y, x.z, x.w};
        const uint32_t d[4] = {x.x ^ y.x, x.y ^ y.y, x.z ^ y.z, x.w ^ y.w};
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                c += ((d[k] >> (8 * b)) & 0xFFu) < lim ? 1u : 0u;
                const uint32_t v = (fa[k] >> (8 * b)) & 0xFFu;
                mx = max(mx, v);
                mn = min(mn, v);
            }
        n = 16u;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        c += (uint32_t)__shfl_xor((int)c, o);
        n += (uint32_t)__shfl_xor((int)n, o);
        mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
        mn = min(mn, (uint32_t)__shfl_xor((int)mn, o));
    }
    band = c;
    spread = mx > mn ? mx - mn : 0u;
    px = n;
}

template <int U, bool PF, bool MAP, int LAYOUT, int GW = kGrayWaves>
__global__ __launch_bounds__(64 * GW) void series_gray_lut_kernel(SeriesArgs a) {
    __shared__ uint32_t lds32[32768];  // the u16 table of the chosen layout
    zero_series(a);
    bool use5 = true;
    if constexpr (LAYOUT == 4) {
        __shared__ uint32_t smp[3 * GW];
        const uint32_t lane = threadIdx.x & 63u, wl = threadIdx.x >> 6;
        uint32_t band, spread, px;
        gray_sample<U, PF>(a, __builtin_amdgcn_readfirstlane(blockIdx.x * (uint32_t)GW + wl), lane,
                           static_cast<const uint8_t*>(a.lut), band, spread, px);
        if (lane == 0u) {
            smp[3 * wl] = band;
            smp[3 * wl + 1] = spread;
            smp[3 * wl + 2] = px;
        }
        __syncthreads();
        uint32_t sb = 0u, ss = 0u, sp = 0u, nw = 0u;
#pragma unroll
        for (int k = 0; k < GW; ++k) {
            sb += smp[3 * k];
            ss += smp[3 * k + 1];
            sp += smp[3 * k + 2];
            nw += smp[3 * k + 2] != 0u ? 1u : 0u;
        }
        sb = __builtin_amdgcn_readfirstlane(sb);
        ss = __builtin_amdgcn_readfirstlane(ss);
        sp = __builtin_amdgcn_readfirstlane(sp);
        nw = __builtin_amdgcn_readfirstlane(nw);
        if (a.probe_min == 0u)
            use5 = true;  // pinned (DIPS_FLAG_GRAY_BAND_TABLE)
        else if (a.probe_min > 1024u)
            use5 = false;  // pinned (DIPS_FLAG_GRAY_PAIR_TABLE)
        else
            use5 = sb * 1024u >= a.probe_min * sp && (sb * 1024u >= a.probe_hi * sp || ss >= a.probe_spread * nw);
    }
    const uint8_t* lut = static_cast<const uint8_t*>(a.lut) + ((LAYOUT == 4 && !use5) ? kGrayLutAllocBytes : 0u);
    {
        const u32x4* src = reinterpret_cast<const u32x4*>(lut);
        u32x4* dst = reinterpret_cast<u32x4*>(lds32);
        for (uint32_t i = threadIdx.x; i < 8192u; i += 64u * GW) dst[i] = src[i];
    }
    __syncthreads();
    const uint8_t* lds = reinterpret_cast<const uint8_t*>(lds32);
    if constexpr (LAYOUT == 4) {
        if (use5)
            gray_walk<U, PF, MAP, 5, GW>(a, lds, lut);
        else
            gray_walk<U, PF, MAP, 2, GW>(a, lds, lut);
    } else {
        gray_walk<U, PF, MAP, LAYOUT, GW>(a, lds, lut);
    }
}

}  // namespace

template <int L>
static const void* gray_ptr(bool per_frame, bool map) {
    return per_frame ? (map ? reinterpret_cast<const void*>(&series_gray_lut_kernel<kUnrollGrayLut, true, true, L>)
                            : reinterpret_cast<const void*>(&series_gray_lut_kernel<kUnrollGrayLut, true, false, L>))
                     : (map ? reinterpret_cast<const void*>(&series_gray_lut_kernel<kUnrollGrayLut, false, true, L>)
                            : reinterpret_cast<const void*>(&series_gray_lut_kernel<kUnrollGrayLut, false, false, L>));
}

// The shipped table kernel: layout 4, layout 5 or 2 per workgroup.
const void* series_gray_lut_kernel_ptr(bool per_frame, bool map) { return gray_ptr<4>(per_frame, map); }

hipError_t launch_gray_lut(uint8_t* tab, float tau, int layout, hipStream_t s) {
    if (layout == 4) {  // auto: layout 5 (+ band word), then layout 2 after it
        const hipError_t e = launch_gray_lut(tab, tau, 5, s);
        return e != hipSuccess ? e : launch_gray_lut(tab + kGrayLutAllocBytes, tau, 2, s);
    }
    if (layout == 3 || layout == 5) {
        const hipError_t e = hipMemsetAsync(tab + kGrayBandOffset, 0, 4, s);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(gray_lut_kernel, dim3(256), dim3(256), 0, s, tab, tau, (uint32_t)layout);
    return hipGetLastError();
}

hipError_t launch_series_gray_lut(const SeriesArgs& a, bool per_frame, bool map, uint32_t blocks, hipStream_t s) {
    const void* k = series_gray_lut_kernel_ptr(per_frame, map);
    if (!k || !a.lut || blocks == 0) return hipErrorInvalidValue;
    SeriesArgs args = a;
    void* params[] = {&args};
    return hipLaunchKernel(k, dim3(blocks), dim3(64 * kGrayWaves), params, 0, s);
}

}  // namespace dips
