// series_v2.hip -- the RGB8/RGBA8 series kernel (hot path of the north star).
//
// Same contract as series_fast_kernel (series_kernels.hip): per (tile, frame)
// one 16-byte record of wave sums {SAD, SJ + count << 20, H, L}, summed per
// frame by series_reduce_kernel.  What differs is how the work is shaped for
// the CDNA4 VALU (measured issue costs: tools/gen_vbench.py, profiles/):
//
//  * intensity without conversions: with J = max+min (integer, needed for SJ
//    anyway) and E = P(max) + P(min), P(c) = the largest power of two <= c,
//        2 * get_intensity = u(max) + u(min) = RNE(J * 65793 * 2^-24 + E * 2^-31)
//    exactly (u(c) = c/255 rounds UP to c*65793*2^-24 + 2^(msb(c)-31); the
//    identity is checked exhaustively in tests/test_oracle.py).  J enters one
//    v_fma_mix_f32 as an f16 DENORMAL (its u16 bits unchanged, value J*2^-24)
//    and E comes from the exponent field of the f16 value c*2^-9 (one packed
//    f16 multiply + an AND): 3.5 packed/mixed ops per pixel pair replace four
//    v_cvt_f32_ubyte and five packed f32 ops.  Intensities live in the 2^22
//    scaled domain I2s = I2 * 2^22 (exact power-of-two scaling);
//  * a 4-slot register ring of frame vecs, rotated by unrolling four frames,
//    so the bytes of frame t double as the SAD reference of frame t+1 with no
//    register copies (the previous kernel spent ~10% of its VALU on v_mov);
//  * U = 5 vecs per lane for RGB8 (1280 px per wave and frame; RGBA8's
//    16-B vecs keep U = 4, the 12-bit offset limit): the per-frame wave
//    reduction and record packing (~22 VALU per lane and frame) spread over
//    20 pixels instead of 16, and a fifth fewer partial records; 116 VGPRs,
//    4 waves per SIMD.  Measured against U = 4 (96 VGPRs, 5 waves) in
//    alternated runs on one box: +0.3-0.7 points (profiles/r05/ab_u5/);
//    U = 2 at 8 waves and U = 3 at 6 had lost to U = 4 the same way;
//  * the two frames of a pair are reduced together and their 8 wave sums are
//    stored straight from the lanes that hold them (no v_readlane).
#include "intensity_v2.h"

namespace dips {

// SJ from the intensity difference: 255 * |dI2| = |dJ| + err, |err| < 1.1e-4
// (u() rounds up by < 2^-24, the sum and difference round by <= 2^-24 each;
// exhaustive in tests/test_oracle.py), so the per-lane f32 sum of
// |dI2s| * 255 * 2^-22 (exact multiplier, <= 20 px x 510 < 16384: rounding
// <= 2^-11 per add) is within 0.015 of the integer SJ.
constexpr float kSjMul = 255.0f / 4194304.0f;

// The integer intensity sum (ISI): for tau >= 2^-5 every selected dI is an
// f32 in [2^-5, 1] whose ulp is >= 2^-28, so a = |dI| * 2^28 -- the
// intensities taken 32 times as large (derive_v2<X32>, an exact power-of-two
// scaling of the reference's f32 arithmetic; threshold and SJ multiplier
// scaled with them) -- is an integer <= 2^28 for every selected pixel: one
// v_cvt_u32_f32 and an integer add per pixel replace v_cvt_f64_f32 +
// v_add_f64 (the f64 add is the most power-hungry VALU class this kernel
// issues, profiles/r02_energy_per_instruction.jsonl), for one packed f16
// multiply per pixel pair.  Two u32 accumulators of <= 12 pixels each stay
// below 2^32 (U = 5: 8 and 12).  The record carries n = sum dI * 2^32 = 16 sum a as H = n >> 15,
// L = n mod 2^15, exactly as the f64 form.
constexpr float kIsiMinTau = 0.03125f;  // 2^-5

// One frame of one tile: accumulate against the reference state `st`
// (updated to this frame's state in per-frame mode) and the reference bytes
// `rb`; produce the 4 per-lane values {SAD, SJ, H, L} and the wave-wide count.
// rb / cur rows hold LR / LC dwords, the first Fmt<C>::NDW of which are the
// vec's bytes (LC = NDW + 1 in the aligned-load form, see load_at).
template <int C, int CH, int U, bool PF, bool MAP, int SAUX = kAuxNT, int LR = Fmt<C>::NDW, int LC = Fmt<C>::NDW,
          int ISI = 0>
__device__ __forceinline__ void frame_v2(const SeriesArgs& a, St2 (&st)[U], const uint32_t (&rb)[U][LR],
                                         const uint32_t (&cur)[U][LC], uint32_t voff, uint32_t t,
                                         uint32_t* vals, uint32_t& cnt) {
    using F = Fmt<C>;
    uint32_t sad = 0, c = 0;
    float sj = 0.5f;  // + 0.5: the final truncation rounds to nearest
    constexpr float sj_mul = ISI ? kSjMul / 32.0f : kSjMul;
    // exact per-lane intensity sum, offset by 2^43 so that the f64's low 52
    // mantissa bits ARE the fixed-point value n = sum(a_s) * 2^9 (ulp(2^43)
    // = 2^-9, the a_s granularity; n < 2^37 keeps every add exact)
    double si = 0x1p43;
    uint32_t si0 = 0, si1 = 0;  // ISI: sum of a over vecs 0 .. U/2-1 and U/2 .. U-1
    uint32_t map[U][F::NDW];
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int k = 0; k < F::NDW; ++k) {
            sad = __builtin_amdgcn_sad_u8(cur[u][k], rb[u][k], sad);
            if constexpr (MAP) map[u][k] = absdiff_bytes(cur[u][k], rb[u][k]);
        }
        St2 n;
        {
            uint32_t cv[F::NDW];
#pragma unroll
            for (int k = 0; k < F::NDW; ++k) cv[k] = cur[u][k];
            derive_v2<C, CH, (ISI != 0)>(cv, n);
        }
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const f32x2 d = n.i[k] - st[u].i[k];
            const float a0 = fabsf(d.x), a1 = fabsf(d.y);
            sj = __builtin_fmaf(a0, sj_mul, sj);
            sj = __builtin_fmaf(a1, sj_mul, sj);
            const bool s0 = a0 > a.thr, s1 = a1 > a.thr;
            const uint64_t m0 = __ballot(s0), m1 = __ballot(s1);
            c += (uint32_t)__builtin_popcountll(m0) + (uint32_t)__builtin_popcountll(m1);
            // (a wave-uniform skip of this exact sum when no lane has a pixel
            // above the threshold measured slower: if-converted by hipcc, or
            // as a forced branch it costs registers and occupancy)
            // (the lane-predicated form `if (s0) si += a0` compiles to an
            // unconditional add and two 32-bit selects of the f64: slower)
            if constexpr (ISI == 1) {
                const uint32_t v = (uint32_t)(s0 ? a0 : 0.0f) + (uint32_t)(s1 ? a1 : 0.0f);
                if (u < U / 2)
                    si0 += v;
                else
                    si1 += v;
            } else {
                si += (double)(s0 ? a0 : 0.0f) + (double)(s1 ? a1 : 0.0f);
            }
        }
        if constexpr (PF) st[u] = n;
    }
    if constexpr (MAP) {
        const __amdgpu_buffer_rsrc_t rm = make_rsrc(a.dmap + (uint64_t)t * a.frame_bytes, a.vec_bytes);
#pragma unroll
        for (int u = 0; u < U; ++u) store_vec<C, SAUX>(rm, voff + (uint32_t)(u * 64 * F::VB), map[u]);
    }
    vals[0] = sad;
    vals[1] = (uint32_t)sj;
    if constexpr (ISI == 1) {
        // n = 16 (si0 + si1): H = n >> 15, L = n mod 2^15 (the 33-bit sum
        // through the carry: add, add-with-carry, alignbit)
        const uint64_t s64 = (uint64_t)si0 + (uint64_t)si1;
        vals[2] = (uint32_t)(s64 >> 11);
        vals[3] = ((uint32_t)s64 & 0x7FFu) << 4;
    } else {
        const uint64_t yb = __builtin_bit_cast(uint64_t, si);
        const uint32_t lo = (uint32_t)yb, hi = (uint32_t)(yb >> 32);
        vals[2] = __builtin_amdgcn_alignbit(hi, lo, 15);  // H = n >> 15 (n < 2^37: no exponent bits)
        vals[3] = lo & 0x7FFFu;                           // L = n mod 2^15
    }
    cnt = c;
}

// Records of frames t, t+1 from their 8 reduced values (lanes 8v hold v);
// the SJ word (1) carries count << 20.
__device__ __forceinline__ void store_pair(__amdgpu_buffer_rsrc_t rpart, uint32_t t, uint32_t rec_off8,
                                           uint32_t lane, uint32_t y, uint32_t cnt0, uint32_t cnt1) {
    const uint32_t add = lane == 8u ? (cnt0 << 20) : (lane == 40u ? (cnt1 << 20) : 0u);
    __builtin_amdgcn_raw_buffer_store_b32(y + add, rpart, rec_off8, t * 16u, 0);
}

__device__ __forceinline__ void store_one(__amdgpu_buffer_rsrc_t rpart, uint32_t t, uint32_t rec_off4,
                                          uint32_t lane, uint32_t y, uint32_t cnt) {
    const uint32_t add = lane == 16u ? (cnt << 20) : 0u;
    __builtin_amdgcn_raw_buffer_store_b32(y + add, rpart, rec_off4, t * 16u, 0);
}

// Minimum waves per SIMD asked of the register allocator: the RGB8
// per-frame kernel fits 64 VGPRs (8 waves) without spilling; the other
// variants hold more state (fixed reference bytes, RGBA vecs, map stores) and
// keep their natural allocation (5-7 waves).
template <int C, int U, bool PF, bool MAP, bool ALIGN = false>
constexpr int v2_min_waves() {
    return ALIGN ? (MAP ? 1 : (U >= 5 ? 3 : 4)) : ((C == 3 && PF && !MAP) ? (U <= 2 ? 8 : (U == 3 ? 6 : (U == 4 ? 5 : 4))) : 1);
}

// The aligned-load form of an RGB8 vec (ALIGN): a frame whose base address
// is not a multiple of 4 (a frame stride W*H*3 that is not, or an offset
// pointer) is read through a descriptor at the dword below its base, one
// aligned dwordx4 per vec, and the vec's 12 bytes are funnel-shifted out of
// the 16 (v_alignbyte_b32 by the wave-uniform byte offset, at first use).
// Byte-unaligned 12-B buffer loads return the same bytes but cost extra
// cache-line requests (62-63 % of 8 TB/s against 71.7 % aligned,
// profiles/r02_fallback_rate_after.jsonl, r02_unaligned_probe.txt).
// RGBA8 frames are off a 4-byte boundary only through an offset pointer
// (their stride is a multiple of 4); their 16-B vec comes out of the lane's
// aligned dwordx4 and the FIRST dword of the next lane's (the vecs of a tile
// are contiguous): one DPP wave_shl:1 move per vec brings it over, lane 63
// takes it from lane 0 of the next vec (v_readlane / v_writelane) or, for
// the tile's last vec, from one wave-uniform dword loaded beside the frame.
// So the ring holds 4 dwords per vec (as aligned frames) and a frame costs
// U + 1 loads per lane-slot instead of 2U (the previous form loaded the
// fifth dword per lane: 65.3 % of 8 TB/s at +2 bytes against 75.1 %
// aligned, profiles/r03/fallback_rate_align.jsonl).
template <int N, int L>
__device__ __forceinline__ void funnel(uint32_t (&v)[L], uint32_t sh) {
    static_assert(L > N, "a funnel needs the dword after the vec");
#pragma unroll
    for (int k = 0; k < N; ++k) v[k] = __builtin_amdgcn_alignbyte(v[k + 1], v[k], sh);
}

// The kernel body; AUX / SAUX are the cache-policy bits of the frame loads /
// map stores (the library kernel below uses nt; probe builds instantiate
// other policies to compare them in one process; profiles/r02_aux_ab_load.txt).
// Schedule: a.part_frames == 0 (and SCHED 0) -- one contiguous (tile, frame)
// range per wave; a.part_frames = L > 0 (or SCHED 1, probe builds) -- the
// frames cut into parts of L, items (part, tile) taken part-major with
// stride n_waves, so concurrent waves read the same frames of adjacent tiles
// (the library's choice for RGB8 / RGBA8 batches, part_geometry in
// dips_abi.hip; tools/alloc_policy_ab.hip measured it 0.3-1.1 points above
// the contiguous ranges on each of four buffers, with 0.7-1.2 % less energy
// per frame).
template <int C, int CH, int U, bool PF, bool MAP, int AUX, int SAUX, int SCHED = 0, bool ALIGN = false,
          int ISI = 0, int WPB = 4>
__device__ __forceinline__ void series_v2_body(const SeriesArgs& a) {
    using F = Fmt<C>;
    static_assert(!ALIGN || C == 3 || C == 4, "the aligned-load form is the RGB8 / RGBA8 one");
    constexpr bool A4 = ALIGN && C == 4;  // RGBA8: the fifth dword from the next lane
    constexpr int LW = (ALIGN && C == 3) ? F::NDW + 1 : F::NDW;  // dwords loaded per vec
    static_assert(U * 64 * F::VB <= 4096, "vec offsets must fit the 12-bit immediate");
    zero_series(a);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * (uint32_t)WPB + (threadIdx.x >> 6));
    if (wave >= a.n_waves) return;
    const uint32_t fb = a.frame_bytes, vb = a.vec_bytes;
    // record dword offsets of the lanes that store reduced values; other
    // lanes point past the descriptor and their stores are dropped
    const uint32_t rec_off8 = (lane & 7u) == 0u ? (lane >> 5) * 16u + ((lane >> 3) & 3u) * 4u : 0x80000000u;
    const uint32_t rec_off4 = (lane & 15u) == 0u ? (lane >> 4) * 4u : 0x80000000u;

    uint64_t i = (uint64_t)wave * a.items / a.n_waves;
    const uint64_t iend = (uint64_t)(wave + 1) * a.items / a.n_waves;
    const bool parts = SCHED == 1 || a.part_frames != 0u;  // wave-uniform (part_geometry)
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
        const uint32_t n = tend - t0;  // frames of this segment (>= 1)
        const uint32_t tlast = tend - 1;
        const uint32_t voff = (tile * U * 64u + lane) * (uint32_t)F::VB;
        const __amdgpu_buffer_rsrc_t rpart =
            make_rsrc(a.partials + 2 * (uint64_t)tile * a.n_frames, a.n_frames * 16u);

        // ALIGN: a descriptor at the dword below p (range rounded up to whole
        // dwords: the dword holding the last byte never crosses a page), one
        // dwordx4 per vec, *sh = p's byte offset in that dword
        // A4: *tl = the dword right after the tile (wave-uniform offset)
        const uint32_t tile_end = (tile + 1u) * U * 64u * (uint32_t)F::VB;
        auto load_at = [&](const uint8_t* p, uint32_t (&dst)[U][LW], uint32_t* sh, uint32_t* tl) {
            if constexpr (ALIGN) {
                const uint32_t d = (uint32_t)(uintptr_t)p & 3u;
                *sh = d;
                const __amdgpu_buffer_rsrc_t r = make_rsrc(p - d, (vb + d + 3u) & ~3u);
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(r, voff + (uint32_t)(u * 64 * F::VB), 0, AUX);
                    dst[u][0] = x.x;
                    dst[u][1] = x.y;
                    dst[u][2] = x.z;
                    dst[u][3] = x.w;
                }
                if constexpr (A4) *tl = __builtin_amdgcn_raw_buffer_load_b32(r, tile_end, 0, AUX);
            } else {
                const __amdgpu_buffer_rsrc_t r = make_rsrc(p, vb);
#pragma unroll
                for (int u = 0; u < U; ++u) load_vec<C, AUX>(r, voff + (uint32_t)(u * 64 * F::VB), dst[u]);
            }
        };
        uint32_t sh[4] = {0u, 0u, 0u, 0u};  // ALIGN: byte offset of each ring slot's frame
        uint32_t tl[4] = {0u, 0u, 0u, 0u};  // A4: the dword after the tile, per ring slot
        auto load_frame = [&](uint32_t tf, uint32_t (&dst)[U][LW], uint32_t* shp, uint32_t* tlp) {
#ifdef DIPS_PROBE_SAMEFRAME
            // probe build only (tools/probe.hip): every load re-reads the
            // segment's first frame -- the kernel's compute-only time
            tf = t0;
#endif
            load_at(a.frames + (uint64_t)min(tf, tlast) * fb, dst, shp, tlp);
        };

        // ring: PF -- frame k of the segment in slot (k+1)&3, its reference
        // (frame k-1) in slot k&3; overall -- frame k in slot k&3, the fixed
        // reference bytes in rb
        uint32_t buf[4][U][LW];
        uint32_t rb[U][LW];  // overall mode only
        St2 st[U];
        // ALIGN: the vec bytes of ring slot j in place (done once per frame, at
        // its first use; in 'per-frame' mode the slot then serves as the next
        // frame's reference as it is)
        // ALIGN: a vec at or past the frame's whole vecs must read as zero,
        // like the plain form's out-of-range loads; with the descriptor range
        // rounded up to a whole dword, the vec right after the last whole one
        // would see the first trailing-pixel bytes in its first dword
        // (which the generic kernel counts), so that dword is masked
        uint32_t keep[U];
#pragma unroll
        for (int u = 0; u < U; ++u) keep[u] = voff + (uint32_t)(u * 64 * F::VB) < vb ? 0xFFFFFFFFu : 0u;
        // the vec bytes out of the aligned words of one ring slot (or the
        // reference), in increasing u: A4 takes vec u's fifth dword from
        // vec u's next lane (lane 63: vec u + 1's lane 0, still unshifted, or
        // the tile's trailing dword) before shifting vec u
        const bool lane63 = lane == 63u;
        auto realign = [&](uint32_t (&v)[U][LW], uint32_t shv, uint32_t tlv) {
            if constexpr (ALIGN) {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    if constexpr (A4) {
                        uint32_t nx = DIPS_DPP(v[u][0], 0x130);  // wave_shl:1 -- lane i gets lane i + 1
                        const uint32_t l63 = u + 1 < U ? (uint32_t)__builtin_amdgcn_readlane((int)v[u + 1][0], 0)
                                                       : __builtin_amdgcn_readfirstlane(tlv);
                        nx = lane63 ? l63 : nx;
#pragma unroll
                        for (int k = 0; k < 3; ++k) v[u][k] = __builtin_amdgcn_alignbyte(v[u][k + 1], v[u][k], shv);
                        v[u][3] = __builtin_amdgcn_alignbyte(nx, v[u][3], shv);
                    } else {
                        funnel<F::NDW>(v[u], shv);
                    }
                    v[u][0] &= keep[u];
                }
            }
        };
        auto settle = [&](int j) {
            if constexpr (ALIGN) realign(buf[j], sh[j], tl[j]);
        };
        {
            const uint8_t* rp = PF ? (t0 == 0 ? a.ref0 : a.frames + (uint64_t)(t0 - 1) * fb) : a.ref0;
            uint32_t (&dref)[U][LW] = PF ? buf[0] : rb;
            uint32_t rsh = 0, rtl = 0;
            load_at(rp, dref, &rsh, &rtl);
            if constexpr (PF) {
                load_frame(t0, buf[1], &sh[1], &tl[1]);
                load_frame(t0 + 1, buf[2], &sh[2], &tl[2]);
                load_frame(t0 + 2, buf[3], &sh[3], &tl[3]);
            } else {
                load_frame(t0, buf[0], &sh[0], &tl[0]);
                load_frame(t0 + 1, buf[1], &sh[1], &tl[1]);
                load_frame(t0 + 2, buf[2], &sh[2], &tl[2]);
                load_frame(t0 + 3, buf[3], &sh[3], &tl[3]);
            }
            if constexpr (ALIGN) realign(dref, rsh, rtl);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                uint32_t dv[F::NDW];
#pragma unroll
                for (int k2 = 0; k2 < F::NDW; ++k2) dv[k2] = dref[u][k2];
                derive_v2<C, CH, (ISI != 0)>(dv, st[u]);
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
                        settle((j + 1) & 3);
                        frame_v2<C, CH, U, PF, MAP, SAUX, LW, LW, ISI>(a, st, buf[j], buf[(j + 1) & 3], voff, tf,
                                                                  v + 4 * q, q ? c1 : c0);
                        __builtin_amdgcn_sched_barrier(0);
                        load_frame(tf + 3, buf[j], &sh[j], &tl[j]);
                    } else {
                        settle(j);
                        frame_v2<C, CH, U, PF, MAP, SAUX, LW, LW, ISI>(a, st, rb, buf[j], voff, tf, v + 4 * q,
                                                                  q ? c1 : c0);
                        __builtin_amdgcn_sched_barrier(0);
                        load_frame(tf + 4, buf[j], &sh[j], &tl[j]);
                    }
                }
                const uint32_t y = wave_sum8_lanes(v, lane);
                store_pair(rpart, t0 + k + 2 * h, rec_off8, lane, y, c0, c1);
            }
        }
        // tail: up to 3 frames, already in flight in their slots
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            if (k + (uint32_t)j < n) {
                uint32_t v[4], c;
                const uint32_t tf = t0 + k + (uint32_t)j;
                if constexpr (PF) {
                    settle(j + 1);
                    frame_v2<C, CH, U, PF, MAP, SAUX, LW, LW, ISI>(a, st, buf[j], buf[j + 1], voff, tf, v, c);
                } else {
                    settle(j);
                    frame_v2<C, CH, U, PF, MAP, SAUX, LW, LW, ISI>(a, st, rb, buf[j], voff, tf, v, c);
                }
                const uint32_t y = wave_sum4_lanes(v);
                store_one(rpart, tf, rec_off4, lane, y, c);
            }
        }
    }
}

template <int C, int CH, int U, bool PF, bool MAP, bool ALIGN = false, int ISI = 0>
__global__ __launch_bounds__(256, (v2_min_waves<C, U, PF, MAP, ALIGN>())) void series_v2_kernel(SeriesArgs a) {
    series_v2_body<C, CH, U, PF, MAP, kAuxNT, kAuxNT, 0, ALIGN, ISI>(a);
}

// ---------------------------------------------------------------------------
// instantiation table
// ---------------------------------------------------------------------------
template <int C, int CH, bool PF, bool MAP, bool ALIGN, int ISI>
static const void* v2_ptr() {
    return reinterpret_cast<const void*>(&series_v2_kernel<C, CH, v2_unroll<C>(), PF, MAP, ALIGN && (C == 3 || C == 4), ISI>);
}

template <int C, bool ALIGN, int ISI>
static const void* pick_v2(int chroma, bool pf, bool map) {
#define DIPS_PICK_V2(CHV)                                                                                   \
    case CHV:                                                                                               \
        return pf ? (map ? v2_ptr<C, CHV, true, true, ALIGN, ISI>() : v2_ptr<C, CHV, true, false, ALIGN, ISI>()) \
                  : (map ? v2_ptr<C, CHV, false, true, ALIGN, ISI>()                                        \
                         : v2_ptr<C, CHV, false, false, ALIGN, ISI>());
    switch (chroma) {
        DIPS_PICK_V2(0)
        DIPS_PICK_V2(1)
        DIPS_PICK_V2(2)
        DIPS_PICK_V2(3)
        default: return nullptr;
    }
#undef DIPS_PICK_V2
}

const void* series_v2_kernel_ptr(int channels, int chroma, bool per_frame, bool map, bool align, int isi) {
    switch (channels) {
        case 3:
            if (isi == 1)
                return align ? pick_v2<3, true, 1>(chroma, per_frame, map) : pick_v2<3, false, 1>(chroma, per_frame, map);
            return align ? pick_v2<3, true, 0>(chroma, per_frame, map) : pick_v2<3, false, 0>(chroma, per_frame, map);
        case 4:
            if (isi == 1)
                return align ? pick_v2<4, true, 1>(chroma, per_frame, map) : pick_v2<4, false, 1>(chroma, per_frame, map);
            return align ? pick_v2<4, true, 0>(chroma, per_frame, map) : pick_v2<4, false, 0>(chroma, per_frame, map);
        default: return nullptr;
    }
}

bool series_v2_isi(float tau) { return tau >= kIsiMinTau; }

}  // namespace dips
