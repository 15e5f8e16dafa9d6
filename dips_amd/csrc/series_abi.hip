// series_abi.hip -- host side of include/dips_hip.h, part 3: the north-star
// per-frame difference series ('overall' against frame 0 or a given
// reference, 'per-frame' against the previous frame; the per-pixel math of
// dips_shader.wgsl:64-82), its host feeds, the synthetic frames and the
// measurement legs bench.py reads (read ceilings, geometry).  Every
// extern "C" body runs inside dips_abi::guard (abi_guard.h).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "dips_handle.h"
#include "dips_kernels.h"

using dips_abi::guard;
using namespace dips_internal;

namespace {

struct FastGeom {
    bool ok = false;
    uint64_t n_tiles = 0, items = 0, n_waves = 0, blocks = 0;
    uint64_t vec_bytes = 0;    // whole vecs of a frame (the vectorised kernel's range)
    uint64_t tail_px0 = 0;     // first pixel of the ragged tail (npx: none)
    uint32_t part_frames = 0;  // part-major schedule: frames per part (0: contiguous ranges)
};

// Resident waves per SIMD for a kernel of `occupancy` waves per SIMD, capped
// by DIPS_SERIES_WAVES_PER_SIMD where `env_cap` (a deployment knob; every
// launch applies it, dips_shard_plan also reports the uncapped count).  No
// launch caps itself: leaving a slot per SIMD free for the halo's RCCL
// kernels beside the sharded 'per-frame' launch cost 2-5 ms per 2,000-5,000
// 4K frames, where the full grid lets the exchange through at +0.03-0.07 ms
// (profiles/r06/halo_contention/).
uint64_t waves_per_simd(uint64_t occupancy, bool env_cap) {
    if (env_cap) {
        if (const char* cap = std::getenv("DIPS_SERIES_WAVES_PER_SIMD")) {
            const unsigned long c = std::strtoul(cap, nullptr, 10);
            if (c >= 1 && c < occupancy) return c;
        }
    }
    return occupancy;
}

// The part-major schedule of the series kernels (series_v2.hip,
// series_gray.hip): the batch's frames cut into P parts of L, items (part,
// tile) dealt to the waves with stride n_waves, so that concurrent waves read
// adjacent tiles of the same frames.  Measured 0.3-1.1 points above one
// contiguous (tile, frame) range per wave on each of four frame buffers,
// 0.7-1.2 % less energy per frame (tools/alloc_policy_ab.hip,
// profiles/r03/alloc/); per-frame 77.3 % against 75.4 % of 8 TB/s, 'overall'
// 74.1 against 72.05 % (profiles/r03/parts/, profiles/r04/l/).  Parts of at
// least 128 frames (each item re-reads its reference tile: +1/L of the
// traffic), P from the one that gives every resident wave slot an item up to
// 4x that: the smallest whose items fill >= 98 % of the slots (k items per
// slot), else the best-filling one (98 rather than 95 %: 8K's 3 parts fill
// 99.9 % against 2 parts' 97.4 %, +0.5 points in alternated runs,
// profiles/r05/ab_fill/; every other config keeps its part count); the
// waves then get ceil(items / n_waves) or one fewer items each (4K RGB8, 5000
// frames, U = 5: L = 1000, 4,050 waves).
// Batches of fewer than 256 frames keep the contiguous ranges.
void part_geometry(FastGeom& g, uint64_t n_frames, uint64_t resident) {
    if (n_frames < 256 || g.n_tiles == 0 || resident == 0) return;
    const uint64_t p_min = std::max<uint64_t>((resident + g.n_tiles - 1) / g.n_tiles, (n_frames + 1249) / 1250);
    const uint64_t p_max = std::min<uint64_t>(4 * p_min, n_frames / 128);
    if (p_max < p_min) return;
    uint64_t best_p = 0;
    double best_fill = -1.0;
    for (uint64_t p = p_min; p <= p_max; ++p) {
        const uint64_t L = (n_frames + p - 1) / p;
        const uint64_t parts = (n_frames + L - 1) / L;
        const uint64_t items = parts * g.n_tiles;
        const uint64_t k = (items + resident - 1) / resident;
        const double fill = (double)items / (double)(k * resident);
        if (fill > best_fill + 1e-9) {
            best_fill = fill;
            best_p = p;
        }
        if (fill >= 0.98) break;
    }
    const uint64_t L = (n_frames + best_p - 1) / best_p;
    const uint64_t items = ((n_frames + L - 1) / L) * g.n_tiles;
    const uint64_t k = (items + resident - 1) / resident;
    g.part_frames = (uint32_t)L;
    g.n_waves = (items + k - 1) / k;
    g.blocks = (g.n_waves + 3) / 4;
}

FastGeom fast_geometry(dips_handle* h, uint32_t width, uint32_t height, uint32_t n_frames, int C, bool pf,
                       bool map, bool align = false, int isi = 0, bool env_cap = true) {
    FastGeom g;
    const uint64_t npx = (uint64_t)width * height;
    const uint64_t fb = npx * (uint64_t)C;
    const int ppv = dips::pixels_per_vec(C);
    // any alignment and pixel count: the vectorised kernel takes the whole
    // vecs of every frame (unaligned frames through unaligned buffer loads,
    // exact on gfx950: tests/test_gpu_series.py::test_unaligned_device_batches), the generic kernel the
    // < ppv trailing pixels
    const uint64_t nvec = npx / (uint64_t)ppv;
    if (nvec == 0 || fb >= (1ull << 31) || n_frames == 0) return g;
    const uint64_t U = (uint64_t)dips::fast_unroll(C);
    g.vec_bytes = nvec * (uint64_t)ppv * (uint64_t)C;
    g.tail_px0 = nvec * (uint64_t)ppv;
    g.n_tiles = (nvec + 64 * U - 1) / (64 * U);
    g.items = g.n_tiles * n_frames;
    const void* k = dips::series_fast_kernel_ptr(C, C == 1 ? 0 : (int)h->p.chroma_filter, pf, map, align, isi);
    if (!k) return g;
    const uint64_t resident = waves_per_simd((uint64_t)occupancy_blocks(h, k), env_cap) * (uint64_t)h->cu_count * 4u;
    g.n_waves = g.items < resident ? g.items : resident;
    g.blocks = (g.n_waves + 3) / 4;
    if (C == 3 || C == 4) part_geometry(g, n_frames, resident);
    g.ok = g.n_tiles < (1ull << 32) && g.blocks < (1ull << 31);
    return g;
}

// GRAY8 runs on the table kernel (series_gray.hip, table layout 4: layout 5
// or 2 per workgroup from a sample of its own items, or the one that
// DIPS_FLAG_GRAY_BAND_TABLE / _PAIR_TABLE pins) unless DIPS_FLAG_CROSSCHECK
// asks for the f32 kernel series_fast_kernel.
//
// Layout 4's choice: layout 5 when the band holds at least kGrayAutoMin of
// the sampled pixels and either kGrayAutoHi of them or the sampled waves'
// frame bytes span kGrayAutoSpread levels on average, else layout 2.  From
// the layouts measured in one process over five 4K contents
// (profiles/r04/d/gray_layout_ab.jsonl; band
// fraction / mean spread of a wave's 1024 pixels; % of 8 TB/s):
//   synthetic (0.64 / 247): layout 5 71.8-72.3, 3 64-70, 2 63-66;
//   random (0.03 / 248): 2 61-63, 5 62-63, 3 60;
//   flat 128 +- 3 (0.51 / 6): 2 70-71, 3 69, 5 58 (bank conflicts);
//   gradient (0.80 / 70): all 69-70;  moving (0.80 / 70): 5 72.2-72.4, 2, 3 68-71.
constexpr double kGrayAutoMin = 0.25, kGrayAutoHi = 0.9;
constexpr uint32_t kGrayAutoSpread = 48;
constexpr int kGrayLayout = 4;

bool gray_lut_enabled(const dips_handle* h) { return !h->crosscheck(); }

FastGeom gray_lut_geometry(dips_handle* h, uint32_t width, uint32_t height, uint32_t n_frames, bool env_cap = true) {
    FastGeom g;
    const uint64_t npx = (uint64_t)width * height;
    const uint64_t nvec = npx / 16u;
    if (nvec == 0 || npx >= (1ull << 31) || n_frames == 0) return g;
    const uint64_t U = (uint64_t)dips::kUnrollGrayLut;
    const uint64_t gw = dips::kGrayLutWaves;
    g.vec_bytes = nvec * 16u;
    g.tail_px0 = nvec * 16u;
    g.n_tiles = (nvec + 64 * U - 1) / (64 * U);
    g.items = g.n_tiles * n_frames;
    // one group per CU (the tables fill its LDS): 4 waves per SIMD
    const uint64_t resident = waves_per_simd(gw / 4u, env_cap) * 4u * (uint64_t)h->cu_count;
    g.n_waves = g.items < resident ? g.items : resident;
    // 'per-frame' batches: the part-major schedule, as for RGB8 (part_geometry)
    if (h->p.mode == DIPS_MODE_PER_FRAME) part_geometry(g, n_frames, resident);
    g.blocks = (g.n_waves + gw - 1) / gw;
    g.ok = g.n_tiles < (1ull << 32) && g.blocks < (1ull << 31);
    return g;
}

// The T_d / T_c tables of the GRAY8 table kernel for the handle's tau.
dips_status ensure_gray_lut(dips_handle* h, hipStream_t s) {
    if (h->gray_lut_valid && h->gray_lut_tau == h->p.tau) return DIPS_OK;
    DIPS_HIP(h, h->gray_lut.ensure(2 * dips::kGrayLutAllocBytes));
    DIPS_HIP(h, dips::launch_gray_lut(h->gray_lut.as<uint8_t>(), h->p.tau, kGrayLayout, s));
    h->gray_lut_valid = true;
    h->gray_lut_tau = h->p.tau;
    return DIPS_OK;
}

// The intensity-sum form of the RGB8 / RGBA8 series kernel for the handle's
// tau (series_v2.hip ISI): 1 (the integer sum) for tau >= 2^-5, 0 (the exact
// f64 sum) below that or with DIPS_FLAG_CROSSCHECK.
int series_isi_form(const dips_handle* h) {
    const int C = (int)h->p.format;
    if (C == 1 || h->crosscheck() || !dips::series_v2_isi(h->p.tau)) return 0;
    return 1;
}

}  // namespace

namespace dips_internal {

// Run the series on device pointers, asynchronously on `s`.
dips_status run_series_device(dips_handle* h, uint32_t width, uint32_t height, const uint8_t* frames,
                              uint32_t n_frames, const uint8_t* ref0, dips_series_entry* series, uint8_t* map,
                              hipStream_t s) {
    const int C = (int)h->p.format;
    const bool pf = h->p.mode == DIPS_MODE_PER_FRAME;
    const uint64_t npx = (uint64_t)width * height;
    const uint64_t fb = npx * (uint64_t)C;
    FastGeom g;
    const bool glut = C == 1 && gray_lut_enabled(h);
    // RGB8 / RGBA8 frames off a 4-byte boundary (an odd frame stride or an
    // offset pointer) run the aligned-load form of the kernel (series_v2.hip
    // ALIGN)
    const bool align = (C == 3 || C == 4) && ((((uintptr_t)frames | (uintptr_t)fb | (uintptr_t)ref0) & 3u) != 0u);
    const int isi = series_isi_form(h);
    if (!(h->p.flags & DIPS_FLAG_FORCE_GENERIC))
        g = glut ? gray_lut_geometry(h, width, height, n_frames)
                 : fast_geometry(h, width, height, n_frames, C, pf, map != nullptr, align, isi);
    // the series starts at zero: the table and RGB(A) kernels clear it
    // themselves (SeriesArgs::zero), saving a fill launch; the others after a
    // fill
    const bool kzero = g.ok && (glut || C != 1) && n_frames < (1u << 30);
    if (!kzero) DIPS_HIP(h, hipMemsetAsync(series, 0, sizeof(dips_series_entry) * (size_t)n_frames, s));
    auto launch_generic = [&](uint64_t px0) -> dips_status {
        const uint64_t bpf = (npx - px0 + 255u) / 256u;  // 256-pixel segments per frame
        if (bpf >= (1ull << 32))
            return fail(h, DIPS_ERR_INVALID, "frame too large for the generic kernel (2^40 pixels)");
        dips::GenericArgs a{};
        a.frames = frames;
        a.ref0 = ref0;
        a.dmap = map;
        a.series = series;
        a.frame_bytes = fb;
        a.n_px = npx;
        a.px0 = px0;
        a.n_frames = n_frames;
        a.blocks_per_frame = (uint32_t)bpf;
        a.mode = h->p.mode;
        a.chroma = C == 1 ? 0u : h->p.chroma_filter;
        a.tau = h->p.tau;
        DIPS_HIP(h, dips::launch_series_generic(a, C, s));
        return DIPS_OK;
    };

    const bool timing = (h->p.flags & DIPS_FLAG_TIME_KERNEL) != 0;
    dips_status st = DIPS_OK;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    // the timing events go back to the free list on every early return; they
    // join ev_pending only once both are recorded
    struct EventReturn {
        dips_handle* h;
        hipEvent_t* e0;
        hipEvent_t* e1;
        ~EventReturn() {
            try {
                if (*e0) h->ev_free.push_back(*e0);
                if (*e1) h->ev_free.push_back(*e1);
            } catch (...) {
            }
        }
    } ev_return{h, &e0, &e1};
    if (timing) {
        e0 = take_event(h);
        e1 = take_event(h);
        if (!e0 || !e1) return fail(h, DIPS_ERR_HIP, "hipEventCreate failed");
    }
    if (g.ok && glut) {
        st = ensure_gray_lut(h, s);  // before e0: the table is not part of the series launch
        if (st != DIPS_OK) return st;
    }
    if (timing) DIPS_HIP(h, hipEventRecord(e0, s));
    if (g.ok) {
        DIPS_HIP(h, h->partials.ensure((size_t)g.items * 16u));
        dips::SeriesArgs a{};
        if (glut) {
            // layout 4's thresholds in 1/1024 of the sampled pixels (each
            // workgroup samples its own items, series_gray.hip gray_sample);
            // a pinned layout: probe_min 0 (always 5) or 1025 (always 2)
            a.probe_min = std::max(1u, (uint32_t)std::ceil(kGrayAutoMin * 1024.0));
            if (h->p.flags & DIPS_FLAG_GRAY_BAND_TABLE) a.probe_min = 0u;
            else if (h->p.flags & DIPS_FLAG_GRAY_PAIR_TABLE) a.probe_min = 1025u;
            a.probe_hi = (uint32_t)std::ceil(kGrayAutoHi * 1024.0);
            a.probe_spread = kGrayAutoSpread;
        }
        if (kzero) {
            a.zero = reinterpret_cast<uint64_t*>(series);
            a.zero_n = 4u * n_frames;
        }
        a.frames = frames;
        a.ref0 = ref0;
        a.dmap = map;
        a.partials = h->partials.as<uint64_t>();
        a.items = g.items;
        a.frame_bytes = (uint32_t)fb;
        a.vec_bytes = (uint32_t)g.vec_bytes;
        a.n_frames = n_frames;
        a.n_tiles = (uint32_t)g.n_tiles;
        a.n_waves = (uint32_t)g.n_waves;
        a.thr = dips::series_threshold(C, h->p.tau, isi);
        a.part_frames = g.part_frames;  // 0: contiguous ranges (part_geometry)
        if (glut) {
            a.lut = h->gray_lut.p;
            DIPS_HIP(h, dips::launch_series_gray_lut(a, pf, map != nullptr, (uint32_t)g.blocks, s));
        } else {
            DIPS_HIP(h, dips::launch_series_fast(a, C, C == 1 ? 0 : (int)h->p.chroma_filter, pf, map != nullptr,
                                                 (uint32_t)g.blocks, s, align, isi));
        }
        // the ragged tail (< pixels_per_vec pixels per frame): its sums go
        // straight into the series by atomics, so the order is free
        if (g.tail_px0 < npx) {
            st = launch_generic(g.tail_px0);
            if (st != DIPS_OK) return st;
        }
    } else {
        st = launch_generic(0);
        if (st != DIPS_OK) return st;
    }
    if (timing) {
        DIPS_HIP(h, hipEventRecord(e1, s));
        h->ev_pending.emplace_back(e0, e1);
        e0 = e1 = nullptr;
    }
    if (g.ok)
        DIPS_HIP(h, dips::launch_series_reduce(h->partials.as<uint64_t>(), n_frames, (uint32_t)g.n_tiles,
                                               C == 1 ? (glut ? 2 : 1) : 0, series, s));
    return DIPS_OK;
}

// Waves of the series launch an aligned batch of this shape runs (0 if the
// shape is not eligible for the fast kernels), with or without the
// DIPS_SERIES_WAVES_PER_SIMD cap.
uint64_t series_waves(dips_handle* h, uint32_t width, uint32_t height, uint32_t n_frames, bool env_cap) {
    const int C = (int)h->p.format;
    FastGeom g = C == 1 && gray_lut_enabled(h)
                     ? gray_lut_geometry(h, width, height, n_frames, env_cap)
                     : fast_geometry(h, width, height, n_frames, C, h->p.mode == DIPS_MODE_PER_FRAME, false, false,
                                     series_isi_form(h), env_cap);
    return g.ok ? g.n_waves : 0;
}

// The series of `n_frames` HOST frames staged through pooled pinned buffers
// and copied to a triple-buffered HBM ring on the side stream, each chunk's
// copy overlapping the previous chunk's series launch (next-1 of SURVEY.md
// s8f); `ref_dev` = the DEVICE reference of the first frame (NULL: overall
// -> the first frame, per-frame -> the first frame itself).  Series into
// the device array `series_dev`, asynchronously on the handle's stream once
// the last chunk is queued (the host frames are all read when it returns).
dips_status run_series_streamed(dips_handle* h, uint32_t width, uint32_t height, const uint8_t* host_frames,
                                uint32_t n_frames, const uint8_t* ref_dev, dips_series_entry* series_dev,
                                uint32_t chunk_frames) {
    if (n_frames == 0) return DIPS_OK;
    const bool pf = h->p.mode == DIPS_MODE_PER_FRAME;
    const size_t fb = (size_t)width * height * (size_t)h->p.format;
    uint32_t chunk = chunk_frames;
    if (chunk == 0) {
        const size_t target = 256u << 20;  // ~256 MiB per DMA chunk
        chunk = (uint32_t)(target / fb);
        if (chunk < 1) chunk = 1;
    }
    if (chunk > n_frames) chunk = n_frames;
    const size_t cbytes = fb * chunk;
    for (auto& r : h->ring) DIPS_HIP(h, r.ensure(cbytes));
    DIPS_HIP(h, h->ring_ref.ensure(fb));
    for (auto& pn : h->pinned) DIPS_HIP(h, pn.ensure(cbytes));
    DIPS_HIP(h, hipStreamSynchronize(h->copy_stream));
    // the ring and the pinned buffers are free once the stream's earlier
    // work (a previous streamed call's kernels) is done
    DIPS_HIP(h, hipStreamSynchronize(h->stream));
    const uint32_t n_chunks = (n_frames + chunk - 1) / chunk;
    for (uint32_t k = 0; k < n_chunks; ++k) {
        const uint32_t b = k % 3u, hb = k % 2u;
        const uint32_t f0 = k * chunk;
        const uint32_t nk = (f0 + chunk <= n_frames) ? chunk : n_frames - f0;
        // pinned[hb] was last read by the DMA of chunk k-2
        if (k >= 2) DIPS_HIP(h, hipEventSynchronize(h->copy_done[(k - 2) % 3u]));
        dips_host::staged_copy(static_cast<uint8_t*>(h->pinned[hb].p), host_frames + (size_t)f0 * fb,
                               (size_t)nk * fb);
        // ring[b] was read by kernel k-3 (frames) and kernel k-2 (per-frame ref)
        if (k >= 2) DIPS_HIP(h, hipStreamWaitEvent(h->copy_stream, h->kernel_done[(k - 2) % 3u], 0));
        // the upload by a copy kernel (1.00-1.15x the DMA engine's rate here)
        DIPS_HIP(h, dips_host::pipe_h2d(h->ring[b].p, h->pinned[hb].p, (size_t)nk * fb, h->copy_stream, true));
        DIPS_HIP(h, hipEventRecord(h->copy_done[b], h->copy_stream));
        DIPS_HIP(h, hipStreamWaitEvent(h->stream, h->copy_done[b], 0));
        const uint8_t* frames_dev = h->ring[b].as<uint8_t>();
        const uint8_t* ref;
        if (pf) {
            if (k == 0) ref = ref_dev ? ref_dev : frames_dev;
            else ref = h->ring[(k - 1) % 3u].as<uint8_t>() + (size_t)(chunk - 1) * fb;
        } else {
            if (k == 0 && !ref_dev)
                DIPS_HIP(h, hipMemcpyAsync(h->ring_ref.p, frames_dev, fb, hipMemcpyDeviceToDevice, h->stream));
            ref = ref_dev ? ref_dev : h->ring_ref.as<uint8_t>();
        }
        dips_status st = run_series_device(h, width, height, frames_dev, nk, ref, series_dev + f0, nullptr, h->stream);
        if (st != DIPS_OK) return st;
        DIPS_HIP(h, hipEventRecord(h->kernel_done[b], h->stream));
    }
    return DIPS_OK;
}

}  // namespace dips_internal

namespace {

// One timed launch of a read-only leg on the handle's stream: *ms = its
// hipEvent duration (synchronous).
template <typename Launch>
dips_status time_leg(dips_handle* h, double* ms, Launch&& launch) {
    DIPS_HIP(h, h->probe_out.ensure(256));
    hipEvent_t e0 = take_event(h), e1 = take_event(h);
    if (!e0 || !e1) return fail(h, DIPS_ERR_HIP, "hipEventCreate failed");
    DIPS_HIP(h, hipEventRecord(e0, h->stream));
    DIPS_HIP(h, launch());
    DIPS_HIP(h, hipEventRecord(e1, h->stream));
    DIPS_HIP(h, hipEventSynchronize(e1));
    float t = 0.0f;
    DIPS_HIP(h, hipEventElapsedTime(&t, e0, e1));
    *ms = t;
    h->ev_free.push_back(e0);
    h->ev_free.push_back(e1);
    return DIPS_OK;
}

}  // namespace

extern "C" {

dips_status dips_diff_series(dips_handle* h, uint32_t width, uint32_t height, const uint8_t* frames,
                             uint32_t n_frames, const uint8_t* ref, dips_series_entry* series, uint8_t* map) {
    return guard(h, [&]() -> dips_status {
        dips_status st = bind(h);
        if (st != DIPS_OK) return st;
        if (n_frames == 0) return DIPS_OK;
        if (!frames || !series || width == 0 || height == 0)
            return fail(h, DIPS_ERR_INVALID, "diff_series: null or empty argument");
        const int C = (int)h->p.format;
        const uint64_t fb = (uint64_t)width * height * (uint64_t)C;
        if (h->p.flags & DIPS_FLAG_DEVICE_PTRS)
            return run_series_device(h, width, height, frames, n_frames, ref ? ref : frames, series, map, h->stream);
        // host pointers: stage through HBM (synchronous call)
        const size_t total = (size_t)fb * n_frames;
        DIPS_HIP(h, h->stage_frames.ensure(total));
        DIPS_HIP(h, h->stage_series.ensure(sizeof(dips_series_entry) * (size_t)n_frames));
        DIPS_HIP(h, hipMemcpyAsync(h->stage_frames.p, frames, total, hipMemcpyHostToDevice, h->stream));
        const uint8_t* ref_dev = h->stage_frames.as<uint8_t>();
        if (ref) {
            DIPS_HIP(h, h->stage_ref.ensure(fb));
            DIPS_HIP(h, hipMemcpyAsync(h->stage_ref.p, ref, fb, hipMemcpyHostToDevice, h->stream));
            ref_dev = h->stage_ref.as<uint8_t>();
        }
        uint8_t* map_dev = nullptr;
        if (map) {
            DIPS_HIP(h, h->stage_map.ensure(total));
            map_dev = h->stage_map.as<uint8_t>();
        }
        st = run_series_device(h, width, height, h->stage_frames.as<uint8_t>(), n_frames, ref_dev,
                               h->stage_series.as<dips_series_entry>(), map_dev, h->stream);
        if (st != DIPS_OK) return st;
        DIPS_HIP(h, hipMemcpyAsync(series, h->stage_series.p, sizeof(dips_series_entry) * (size_t)n_frames,
                                   hipMemcpyDeviceToHost, h->stream));
        if (map) DIPS_HIP(h, hipMemcpyAsync(map, map_dev, total, hipMemcpyDeviceToHost, h->stream));
        DIPS_HIP(h, hipStreamSynchronize(h->stream));
        return DIPS_OK;
    });
}

dips_status dips_diff_series_streamed(dips_handle* h, uint32_t width, uint32_t height, const uint8_t* host_frames,
                                      uint32_t n_frames, const uint8_t* host_ref, dips_series_entry* series,
                                      uint32_t chunk_frames) {
    return guard(h, [&]() -> dips_status {
        dips_status st = bind(h);
        if (st != DIPS_OK) return st;
        if (n_frames == 0) return DIPS_OK;
        if (!host_frames || !series || width == 0 || height == 0)
            return fail(h, DIPS_ERR_INVALID, "diff_series_streamed: null or empty argument");
        const size_t fb = (size_t)width * height * (size_t)h->p.format;
        DIPS_HIP(h, h->stage_series.ensure(sizeof(dips_series_entry) * (size_t)n_frames));
        dips_series_entry* series_dev = h->stage_series.as<dips_series_entry>();
        const uint8_t* ref_dev = nullptr;
        if (host_ref) {
            DIPS_HIP(h, hipStreamSynchronize(h->stream));  // ring_ref may still be read by earlier work
            DIPS_HIP(h, h->ring_ref.ensure(fb));
            DIPS_HIP(h, h->pinned[1].ensure(fb));
            DIPS_HIP(h, hipStreamSynchronize(h->copy_stream));
            std::memcpy(h->pinned[1].p, host_ref, fb);
            DIPS_HIP(h, hipMemcpyAsync(h->ring_ref.p, h->pinned[1].p, fb, hipMemcpyHostToDevice, h->copy_stream));
            DIPS_HIP(h, hipStreamSynchronize(h->copy_stream));
            ref_dev = h->ring_ref.as<uint8_t>();
        }
        st = run_series_streamed(h, width, height, host_frames, n_frames, ref_dev, series_dev, chunk_frames);
        if (st != DIPS_OK) return st;
        DIPS_HIP(h, hipMemcpyAsync(series, series_dev, sizeof(dips_series_entry) * (size_t)n_frames,
                                   hipMemcpyDeviceToHost, h->stream));
        DIPS_HIP(h, hipStreamSynchronize(h->stream));
        return DIPS_OK;
    });
}

dips_status dips_synth_frames(dips_handle* h, uint32_t width, uint32_t height, uint64_t seed, uint64_t t0,
                              uint32_t n_frames, uint8_t* dst) {
    return guard(h, [&]() -> dips_status {
        dips_status st = bind(h);
        if (st != DIPS_OK) return st;
        if (n_frames == 0) return DIPS_OK;
        if (!dst || width == 0 || height == 0)
            return fail(h, DIPS_ERR_INVALID, "synth_frames: null or empty argument");
        dips::SynthArgs a{};
        a.dst = dst;
        a.channels = h->p.format;
        a.width = width;
        a.height = height;
        a.frame_bytes = (uint64_t)width * height * a.channels;
        a.total_bytes = a.frame_bytes * n_frames;
        a.seed = seed;
        a.t0 = t0;
        a.radius = height / 8u > 0 ? height / 8u : 1u;
        DIPS_HIP(h, dips::launch_synth(a, h->stream));
        return DIPS_OK;
    });
}

dips_status dips_read_ceiling(dips_handle* h, const uint8_t* dev_bytes, uint64_t bytes, double* ms) {
    return guard(h, [&]() -> dips_status {
        dips_status st = bind(h);
        if (st != DIPS_OK) return st;
        if (!dev_bytes || !ms) return fail(h, DIPS_ERR_INVALID, "read_ceiling: null argument");
        return time_leg(h, ms, [&]() {
            return dips::launch_read_ceiling(dev_bytes, bytes, h->probe_out.as<uint32_t>(), h->stream);
        });
    });
}

dips_status dips_read_ceiling_walk(dips_handle* h, const uint8_t* dev_frames, uint32_t width, uint32_t height,
                                   uint32_t n_frames, double* ms) {
    return guard(h, [&]() -> dips_status {
        dips_status st = bind(h);
        if (st != DIPS_OK) return st;
        if (!dev_frames || !ms) return fail(h, DIPS_ERR_INVALID, "read_ceiling_walk: null argument");
        const int C = (int)h->p.format;
        if (C != 3 && C != 4) return fail(h, DIPS_ERR_INVALID, "read_ceiling_walk: RGB8 / RGBA8 only");
        // the geometry and schedule an aligned batch of this shape runs with
        // (part-major for batches of >= 256 frames, either mode)
        FastGeom g = fast_geometry(h, width, height, n_frames, C, h->p.mode == DIPS_MODE_PER_FRAME, false, false,
                                   series_isi_form(h));
        if (!g.ok) return fail(h, DIPS_ERR_INVALID, "read_ceiling_walk: shape not eligible for the series kernel");
        dips::SeriesArgs a{};
        a.frames = dev_frames;
        a.items = g.items;
        a.frame_bytes = (uint32_t)((uint64_t)width * height * (uint64_t)C);
        a.vec_bytes = (uint32_t)g.vec_bytes;
        a.n_frames = n_frames;
        a.n_tiles = (uint32_t)g.n_tiles;
        a.n_waves = (uint32_t)g.n_waves;
        a.part_frames = g.part_frames;
        return time_leg(h, ms, [&]() {
            return dips::launch_read_walk(a, C == 3 ? 12 : 16, (uint32_t)g.blocks, h->probe_out.as<uint32_t>(),
                                          h->stream);
        });
    });
}

dips_status dips_series_geometry(dips_handle* h, uint32_t width, uint32_t height, uint32_t n_frames,
                                 uint64_t* waves, uint64_t* tiles, uint64_t* partial_bytes) {
    return guard(h, [&]() -> dips_status {
        dips_status st = bind(h);
        if (st != DIPS_OK) return st;
        const int C = (int)h->p.format;
        // the kernel an aligned batch of this shape runs (its occupancy sets
        // the wave slots)
        FastGeom g = C == 1 && gray_lut_enabled(h)
                         ? gray_lut_geometry(h, width, height, n_frames)
                         : fast_geometry(h, width, height, n_frames, C, h->p.mode == DIPS_MODE_PER_FRAME, false,
                                         false, series_isi_form(h));
        if (waves) *waves = g.ok ? g.n_waves : 0;
        if (tiles) *tiles = g.ok ? g.n_tiles : 0;
        if (partial_bytes) *partial_bytes = g.ok ? g.n_tiles * 16u : 0;
        return g.ok ? DIPS_OK : fail(h, DIPS_ERR_INVALID, "shape not eligible for the fast kernel");
    });
}

}  // extern "C"
