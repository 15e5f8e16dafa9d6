// dips_abi.hip -- host side of the C ABI declared in include/dips_hip.h.
//
// The handle plays the role of the reference's ComputeState
// (dips/src/gpu/mod.rs:39-56): it owns the HIP device binding, the stream,
// the temporal ring of the dips-compat path and the workspace of the batch
// series path.  No C++ exception leaves this file: every entry point returns
// a dips_status (or the documented int) and records a message for
// dips_last_error().
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cctype>
#include <cstring>
#include <fstream>
#include <map>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/dips_hip.h"
#include "dips_kernels.h"
#include "host_buffers.h"
#include "host_stream.h"

namespace {

using dips_host::DevBuf;
using dips_host::HostPinned;
using dips_host::staged_copy;

std::mutex g_err_mu;
std::string g_create_err;

}  // namespace

struct dips_handle {
    dips_params p{};
    int device = 0;
    int cu_count = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    hipStream_t copy_stream = nullptr;
    hipEvent_t switch_ev = nullptr;  // orders a newly set stream after the previous one
    hipEvent_t join_ev = nullptr;    // orders the stream after copy_stream (deferred W > 1 upload)
    std::string err;

    // batch series workspace
    DevBuf partials, stage_frames, stage_ref, stage_series, stage_map;
    DevBuf probe_out;  // sink of the read-ceiling kernel
    std::map<const void*, int> occupancy;

    // streamed feed
    DevBuf ring[3];
    DevBuf ring_ref;
    HostPinned pinned[2];
    hipEvent_t copy_done[3] = {nullptr, nullptr, nullptr};
    hipEvent_t kernel_done[3] = {nullptr, nullptr, nullptr};

    // kernel timing
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pending;
    std::vector<hipEvent_t> ev_free;
    double t_ms = 0.0;
    uint64_t t_launches = 0;
    std::vector<double> t_each;  // per-launch times since the last reset

    // dips-compat ComputeState
    uint32_t width = 0, height = 0;
    int n_queued = 0;
    bool main_init = false;
    uint32_t ring_idx = 0;     // UCircularIndex (utils/indexing.rs:1-34)
    uint32_t uniform_idx = 0;  // starting_index uniform (bind_groups.rs:317-321)
    DevBuf slots[4], raw, start, out;
    HostPinned io;
    uint64_t added = 0;       // frames added so far (global frame index of the next one)
    DevBuf slots_alt[4];      // second ring for the multi-chunk batch kernel (swapped in after it)
    DevBuf filtered;          // W > 1 batch: ring texels of a chunk of frames (compat_filter_frames)
    dips_host::StreamPipe pipe;  // host-pointer feed of dips_frame_callback_batch
    dips_host::PieceEvents pieces;  // per-piece completion of the per-frame readback
    dips_host::PieceEvents up_pieces;  // per-stripe upload completion (striped frame_callback)
    HostPinned io_out;                 // readback staging of the striped frame_callback
    dips_host::CallPhases cb_phases;   // where the last zero-copy frame_callback's time went
    bool cb_phases_valid = false;
    // deferred add_texture (steady state, W = 1, host frame): add_texture
    // stages the frame into `io` and launches, stripe by stripe, the
    // compute_main of the dispatch that normally follows (zero-copy, output
    // into `io_out`, the raw frame into its slot); that dispatch only collects
    // the stripes and quantises the slot; any other call first lets the
    // speculative kernels finish (flush_pending) and leaves the slot raw, as
    // an add_texture without a dispatch does in the reference
    bool pending = false;
    uint32_t pending_slot = 0;
    dips_host::DirectGeom pend_geom;  // stripes of the speculative dispatch
    int pend_key = 0;                 // its output form in io_out (compact_out_keys)
    // slots holding a raw frame (added, not yet quantised by a dispatch): the
    // reference reads their unquantised intensity, which the
    // batch kernel's gray-texel ring cannot express
    bool slot_raw[4] = {false, false, false, false};
    int cb_occupancy = 0;
    DevBuf gray_lut;          // T_d / T_c tables of series_gray_lut_kernel (128 KiB) for gray_lut_tau
                              // (layout 4: layout 3's and layout 2's, kGrayLutAllocBytes apart)
    DevBuf pk_in, pk_out;     // DIPS_CALLBACK_DIRECT=2: packed input / keys of the per-frame call in HBM
    bool gray_lut_valid = false;
    float gray_lut_tau = 0.0f;
    int gray_lut_layout = 0;
    DevBuf cb_lut;            // epilogue table of compat_batch_lut_kernel (128 KiB)
    bool cb_lut_valid = false;
    uint32_t cb_lut_filter = 0, cb_lut_col = 0;
    float cb_lut_k = 0.0f;
};

namespace {

dips_status fail(dips_handle* h, dips_status st, const std::string& msg) {
    if (h) h->err = msg;
    return st;
}

dips_status flush_pending(dips_handle* h);  // below, with add_texture

dips_status hip_fail(dips_handle* h, hipError_t e, const char* what) {
    std::string m = std::string(what) + ": " + hipGetErrorString(e);
    return fail(h, e == hipErrorOutOfMemory ? DIPS_ERR_NOMEM : DIPS_ERR_HIP, m);
}

#define DIPS_HIP(h, call)                                   \
    do {                                                    \
        hipError_t e_ = (call);                             \
        if (e_ != hipSuccess) return hip_fail((h), e_, #call); \
    } while (0)

dips_status validate_params(const dips_params* p, std::string* why) {
    if (p->spatial_window_size < 1 || p->spatial_window_size > 11) {
        *why = "spatial_window_size must be in [1, 11] (dips_shader.wgsl:27 MAX_WIN_SIZE_SQUARE = 11*11)";
        return DIPS_ERR_INVALID;
    }
    if (p->chroma_filter > 3u) {
        *why = "chroma_filter must be 0..3 (dips/src/lib.rs:43-61)";
        return DIPS_ERR_INVALID;
    }
    if (p->mode > 1u) {
        *why = "mode must be DIPS_MODE_OVERALL or DIPS_MODE_PER_FRAME";
        return DIPS_ERR_INVALID;
    }
    if (p->format != DIPS_FMT_GRAY8 && p->format != DIPS_FMT_RGB8 && p->format != DIPS_FMT_RGBA8) {
        *why = "format must be DIPS_FMT_GRAY8, DIPS_FMT_RGB8 or DIPS_FMT_RGBA8";
        return DIPS_ERR_INVALID;
    }
    if (!(p->tau >= 0.0f) || std::isinf(p->tau)) {
        *why = "tau must be finite and >= 0";
        return DIPS_ERR_INVALID;
    }
    if (!std::isfinite(p->sensitivity)) {
        *why = "sensitivity must be finite";
        return DIPS_ERR_INVALID;
    }
    return DIPS_OK;
}

hipEvent_t take_event(dips_handle* h) {
    if (!h->ev_free.empty()) {
        hipEvent_t e = h->ev_free.back();
        h->ev_free.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

int occupancy_blocks(dips_handle* h, const void* kernel) {
    auto it = h->occupancy.find(kernel);
    if (it != h->occupancy.end()) return it->second;
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, 256, 0) != hipSuccess || nb < 1) nb = 1;
    h->occupancy[kernel] = nb;
    return nb;
}

struct FastGeom {
    bool ok = false;
    uint64_t n_tiles = 0, items = 0, n_waves = 0, blocks = 0;
    uint64_t vec_bytes = 0;  // whole vecs of a frame (the vectorised kernel's range)
    uint64_t tail_px0 = 0;   // first pixel of the ragged tail (npx: none)
    uint32_t part_frames = 0;  // series_v2 part-major schedule: frames per part (0: contiguous ranges)
};

// The part-major schedule of the RGB8 / RGBA8 series kernel (series_v2.hip):
// the batch's frames cut into P parts of L, items (part, tile) dealt to the
// waves with stride n_waves, so that concurrent waves read adjacent tiles of
// the same frames.  Measured 0.3-1.1 points above one contiguous (tile,
// frame) range per wave on each of four frame buffers, 0.7-1.2 % less energy
// per frame (tools/alloc_policy_ab.hip, profiles/r03/alloc/).  Parts of at
// least 128 frames (each item re-reads its reference tile: +1/L of the
// traffic), P from the one that gives every resident wave slot an item up
// to 4x that: the smallest whose items fill >= 95 % of the slots (k items per
// slot), else the best-filling one; the waves then get ceil(items / n_waves)
// or one fewer items each (4K RGB8, 5000 frames: L = 1000, 5,063 waves).  Batches of
// fewer than 256 frames keep the contiguous ranges (DIPS_SERIES_PARTS=0:
// always, A/B runs).  In one process, alternated (tools/isi_ab.py,
// profiles/r03/parts/), per-frame 77.3 % against 75.4 % of 8 TB/s with 1.2 %
// less energy per frame; 'overall' measured 73.8 against 73.9 % in round 3
// and 74.1 against 72.05 % in round 4 (profiles/r04/l/), so since round 4
// 'overall' batches take it too (fast_geometry).
void part_geometry(FastGeom& g, uint64_t n_frames, uint64_t resident) {
    const char* e = std::getenv("DIPS_SERIES_PARTS");
    if ((e && e[0] == '0') || n_frames < 256 || g.n_tiles == 0 || resident == 0) return;
    const uint64_t p_min = std::max<uint64_t>((resident + g.n_tiles - 1) / g.n_tiles, (n_frames + 1249) / 1250);
    const uint64_t p_max = std::min<uint64_t>(4 * p_min, n_frames / 128);
    if (p_max < p_min) return;
    // the fewest parts (the longest L) whose items fill >= 95 % of the
    // slots, else the best-filling P
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
        if (fill >= 0.95) break;
    }
    const uint64_t L = (n_frames + best_p - 1) / best_p;
    const uint64_t items = ((n_frames + L - 1) / L) * g.n_tiles;
    const uint64_t k = (items + resident - 1) / resident;
    g.part_frames = (uint32_t)L;
    g.n_waves = (items + k - 1) / k;
    g.blocks = (g.n_waves + 3) / 4;
}

FastGeom fast_geometry(dips_handle* h, uint32_t width, uint32_t height, uint32_t n_frames, int C, bool pf,
                       bool map, bool align = false, int isi = 0) {
    FastGeom g;
    const uint64_t npx = (uint64_t)width * height;
    const uint64_t fb = npx * (uint64_t)C;
    const int ppv = dips::pixels_per_vec(C);
    // any alignment and pixel count: the vectorised kernel takes the whole
    // vecs of every frame (unaligned frames through unaligned buffer loads,
    // exact on gfx950: tools/unaligned_probe.hip), the generic kernel the
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
    // waves per SIMD: the kernel's occupancy, optionally capped by
    // DIPS_SERIES_WAVES_PER_SIMD (bench.py sets 4 at N > 1 so that RCCL's
    // halo kernels find a free slot beside the persistent grid instead of
    // delaying part of it; 3-5 waves per SIMD run at the same speed,
    // profiles/r01_wave_count_probe.txt)
    uint64_t per_simd = (uint64_t)occupancy_blocks(h, k);
    if (const char* cap = std::getenv("DIPS_SERIES_WAVES_PER_SIMD")) {
        const unsigned long c = std::strtoul(cap, nullptr, 10);
        if (c >= 1 && c < per_simd) per_simd = c;
    }
    const uint64_t resident = per_simd * (uint64_t)h->cu_count * 4u;
    g.n_waves = g.items < resident ? g.items : resident;
    g.blocks = (g.n_waves + 3) / 4;
    // the part-major schedule for 'per-frame' and 'overall' batches alike
    // (DIPS_SERIES_PARTS=1: 'per-frame' only, the round-3 default; =0: off).
    // 'Overall' at 4K, three alternated rounds in one process
    // (tools/isi_ab.py, profiles/r04/l/): 74.1 % of 8 TB/s against 72.05 %
    // with contiguous ranges, 5.37 against 5.62 mJ per frame
    const char* pe = std::getenv("DIPS_SERIES_PARTS");
    if ((C == 3 || C == 4) && (pf || !(pe && pe[0] == '1'))) part_geometry(g, n_frames, resident);
    g.ok = g.n_tiles < (1ull << 32) && g.blocks < (1ull << 31);
    return g;
}

// GRAY8 runs on the table kernel (series_gray.hip) unless DIPS_GRAY_LUT=0
// (the f32 kernel series_fast_kernel; kept for A/B runs and as a cross-check).
// Table layout: 4 auto (default): layout 5 or 2 per launch from a sample of
// the batch's content; 5 the u16 table keyed by (a ^ b, a) with the band
// clamp, 3 the same with a bank swizzle, 2 the u16 table keyed by (a, b)
// (swizzled), 1 two byte tables,
// 0 the f32 series_fast_kernel (DIPS_GRAY_LUT, read per call: A/B runs and
// tests)
int gray_lut_layout() {
    if (const char* e = std::getenv("DIPS_GRAY_LUT")) {
        if (e[0] == '0') return 0;
        if (e[0] == '1') return 1;
        if (e[0] == '2') return 2;
        if (e[0] == '3') return 3;
        if (e[0] == '5') return 5;
    }
    return 4;
}

// Layout 4's choice (series_gray.hip): layout 5 when the band holds at least
// kGrayAutoMin of the sampled pixels and either kGrayAutoHi of them or the
// sampled waves' frame bytes span kGrayAutoSpread levels on average, else
// layout 2.  From the layouts measured in one process over five 4K contents
// (tools/gray_layout_ab.py, profiles/r04/d/gray_layout_ab.jsonl; band
// fraction / mean spread of a wave's 1024 pixels; % of 8 TB/s):
//   synthetic (0.64 / 247): layout 5 71.8-72.3, 3 64-70, 2 63-66;
//   random (0.03 / 248): 2 61-63, 5 62-63, 3 60;
//   flat 128 +- 3 (0.51 / 6): 2 70-71, 3 69, 5 58 (bank conflicts);
//   gradient (0.80 / 70): all 69-70;  moving (0.80 / 70): 5 72.2-72.4, 2, 3 68-71.
// DIPS_GRAY_AUTO_FRAC overrides kGrayAutoMin (0: always layout 5, > 1:
// always layout 2; tests).
constexpr double kGrayAutoMin = 0.25, kGrayAutoHi = 0.9;
constexpr uint32_t kGrayAutoSpread = 48;
double gray_auto_frac() {
    if (const char* e = std::getenv("DIPS_GRAY_AUTO_FRAC")) {
        const double v = std::strtod(e, nullptr);
        if (v >= 0.0 && v <= 2.0) return v;
    }
    return kGrayAutoMin;
}
bool gray_lut_enabled() { return gray_lut_layout() != 0; }

FastGeom gray_lut_geometry(dips_handle* h, uint32_t width, uint32_t height, uint32_t n_frames) {
    FastGeom g;
    const uint64_t npx = (uint64_t)width * height;
    const uint64_t nvec = npx / 16u;
    if (nvec == 0 || npx >= (1ull << 31) || n_frames == 0) return g;
    const int layout = gray_lut_layout();
    const int alu = layout == 2 ? dips::gray_alu_vecs(h->p.tau) : 0;
    const uint64_t U = (uint64_t)(layout == 4 ? 4 : layout >= 2 ? (alu > 0 ? 4 : dips::gray_lut_unroll())
                                                               : dips::kUnrollGrayLut);
    const uint64_t gw = dips::gray_lut_waves(layout, alu);
    g.vec_bytes = nvec * 16u;
    g.tail_px0 = nvec * 16u;
    g.n_tiles = (nvec + 64 * U - 1) / (64 * U);
    g.items = g.n_tiles * n_frames;
    // one group per CU (the tables fill its LDS): 4 (3) waves per SIMD
    uint64_t per_simd = gw / 4u;
    if (const char* cap = std::getenv("DIPS_SERIES_WAVES_PER_SIMD")) {
        const unsigned long c = std::strtoul(cap, nullptr, 10);
        if (c >= 1 && c < per_simd) per_simd = c;
    }
    const uint64_t resident = per_simd * 4u * (uint64_t)h->cu_count;
    g.n_waves = g.items < resident ? g.items : resident;
    // 'per-frame' batches: the part-major schedule, as for RGB8 (part_geometry)
    if (h->p.mode == DIPS_MODE_PER_FRAME) part_geometry(g, n_frames, resident);
    g.blocks = (g.n_waves + gw - 1) / gw;
    g.ok = g.n_tiles < (1ull << 32) && g.blocks < (1ull << 31);
    return g;
}

// The T_d / T_c tables of the GRAY8 table kernel for the handle's tau.
dips_status ensure_gray_lut(dips_handle* h, hipStream_t s) {
    const int layout = gray_lut_layout();
    if (h->gray_lut_valid && h->gray_lut_tau == h->p.tau && h->gray_lut_layout == layout) return DIPS_OK;
    DIPS_HIP(h, h->gray_lut.ensure(2 * dips::kGrayLutAllocBytes));
    DIPS_HIP(h, dips::launch_gray_lut(h->gray_lut.as<uint8_t>(), h->p.tau, layout, s));
    h->gray_lut_valid = true;
    h->gray_lut_tau = h->p.tau;
    h->gray_lut_layout = layout;
    return DIPS_OK;
}

// The intensity-sum form of the RGB8 / RGBA8 series kernel for the handle's
// tau (series_v2.hip ISI): 1 (the integer sum) for tau >= 2^-5, or 2 (SADI)
// with DIPS_SERIES_ISI=2 and tau < 1; 0 (the exact f64 sum) below 2^-5 or
// with DIPS_SERIES_ISI=0 (A/B runs).  Read per call.
int series_isi_form(const dips_handle* h) {
    const int C = (int)h->p.format;
    if (C == 1 || !dips::series_v2_isi(h->p.tau)) return 0;
    const char* isi_env = std::getenv("DIPS_SERIES_ISI");
    if (isi_env && isi_env[0] == '0') return 0;
    if (isi_env && isi_env[0] == '2' && dips::series_v2_sadi(h->p.tau)) return 2;
    return 1;
}

// Run the series on device pointers, asynchronously on `s`.
dips_status run_series_device(dips_handle* h, uint32_t width, uint32_t height, const uint8_t* frames,
                              uint32_t n_frames, const uint8_t* ref0, dips_series_entry* series, uint8_t* map,
                              hipStream_t s) {
    const int C = (int)h->p.format;
    const bool pf = h->p.mode == DIPS_MODE_PER_FRAME;
    const uint64_t npx = (uint64_t)width * height;
    const uint64_t fb = npx * (uint64_t)C;
    FastGeom g;
    const bool glut = C == 1 && gray_lut_enabled();
    // RGB8 / RGBA8 frames off a 4-byte boundary (an odd frame stride or an
    // offset pointer) run the aligned-load form of the kernel (series_v2.hip
    // ALIGN) (DIPS_SERIES_ALIGN=0: the byte-unaligned 12-/16-B loads instead,
    // A/B)
    const char* align_env = std::getenv("DIPS_SERIES_ALIGN");
    const bool align = (C == 3 || C == 4) && ((((uintptr_t)frames | (uintptr_t)fb | (uintptr_t)ref0) & 3u) != 0u) &&
                       !(align_env && align_env[0] == '0');
    // RGB8 / RGBA8 with tau >= 2^-5: the integer intensity sum (series_v2.hip
    // ISI = 1, or 2 = SADI with DIPS_SERIES_ISI=2; DIPS_SERIES_ISI=0 keeps the
    // f64 sum; A/B runs)
    const int isi = series_isi_form(h);
    if (!(h->p.flags & DIPS_FLAG_FORCE_GENERIC))
        g = glut ? gray_lut_geometry(h, width, height, n_frames)
                 : fast_geometry(h, width, height, n_frames, C, pf, map != nullptr, align, isi);
    // the series starts at zero: the table and RGB(A) kernels clear it
    // themselves (SeriesArgs::zero), saving a fill launch; the others after a
    // fill (DIPS_SERIES_KZERO=0: always the fill, A/B runs)
    const char* kz_env = std::getenv("DIPS_SERIES_KZERO");
    const bool kzero = g.ok && (glut || C != 1) && n_frames < (1u << 30) && !(kz_env && kz_env[0] == '0');
    if (!kzero) DIPS_HIP(h, hipMemsetAsync(series, 0, sizeof(dips_series_entry) * (size_t)n_frames, s));
    auto launch_generic = [&](uint64_t px0) -> dips_status {
        const uint64_t bpf = (npx - px0 + 255u) / 256u;
        if (bpf * (uint64_t)n_frames >= (1ull << 31))
            return fail(h, DIPS_ERR_INVALID, "frame batch too large for the generic kernel; split the batch");
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
        if (glut && h->gray_lut_layout == 4) {
            // layout 4's thresholds in 1/1024 of the sampled pixels (each
            // workgroup samples its own items, series_gray.hip gray_sample);
            // the forced settings: 0 -> always layout 5, > 1024 -> always 2
            const double fmin = gray_auto_frac();
            a.probe_min = fmin == 0.0 ? 0u : (fmin > 1.0 ? 1025u : std::max(1u, (uint32_t)std::ceil(fmin * 1024.0)));
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
        a.thr_int = isi == 2 ? dips::series_sadi_threshold(h->p.tau) : 0u;
        a.part_frames = g.part_frames;  // 0: contiguous ranges (part_geometry)
        if (glut) {
            a.lut = h->gray_lut.p;
            const int alu = h->gray_lut_layout == 2 ? dips::gray_alu_vecs(h->p.tau) : 0;
            DIPS_HIP(h, dips::launch_series_gray_lut(a, pf, map != nullptr, h->gray_lut_layout, (uint32_t)g.blocks, s,
                                                     alu));
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
    }
    if (g.ok)
        DIPS_HIP(h, dips::launch_series_reduce(h->partials.as<uint64_t>(), n_frames, (uint32_t)g.n_tiles,
                                               C == 1 ? (glut ? 2 : 1) : (isi == 2 ? 3 : 0), series, s,
                                               isi == 2 ? dips::series_sadi_threshold(h->p.tau) : 0u));
    return DIPS_OK;
}

dips_status bind(dips_handle* h) {
    if (!h) return DIPS_ERR_INVALID;
    hipError_t e = hipSetDevice(h->device);
    if (e != hipSuccess) return hip_fail(h, e, "hipSetDevice");
    return DIPS_OK;
}

}  // namespace

extern "C" {

int dips_abi_version(void) { return DIPS_ABI_VERSION; }

dips_status dips_params_default(dips_params* p) {
    if (!p) return DIPS_ERR_INVALID;
    std::memset(p, 0, sizeof(*p));
    p->colorize = 0;
    p->spatial_window_size = 1;
    p->sensitivity = 5.0f;
    p->filter_type = DIPS_FILTER_UNFILTERED;
    p->chroma_filter = DIPS_CHROMA_NONE;
    p->mode = DIPS_MODE_OVERALL;
    p->format = DIPS_FMT_RGB8;
    p->tau = 0.0f;
    p->flags = 0;
    return DIPS_OK;
}

// DIPS_COPY_AFFINITY=1: pin the copy pool's workers to the CPUs of the NUMA
// node the device hangs off (sysfs numa_node of its PCI function), once per
// process, at the first handle (A/B runs: tools/pfc_threads_ab.py).
void maybe_pin_copy_pool(int device) {
    static std::once_flag once;
    const char* e = std::getenv("DIPS_COPY_AFFINITY");
    if (!e || e[0] != '1') return;
    std::call_once(once, [device]() {
        char bus[64] = {0};
        if (hipDeviceGetPCIBusId(bus, (int)sizeof bus, device) != hipSuccess) return;
        for (char* c = bus; *c; ++c) *c = (char)std::tolower((unsigned char)*c);
        std::ifstream f(std::string("/sys/bus/pci/devices/") + bus + "/numa_node");
        int node = -1;
        if (!(f >> node) || node < 0) return;
        const unsigned n = dips_host::CopyPool::global().pin_workers_to_node(node);
        if (std::getenv("DIPS_STRIPE_TRACE"))
            std::fprintf(stderr, "copy pool pinned to NUMA node %d of %s: %u CPUs\n", node, bus, n);
    });
}

dips_status dips_create(const dips_params* params, int device, dips_handle** out) {
    if (!out) return DIPS_ERR_INVALID;
    *out = nullptr;
    dips_params p;
    if (params) p = *params;
    else dips_params_default(&p);
    std::string why;
    if (validate_params(&p, &why) != DIPS_OK) {
        std::lock_guard<std::mutex> lk(g_err_mu);
        g_create_err = why;
        return DIPS_ERR_INVALID;
    }
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess || count <= 0 || device < 0 || device >= count) {
        std::lock_guard<std::mutex> lk(g_err_mu);
        g_create_err = std::string("no HIP device ") + std::to_string(device) + " (" +
                       (e == hipSuccess ? std::to_string(count) + " visible" : hipGetErrorString(e)) + ")";
        return DIPS_ERR_NODEVICE;
    }
    dips_handle* h = new (std::nothrow) dips_handle();
    if (!h) return DIPS_ERR_NOMEM;
    h->p = p;
    h->device = device;
    e = hipSetDevice(device);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&h->cu_count, hipDeviceAttributeMultiprocessorCount, device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&h->own_stream, hipStreamDefault);  // blocking: ordered with stream 0 (see dips_set_stream)
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&h->copy_stream, hipStreamNonBlocking);
    for (int i = 0; i < 3 && e == hipSuccess; ++i) {
        e = hipEventCreateWithFlags(&h->copy_done[i], hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&h->kernel_done[i], hipEventDisableTiming);
    }
    if (e != hipSuccess) {
        std::lock_guard<std::mutex> lk(g_err_mu);
        g_create_err = std::string("HIP initialisation failed: ") + hipGetErrorString(e);
        dips_destroy(h);
        return DIPS_ERR_HIP;
    }
    h->stream = h->own_stream;
    maybe_pin_copy_pool(device);
    *out = h;
    return DIPS_OK;
}

void dips_destroy(dips_handle* h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    if (h->copy_stream) (void)hipStreamSynchronize(h->copy_stream);
    for (auto& pr : h->ev_pending) {
        (void)hipEventDestroy(pr.first);
        (void)hipEventDestroy(pr.second);
    }
    for (auto e : h->ev_free) (void)hipEventDestroy(e);
    for (int i = 0; i < 3; ++i) {
        if (h->copy_done[i]) (void)hipEventDestroy(h->copy_done[i]);
        if (h->kernel_done[i]) (void)hipEventDestroy(h->kernel_done[i]);
        h->ring[i].release();
    }
    h->ring_ref.release();
    h->pinned[0].release();
    h->pinned[1].release();
    h->partials.release();
    h->stage_frames.release();
    h->stage_ref.release();
    h->stage_series.release();
    h->stage_map.release();
    for (auto& s : h->slots) s.release();
    for (auto& s : h->slots_alt) s.release();
    h->pipe.release();
    h->pieces.release();
    h->up_pieces.release();
    h->probe_out.release();
    h->io_out.release();
    h->raw.release();
    h->filtered.release();
    h->cb_lut.release();
    h->pk_in.release();
    h->pk_out.release();
    h->gray_lut.release();
    h->start.release();
    h->out.release();
    h->io.release();
    if (h->switch_ev) (void)hipEventDestroy(h->switch_ev);
    if (h->join_ev) (void)hipEventDestroy(h->join_ev);
    if (h->own_stream) (void)hipStreamDestroy(h->own_stream);
    if (h->copy_stream) (void)hipStreamDestroy(h->copy_stream);
    delete h;
}

const char* dips_last_error(const dips_handle* h) {
    if (h) return h->err.c_str();
    std::lock_guard<std::mutex> lk(g_err_mu);
    return g_create_err.c_str();
}

dips_status dips_set_stream(dips_handle* h, void* stream) {
    if (!h) return DIPS_ERR_INVALID;
    hipStream_t next = stream ? static_cast<hipStream_t>(stream) : h->own_stream;
    if (next == h->stream) return DIPS_OK;
    // the handle's scratch (partials, tables, staging) serves every stream:
    // work issued on the new stream waits for all work issued on the old one
    dips_status st = bind(h);
    if (st != DIPS_OK) return st;
    st = flush_pending(h);  // on the old stream, ordered before the switch
    if (st != DIPS_OK) return st;
    if (!h->switch_ev) DIPS_HIP(h, hipEventCreateWithFlags(&h->switch_ev, hipEventDisableTiming));
    DIPS_HIP(h, hipEventRecord(h->switch_ev, h->stream));
    DIPS_HIP(h, hipStreamWaitEvent(next, h->switch_ev, 0));
    h->stream = next;
    return DIPS_OK;
}

dips_status dips_synchronize(dips_handle* h) {
    dips_status st = bind(h);
    if (st != DIPS_OK) return st;
    st = flush_pending(h);  // a deferred frame into its slot first
    if (st != DIPS_OK) return st;
    DIPS_HIP(h, hipStreamSynchronize(h->stream));
    return DIPS_OK;
}

// ---------------------------------------------------------------------------
// dips-compat ComputeState
// ---------------------------------------------------------------------------

}  // extern "C"

namespace {

// A deferred frame (see dips_handle::pending) abandoned by its dispatch: the
// speculative kernels have stored the raw frame into its slot (what the
// reference's add_texture leaves there); the odd stripes ran on copy_stream,
// so wait for them -- later work on the stream is ordered after the even
// ones.  Every entry point except dispatch calls this first.
dips_status flush_pending(dips_handle* h) {
    if (!h->pending) return DIPS_OK;
    h->pending = false;
    DIPS_HIP(h, hipStreamSynchronize(h->copy_stream));
    return DIPS_OK;
}

// Bytes per pixel the zero-copy compute_main writes into pinned memory: the
// texel's key (1: gray, 2: colorized; compat_main_host_kernel) instead of the
// RGBA8 texel, rebuilt by the copy-out threads.  DIPS_COMPACT_OUT=0 keeps
// RGBA8 (A/B, tests).  Read on the calling thread.
int compact_out_keys(const dips_handle* h) {
    const char* e = std::getenv("DIPS_COMPACT_OUT");
    if (e && e[0] == '0') return 0;
    return h->p.colorize ? 2 : 1;
}

// Bytes per pixel of the zero-copy input (W = 1, keyed output only): the
// copy pool packs each staged piece into what get_intensity reads -- (max,
// min) of R, G, B (2, chroma None) or the chroma channel (1) -- instead of
// the RGBA8 texel (0: DIPS_COMPACT_IN=0, A/B).  Read on the calling thread.
int compact_in_bytes(const dips_handle* h, int out_key) {
    const char* e = std::getenv("DIPS_COMPACT_IN");
    if (out_key == 0 || h->p.spatial_window_size != 1 || (e && e[0] == '0')) return 0;
    return h->p.chroma_filter == DIPS_CHROMA_NONE ? 2 : 1;
}

// Two pixels per thread in the keyed zero-copy kernel (DIPS_HOST_PX=2; the
// default one pixel per thread measured faster: 1,042-1,089 against 950-975
// 4K frames/s, profiles/r03/compact_out_ab_px.jsonl).  Read on the calling
// thread: the launches run on the copy pool's.
uint32_t host_pairs() {
    const char* e = std::getenv("DIPS_HOST_PX");
    return (e && e[0] == '2') ? 1u : 0u;
}

// Deferral of host frames in steady state (DIPS_DEFER_UPLOAD=0 turns it off).
bool defer_upload(const dips_handle* h) {
    if (!h->main_init || (h->p.flags & DIPS_FLAG_DEVICE_PTRS)) return false;
    const char* e = std::getenv("DIPS_DEFER_UPLOAD");
    return !(e && e[0] == '0');
}

// ComputeState::add_texture (dips/src/gpu/mod.rs:170-216) from a host frame
// (through the pinned staging buffer) or a device frame (D2D).  In steady
// state with W = 1 a host frame is staged into the pinned buffer and the
// compute of the dispatch that normally follows is launched on it, stripe by
// stripe (zero-copy, both PCIe directions at once, as in
// frame_callback_striped; see dips_handle::pending); the ring bookkeeping is
// the same.
dips_status add_texture_impl(dips_handle* h, uint32_t width, uint32_t height, const uint8_t* frame, size_t len,
                             bool device_src) {
    if (!frame || width == 0 || height == 0) return fail(h, DIPS_ERR_INVALID, "add_texture: empty frame");
    const size_t fb = (size_t)width * height * 4u;
    if (len != fb) return fail(h, DIPS_ERR_INVALID, "add_texture: len != width*height*4 (RGBA8, stride width*4)");
    if (h->n_queued > 0 && (width != h->width || height != h->height))
        return fail(h, DIPS_ERR_INVALID, "add_texture: frame size changed after the first frame");
    dips_status fst = flush_pending(h);
    if (fst != DIPS_OK) return fst;
    if (!device_src && defer_upload(h)) {
        DIPS_HIP(h, h->io_out.ensure(fb));
        // io / io_out are free once both streams have drained
        DIPS_HIP(h, hipStreamSynchronize(h->stream));
        DIPS_HIP(h, hipStreamSynchronize(h->copy_stream));
        // update_temporal_texture (bind_groups.rs:407-427)
        const uint32_t slot = h->ring_idx;
        h->slot_raw[slot] = true;
        h->uniform_idx = slot;
        h->ring_idx = (slot + 1u) % 4u;
        h->added += 1;
        // the speculative compute_main, stripe by stripe as the pool stages them
        void *din = nullptr, *dout = nullptr;
        DIPS_HIP(h, hipHostGetDevicePointer(&din, h->io.p, 0));
        DIPS_HIP(h, hipHostGetDevicePointer(&dout, h->io_out.p, 0));
        dips::CompatArgs a{};
        for (int k = 0; k < 4; ++k) a.slots[k] = h->slots[k].as<uint8_t>();
        a.start = h->start.as<uint8_t>();
        a.raw = static_cast<const uint8_t*>(din);
        a.out = static_cast<uint8_t*>(dout);
        a.width = width;
        a.height = height;
        a.newest = slot;
        a.window = 1;
        a.chroma = h->p.chroma_filter;
        a.filter = h->p.filter_type;
        a.sensitivity = h->p.sensitivity;
        a.colorize = h->p.colorize ? 1u : 0u;
        a.out_key = (uint32_t)compact_out_keys(h);
        a.host_pairs = host_pairs();
        a.in_key = (uint32_t)compact_in_bytes(h, (int)a.out_key);
        h->pend_key = (int)a.out_key;
        const size_t row = (size_t)width * 4u;
        h->pend_geom.init(height, row);
        const hipStream_t cs[2] = {h->stream, h->copy_stream};
        const int32_t win = h->p.spatial_window_size;
        if (win == 1) {
            DIPS_HIP(h, dips_host::direct_stage_launch(frame, h->io.bytes(), cs, h->device, h->pieces, h->pend_geom,
                                                       [&](uint32_t y0, uint32_t y1, hipStream_t st) {
                                                           a.y0 = y0;
                                                           a.y1 = y1;
                                                           return dips::launch_compat_main_host(a, st, 1);
                                                       },
                                                       (int)a.in_key, (int)a.chroma - 1));
        } else {
            // W > 1: the filter needs the whole frame, so the stripes first go
            // into the slot (copy kernels from the pinned buffer, launched as
            // the pool stages them), then the spatial filter of the newest
            // slot into `raw` (dips_shader.wgsl:120-170, as dispatch_impl),
            // then compute_main per stripe with its output into io_out
            uint8_t* dslot = h->slots[slot].as<uint8_t>();
            const uint8_t* dsrc = static_cast<const uint8_t*>(din);
            DIPS_HIP(h, dips_host::direct_stage_launch(frame, h->io.bytes(), cs, h->device, h->up_pieces,
                                                       h->pend_geom, [&](uint32_t y0, uint32_t y1, hipStream_t st) {
                                                           return dips::launch_copy_from_host(
                                                               dsrc + (size_t)y0 * row, dslot + (size_t)y0 * row,
                                                               (uint64_t)(y1 - y0) * row, st);
                                                       }));
            if (!h->join_ev) DIPS_HIP(h, hipEventCreateWithFlags(&h->join_ev, hipEventDisableTiming));
            DIPS_HIP(h, hipEventRecord(h->join_ev, h->copy_stream));
            DIPS_HIP(h, hipStreamWaitEvent(h->stream, h->join_ev, 0));
            DIPS_HIP(h, dips::launch_compat_filter_frames(dslot, h->raw.as<uint8_t>(), width, height, 1, win,
                                                          h->p.chroma_filter, h->stream));
            a.raw = h->raw.as<uint8_t>();
            a.in_key = 0;  // (compact_in_bytes is 0 for W > 1 anyway)
            DIPS_HIP(h, h->pieces.ensure(h->pend_geom.n_s));
            for (uint32_t si = 0; si < h->pend_geom.n_s; ++si) {
                a.y0 = h->pend_geom.y0(si);
                a.y1 = h->pend_geom.y1(si);
                DIPS_HIP(h, dips::launch_compat_main_host(a, h->stream, 2));
                DIPS_HIP(h, hipEventRecord(h->pieces.ev[si], h->stream));
            }
        }
        h->pending = true;
        h->pending_slot = slot;
        return DIPS_OK;
    }
    if (h->n_queued == 0) {
        for (auto& s : h->slots) DIPS_HIP(h, s.ensure(fb));
        DIPS_HIP(h, h->raw.ensure(fb));
        DIPS_HIP(h, h->start.ensure(fb));
        DIPS_HIP(h, h->out.ensure(fb));
        DIPS_HIP(h, h->io.ensure(fb));
        h->width = width;
        h->height = height;
    }
    // host frames go up through the pinned staging buffer in pieces (host
    // copy and PCIe transfer overlapped); device frames are copied in HBM
    auto put = [&](void* dst) -> hipError_t {
        if (device_src) return hipMemcpyAsync(dst, frame, fb, hipMemcpyDeviceToDevice, h->stream);
        const hipError_t e = hipStreamSynchronize(h->stream);  // the staging buffer is free again
        return e != hipSuccess ? e : dips_host::upload_via(dst, frame, fb, h->io.bytes(), h->stream);
    };
    if (!h->main_init) {
        // VecDeque phase (dips/src/gpu/mod.rs:171-177): frames 0..3 fill slots 0..3
        DIPS_HIP(h, put(h->slots[h->n_queued].p));
        h->slot_raw[h->n_queued] = true;
        h->n_queued += 1;
        if (h->n_queued == 4) {
            // PreComputeBindGroups::initialize + run_precompute_pipeline (:178-188)
            dips::CompatArgs a{};
            for (int k = 0; k < 4; ++k) a.slots[k] = h->slots[k].as<uint8_t>();
            a.start = h->start.as<uint8_t>();
            a.width = width;
            a.height = height;
            a.window = h->p.spatial_window_size;
            a.chroma = h->p.chroma_filter;
            DIPS_HIP(h, dips::launch_compat_precompute(a, h->stream));
            // MainComputeBindGroups::initialize with starting index 0 (bind_groups.rs:73)
            h->main_init = true;
            h->ring_idx = 0;
            h->uniform_idx = 0;
        }
    } else {
        // update_temporal_texture (bind_groups.rs:407-427)
        DIPS_HIP(h, put(h->slots[h->ring_idx].p));
        h->slot_raw[h->ring_idx] = true;
        h->uniform_idx = h->ring_idx;
        h->ring_idx = (h->ring_idx + 1u) % 4u;
    }
    h->added += 1;
    if (!device_src) DIPS_HIP(h, hipStreamSynchronize(h->stream));
    return DIPS_OK;
}

// ComputeState::dispatch (dips/src/gpu/mod.rs:306-397) into `out`: a host
// buffer (synchronous readback) or a device buffer (asynchronous).
int dispatch_impl(dips_handle* h, uint8_t* out, size_t cap, bool device_dst) {
    if (!h->main_init) return 0;  // None (dips/src/gpu/mod.rs:394-396)
    const size_t fb = (size_t)h->width * h->height * 4u;
    if (!out) return fail(h, DIPS_ERR_INVALID, "dispatch: null output");
    if (cap < fb) return fail(h, DIPS_ERR_CAPACITY, "dispatch: output buffer smaller than width*height*4");
    if (h->pending && !device_dst) {
        // the speculative compute_main of the deferred add_texture: collect
        // its stripes, then store the gray texel into the newest slot (every
        // stripe's kernel has finished once collected): W = 1 quantises the
        // raw frame in place, W > 1 copies the filtered texel from `raw`
        h->pending = false;
        DIPS_HIP(h, dips_host::direct_collect(out, h->io_out.bytes(), h->pieces, h->pend_geom, h->pend_key));
        uint8_t* dslot = h->slots[h->pending_slot].as<uint8_t>();
        if (h->p.spatial_window_size == 1)
            DIPS_HIP(h, dips::launch_compat_quantise_slot(dslot, (uint64_t)h->width * h->height, h->p.chroma_filter,
                                                          h->stream));
        else
            DIPS_HIP(h, dips::launch_copy_from_host(h->raw.as<uint8_t>(), dslot, fb, h->stream));
        h->slot_raw[h->pending_slot] = false;
        return 1;
    }
    dips_status fst = flush_pending(h);
    if (fst != DIPS_OK) return fst;
    dips::CompatArgs a{};
    for (int k = 0; k < 4; ++k) a.slots[k] = h->slots[k].as<uint8_t>();
    a.start = h->start.as<uint8_t>();
    a.out = device_dst ? out : h->out.as<uint8_t>();
    a.width = h->width;
    a.height = h->height;
    a.newest = h->uniform_idx;
    a.window = h->p.spatial_window_size;
    a.chroma = h->p.chroma_filter;
    a.filter = h->p.filter_type;
    a.sensitivity = h->p.sensitivity;
    a.colorize = h->p.colorize ? 1u : 0u;
    if (a.window == 1) {
        a.raw = a.slots[a.newest];  // per-pixel in-place filter is race free
    } else {
        // spatial_median_filter of the newest slot as it was before the
        // dispatch (dips_shader.wgsl:120-170), stored as the gray ring texel
        DIPS_HIP(h, dips::launch_compat_filter_frames(a.slots[a.newest], h->raw.as<uint8_t>(), h->width, h->height, 1,
                                                      a.window, a.chroma, h->stream));
        a.raw = h->raw.as<uint8_t>();
    }
    DIPS_HIP(h, dips::launch_compat_main(a, h->stream));
    h->slot_raw[a.newest] = false;  // compute_main stored the quantised texel
    if (device_dst) return 1;
    // readback (copy_texture_to_buffer + map, gpu/mod.rs:342-393) in pieces,
    // each copied out as soon as its DMA lands
    DIPS_HIP(h, dips_host::download_via(out, h->out.p, fb, h->io.bytes(), h->stream, h->pieces));
    return 1;
}

dips_status batch_steady(dips_handle* h, const uint8_t* bf, uint8_t* bo, uint32_t m, const uint8_t* filter_src);

// frame_callback over frames[0..n) (device pointers), asynchronous: the
// first frames of the stream one by one (start texture, unquantised ring),
// then the steady state (global frame >= 7) in one batch kernel; for W > 1
// the frames are first replaced by their filtered ring texels, a chunk at a
// time (compat_filter_frames), and the batch kernel runs on those.
dips_status frame_callback_device(dips_handle* h, uint32_t width, uint32_t height, const uint8_t* frames, uint32_t n,
                                  uint8_t* out) {
    const size_t fb = (size_t)width * height * 4u;
    uint32_t t = 0;
    // one by one while the batch kernel cannot take the state: the stream's
    // first frames, or a raw frame among the three slots it reads as the ring
    auto ring_raw = [&]() {
        return h->slot_raw[(h->ring_idx + 1u) % 4u] || h->slot_raw[(h->ring_idx + 2u) % 4u] ||
               h->slot_raw[(h->ring_idx + 3u) % 4u];
    };
    for (; t < n && (h->added < 7 || ring_raw()); ++t) {
        dips_status st = add_texture_impl(h, width, height, frames + (size_t)t * fb, fb, true);
        if (st != DIPS_OK) return st;
        const int r = dispatch_impl(h, out + (size_t)t * fb, fb, true);
        if (r < 0) return (dips_status)r;
        if (r == 0)  // frame_data.to_vec() (dips/src/lib.rs:244)
            DIPS_HIP(h, hipMemcpyAsync(out + (size_t)t * fb, frames + (size_t)t * fb, fb, hipMemcpyDeviceToDevice,
                                       h->stream));
    }
    if (t == n) return DIPS_OK;
    if (width != h->width || height != h->height)
        return fail(h, DIPS_ERR_INVALID, "frame_callback_batch: frame size changed after the first frame");
    const uint8_t* bf = frames + (size_t)t * fb;
    uint8_t* bo = out + (size_t)t * fb;
    const uint32_t m = n - t;
    const uint64_t npx = (uint64_t)width * height;
    auto a16 = [](const void* q) { return ((uintptr_t)q & 15u) == 0; };
    if (npx % 4u != 0 || fb >= (1ull << 31) || !a16(bf) || !a16(bo)) {
        for (; t < n; ++t) {  // shapes the batch kernel does not take: frame by frame
            dips_status st = add_texture_impl(h, width, height, frames + (size_t)t * fb, fb, true);
            if (st != DIPS_OK) return st;
            const int r = dispatch_impl(h, out + (size_t)t * fb, fb, true);
            if (r < 0) return (dips_status)r;
        }
        return DIPS_OK;
    }
    const int32_t window = h->p.spatial_window_size;
    if (window == 1) {
        const dips_status st = batch_steady(h, bf, bo, m, nullptr);
        if (st == DIPS_OK)
            for (auto& r : h->slot_raw) r = false;  // the batch leaves gray ring texels
        return st;
    }
    // filtered ring texels of up to g frames at a time (~1 GiB of scratch)
    uint64_t g = std::max<uint64_t>(16u, (1ull << 30) / fb);
    if (const char* e = std::getenv("DIPS_WINDOW_BATCH_FRAMES")) g = std::max(1ul, std::strtoul(e, nullptr, 10));
    g = std::min<uint64_t>(std::min<uint64_t>(g, m), 65535u);
    DIPS_HIP(h, h->filtered.ensure(g * fb));
    for (uint32_t s0 = 0; s0 < m; s0 += (uint32_t)g) {
        const uint32_t gn = (uint32_t)std::min<uint64_t>(g, m - s0);
        dips_status st = batch_steady(h, h->filtered.as<uint8_t>(), bo + (size_t)s0 * fb, gn, bf + (size_t)s0 * fb);
        if (st != DIPS_OK) return st;
    }
    for (auto& r : h->slot_raw) r = false;  // the batch leaves gray ring texels
    return DIPS_OK;
}

// The batch kernel over m steady-state frames at bf (device, 16-B aligned),
// outputs to bo; the ring slots are read before and rewritten after.  With
// filter_src, the m frames there are first filtered into bf (W > 1).
dips_status batch_steady(dips_handle* h, const uint8_t* bf, uint8_t* bo, uint32_t m, const uint8_t* filter_src) {
    const uint32_t width = h->width, height = h->height;
    const size_t fb = (size_t)width * height * 4u;
    const uint64_t npx = (uint64_t)width * height;
    const bool fast = dips::alt_fast_epilogue_ok(h->p.filter_type, h->p.sensitivity);
    // the epilogue-table kernel (default) or the per-pixel arithmetic one
    // (DIPS_COMPAT_LUT=0: kept for A/B runs and as a cross-check in the tests)
    bool lut = true;
    if (const char* e = std::getenv("DIPS_COMPAT_LUT"))
        if (e[0] == '0') lut = false;
    const void* k = lut ? dips::compat_batch_lut_kernel_ptr((int)h->p.chroma_filter)
                        : dips::compat_batch_kernel_ptr((int)h->p.chroma_filter, (int)h->p.filter_type,
                                                        h->p.colorize != 0, fast);
    if (!k) return fail(h, DIPS_ERR_INVALID, "no batch kernel for these parameters");
    uint64_t resident = 0;
    if (lut) {
        resident = (uint64_t)dips::kCompatLutWaves * (uint64_t)h->cu_count;  // one workgroup per CU (LDS)
    } else {
        if (h->cb_occupancy == 0) {
            int nb = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, 256, 0) != hipSuccess || nb < 1) nb = 1;
            h->cb_occupancy = nb;
        }
        resident = (uint64_t)h->cb_occupancy * 4u * (uint64_t)h->cu_count;
    }
    const uint64_t n_vec = npx / 4u;
    const uint64_t U = lut ? (uint64_t)dips::compat_lut_unroll() : (uint64_t)dips::kUnrollCompatBatch;
    const uint64_t n_tiles = (n_vec + 64u * U - 1) / (64u * U);
    uint64_t n_chunks = (resident + n_tiles - 1) / n_tiles;
    n_chunks = std::min<uint64_t>(n_chunks, (m + 15u) / 16u);
    n_chunks = std::max<uint64_t>(n_chunks, 1);
    const uint32_t chunk = (uint32_t)((m + n_chunks - 1) / n_chunks);
    n_chunks = (m + chunk - 1) / chunk;
    if (n_tiles * n_chunks >= (1ull << 31)) return fail(h, DIPS_ERR_INVALID, "batch too large; split it");

    dips::CompatBatchArgs a{};
    a.frames = bf;
    a.out = bo;
    a.start = h->start.as<uint8_t>();
    const uint32_t r0 = h->ring_idx;  // slot of the batch's first frame
    for (uint32_t j = 0; j < 3; ++j) a.pre[j] = h->slots[(r0 + 3u - j) % 4u].as<uint8_t>();
    // with several chunks the last one would overwrite ring slots the first
    // one still reads: write the new ring into the second set and swap
    const bool swap = n_chunks > 1;
    if (swap)
        for (auto& sb : h->slots_alt) DIPS_HIP(h, sb.ensure(fb));
    for (uint32_t j = 0; j < 4; ++j) {
        a.post[j] = nullptr;
        if (j < m) {
            const uint32_t slot = (uint32_t)((r0 + (uint64_t)(m - 1 - j)) % 4u);
            a.post[j] = (swap ? h->slots_alt[slot] : h->slots[slot]).as<uint8_t>();
        }
    }
    a.frame_bytes = (uint32_t)fb;
    a.n_vec = (uint32_t)n_vec;
    a.n_frames = m;
    a.chunk = chunk;
    a.n_chunks = (uint32_t)n_chunks;
    a.n_tiles = (uint32_t)n_tiles;
    a.k = h->p.sensitivity;
    a.kneg_half = -h->p.sensitivity * 0.5f;
    if (lut) {
        // (re)build the table when the properties changed since the last batch
        const uint32_t col = h->p.colorize != 0 ? 1u : 0u;
        if (!h->cb_lut_valid || h->cb_lut_filter != h->p.filter_type || h->cb_lut_col != col ||
            !(h->cb_lut_k == h->p.sensitivity)) {
            DIPS_HIP(h, h->cb_lut.ensure(65536u * sizeof(uint16_t)));
            DIPS_HIP(h, dips::launch_compat_lut(h->cb_lut.as<uint16_t>(), h->p.filter_type, h->p.sensitivity,
                                                col != 0, h->stream));
            h->cb_lut_valid = true;
            h->cb_lut_filter = h->p.filter_type;
            h->cb_lut_col = col;
            h->cb_lut_k = h->p.sensitivity;
        }
        a.lut = h->cb_lut.as<uint16_t>();
    }
    const bool timing = (h->p.flags & DIPS_FLAG_TIME_KERNEL) != 0;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (timing) {
        e0 = take_event(h);
        e1 = take_event(h);
        if (!e0 || !e1) return fail(h, DIPS_ERR_HIP, "hipEventCreate failed");
        DIPS_HIP(h, hipEventRecord(e0, h->stream));
    }
    if (filter_src)
        DIPS_HIP(h, dips::launch_compat_filter_frames(filter_src, const_cast<uint8_t*>(bf), width, height, m,
                                                      h->p.spatial_window_size, h->p.chroma_filter, h->stream));
    if (lut)
        DIPS_HIP(h, dips::launch_compat_batch_lut(
                        a, (int)h->p.chroma_filter,
                        (uint32_t)((n_tiles * n_chunks + dips::kCompatLutWaves - 1) / dips::kCompatLutWaves), h->stream));
    else
        DIPS_HIP(h, dips::launch_compat_batch(a, (int)h->p.chroma_filter, (int)h->p.filter_type, h->p.colorize != 0,
                                              fast, (uint32_t)((n_tiles * n_chunks + 3u) / 4u), h->stream));
    if (timing) {
        DIPS_HIP(h, hipEventRecord(e1, h->stream));
        h->ev_pending.emplace_back(e0, e1);
    }
    if (swap) {
        // m >= 16: all four slots were rewritten
        for (int j = 0; j < 4; ++j) std::swap(h->slots[j], h->slots_alt[j]);
    }
    h->ring_idx = (uint32_t)((r0 + (uint64_t)m) % 4u);
    h->uniform_idx = (h->ring_idx + 3u) % 4u;
    h->added += m;
    return DIPS_OK;
}

// frame_callback in steady state (ComputeState initialised, W = 1, host
// pointers): add_texture + dispatch with the frame cut into ~4 MiB row
// stripes.  Stripe s is staged by the copy pool and DMA'd on copy_stream;
// the main kernel of stripe s (W = 1 is per pixel) runs as soon as its rows
// have landed and the stripe's readback follows on the compute stream, so
// stripe s comes back while stripes s+1.. still go up (both PCIe directions
// at once).  Same outputs and ring state as add_texture + dispatch.
int frame_callback_striped(dips_handle* h, const uint8_t* frame, uint8_t* out) {
    const auto t_call = std::chrono::steady_clock::now();
    auto us_since_call = [&]() {
        return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_call).count();
    };
    dips_status st = flush_pending(h);  // a deferred frame into its slot first
    if (st != DIPS_OK) return st;
    const uint32_t W = h->width, H = h->height;
    const size_t row = (size_t)W * 4u, fb = row * H;
    DIPS_HIP(h, h->io_out.ensure(fb));
    // the previous call's transfers out of io / into io_out are complete
    // once both streams have drained (the compute stream waited for every
    // upload; the upload stream is synchronised too in case an earlier call
    // failed between its uploads and its kernels)
    DIPS_HIP(h, hipStreamSynchronize(h->stream));
    DIPS_HIP(h, hipStreamSynchronize(h->copy_stream));
    // update_temporal_texture (bind_groups.rs:407-427)
    uint8_t* slot = h->slots[h->ring_idx].as<uint8_t>();
    h->slot_raw[h->ring_idx] = false;  // compute_main stores the quantised texel
    h->uniform_idx = h->ring_idx;
    h->ring_idx = (h->ring_idx + 1u) % 4u;
    h->added += 1;
    dips::CompatArgs a{};
    for (int k = 0; k < 4; ++k) a.slots[k] = h->slots[k].as<uint8_t>();
    a.start = h->start.as<uint8_t>();
    a.out = h->out.as<uint8_t>();
    a.raw = slot;  // W = 1: the per-pixel in-place filter is race free
    a.width = W;
    a.height = H;
    a.newest = h->uniform_idx;
    a.window = 1;
    a.chroma = h->p.chroma_filter;
    a.filter = h->p.filter_type;
    a.sensitivity = h->p.sensitivity;
    a.colorize = h->p.colorize ? 1u : 0u;
    // zero-copy form (default; DIPS_CALLBACK_DIRECT=0 selects the DMA form
    // after this block): the main kernel reads the staged stripe from pinned
    // host memory and writes its output there, the pool copies stripes in and
    // out
    const char* direct_env = std::getenv("DIPS_CALLBACK_DIRECT");
    // DIPS_CALLBACK_DIRECT=2: the compact forms through the copy engines
    // (run_striped_frame_dma_keys; A/B against the zero-copy form)
    if (direct_env && direct_env[0] == '2') {
        a.out_key = (uint32_t)compact_out_keys(h);
        a.in_key = a.out_key ? (uint32_t)compact_in_bytes(h, (int)a.out_key) : 0u;
        if (a.out_key != 0u && a.in_key != 0u) {
            const size_t npx = (size_t)W * H;
            DIPS_HIP(h, h->pk_in.ensure(npx * a.in_key));
            DIPS_HIP(h, h->pk_out.ensure(npx * a.out_key));
            a.raw = h->pk_in.as<uint8_t>();
            a.out = h->pk_out.as<uint8_t>();
            a.host_pairs = 0u;
            dips_host::CallPhases ph;
            ph.sync_us = us_since_call();
            h->cb_phases_valid = false;
            DIPS_HIP(h, dips_host::run_striped_frame_dma_keys(
                            frame, out, H, row, h->io.bytes(), h->io_out.bytes(), h->pk_in.as<uint8_t>(),
                            h->pk_out.as<uint8_t>(), h->copy_stream, h->stream, h->device, h->up_pieces, h->pieces,
                            [&](uint32_t y0, uint32_t y1, hipStream_t s) {
                                a.y0 = y0;
                                a.y1 = y1;
                                return dips::launch_compat_main_host(a, s);
                            },
                            (int)a.out_key, (int)a.in_key, (int)a.chroma - 1, &ph, t_call));
            ph.wall_us = us_since_call();
            h->cb_phases = ph;
            h->cb_phases_valid = true;
            return 1;
        }
    }
    if (!direct_env || direct_env[0] != '0') {
        void *din = nullptr, *dout = nullptr;
        DIPS_HIP(h, hipHostGetDevicePointer(&din, h->io.p, 0));
        DIPS_HIP(h, hipHostGetDevicePointer(&dout, h->io_out.p, 0));
        a.raw = static_cast<const uint8_t*>(din);
        a.out = static_cast<uint8_t*>(dout);
        a.out_key = (uint32_t)compact_out_keys(h);
        a.host_pairs = host_pairs();
        a.in_key = (uint32_t)compact_in_bytes(h, (int)a.out_key);
        // odd stripes on copy_stream (idle here, synchronised above); every
        // stripe's kernel has finished when the call returns
        const char* one_env = std::getenv("DIPS_DIRECT_STREAMS");  // "1": every stripe on the compute stream (A/B)
        const hipStream_t cs[2] = {h->stream, (one_env && one_env[0] == '1') ? h->stream : h->copy_stream};
        dips_host::CallPhases ph;
        ph.sync_us = us_since_call();
        h->cb_phases_valid = false;
        DIPS_HIP(h, dips_host::run_striped_frame_direct(frame, out, H, row, h->io.bytes(), h->io_out.bytes(), cs,
                                                        h->device, h->pieces,
                                                        [&](uint32_t y0, uint32_t y1, hipStream_t s) {
                                                            a.y0 = y0;
                                                            a.y1 = y1;
                                                            return dips::launch_compat_main_host(a, s);
                                                        },
                                                        (int)a.out_key, (int)a.in_key, (int)a.chroma - 1, &ph,
                                                        t_call));
        ph.wall_us = us_since_call();
        h->cb_phases = ph;
        h->cb_phases_valid = true;
        return 1;
    }
    DIPS_HIP(h, dips_host::run_striped_frame(frame, out, H, row, h->io.bytes(), h->io_out.bytes(), slot,
                                             h->out.as<uint8_t>(), h->copy_stream, h->stream, h->up_pieces,
                                             h->pieces, [&](uint32_t y0, uint32_t y1) {
                                                 a.y0 = y0;
                                                 a.y1 = y1;
                                                 return dips::launch_compat_main(a, h->stream);
                                             }));
    return 1;
}

}  // namespace

extern "C" {

dips_status dips_add_texture(dips_handle* h, uint32_t width, uint32_t height, const uint8_t* frame, size_t len) {
    dips_status st = bind(h);
    if (st != DIPS_OK) return st;
    return add_texture_impl(h, width, height, frame, len, false);
}

int dips_dispatch(dips_handle* h, uint8_t* out, size_t cap) {
    dips_status st = bind(h);
    if (st != DIPS_OK) return st;
    return dispatch_impl(h, out, cap, false);
}

int dips_frame_callback(dips_handle* h, uint32_t width, uint32_t height, const uint8_t* frame, size_t len,
                        uint8_t* out, size_t cap) {
    if (!h) return DIPS_ERR_INVALID;
    if (!out || cap < len) return fail(h, DIPS_ERR_CAPACITY, "frame_callback: output buffer too small");
    const char* striped_env = std::getenv("DIPS_CALLBACK_STRIPED");  // "0": plain add_texture + dispatch
    if ((!striped_env || striped_env[0] != '0') && h->main_init && h->p.spatial_window_size == 1 &&
        !(h->p.flags & DIPS_FLAG_DEVICE_PTRS) && frame &&
        width == h->width && height == h->height && len == (size_t)width * height * 4u) {
        dips_status st = bind(h);
        if (st != DIPS_OK) return st;
        return frame_callback_striped(h, frame, out);
    }
    dips_status st = dips_add_texture(h, width, height, frame, len);
    if (st != DIPS_OK) return st;
    const int r = dips_dispatch(h, out, cap);
    if (r == 0) dips_host::pool_copy(out, frame, len);  // frame_data.to_vec() (dips/src/lib.rs:244)
    return r;
}

dips_status dips_compat_resume(dips_handle* h, uint32_t width, uint32_t height, const uint8_t* start_rgba,
                               const uint8_t* halo, uint64_t t0) {
    dips_status st = bind(h);
    if (st != DIPS_OK) return st;
    if (!start_rgba || !halo || width == 0 || height == 0)
        return fail(h, DIPS_ERR_INVALID, "compat_resume: null or empty argument");
    if (t0 < 7) return fail(h, DIPS_ERR_INVALID, "compat_resume: t0 must be >= 7 (steady state of the ring)");
    // a deferred frame's speculative kernels (odd stripes on copy_stream) must
    // land before the slots are rewritten below on h->stream
    st = flush_pending(h);
    if (st != DIPS_OK) return st;
    const size_t fb = (size_t)width * height * 4u;
    const bool dev = (h->p.flags & DIPS_FLAG_DEVICE_PTRS) != 0;
    for (auto& sl : h->slots) DIPS_HIP(h, sl.ensure(fb));
    DIPS_HIP(h, h->raw.ensure(fb));
    DIPS_HIP(h, h->start.ensure(fb));
    DIPS_HIP(h, h->out.ensure(fb));
    DIPS_HIP(h, h->io.ensure(fb));
    DIPS_HIP(h, hipStreamSynchronize(h->stream));
    const hipMemcpyKind kind = dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    DIPS_HIP(h, hipMemcpyAsync(h->start.p, start_rgba, fb, kind, h->stream));
    // slot (t0-1-j) mod 4 <- ring texel of frame t0-1-j (halo[2-j]); the
    // raw frame goes through h->raw when it comes from the host
    for (int j = 0; j < 3; ++j) {
        const uint8_t* src = halo + (size_t)(2 - j) * fb;
        if (!dev) {
            DIPS_HIP(h, hipMemcpyAsync(h->raw.p, src, fb, hipMemcpyHostToDevice, h->stream));
            src = h->raw.as<uint8_t>();
        }
        uint8_t* slot = h->slots[(t0 - 1 - (uint64_t)j) % 4u].as<uint8_t>();
        if (h->p.spatial_window_size == 1)
            DIPS_HIP(h, dips::launch_compat_gray(src, slot, (uint64_t)width * height, h->p.chroma_filter, h->stream));
        else  // the filtered texel compute_main stored (dips_shader.wgsl:120-170, 187)
            DIPS_HIP(h, dips::launch_compat_filter_frames(src, slot, width, height, 1, h->p.spatial_window_size,
                                                          h->p.chroma_filter, h->stream));
    }
    DIPS_HIP(h, hipMemsetAsync(h->slots[t0 % 4u].p, 0, fb, h->stream));
    if (!dev) DIPS_HIP(h, hipStreamSynchronize(h->stream));  // host buffers are borrowed for the call only
    h->width = width;
    h->height = height;
    h->n_queued = 4;
    h->main_init = true;
    for (auto& r : h->slot_raw) r = false;  // gray texels, as the ring of a continuous run
    h->ring_idx = (uint32_t)(t0 % 4u);
    h->uniform_idx = (uint32_t)((t0 - 1) % 4u);
    h->added = t0;
    return DIPS_OK;
}

dips_status dips_frame_callback_batch(dips_handle* h, uint32_t width, uint32_t height, const uint8_t* frames,
                                      uint32_t n_frames, uint8_t* out) {
    dips_status st = bind(h);
    if (st != DIPS_OK) return st;
    st = flush_pending(h);  // a deferred frame into its slot first
    if (st != DIPS_OK) return st;
    if (n_frames == 0) return DIPS_OK;
    if (!frames || !out || width == 0 || height == 0)
        return fail(h, DIPS_ERR_INVALID, "frame_callback_batch: null or empty argument");
    if (h->p.flags & DIPS_FLAG_DEVICE_PTRS) return frame_callback_device(h, width, height, frames, n_frames, out);
    // host frames: pipelined upload / batch kernel / download in chunks
    const size_t fb = (size_t)width * height * 4u;
    const uint64_t chunk = dips_host::feed_chunk_frames(fb);
    int fst = 0;
    DIPS_HIP(h, dips_host::run_stream_pipe(
                    h->pipe, h->stream, n_frames, fb, fb, chunk, frames, out,
                    [&](const uint8_t* din, uint8_t* dout, uint64_t m) {
                        return (int)frame_callback_device(h, width, height, din, (uint32_t)m, dout);
                    },
                    &fst));
    if (fst < 0) return (dips_status)fst;
    DIPS_HIP(h, hipStreamSynchronize(h->stream));
    return DIPS_OK;
}

int dips_start_texture(dips_handle* h, uint8_t* out, size_t cap) {
    dips_status st = bind(h);
    if (st != DIPS_OK) return st;
    st = flush_pending(h);  // a deferred frame into its slot first
    if (st != DIPS_OK) return st;
    if (!h->main_init) return 0;
    const size_t fb = (size_t)h->width * h->height * 4u;
    if (!out || cap < fb) return fail(h, DIPS_ERR_CAPACITY, "start_texture: output buffer too small");
    if (h->p.flags & DIPS_FLAG_DEVICE_PTRS) {  // device destination, asynchronous on the stream
        DIPS_HIP(h, hipMemcpyAsync(out, h->start.p, fb, hipMemcpyDeviceToDevice, h->stream));
        return 1;
    }
    DIPS_HIP(h, hipMemcpyAsync(h->io.p, h->start.p, fb, hipMemcpyDeviceToHost, h->stream));
    DIPS_HIP(h, hipStreamSynchronize(h->stream));
    std::memcpy(out, h->io.p, fb);
    return 1;
}

// ---------------------------------------------------------------------------
// Batch series
// ---------------------------------------------------------------------------

double dips_series_si(const dips_series_entry* e) { return e ? std::ldexp((double)e->si_fixed, -32) : 0.0; }

dips_status dips_diff_series(dips_handle* h, uint32_t width, uint32_t height, const uint8_t* frames,
                             uint32_t n_frames, const uint8_t* ref, dips_series_entry* series, uint8_t* map) {
    dips_status st = bind(h);
    if (st != DIPS_OK) return st;
    if (n_frames == 0) return DIPS_OK;
    if (!frames || !series || width == 0 || height == 0) return fail(h, DIPS_ERR_INVALID, "diff_series: null or empty argument");
    const int C = (int)h->p.format;
    const uint64_t fb = (uint64_t)width * height * (uint64_t)C;
    if (h->p.flags & DIPS_FLAG_DEVICE_PTRS) {
        return run_series_device(h, width, height, frames, n_frames, ref ? ref : frames, series, map, h->stream);
    }
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
}

dips_status dips_diff_series_streamed(dips_handle* h, uint32_t width, uint32_t height, const uint8_t* host_frames,
                                      uint32_t n_frames, const uint8_t* host_ref, dips_series_entry* series,
                                      uint32_t chunk_frames) {
    dips_status st = bind(h);
    if (st != DIPS_OK) return st;
    if (n_frames == 0) return DIPS_OK;
    if (!host_frames || !series || width == 0 || height == 0)
        return fail(h, DIPS_ERR_INVALID, "diff_series_streamed: null or empty argument");
    const int C = (int)h->p.format;
    const bool pf = h->p.mode == DIPS_MODE_PER_FRAME;
    const size_t fb = (size_t)width * height * (size_t)C;
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
    DIPS_HIP(h, h->stage_series.ensure(sizeof(dips_series_entry) * (size_t)n_frames));
    dips_series_entry* series_dev = h->stage_series.as<dips_series_entry>();
    DIPS_HIP(h, hipStreamSynchronize(h->stream));
    DIPS_HIP(h, hipStreamSynchronize(h->copy_stream));
    if (host_ref) {
        std::memcpy(h->pinned[1].p, host_ref, fb);
        DIPS_HIP(h, hipMemcpyAsync(h->ring_ref.p, h->pinned[1].p, fb, hipMemcpyHostToDevice, h->copy_stream));
        DIPS_HIP(h, hipStreamSynchronize(h->copy_stream));
    }
    const uint32_t n_chunks = (n_frames + chunk - 1) / chunk;
    for (uint32_t k = 0; k < n_chunks; ++k) {
        const uint32_t b = k % 3u, hb = k % 2u;
        const uint32_t f0 = k * chunk;
        const uint32_t nk = (f0 + chunk <= n_frames) ? chunk : n_frames - f0;
        // pinned[hb] was last read by the DMA of chunk k-2
        if (k >= 2) DIPS_HIP(h, hipEventSynchronize(h->copy_done[(k - 2) % 3u]));
        staged_copy(static_cast<uint8_t*>(h->pinned[hb].p), host_frames + (size_t)f0 * fb, (size_t)nk * fb);
        // ring[b] was read by kernel k-3 (frames) and kernel k-2 (per-frame ref)
        if (k >= 2) DIPS_HIP(h, hipStreamWaitEvent(h->copy_stream, h->kernel_done[(k - 2) % 3u], 0));
        DIPS_HIP(h, dips_host::pipe_h2d(h->ring[b].p, h->pinned[hb].p, (size_t)nk * fb, h->copy_stream, true));
        DIPS_HIP(h, hipEventRecord(h->copy_done[b], h->copy_stream));
        DIPS_HIP(h, hipStreamWaitEvent(h->stream, h->copy_done[b], 0));
        const uint8_t* frames_dev = h->ring[b].as<uint8_t>();
        const uint8_t* ref_dev;
        if (pf) {
            if (k == 0) ref_dev = host_ref ? h->ring_ref.as<uint8_t>() : frames_dev;
            else ref_dev = h->ring[(k - 1) % 3u].as<uint8_t>() + (size_t)(chunk - 1) * fb;
        } else {
            if (k == 0 && !host_ref) {
                DIPS_HIP(h, hipMemcpyAsync(h->ring_ref.p, frames_dev, fb, hipMemcpyDeviceToDevice, h->stream));
            }
            ref_dev = h->ring_ref.as<uint8_t>();
        }
        st = run_series_device(h, width, height, frames_dev, nk, ref_dev, series_dev + f0, nullptr, h->stream);
        if (st != DIPS_OK) return st;
        DIPS_HIP(h, hipEventRecord(h->kernel_done[b], h->stream));
    }
    DIPS_HIP(h, hipMemcpyAsync(series, series_dev, sizeof(dips_series_entry) * (size_t)n_frames,
                               hipMemcpyDeviceToHost, h->stream));
    DIPS_HIP(h, hipStreamSynchronize(h->stream));
    return DIPS_OK;
}

dips_status dips_synth_frames(dips_handle* h, uint32_t width, uint32_t height, uint64_t seed, uint64_t t0,
                              uint32_t n_frames, uint8_t* dst) {
    dips_status st = bind(h);
    if (st != DIPS_OK) return st;
    if (n_frames == 0) return DIPS_OK;
    if (!dst || width == 0 || height == 0) return fail(h, DIPS_ERR_INVALID, "synth_frames: null or empty argument");
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
}

dips_status dips_kernel_time(dips_handle* h, double* total_ms, uint64_t* launches) {
    dips_status st = bind(h);
    if (st != DIPS_OK) return st;
    for (auto& pr : h->ev_pending) {
        DIPS_HIP(h, hipEventSynchronize(pr.second));
        float ms = 0.0f;
        DIPS_HIP(h, hipEventElapsedTime(&ms, pr.first, pr.second));
        h->t_ms += ms;
        h->t_launches += 1;
        h->t_each.push_back(ms);
        h->ev_free.push_back(pr.first);
        h->ev_free.push_back(pr.second);
    }
    h->ev_pending.clear();
    if (total_ms) *total_ms = h->t_ms;
    if (launches) *launches = h->t_launches;
    return DIPS_OK;
}

dips_status dips_kernel_time_reset(dips_handle* h) {
    dips_status st = dips_kernel_time(h, nullptr, nullptr);
    if (st != DIPS_OK) return st;
    h->t_ms = 0.0;
    h->t_launches = 0;
    h->t_each.clear();
    return DIPS_OK;
}

dips_status dips_kernel_time_each(dips_handle* h, double* ms_each, uint64_t cap, uint64_t* launches) {
    dips_status st = dips_kernel_time(h, nullptr, nullptr);
    if (st != DIPS_OK) return st;
    const uint64_t n = h->t_each.size();
    if (ms_each)
        for (uint64_t i = 0; i < n && i < cap; ++i) ms_each[i] = h->t_each[i];
    if (launches) *launches = n;
    return DIPS_OK;
}

dips_status dips_read_ceiling(dips_handle* h, const uint8_t* dev_bytes, uint64_t bytes, double* ms) {
    dips_status st = bind(h);
    if (st != DIPS_OK) return st;
    if (!dev_bytes || !ms) return fail(h, DIPS_ERR_INVALID, "read_ceiling: null argument");
    DIPS_HIP(h, h->probe_out.ensure(256));
    hipEvent_t e0 = take_event(h), e1 = take_event(h);
    if (!e0 || !e1) return fail(h, DIPS_ERR_HIP, "hipEventCreate failed");
    DIPS_HIP(h, hipEventRecord(e0, h->stream));
    DIPS_HIP(h, dips::launch_read_ceiling(dev_bytes, bytes, h->probe_out.as<uint32_t>(), h->stream));
    DIPS_HIP(h, hipEventRecord(e1, h->stream));
    DIPS_HIP(h, hipEventSynchronize(e1));
    float t = 0.0f;
    DIPS_HIP(h, hipEventElapsedTime(&t, e0, e1));
    *ms = t;
    h->ev_free.push_back(e0);
    h->ev_free.push_back(e1);
    return DIPS_OK;
}

dips_status dips_read_ceiling_walk(dips_handle* h, const uint8_t* dev_frames, uint32_t width, uint32_t height,
                                   uint32_t n_frames, double* ms) {
    dips_status st = bind(h);
    if (st != DIPS_OK) return st;
    if (!dev_frames || !ms) return fail(h, DIPS_ERR_INVALID, "read_ceiling_walk: null argument");
    const int C = (int)h->p.format;
    if (C != 3 && C != 4) return fail(h, DIPS_ERR_INVALID, "read_ceiling_walk: RGB8 / RGBA8 only");
    // the geometry and schedule an aligned batch of this shape runs with
    // (part-major for 'per-frame' batches of >= 256 frames)
    FastGeom g = fast_geometry(h, width, height, n_frames, C, h->p.mode == DIPS_MODE_PER_FRAME, false, false,
                               series_isi_form(h));
    if (!g.ok) return fail(h, DIPS_ERR_INVALID, "read_ceiling_walk: shape not eligible for the series kernel");
    DIPS_HIP(h, h->probe_out.ensure(256));
    dips::SeriesArgs a{};
    a.frames = dev_frames;
    a.items = g.items;
    a.frame_bytes = (uint32_t)((uint64_t)width * height * (uint64_t)C);
    a.vec_bytes = (uint32_t)g.vec_bytes;
    a.n_frames = n_frames;
    a.n_tiles = (uint32_t)g.n_tiles;
    a.n_waves = (uint32_t)g.n_waves;
    a.part_frames = g.part_frames;
    hipEvent_t e0 = take_event(h), e1 = take_event(h);
    if (!e0 || !e1) return fail(h, DIPS_ERR_HIP, "hipEventCreate failed");
    DIPS_HIP(h, hipEventRecord(e0, h->stream));
    DIPS_HIP(h, dips::launch_read_walk(a, C == 3 ? 12 : 16, (uint32_t)g.blocks, h->probe_out.as<uint32_t>(), h->stream));
    DIPS_HIP(h, hipEventRecord(e1, h->stream));
    DIPS_HIP(h, hipEventSynchronize(e1));
    float t = 0.0f;
    DIPS_HIP(h, hipEventElapsedTime(&t, e0, e1));
    *ms = t;
    h->ev_free.push_back(e0);
    h->ev_free.push_back(e1);
    return DIPS_OK;
}

dips_status dips_callback_phases(const dips_handle* h, double* us, uint32_t cap, uint32_t* n) {
    if (!h || (!us && cap)) return DIPS_ERR_INVALID;
    if (!h->cb_phases_valid) return DIPS_ERR_STATE;
    const dips_host::CallPhases& p = h->cb_phases;
    const double v[DIPS_CALLBACK_PHASES] = {p.sync_us,     p.staged_us,     p.launched_us, p.kernels_us, p.wall_us,
                                            p.pack_cpu_us, p.expand_cpu_us, p.wait_cpu_us, p.threads,    p.stripes,
                                            p.expand_us};
    for (uint32_t i = 0; i < cap && i < DIPS_CALLBACK_PHASES; ++i) us[i] = v[i];
    if (n) *n = DIPS_CALLBACK_PHASES;
    return DIPS_OK;
}

dips_status dips_series_geometry(dips_handle* h, uint32_t width, uint32_t height, uint32_t n_frames,
                                 uint64_t* waves, uint64_t* tiles, uint64_t* partial_bytes) {
    dips_status st = bind(h);
    if (st != DIPS_OK) return st;
    const int C = (int)h->p.format;
    // the kernel an aligned batch of this shape runs (its occupancy sets the
    // wave slots)
    FastGeom g = C == 1 && gray_lut_enabled()
                     ? gray_lut_geometry(h, width, height, n_frames)
                     : fast_geometry(h, width, height, n_frames, C, h->p.mode == DIPS_MODE_PER_FRAME, false, false,
                                     series_isi_form(h));
    if (waves) *waves = g.ok ? g.n_waves : 0;
    if (tiles) *tiles = g.ok ? g.n_tiles : 0;
    if (partial_bytes) *partial_bytes = g.ok ? g.n_tiles * 16u : 0;
    return g.ok ? DIPS_OK : fail(h, DIPS_ERR_INVALID, "shape not eligible for the fast kernel");
}

}  // extern "C"
