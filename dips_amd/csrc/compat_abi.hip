// compat_abi.hip -- host side of include/dips_hip.h, part 2: the dips-compat
// ComputeState.  add_texture (dips/src/gpu/mod.rs:170-216), dispatch
// (:306-397), frame_callback (dips/src/lib.rs:233-246), its batch form, the
// start texture and the frame-range resume of the sharded path.  Every
// extern "C" body runs inside dips_abi::guard (abi_guard.h).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <utility>

#include "dips_handle.h"
#include "dips_kernels.h"

using dips_abi::guard;
using namespace dips_internal;

namespace dips_internal {

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

}  // namespace dips_internal

namespace {

// Bytes per pixel the zero-copy compute_main writes into pinned memory: the
// texel's key (1: gray, 2: colorized; compat_main_host_kernel) instead of the
// RGBA8 texel, rebuilt by the copy-out threads.
int compact_out_keys(const dips_handle* h) { return h->p.colorize ? 2 : 1; }

// Bytes per pixel of the zero-copy input (W = 1): the copy pool packs each
// staged piece into what get_intensity reads -- (max, min) of R, G, B (2,
// chroma None) or the chroma channel (1) -- instead of the RGBA8 texel.
int compact_in_bytes(const dips_handle* h) {
    if (h->p.spatial_window_size != 1) return 0;
    return h->p.chroma_filter == DIPS_CHROMA_NONE ? 2 : 1;
}

// Deferral of host frames in steady state (off with DIPS_FLAG_CROSSCHECK).
bool defer_upload(const dips_handle* h) {
    return h->main_init && !(h->p.flags & DIPS_FLAG_DEVICE_PTRS) && !h->crosscheck();
}

// ComputeState::add_texture (dips/src/gpu/mod.rs:170-216) from a host frame
// (through the pinned staging buffer) or a device frame (D2D).  In steady
// state a host frame is staged into the pinned buffer and the compute of the
// dispatch that normally follows is launched on it, stripe by stripe
// (zero-copy, both PCIe directions at once, as in frame_callback_striped;
// see dips_handle::pending); the ring bookkeeping is the same.
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
        a.in_key = (uint32_t)compact_in_bytes(h);
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
    // filtered ring texels of up to g frames at a time (~1 GiB of scratch;
    // DIPS_WINDOW_BATCH_FRAMES sets g)
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
    // the epilogue-table kernel, or the per-pixel arithmetic one (DIPS_FLAG_CROSSCHECK)
    const bool lut = !h->crosscheck();
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
    const uint64_t U = lut ? (uint64_t)dips::kUnrollCompatLut : (uint64_t)dips::kUnrollCompatBatch;
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
// pointers): add_texture + dispatch in one zero-copy pass.  The frame is cut
// into ~4 MiB row stripes; the copy pool packs each stripe into pinned
// memory in the compact input form (compact_in_bytes), the thread that
// stages a stripe's last piece launches its compute_main, which reads the
// stripe over PCIe, stores the quantised texel into the ring slot and writes
// the output keys (compact_out_keys) back into pinned memory, and the pool
// expands each stripe's keys into `out` as soon as its kernel has finished
// -- both PCIe directions at once.  Same outputs and ring state as
// add_texture + dispatch.
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
    h->slot_raw[h->ring_idx] = false;  // compute_main stores the quantised texel
    h->uniform_idx = h->ring_idx;
    h->ring_idx = (h->ring_idx + 1u) % 4u;
    h->added += 1;
    dips::CompatArgs a{};
    for (int k = 0; k < 4; ++k) a.slots[k] = h->slots[k].as<uint8_t>();
    a.start = h->start.as<uint8_t>();
    a.width = W;
    a.height = H;
    a.newest = h->uniform_idx;
    a.window = 1;
    a.chroma = h->p.chroma_filter;
    a.filter = h->p.filter_type;
    a.sensitivity = h->p.sensitivity;
    a.colorize = h->p.colorize ? 1u : 0u;
    void *din = nullptr, *dout = nullptr;
    DIPS_HIP(h, hipHostGetDevicePointer(&din, h->io.p, 0));
    DIPS_HIP(h, hipHostGetDevicePointer(&dout, h->io_out.p, 0));
    a.raw = static_cast<const uint8_t*>(din);
    a.out = static_cast<uint8_t*>(dout);
    a.out_key = (uint32_t)compact_out_keys(h);
    a.in_key = (uint32_t)compact_in_bytes(h);
    // odd stripes on copy_stream (idle here, synchronised above); every
    // stripe's kernel has finished when the call returns
    const hipStream_t cs[2] = {h->stream, h->copy_stream};
    dips_host::CallPhases ph;
    ph.sync_us = us_since_call();
    DIPS_HIP(h, dips_host::run_striped_frame_direct(frame, out, H, row, h->io.bytes(), h->io_out.bytes(), cs, h->device,
                                                    h->pieces,
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

}  // namespace

namespace dips_internal {

dips_status compat_resume_impl(dips_handle* h, uint32_t width, uint32_t height, const uint8_t* start_rgba,
                               const uint8_t* halo, uint64_t t0, bool dev) {
    if (!start_rgba || !halo || width == 0 || height == 0)
        return fail(h, DIPS_ERR_INVALID, "compat_resume: null or empty argument");
    if (t0 < 7) return fail(h, DIPS_ERR_INVALID, "compat_resume: t0 must be >= 7 (steady state of the ring)");
    // a deferred frame's speculative kernels (odd stripes on copy_stream)
    // must land before the slots are rewritten below on h->stream
    dips_status st = flush_pending(h);
    if (st != DIPS_OK) return st;
    const size_t fb = (size_t)width * height * 4u;

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
            DIPS_HIP(h, dips::launch_compat_gray(src, slot, (uint64_t)width * height, h->p.chroma_filter,
                                                 h->stream));
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

}  // namespace dips_internal

extern "C" {

dips_status dips_add_texture(dips_handle* h, uint32_t width, uint32_t height, const uint8_t* frame, size_t len) {
    return guard(h, [&]() -> dips_status {
        dips_status st = bind(h);
        if (st != DIPS_OK) return st;
        return add_texture_impl(h, width, height, frame, len, false);
    });
}

int dips_dispatch(dips_handle* h, uint8_t* out, size_t cap) {
    return guard(h, [&]() -> int {
        dips_status st = bind(h);
        if (st != DIPS_OK) return st;
        return dispatch_impl(h, out, cap, false);
    });
}

int dips_frame_callback(dips_handle* h, uint32_t width, uint32_t height, const uint8_t* frame, size_t len,
                        uint8_t* out, size_t cap) {
    return guard(h, [&]() -> int {
        if (!h) return DIPS_ERR_INVALID;
        h->cb_phases_valid = false;  // set again only by a completed zero-copy call
        if (!out || cap < len) return fail(h, DIPS_ERR_CAPACITY, "frame_callback: output buffer too small");
        if (!h->crosscheck() && h->main_init && h->p.spatial_window_size == 1 &&
            !(h->p.flags & DIPS_FLAG_DEVICE_PTRS) && frame && width == h->width && height == h->height &&
            len == (size_t)width * height * 4u) {
            dips_status st = bind(h);
            if (st != DIPS_OK) return st;
            return frame_callback_striped(h, frame, out);
        }
        dips_status st = dips_add_texture(h, width, height, frame, len);
        if (st != DIPS_OK) return st;
        const int r = dips_dispatch(h, out, cap);
        if (r == 0) dips_host::pool_copy(out, frame, len);  // frame_data.to_vec() (dips/src/lib.rs:244)
        return r;
    });
}

dips_status dips_compat_resume(dips_handle* h, uint32_t width, uint32_t height, const uint8_t* start_rgba,
                               const uint8_t* halo, uint64_t t0) {
    return guard(h, [&]() -> dips_status {
        dips_status st = bind(h);
        if (st != DIPS_OK) return st;
        return compat_resume_impl(h, width, height, start_rgba, halo, t0, (h->p.flags & DIPS_FLAG_DEVICE_PTRS) != 0);
    });
}

dips_status dips_frame_callback_batch(dips_handle* h, uint32_t width, uint32_t height, const uint8_t* frames,
                                      uint32_t n_frames, uint8_t* out) {
    return guard(h, [&]() -> dips_status {
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
        const uint64_t chunk = dips_host::feed_chunk_frames(fb, n_frames);
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
    });
}

int dips_start_texture(dips_handle* h, uint8_t* out, size_t cap) {
    return guard(h, [&]() -> int {
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
    });
}

dips_status dips_callback_phases(const dips_handle* h, double* us, uint32_t cap, uint32_t* n) {
    return guard(h, [&]() -> dips_status {
        if (!h || (!us && cap)) return DIPS_ERR_INVALID;
        if (!h->cb_phases_valid) return DIPS_ERR_STATE;
        const dips_host::CallPhases& p = h->cb_phases;
        const double v[DIPS_CALLBACK_PHASES] = {p.sync_us,     p.staged_us,     p.launched_us, p.kernels_us,
                                                p.wall_us,     p.pack_cpu_us,   p.expand_cpu_us, p.wait_cpu_us,
                                                p.threads,     p.stripes,       p.expand_us};
        for (uint32_t i = 0; i < cap && i < DIPS_CALLBACK_PHASES; ++i) us[i] = v[i];
        if (n) *n = DIPS_CALLBACK_PHASES;
        return DIPS_OK;
    });
}

}  // extern "C"
