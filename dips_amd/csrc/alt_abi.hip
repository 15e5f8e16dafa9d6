// alt_abi.hip -- host side of the dips_alt operator's C ABI (include/dips_hip.h,
// "dips_alt operator").  The handle plays DiPsCompute
// (dips_alt/src/dips_compute/mod.rs:243-267: texture slots, texture_index,
// snapshot texture, output) plus the loop state of run_dips_on_file
// (dips_alt/src/lib.rs:566-567: index, overall_frame).  Every extern "C"
// body runs inside dips_abi::guard (abi_guard.h): no C++ exception leaves
// the library; every entry point returns a dips_status.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <utility>
#include <vector>

#include "../../include/dips_hip.h"
#include "abi_guard.h"
#include "comm.h"
#include "alt_lut.h"
#include "dips_kernels.h"
#include "host_buffers.h"
#include "host_stream.h"

namespace dips {

// The exact two-level index of alt_lut.h.  The value set is enumerated with
// the device's f32 arithmetic: u(c) = c / 255 (IEEE division, correctly
// rounded like __fdiv_rn), I = (u(max) + u(min)) / 2, diff = u(S) - I, and the
// cluster from fmaf(diff, 510, 1.5 * 2^23) like v_fma_f32.
const AltLutIndex& alt_lut_index() {
    static AltLutIndex idx;
    static std::once_flag once;
    std::call_once(once, [] {
        float u[256];
        for (int c = 0; c < 256; ++c) u[c] = (float)c / 255.0f;
        std::vector<float> iv;
        iv.reserve(32896);
        for (int mx = 0; mx < 256; ++mx)
            for (int mn = 0; mn <= mx; ++mn) iv.push_back((u[mx] + u[mn]) / 2.0f);
        std::sort(iv.begin(), iv.end());
        iv.erase(std::unique(iv.begin(), iv.end()), iv.end());
        std::vector<uint32_t> bits;
        bits.reserve(256 * iv.size());
        for (int s = 0; s < 256; ++s)
            for (float i : iv) {
                const float d = u[s] - i;
                uint32_t b;
                std::memcpy(&b, &d, 4);
                bits.push_back(b);
            }
        std::sort(bits.begin(), bits.end());
        bits.erase(std::unique(bits.begin(), bits.end()), bits.end());
        // clusters
        std::vector<std::vector<uint32_t>> cl(kAltLutClusters);
        for (uint32_t b : bits) {
            float d;
            std::memcpy(&d, &b, 4);
            const float t = std::fmaf(d, 510.0f, kAltLutRound);
            uint32_t tb;
            std::memcpy(&tb, &t, 4);
            const uint32_t c = tb - (0x4B400000u - 510u);  // |diff| <= 1: always in range
            if (c < (uint32_t)kAltLutClusters) cl[c].push_back(b);
        }
        uint32_t off = 0;
        idx.diffs.clear();
        idx.slots.clear();
        for (int c = 0; c < kAltLutClusters; ++c) {
            const auto& m = cl[c];
            uint32_t best_sh = 0, best_span = 0, best_base = 0;
            bool found = false;
            for (uint32_t sh = 0; sh < 32 && !m.empty(); ++sh) {
                std::vector<uint32_t> v;
                for (uint32_t b : m) v.push_back(b >> sh);
                std::sort(v.begin(), v.end());
                if (std::adjacent_find(v.begin(), v.end()) != v.end()) continue;  // not injective
                const uint32_t span = v.back() - v.front() + 1;
                if (!found || span < best_span) {
                    found = true;
                    best_sh = sh;
                    best_span = span;
                    best_base = v.front();
                }
            }
            if (m.empty()) {  // no member: never read
                idx.l1[2 * c] = 0;
                idx.l1[2 * c + 1] = 0;
                continue;
            }
            // byte address = ((bits >> sh) << 1) + x = 2 * (off + (bits >> sh) - base)
            idx.l1[2 * c] = 2u * off - 2u * best_base;
            idx.l1[2 * c + 1] = best_sh;
            for (uint32_t b : m) {
                float d;
                std::memcpy(&d, &b, 4);
                idx.diffs.push_back(d);
                idx.slots.push_back((uint16_t)(off + (b >> best_sh) - best_base));
            }
            off += best_span;
        }
        idx.l2_entries = off;
    });
    return idx;
}

}  // namespace dips

namespace {

using dips_host::DevBuf;
using dips_host::HostPinned;

std::mutex g_alt_err_mu;
std::string g_alt_create_err;

constexpr uint64_t kFrameCount = 2;  // FRAME_COUNT, dips_alt/src/lib.rs:36

}  // namespace

struct dips_alt_handle {
    dips_alt_params p{};
    int device = 0;
    int cu_count = 0;
    uint32_t width = 0, height = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    hipEvent_t switch_ev = nullptr;  // orders a newly set stream after the previous one
    hipEvent_t join_ev = nullptr;    // orders the stream after meta_stream (zero-copy W > 1 upload)
    std::string err;

    DevBuf slots[dips::kAltMaxTextures];  // input_textures (mod.rs:279-301)
    DevBuf snap[2];                       // snapshot texture (.r), double-buffered for the batch kernel
    int cur = 0;                          // snap[cur] is the snapshot texture
    uint64_t sent = 0;                    // frames sent; texture_index = sent % N (mod.rs:494, 523)
    uint64_t index = 0, overall = 0;      // run_dips_on_file loop state (lib.rs:566-567)

    DevBuf out1, meta;
    dips_host::StreamPipe pipe;  // host-pointer feed of dips_alt_send_frames
    dips_host::PieceEvents pieces;  // per-piece completion of send_frame's readback
    dips_host::PieceEvents up_pieces;  // per-stripe upload completion of send_frame
    HostPinned io_out;                 // send_frame readback staging (striped)
    HostPinned io;
    HostPinned meta_pin[2];  // per-batch flags + chunk table, pinned so the upload stays asynchronous
    hipEvent_t meta_done[2] = {nullptr, nullptr};
    hipEvent_t meta_free = nullptr;     // the last batch kernel that read the device table
    hipStream_t meta_stream = nullptr;  // uploads of the table
    bool meta_pending[2] = {false, false};
    int meta_turn = 0;
    int occupancy = 0;
    int occupancy_pre = 0;  // the prefiltered (W > 1) batch kernel
    int occupancy_lut = 0, occupancy_lut_pre = 0;  // the epilogue-table forms
    const void* occ_kernel = nullptr;  // the kernel each occupancy was computed for
    const void* occ_kernel_pre = nullptr;
    const void* occ_kernel_lut = nullptr;
    const void* occ_kernel_lut_pre = nullptr;
    // epilogue table (alt_lut.h): the index (uploaded once) and the u16
    // contents for the current properties
    DevBuf lut_l1, lut_diffs, lut_slots, lut_l2;
    bool lut_index_ready = false, lut_valid = false;
    uint32_t lut_filter = 0, lut_col = 0;
    float lut_k = 0.0f;
    DevBuf filtered;        // W > 1 batch: filtered f32 intensities of a chunk of frames (+ the one before)
    // the sharded run loop (dips_alt_run_sharded): frames received from
    // other ranks, the replay sequence built from them, its discarded
    // outputs, and the staging of a host frame this rank sends
    DevBuf shard_recv, shard_replay, shard_scratch, shard_stage;

    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pending;
    std::vector<hipEvent_t> ev_free;
    double t_ms = 0.0;
    uint64_t t_launches = 0;

    size_t frame_bytes() const { return (size_t)width * height * 4u; }
    size_t n_px() const { return (size_t)width * height; }
    bool crosscheck() const { return (p.flags & DIPS_FLAG_CROSSCHECK) != 0; }
};

namespace dips_abi {

void note_error(dips_alt_handle* h, const char* msg) noexcept {
    if (!h) return;
    try {
        h->err = msg;
    } catch (...) {
    }
}

void note_error(AltCreateTag, const char* msg) noexcept {
    try {
        std::lock_guard<std::mutex> lk(g_alt_err_mu);
        g_alt_create_err = msg;
    } catch (...) {
    }
}

}  // namespace dips_abi

using dips_abi::guard;

namespace {

dips_status fail(dips_alt_handle* h, dips_status st, const std::string& msg) {
    if (h) h->err = msg;
    return st;
}

dips_status hip_fail(dips_alt_handle* h, hipError_t e, const char* what) {
    return fail(h, e == hipErrorOutOfMemory ? DIPS_ERR_NOMEM : DIPS_ERR_HIP,
                std::string(what) + ": " + hipGetErrorString(e));
}

#define ALT_HIP(h, call)                                        \
    do {                                                        \
        hipError_t e_ = (call);                                 \
        if (e_ != hipSuccess) return hip_fail((h), e_, #call); \
    } while (0)

dips_status bind(dips_alt_handle* h) {
    if (!h) return DIPS_ERR_INVALID;
    hipError_t e = hipSetDevice(h->device);
    if (e != hipSuccess) return hip_fail(h, e, "hipSetDevice");
    return DIPS_OK;
}

dips_status validate(const dips_alt_params* p, uint32_t w, uint32_t hgt, std::string* why) {
    if (p->num_textures < 1 || p->num_textures > (uint32_t)dips::kAltMaxTextures) {
        *why = "num_textures must be in [1, 16] (MAX_TEMPORAL_ARRAY_SIZE, dips_alt pre_compute_shader.wgsl:12)";
        return DIPS_ERR_INVALID;
    }
    if (p->window_size < 1 || p->window_size > 11) {
        *why = "window_size must be in [1, 11] (MAX_WIN_SIZE_SQUARE = 11*11, pre_compute_shader.wgsl:28)";
        return DIPS_ERR_INVALID;
    }
    if (p->chroma_filter > 3u) {
        *why = "chroma_filter must be 0..3 (dips_alt/src/dips_compute/mod.rs:158-165)";
        return DIPS_ERR_INVALID;
    }
    if (!std::isfinite(p->sigmoid_horizontal_scalar)) {
        *why = "sigmoid_horizontal_scalar must be finite";
        return DIPS_ERR_INVALID;
    }
    if (w == 0 || hgt == 0) {
        *why = "width and height must be non-zero";
        return DIPS_ERR_INVALID;
    }
    if ((uint64_t)w * hgt * 4u >= (1ull << 31)) {
        *why = "frame larger than 2 GiB";
        return DIPS_ERR_INVALID;
    }
    return DIPS_OK;
}

hipEvent_t take_event(dips_alt_handle* h) {
    if (!h->ev_free.empty()) {
        hipEvent_t e = h->ev_free.back();
        h->ev_free.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

bool fast_eligible(const dips_alt_handle* h, const uint8_t* frames, const uint8_t* out) {
    auto a16 = [](const void* q) { return ((uintptr_t)q & 15u) == 0; };
    return h->p.num_textures == 2 && h->p.window_size == 1 && !(h->p.flags & DIPS_FLAG_FORCE_GENERIC) &&
           h->n_px() % 4u == 0 && a16(frames) && a16(out);
}

// Slot k's content at global frame g (the latest frame G <= g with
// G = k mod N): a batch frame if G >= sent, else the slot buffer.
const uint8_t* slot_at(const dips_alt_handle* h, const uint8_t* frames, uint64_t g, uint32_t k) {
    const uint64_t N = h->p.num_textures;
    const uint64_t back = (g + N - k) % N;  // (g - k) mod N, k < N
    if (back <= g && g - back >= h->sent) return frames + (size_t)(g - back - h->sent) * h->frame_bytes();
    return h->slots[k].as<uint8_t>();
}

// W > 1, N = 2: the same batch kernel on prefiltered intensities
// (launch_alt_filter_frames), so each frame is filtered once instead of once
// per slot and frame.
bool window_eligible(const dips_alt_handle* h, const uint8_t* frames, const uint8_t* out) {
    return h->p.num_textures == 2 && h->p.window_size > 1 && !(h->p.flags & DIPS_FLAG_FORCE_GENERIC) &&
           h->n_px() % 4u == 0 && ((uintptr_t)frames & 3u) == 0 && ((uintptr_t)out & 15u) == 0;
}

// The epilogue table of alt_lut.h for the handle's properties: the index is
// uploaded once, the u16 contents are refilled when the properties change.
dips_status ensure_lut(dips_alt_handle* h, hipStream_t s) {
    const dips::AltLutIndex& ix = dips::alt_lut_index();
    if (ix.l2_entries > (uint32_t)dips::kAltLutL2Max || ix.diffs.empty())
        return fail(h, DIPS_ERR_INVALID, "alt epilogue table: index larger than its LDS allocation");
    {
        if (!h->lut_index_ready) {
            ALT_HIP(h, h->lut_l1.ensure(sizeof(ix.l1)));
            ALT_HIP(h, h->lut_diffs.ensure(ix.diffs.size() * sizeof(float)));
            ALT_HIP(h, h->lut_slots.ensure(ix.slots.size() * sizeof(uint16_t)));
            ALT_HIP(h, h->lut_l2.ensure((size_t)dips::kAltLutL2Max * sizeof(uint16_t)));
            ALT_HIP(h, hipMemcpyAsync(h->lut_l1.p, ix.l1, sizeof(ix.l1), hipMemcpyHostToDevice, s));
            ALT_HIP(h, hipMemcpyAsync(h->lut_diffs.p, ix.diffs.data(), ix.diffs.size() * sizeof(float),
                                      hipMemcpyHostToDevice, s));
            ALT_HIP(h, hipMemcpyAsync(h->lut_slots.p, ix.slots.data(), ix.slots.size() * sizeof(uint16_t),
                                      hipMemcpyHostToDevice, s));
            ALT_HIP(h, hipMemsetAsync(h->lut_l2.p, 0, (size_t)dips::kAltLutL2Max * sizeof(uint16_t), s));
            // (the host sources are the process-lifetime index: no wait needed)
            h->lut_index_ready = true;
        }
        const uint32_t col = h->p.colorize != 0 ? 1u : 0u;
        if (!h->lut_valid || h->lut_filter != h->p.filter_type || h->lut_col != col ||
            !(h->lut_k == h->p.sigmoid_horizontal_scalar)) {
            ALT_HIP(h, dips::launch_alt_lut_fill(h->lut_l2.as<uint16_t>(), h->lut_diffs.as<float>(),
                                                 h->lut_slots.as<uint16_t>(), (uint32_t)ix.diffs.size(),
                                                 h->p.filter_type, h->p.sigmoid_horizontal_scalar, col != 0, s));
            h->lut_valid = true;
            h->lut_filter = h->p.filter_type;
            h->lut_col = col;
            h->lut_k = h->p.sigmoid_horizontal_scalar;
        }
    }
    return DIPS_OK;
}

// prev0 / prefiltered: frames and prev0 hold f32 intensities (chroma -1
// kernel); otherwise prev0 = the slot of the frame before frames[0].
dips_status run_fast(dips_alt_handle* h, const uint8_t* frames, uint32_t n, const uint8_t* flags, uint8_t* out,
                     hipStream_t s, const uint8_t* prev0 = nullptr) {
    const bool pre = prev0 != nullptr;
    const int chroma = pre ? -1 : (int)h->p.chroma_filter;
    const bool fast = dips::alt_fast_epilogue_ok(h->p.filter_type, h->p.sigmoid_horizontal_scalar);
    // the epilogue-table kernel, or the per-pixel arithmetic one (DIPS_FLAG_CROSSCHECK)
    const bool lut = !h->crosscheck();
    const void* k = lut ? dips::alt_batch_lut_kernel_ptr(chroma)
                        : dips::alt_batch_kernel_ptr(chroma, (int)h->p.filter_type, h->p.colorize != 0, fast);
    if (!k) return fail(h, DIPS_ERR_INVALID, "no batch kernel for these parameters");
    int& occ = lut ? (pre ? h->occupancy_lut_pre : h->occupancy_lut) : (pre ? h->occupancy_pre : h->occupancy);
    const void*& occ_k = lut ? (pre ? h->occ_kernel_lut_pre : h->occ_kernel_lut) : (pre ? h->occ_kernel_pre : h->occ_kernel);
    if (occ == 0 || occ_k != k) {
        occ_k = k;
        int nb = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, 256, 0) != hipSuccess || nb < 1) nb = 1;
        occ = nb;
    }
    if (lut) {
        const dips_status st = ensure_lut(h, s);
        if (st != DIPS_OK) return st;
    }
    const uint64_t n_vec = h->n_px() / 4u;
    const uint64_t U = lut ? (uint64_t)dips::kUnrollAltLut : (uint64_t)dips::kUnrollAlt;
    const uint64_t n_tiles = (n_vec + 64u * U - 1) / (64u * U);
    const uint64_t resident = (uint64_t)occ * 4u * (uint64_t)h->cu_count;
    // chunks of >= 16 frames; enough (tile, chunk) items to fill the chip
    uint64_t n_chunks = (resident + n_tiles - 1) / n_tiles;
    n_chunks = std::min<uint64_t>(n_chunks, (n + 15u) / 16u);
    n_chunks = std::max<uint64_t>(n_chunks, 1);
    const uint32_t chunk = (uint32_t)((n + n_chunks - 1) / n_chunks);
    n_chunks = (n + chunk - 1) / chunk;
    if (n_tiles * n_chunks >= (1ull << 31)) return fail(h, DIPS_ERR_INVALID, "batch too large; split it");

    // per-frame flags and per-chunk "last snapshot before the chunk", staged
    // in one of two pinned buffers (reused once its previous upload is done)
    const size_t flag_bytes = ((size_t)n + 3u) & ~(size_t)3u;
    const size_t meta_bytes = flag_bytes + 4u * n_chunks;
    const int mb = h->meta_turn;
    h->meta_turn ^= 1;
    if (h->meta_pending[mb]) {
        ALT_HIP(h, hipEventSynchronize(h->meta_done[mb]));
        h->meta_pending[mb] = false;
    }
    ALT_HIP(h, h->meta_pin[mb].ensure(meta_bytes));
    uint8_t* meta_host = h->meta_pin[mb].bytes();
    std::memset(meta_host, 0, meta_bytes);
    int32_t last = -1;
    std::vector<int32_t> cs(n_chunks, -1);
    for (uint32_t t = 0; t < n; ++t) {
        if (t % chunk == 0) cs[t / chunk] = last;
        const uint8_t f = flags && flags[t] ? 1 : 0;
        meta_host[t] = f;
        if (f) last = (int32_t)t;
    }
    std::memcpy(meta_host + flag_bytes, cs.data(), 4u * n_chunks);
    if (meta_bytes > h->meta.cap) {
        ALT_HIP(h, hipStreamSynchronize(s));  // the old table may still be read by a queued kernel
        ALT_HIP(h, hipStreamSynchronize(h->meta_stream));
        ALT_HIP(h, h->meta.ensure(meta_bytes));
    }
    // on its own idle stream: a small host-to-device copy queued behind
    // other work on `s` can hold the host until `s` drains (measured: it
    // serialised the pipelined host feed)
    ALT_HIP(h, hipStreamWaitEvent(h->meta_stream, h->meta_free, 0));
    ALT_HIP(h, hipMemcpyAsync(h->meta.p, meta_host, meta_bytes, hipMemcpyHostToDevice, h->meta_stream));
    ALT_HIP(h, hipEventRecord(h->meta_done[mb], h->meta_stream));
    ALT_HIP(h, hipStreamWaitEvent(s, h->meta_done[mb], 0));
    h->meta_pending[mb] = true;

    dips::AltBatchArgs a{};
    a.frames = frames;
    a.prev0 = pre ? prev0 : h->slots[(h->sent + 1u) % 2u].as<uint8_t>();
    a.snap_in = h->snap[h->cur].as<uint8_t>();
    a.snap_out = h->snap[1 - h->cur].as<uint8_t>();
    a.out = out;
    a.flags = h->meta.as<uint8_t>();
    a.chunk_snap = reinterpret_cast<const int32_t*>(h->meta.as<uint8_t>() + flag_bytes);
    a.frame_bytes = (uint32_t)h->frame_bytes();
    a.n_vec = (uint32_t)n_vec;
    a.n_frames = n;
    a.chunk = chunk;
    a.n_chunks = (uint32_t)n_chunks;
    a.n_tiles = (uint32_t)n_tiles;
    a.last_snap = last;
    a.scalar = h->p.sigmoid_horizontal_scalar;
    a.kneg_half = -h->p.sigmoid_horizontal_scalar * 0.5f;
    a.lut_l1 = lut ? h->lut_l1.as<uint32_t>() : nullptr;
    a.lut_l2 = lut ? h->lut_l2.as<uint16_t>() : nullptr;
    const uint32_t blocks = (uint32_t)((n_tiles * n_chunks + 3u) / 4u);

    const bool timing = (h->p.flags & DIPS_FLAG_TIME_KERNEL) != 0;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (timing) {
        e0 = take_event(h);
        e1 = take_event(h);
        if (!e0 || !e1) return fail(h, DIPS_ERR_HIP, "hipEventCreate failed");
        ALT_HIP(h, hipEventRecord(e0, s));
    }
    if (lut)
        ALT_HIP(h, dips::launch_alt_batch_lut(a, chroma, blocks, s));
    else
        ALT_HIP(h, dips::launch_alt_batch(a, chroma, (int)h->p.filter_type, h->p.colorize != 0, fast, blocks, s));
    if (timing) {
        ALT_HIP(h, hipEventRecord(e1, s));
        h->ev_pending.emplace_back(e0, e1);
    }
    ALT_HIP(h, hipEventRecord(h->meta_free, s));  // the next table upload waits for this kernel
    if (last >= 0) h->cur = 1 - h->cur;
    return DIPS_OK;
}

// W > 1, N = 2: filter a chunk of frames (plus the one before it) into
// f32 intensities, then the batch kernel over them; ~1 GiB of scratch.
dips_status run_prefiltered(dips_alt_handle* h, const uint8_t* frames, uint32_t n, const uint8_t* flags,
                            uint8_t* out, hipStream_t s) {
    const size_t fb = h->frame_bytes();
    // DIPS_WINDOW_BATCH_FRAMES sets the frames per chunk
    uint64_t g = std::max<uint64_t>(16u, (1ull << 30) / fb);
    if (const char* e = std::getenv("DIPS_WINDOW_BATCH_FRAMES")) g = std::max(1ul, std::strtoul(e, nullptr, 10));
    g = std::min<uint64_t>(std::min<uint64_t>(g, n), 65534u);
    ALT_HIP(h, h->filtered.ensure((g + 1) * fb));
    float* G = h->filtered.as<float>();
    const uint8_t* G8 = h->filtered.as<uint8_t>();
    const int32_t win = h->p.window_size;
    const uint32_t ch = h->p.chroma_filter;
    for (uint32_t s0 = 0; s0 < n; s0 += (uint32_t)g) {
        const uint32_t gn = (uint32_t)std::min<uint64_t>(g, n - s0);
        if (s0 == 0) {  // the frame before the batch: slot (sent + 1) mod 2 (zeros before the first frame)
            ALT_HIP(h, dips::launch_alt_filter_frames(h->slots[(h->sent + 1u) % 2u].as<uint8_t>(), G, h->width,
                                                      h->height, 1, win, ch, s));
            ALT_HIP(h, dips::launch_alt_filter_frames(frames, G + h->n_px(), h->width, h->height, gn, win, ch, s));
        } else {
            ALT_HIP(h, dips::launch_alt_filter_frames(frames + (size_t)(s0 - 1) * fb, G, h->width, h->height, gn + 1,
                                                      win, ch, s));
        }
        dips_status st = run_fast(h, G8 + fb, gn, flags ? flags + s0 : nullptr, out + (size_t)s0 * fb, s, G8);
        if (st != DIPS_OK) return st;
    }
    return DIPS_OK;
}

dips_status run_generic(dips_alt_handle* h, const uint8_t* frames, uint32_t n, const uint8_t* flags, uint8_t* out,
                        hipStream_t s) {
    dips::AltArgs a{};
    a.width = h->width;
    a.height = h->height;
    a.n_tex = h->p.num_textures;
    a.window = h->p.window_size;
    a.chroma = h->p.chroma_filter;
    a.filter = h->p.filter_type;
    a.scalar = h->p.sigmoid_horizontal_scalar;
    a.colorize = h->p.colorize ? 1u : 0u;
    a.snap = h->snap[h->cur].as<uint8_t>();
    for (uint32_t t = 0; t < n; ++t) {
        const uint64_t g = h->sent + t;
        for (uint32_t k = 0; k < h->p.num_textures; ++k) a.slots[k] = slot_at(h, frames, g, k);
        a.snapshot = flags && flags[t] ? 1u : 0u;
        a.out = out + (size_t)t * h->frame_bytes();
        ALT_HIP(h, dips::launch_alt_frame(a, s));
    }
    return DIPS_OK;
}

// n consecutive send_frame calls on device pointers, asynchronous on s.
dips_status send_frames_device(dips_alt_handle* h, const uint8_t* frames, uint32_t n, const uint8_t* flags,
                               uint8_t* out, hipStream_t s) {
    if (n == 0) return DIPS_OK;
    dips_status st = fast_eligible(h, frames, out)     ? run_fast(h, frames, n, flags, out, s)
                     : window_eligible(h, frames, out) ? run_prefiltered(h, frames, n, flags, out, s)
                                                       : run_generic(h, frames, n, flags, out, s);
    if (st != DIPS_OK) return st;
    // the texture slots now hold the batch's last N frames (write_texture, mod.rs:510-521)
    const uint64_t N = h->p.num_textures;
    const uint64_t end = h->sent + n;
    const uint64_t beg = end > h->sent + N ? end - N : h->sent;
    const size_t fb = h->frame_bytes();
    const bool vec = fb % 16u == 0 && ((uintptr_t)frames & 15u) == 0;
    dips::CopyFramesArgs ca{};
    ca.n16 = fb / 16u;
    uint32_t nc = 0;
    for (uint64_t G = std::max(beg, h->sent); G < end; ++G) {
        const uint8_t* src = frames + (size_t)(G - h->sent) * fb;
        if (vec && N <= 2) {
            ca.src[nc] = src;
            ca.dst[nc] = h->slots[G % N].as<uint8_t>();
            ++nc;
        } else {
            ALT_HIP(h, hipMemcpyAsync(h->slots[G % N].p, src, fb, hipMemcpyDeviceToDevice, s));
        }
    }
    ALT_HIP(h, dips::launch_copy_frames(ca, nc, s));
    h->sent = end;
    return DIPS_OK;
}

}  // namespace

extern "C" {

dips_status dips_alt_params_default(dips_alt_params* p) {
    return guard(nullptr, [&]() -> dips_status {
        if (!p) return DIPS_ERR_INVALID;
        std::memset(p, 0, sizeof(*p));
        p->colorize = 1;
        p->window_size = 1;
        p->sigmoid_horizontal_scalar = 5.0f;
        p->filter_type = DIPS_FILTER_SIGMOID;
        p->chroma_filter = DIPS_CHROMA_NONE;
        p->num_textures = (uint32_t)kFrameCount;
        p->flags = 0;
        return DIPS_OK;
    });
}

dips_status dips_alt_create(const dips_alt_params* params, uint32_t width, uint32_t height, int device,
                            dips_alt_handle** out) {
    return guard(dips_abi::AltCreateTag{}, [&]() -> dips_status {
        if (!out) return DIPS_ERR_INVALID;
        *out = nullptr;
        dips_alt_params p;
        if (params) p = *params;
        else dips_alt_params_default(&p);
        std::string why;
        if (validate(&p, width, height, &why) != DIPS_OK) {
            std::lock_guard<std::mutex> lk(g_alt_err_mu);
            g_alt_create_err = why;
            return DIPS_ERR_INVALID;
        }
        int count = 0;
        hipError_t e = hipGetDeviceCount(&count);
        if (e != hipSuccess || count <= 0 || device < 0 || device >= count) {
            std::lock_guard<std::mutex> lk(g_alt_err_mu);
            g_alt_create_err = std::string("no HIP device ") + std::to_string(device) + " (" +
                               (e == hipSuccess ? std::to_string(count) + " visible" : hipGetErrorString(e)) + ")";
            return DIPS_ERR_NODEVICE;
        }
        dips_alt_handle* h = new (std::nothrow) dips_alt_handle();
        if (!h) return DIPS_ERR_NOMEM;
        h->p = p;
        h->device = device;
        h->width = width;
        h->height = height;
        e = hipSetDevice(device);
        if (e == hipSuccess) e = hipDeviceGetAttribute(&h->cu_count, hipDeviceAttributeMultiprocessorCount, device);
        // blocking: ordered with stream 0 (see dips_set_stream)
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&h->own_stream, hipStreamDefault);
        for (int k = 0; k < 2 && e == hipSuccess; ++k)
            e = hipEventCreateWithFlags(&h->meta_done[k], hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&h->meta_free, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventRecord(h->meta_free, h->own_stream);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&h->meta_stream, hipStreamNonBlocking);
        // wgpu zero-initialises textures: slots, snapshot and output start at 0
        for (uint32_t k = 0; k < p.num_textures && e == hipSuccess; ++k) {
            e = h->slots[k].ensure(h->frame_bytes());
            if (e == hipSuccess) e = hipMemsetAsync(h->slots[k].p, 0, h->frame_bytes(), h->own_stream);
        }
        for (int k = 0; k < 2 && e == hipSuccess; ++k) {
            e = h->snap[k].ensure(h->n_px());
            if (e == hipSuccess) e = hipMemsetAsync(h->snap[k].p, 0, h->n_px(), h->own_stream);
        }
        if (e == hipSuccess) e = hipStreamSynchronize(h->own_stream);
        if (e != hipSuccess) {
            {
                std::lock_guard<std::mutex> lk(g_alt_err_mu);
                g_alt_create_err = std::string("HIP initialisation failed: ") + hipGetErrorString(e);
            }
            dips_alt_destroy(h);
            return e == hipErrorOutOfMemory ? DIPS_ERR_NOMEM : DIPS_ERR_HIP;
        }
        h->stream = h->own_stream;
        *out = h;
        return DIPS_OK;
    });
}

void dips_alt_destroy(dips_alt_handle* h) {
    guard(h, [&]() -> void {
        if (!h) return;
        (void)hipSetDevice(h->device);
        if (h->stream) (void)hipStreamSynchronize(h->stream);
        for (auto& pr : h->ev_pending) {
            (void)hipEventDestroy(pr.first);
            (void)hipEventDestroy(pr.second);
        }
        for (auto e : h->ev_free) (void)hipEventDestroy(e);
        if (h->meta_stream) (void)hipStreamSynchronize(h->meta_stream);
        for (auto& ev : h->meta_done)
            if (ev) (void)hipEventDestroy(ev);
        if (h->meta_free) (void)hipEventDestroy(h->meta_free);
        if (h->switch_ev) (void)hipEventDestroy(h->switch_ev);
        if (h->join_ev) (void)hipEventDestroy(h->join_ev);
        if (h->meta_stream) (void)hipStreamDestroy(h->meta_stream);
        for (auto& mp : h->meta_pin) mp.release();
        for (auto& s : h->slots) s.release();
        for (auto& s : h->snap) s.release();
        h->filtered.release();
        h->lut_l1.release();
        h->lut_diffs.release();
        h->lut_slots.release();
        h->lut_l2.release();
        h->out1.release();
        h->pipe.release();
        h->pieces.release();
        h->up_pieces.release();
        h->io_out.release();
        h->meta.release();
        h->io.release();
        h->shard_recv.release();
        h->shard_replay.release();
        h->shard_scratch.release();
        h->shard_stage.release();
        if (h->own_stream) (void)hipStreamDestroy(h->own_stream);
        delete h;
    });
}

const char* dips_alt_last_error(const dips_alt_handle* h) {
    return guard(h, [&]() -> const char* {
        if (h) return h->err.c_str();
        // this thread's copy (see dips_last_error)
        thread_local std::string copy;
        std::lock_guard<std::mutex> lk(g_alt_err_mu);
        copy = g_alt_create_err;
        return copy.c_str();
    });
}

dips_status dips_alt_set_stream(dips_alt_handle* h, void* stream) {
    return guard(h, [&]() -> dips_status {
        if (!h) return DIPS_ERR_INVALID;
        hipStream_t next = stream ? static_cast<hipStream_t>(stream) : h->own_stream;
        if (next == h->stream) return DIPS_OK;
        // slots, snapshot and tables serve every stream: work issued on the new
        // stream waits for all work issued on the old one
        dips_status st = bind(h);
        if (st != DIPS_OK) return st;
        if (!h->switch_ev) ALT_HIP(h, hipEventCreateWithFlags(&h->switch_ev, hipEventDisableTiming));
        ALT_HIP(h, hipEventRecord(h->switch_ev, h->stream));
        ALT_HIP(h, hipStreamWaitEvent(next, h->switch_ev, 0));
        h->stream = next;
        return DIPS_OK;
    });
}

dips_status dips_alt_synchronize(dips_alt_handle* h) {
    return guard(h, [&]() -> dips_status {
        dips_status st = bind(h);
        if (st != DIPS_OK) return st;
        ALT_HIP(h, hipStreamSynchronize(h->stream));
        return DIPS_OK;
    });
}

dips_status dips_alt_send_frame(dips_alt_handle* h, const uint8_t* frame, size_t len, int snapshot, uint8_t* out,
                                size_t cap) {
    return guard(h, [&]() -> dips_status {
        dips_status st = bind(h);
        if (st != DIPS_OK) return st;
        const size_t fb = h->frame_bytes();
        if (!frame || len != fb)
            return fail(h, DIPS_ERR_INVALID, "send_frame: len != width*height*4 (RGBA8, stride width*4)");
        if (!out || cap < fb) return fail(h, DIPS_ERR_CAPACITY, "send_frame: output buffer smaller than width*height*4");
        ALT_HIP(h, h->io.ensure(fb));
        ALT_HIP(h, h->out1.ensure(fb));
        ALT_HIP(h, hipStreamSynchronize(h->stream));
        // queue.write_texture into slot texture_index, then texture_index += 1
        const uint32_t N = h->p.num_textures;
        uint8_t* slot = h->slots[h->sent % N].as<uint8_t>();
        // the zero-copy forms (W = 1: per pixel in row stripes; W > 1: the
        // stripes into the slot by copy kernels, the frame kernel on the
        // whole frame, its output back by copy kernels), or whole-frame DMA
        // transfers through the pinned buffer (DIPS_FLAG_CROSSCHECK, and
        // frames of a byte count off a multiple of 4 with W > 1)
        const bool striped = h->p.window_size == 1 && !h->crosscheck();
        const bool window_direct = h->p.window_size > 1 && fb % 4u == 0 && !h->crosscheck();
        if (!striped && !window_direct) ALT_HIP(h, dips_host::upload_via(slot, frame, fb, h->io.bytes(), h->stream));
        h->sent += 1;
        dips::AltArgs a{};
        for (uint32_t k = 0; k < N; ++k) a.slots[k] = h->slots[k].as<uint8_t>();
        a.snap = h->snap[h->cur].as<uint8_t>();
        a.out = h->out1.as<uint8_t>();
        a.width = h->width;
        a.height = h->height;
        a.n_tex = N;
        a.window = h->p.window_size;
        a.chroma = h->p.chroma_filter;
        a.filter = h->p.filter_type;
        a.scalar = h->p.sigmoid_horizontal_scalar;
        a.colorize = h->p.colorize ? 1u : 0u;
        a.snapshot = snapshot ? 1u : 0u;
        if (window_direct) {
            ALT_HIP(h, h->io_out.ensure(fb));
            ALT_HIP(h, hipStreamSynchronize(h->meta_stream));
            void *din = nullptr, *dout = nullptr;
            ALT_HIP(h, hipHostGetDevicePointer(&din, h->io.p, 0));
            ALT_HIP(h, hipHostGetDevicePointer(&dout, h->io_out.p, 0));
            const size_t row = (size_t)h->width * 4u;
            dips_host::DirectGeom g;
            g.init(h->height, row);
            const hipStream_t cs[2] = {h->stream, h->meta_stream};
            const uint8_t* src = static_cast<const uint8_t*>(din);
            ALT_HIP(h, dips_host::direct_stage_launch(frame, h->io.bytes(), cs, h->device, h->up_pieces, g,
                                                      [&](uint32_t y0, uint32_t y1, hipStream_t st) {
                                                          return dips::launch_copy_from_host(
                                                              src + (size_t)y0 * row, slot + (size_t)y0 * row,
                                                              (uint64_t)(y1 - y0) * row, st);
                                                      }));
            if (!h->join_ev) ALT_HIP(h, hipEventCreateWithFlags(&h->join_ev, hipEventDisableTiming));
            ALT_HIP(h, hipEventRecord(h->join_ev, h->meta_stream));
            ALT_HIP(h, hipStreamWaitEvent(h->stream, h->join_ev, 0));
            ALT_HIP(h, dips::launch_alt_frame(a, h->stream));
            ALT_HIP(h, h->pieces.ensure(g.n_s));
            const uint8_t* o1 = h->out1.as<uint8_t>();
            uint8_t* dst = static_cast<uint8_t*>(dout);
            for (uint32_t si = 0; si < g.n_s; ++si) {
                const size_t o = (size_t)g.y0(si) * row, len2 = (size_t)(g.y1(si) - g.y0(si)) * row;
                ALT_HIP(h, dips::launch_copy_to_host(o1 + o, dst + o, len2, h->stream));
                ALT_HIP(h, hipEventRecord(h->pieces.ev[si], h->stream));
            }
            ALT_HIP(h, dips_host::direct_collect(out, h->io_out.bytes(), h->pieces, g));
            return DIPS_OK;
        }
        if (!striped) {
            ALT_HIP(h, dips::launch_alt_frame(a, h->stream));
            // copy_texture_to_buffer + map_async + de-pad (mod.rs:597-643)
            ALT_HIP(h, dips_host::download_via(out, h->out1.p, fb, h->io.bytes(), h->stream, h->pieces));
            return DIPS_OK;
        }
        // W = 1 (per pixel), zero-copy: ~4 MiB row stripes; the kernel reads
        // the staged stripe from pinned host memory, stores it into the slot
        // and writes its output to pinned host memory; odd stripes on
        // meta_stream (idle once synchronised here)
        ALT_HIP(h, h->io_out.ensure(fb));
        ALT_HIP(h, hipStreamSynchronize(h->meta_stream));  // no upload of an earlier call still reads `io`
        void *din = nullptr, *dout = nullptr;
        ALT_HIP(h, hipHostGetDevicePointer(&din, h->io.p, 0));
        ALT_HIP(h, hipHostGetDevicePointer(&dout, h->io_out.p, 0));
        a.out = static_cast<uint8_t*>(dout);
        const uint32_t newest = (uint32_t)((h->sent - 1) % N);
        const hipStream_t cs[2] = {h->stream, h->meta_stream};
        ALT_HIP(h, dips_host::run_striped_frame_direct(
                       frame, out, h->height, (size_t)h->width * 4u, h->io.bytes(), h->io_out.bytes(), cs, h->device,
                       h->pieces, [&](uint32_t y0, uint32_t y1, hipStream_t s) {
                           a.y0 = y0;
                           a.y1 = y1;
                           return dips::launch_alt_frame_host(a, static_cast<const uint8_t*>(din), slot, newest, s);
                       }));
        return DIPS_OK;
    });
}

dips_status dips_alt_send_frames(dips_alt_handle* h, const uint8_t* frames, uint32_t n, const uint8_t* flags,
                                 uint8_t* out) {
    return guard(h, [&]() -> dips_status {
        dips_status st = bind(h);
        if (st != DIPS_OK) return st;
        if (n == 0) return DIPS_OK;
        if (!frames || !out) return fail(h, DIPS_ERR_INVALID, "send_frames: null frames or output");
        if (h->p.flags & DIPS_FLAG_DEVICE_PTRS) return send_frames_device(h, frames, n, flags, out, h->stream);
        // host frames: pipelined upload / batch kernel / download in chunks
        const size_t fb = h->frame_bytes();
        const uint64_t chunk = dips_host::feed_chunk_frames(fb, n);
        uint64_t done = 0;
        int fst = 0;
        ALT_HIP(h, dips_host::run_stream_pipe(
                       h->pipe, h->stream, n, fb, fb, chunk, frames, out,
                       [&](const uint8_t* din, uint8_t* dout, uint64_t m) {
                           const int r = (int)send_frames_device(h, din, (uint32_t)m, flags ? flags + done : nullptr,
                                                                 dout, h->stream);
                           done += m;
                           return r;
                       },
                       &fst));
        if (fst < 0) return (dips_status)fst;
        ALT_HIP(h, hipStreamSynchronize(h->stream));
        return DIPS_OK;
    });
}

dips_status dips_alt_run(dips_alt_handle* h, const uint8_t* frames, uint32_t n, const uint64_t* markers,
                         uint32_t n_markers, uint8_t* out) {
    return guard(h, [&]() -> dips_status {
        if (!h) return DIPS_ERR_INVALID;
        if (n_markers && !markers) return fail(h, DIPS_ERR_INVALID, "run: null refresh markers");
        std::vector<uint8_t> flags(n);
        for (uint32_t t = 0; t < n; ++t) {
            flags[t] = h->index == kFrameCount ? 1 : 0;  // match index { FRAME_COUNT => Some(()) } (lib.rs:636-639)
            if (h->index <= kFrameCount) h->index += 1;  // lib.rs:662-664
            h->overall += 1;                             // lib.rs:666
            for (uint32_t k = 0; k < n_markers; ++k)     // refresh_markers.contains (lib.rs:668-670)
                if (markers[k] == h->overall) {
                    h->index = 0;
                    break;
                }
        }
        return dips_alt_send_frames(h, frames, n, flags.data(), out);
    });
}

dips_status dips_alt_run_sharded(dips_alt_handle* h, dips_comm* comm, const uint8_t* frames, uint32_t n_local,
                                 uint64_t n_total, const uint64_t* markers, uint32_t n_markers, uint8_t* out) {
    return guard(h, [&]() -> dips_status {
        dips_status st = bind(h);
        if (st != DIPS_OK) return st;
        if (!comm) return fail(h, DIPS_ERR_INVALID, "alt sharded: null communicator");
        if (comm->device != h->device) return fail(h, DIPS_ERR_INVALID, "alt sharded: device mismatch");
        if (n_markers && !markers) return fail(h, DIPS_ERR_INVALID, "alt sharded: null refresh markers");
        if (n_total >= (1ull << 32)) return fail(h, DIPS_ERR_INVALID, "alt sharded: 2^32 frames or more");
        const int G = comm->nranks, r = comm->rank;
        const uint64_t N = h->p.num_textures;
        auto range = [&](int k, uint64_t* f, uint64_t* c) {
            const unsigned __int128 nt = n_total;
            *f = (uint64_t)(nt * (unsigned)k / (unsigned)G);
            *c = (uint64_t)(nt * (unsigned)(k + 1) / (unsigned)G) - *f;
        };
        uint64_t first = 0, count = 0;
        range(r, &first, &count);
        if ((uint64_t)n_local != count)
            return fail(h, DIPS_ERR_INVALID, "alt sharded: rank " + std::to_string(r) + " owns " +
                                                 std::to_string(count) + " frames, n_local is " + std::to_string(n_local));
        if (count && (!frames || !out)) return fail(h, DIPS_ERR_INVALID, "alt sharded: null frames or output");
        if (h->sent != 0 || h->overall != 0)
            return fail(h, DIPS_ERR_STATE, "alt sharded: the handle must be fresh (no frame sent yet)");

        // the run_dips_on_file loop over every frame (lib.rs:588-683, as
        // dips_alt_run): the snapshot flags, and the loop state after this
        // rank's last frame
        std::vector<uint8_t> flags((size_t)n_total);
        uint64_t index = 0, overall = 0, end_index = 0, end_overall = 0;
        for (uint64_t t = 0; t < n_total; ++t) {
            flags[t] = index == kFrameCount ? 1 : 0;
            if (index <= kFrameCount) index += 1;
            overall += 1;
            for (uint32_t k = 0; k < n_markers; ++k)
                if (markers[k] == overall) {
                    index = 0;
                    break;
                }
            if (t + 1 == first + count) {
                end_index = index;
                end_overall = overall;
            }
        }
        // what rank k replays through its fresh operator before its own
        // frames: the source frames of the last snapshot before its first
        // frame t0 (that one flagged), then its halo, the min(N, t0) frames
        // before t0 -- the slots and the snapshot texture as the single loop
        // has them at frame t0.  With t0 < N the single loop still holds
        // N - t0 never-written (zero) slots, the oldest; after a snapshot
        // replay that many zero frames (kZeroFrame) go before the halo.
        constexpr uint64_t kZeroFrame = ~0ull;
        auto replay_of = [&](int k) {
            std::vector<std::pair<uint64_t, uint8_t>> rp;
            uint64_t t0 = 0, c = 0;
            range(k, &t0, &c);
            if (t0 == 0 || c == 0) return rp;
            for (uint64_t sf = t0; sf-- > 0;) {
                if (flags[sf]) {
                    for (uint64_t g = sf + 1 > N ? sf + 1 - N : 0; g <= sf; ++g) rp.emplace_back(g, g == sf ? 1 : 0);
                    break;
                }
            }
            const uint64_t halo = std::min<uint64_t>(N, t0);
            if (!rp.empty())
                for (uint64_t z = halo; z < N; ++z) rp.emplace_back(kZeroFrame, 0);
            for (uint64_t g = t0 - halo; g < t0; ++g) rp.emplace_back(g, 0);
            return rp;
        };
        auto distinct = [&](const std::vector<std::pair<uint64_t, uint8_t>>& rp) {
            std::vector<uint64_t> v;
            for (auto& e : rp)
                if (e.first != kZeroFrame) v.push_back(e.first);
            std::sort(v.begin(), v.end());
            v.erase(std::unique(v.begin(), v.end()), v.end());
            return v;
        };
        auto owner = [&](uint64_t g) {
            int k = (int)((unsigned __int128)g * (unsigned)G / n_total);  // first guess, then adjust
            uint64_t f = 0, c = 0;
            for (;;) {
                range(k, &f, &c);
                if (g < f) --k;
                else if (g >= f + c) ++k;
                else return k;
            }
        };
        const size_t fb = h->frame_bytes();
        const bool dev = (h->p.flags & DIPS_FLAG_DEVICE_PTRS) != 0;
        hipStream_t s = h->stream;

        // every (frame, owner, destination) transfer, in one order on every
        // rank; each rank takes part in each exchange (the loopback meets
        // all ranks), passing -1 where it neither sends nor receives
        const auto mine = replay_of(r);
        const std::vector<uint64_t> want = distinct(mine);  // the frames this rank receives
        if (!want.empty()) ALT_HIP(h, h->shard_recv.ensure(want.size() * fb));
        if (!dev) ALT_HIP(h, h->shard_stage.ensure(fb));
        for (int k = 1; k < G; ++k) {
            for (uint64_t g : distinct(replay_of(k))) {
                const int o = owner(g);
                if (o == k) continue;  // (never: replayed frames precede the rank's own)
                const void* send = nullptr;
                void* recv = nullptr;
                if (r == o) {
                    const uint8_t* src = frames + (size_t)(g - first) * fb;
                    if (!dev) {
                        ALT_HIP(h, hipMemcpyAsync(h->shard_stage.p, src, fb, hipMemcpyHostToDevice, s));
                        src = static_cast<const uint8_t*>(h->shard_stage.p);
                    }
                    send = src;
                }
                if (r == k)
                    recv = h->shard_recv.as<uint8_t>() +
                           (size_t)(std::lower_bound(want.begin(), want.end(), g) - want.begin()) * fb;
                const dips_status cs = comm->exchange(send, r == o ? k : -1, recv, r == k ? o : -1, fb, s);
                if (cs != DIPS_OK)
                    return fail(h, cs, "alt sharded: communicator (rank " + std::to_string(r) + "): " + comm->err);
            }
        }

        // replay (outputs discarded), then this rank's frames with its flags
        if (!mine.empty()) {
            ALT_HIP(h, h->shard_replay.ensure(mine.size() * fb));
            ALT_HIP(h, h->shard_scratch.ensure(mine.size() * fb));
            std::vector<uint8_t> rflags(mine.size());
            for (size_t i = 0; i < mine.size(); ++i) {
                uint8_t* dst = h->shard_replay.as<uint8_t>() + i * fb;
                if (mine[i].first == kZeroFrame) {
                    ALT_HIP(h, hipMemsetAsync(dst, 0, fb, s));
                } else {
                    const size_t at =
                        (size_t)(std::lower_bound(want.begin(), want.end(), mine[i].first) - want.begin());
                    ALT_HIP(h, hipMemcpyAsync(dst, h->shard_recv.as<uint8_t>() + at * fb, fb,
                                              hipMemcpyDeviceToDevice, s));
                }
                rflags[i] = mine[i].second;
            }
            st = send_frames_device(h, h->shard_replay.as<uint8_t>(), (uint32_t)mine.size(), rflags.data(),
                                    h->shard_scratch.as<uint8_t>(), s);
            if (st != DIPS_OK) return st;
        }
        if (count) {
            st = dev ? send_frames_device(h, frames, (uint32_t)count, flags.data() + first, out, s)
                     : dips_alt_send_frames(h, frames, (uint32_t)count, flags.data() + first, out);
            if (st != DIPS_OK) return st;
        }
        h->index = end_index;  // the loop state of the single loop after this rank's last frame
        h->overall = end_overall;
        if (dev) ALT_HIP(h, hipStreamSynchronize(s));  // synchronous in both pointer modes
        return DIPS_OK;
    });
}

dips_status dips_alt_snapshot_texture(dips_alt_handle* h, uint8_t* out, size_t cap) {
    return guard(h, [&]() -> dips_status {
        dips_status st = bind(h);
        if (st != DIPS_OK) return st;
        if (!out || cap < h->n_px())
            return fail(h, DIPS_ERR_CAPACITY, "snapshot_texture: output smaller than width*height");
        ALT_HIP(h, hipMemcpyAsync(out, h->snap[h->cur].p, h->n_px(), hipMemcpyDeviceToHost, h->stream));
        ALT_HIP(h, hipStreamSynchronize(h->stream));
        return DIPS_OK;
    });
}

dips_status dips_alt_kernel_time(dips_alt_handle* h, double* total_ms, uint64_t* launches) {
    return guard(h, [&]() -> dips_status {
        dips_status st = bind(h);
        if (st != DIPS_OK) return st;
        for (auto& pr : h->ev_pending) {
            ALT_HIP(h, hipEventSynchronize(pr.second));
            float ms = 0.0f;
            ALT_HIP(h, hipEventElapsedTime(&ms, pr.first, pr.second));
            h->t_ms += ms;
            h->t_launches += 1;
            h->ev_free.push_back(pr.first);
            h->ev_free.push_back(pr.second);
        }
        h->ev_pending.clear();
        if (total_ms) *total_ms = h->t_ms;
        if (launches) *launches = h->t_launches;
        return DIPS_OK;
    });
}

dips_status dips_alt_kernel_time_reset(dips_alt_handle* h) {
    return guard(h, [&]() -> dips_status {
        dips_status st = dips_alt_kernel_time(h, nullptr, nullptr);
        if (st != DIPS_OK) return st;
        h->t_ms = 0.0;
        h->t_launches = 0;
        return DIPS_OK;
    });
}

dips_status dips_alt_lut_index(uint32_t* l1, uint32_t l1_cap, float* diffs, uint16_t* slots, uint32_t cap,
                               uint32_t* n_diffs, uint32_t* l2_entries) {
    return guard(nullptr, [&]() -> dips_status {
        const dips::AltLutIndex& ix = dips::alt_lut_index();
        if (n_diffs) *n_diffs = (uint32_t)ix.diffs.size();
        if (l2_entries) *l2_entries = ix.l2_entries;
        if (l1) {
            if (l1_cap < 2u * dips::kAltLutClusters) return DIPS_ERR_CAPACITY;
            std::memcpy(l1, ix.l1, sizeof(ix.l1));
        }
        if (diffs || slots) {
            if (cap < ix.diffs.size()) return DIPS_ERR_CAPACITY;
            if (diffs) std::memcpy(diffs, ix.diffs.data(), ix.diffs.size() * sizeof(float));
            if (slots) std::memcpy(slots, ix.slots.data(), ix.slots.size() * sizeof(uint16_t));
        }
        return DIPS_OK;
    });
}

dips_status dips_alt_lut_selfcheck(dips_alt_handle* h, uint64_t* mismatches) {
    return guard(h, [&]() -> dips_status {
        dips_status st = bind(h);
        if (st != DIPS_OK) return st;
        if (!mismatches) return fail(h, DIPS_ERR_INVALID, "lut_selfcheck: null argument");
        st = ensure_lut(h, h->stream);
        if (st != DIPS_OK) return st;
        DevBuf bad;
        ALT_HIP(h, bad.ensure(sizeof(unsigned long long)));
        ALT_HIP(h, hipMemsetAsync(bad.p, 0, sizeof(unsigned long long), h->stream));
        const hipError_t e = dips::launch_alt_lut_check(h->lut_l1.as<uint32_t>(), h->lut_l2.as<uint16_t>(),
                                                        h->p.filter_type, h->p.sigmoid_horizontal_scalar,
                                                        h->p.colorize != 0, bad.as<unsigned long long>(), h->stream);
        unsigned long long n = 0;
        hipError_t e2 =
            e == hipSuccess ? hipMemcpyAsync(&n, bad.p, sizeof(n), hipMemcpyDeviceToHost, h->stream) : e;
        if (e2 == hipSuccess) e2 = hipStreamSynchronize(h->stream);
        bad.release();
        if (e2 != hipSuccess) return hip_fail(h, e2, "lut_selfcheck");
        *mismatches = n;
        return DIPS_OK;
    });
}

}  // extern "C"
