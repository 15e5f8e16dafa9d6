// host_stream.h -- pipelined host-memory feed for the batch operators
// (internal to libdips_hip.so): frames in pageable host memory are copied
// into pinned buffers by several threads, DMA'd to HBM on an upload stream,
// processed on the compute stream and DMA'd back on a download stream, two
// chunks in flight, so the PCIe transfers in both directions, the host copies
// and the kernels overlap.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "copy_pool.h"
#include "host_buffers.h"

namespace dips {  // compat_kernels.hip (also declared in dips_kernels.h)
hipError_t launch_copy_from_host(const uint8_t* src, uint8_t* dst, uint64_t bytes, hipStream_t s);
hipError_t launch_copy_to_host(const uint8_t* src, uint8_t* dst, uint64_t bytes, hipStream_t s);
}  // namespace dips

namespace dips_host {

// Chunk copies of the host-fed pipelines between a pinned buffer and HBM: a
// copy kernel (system-scope accesses to the pinned side) or hipMemcpyAsync
// (a DMA engine), per call site.  Measured in one process
// (profiles/r02_pipe_kernel_copy_ab_box*.jsonl): the streamed series' uploads by kernel ran
// 1.00-1.15x the DMA rate (`kernel` there), the visual operators' two-way
// pipe 0.81-0.82x with a kernel upload (DMA kept).
inline hipError_t pipe_h2d(void* dev, const void* pin, size_t bytes, hipStream_t s, bool kernel = false) {
    if (kernel && bytes % 4u == 0) {
        void* pd = nullptr;
        const hipError_t e = hipHostGetDevicePointer(&pd, const_cast<void*>(pin), 0);
        if (e != hipSuccess) return e;
        return dips::launch_copy_from_host(static_cast<const uint8_t*>(pd), static_cast<uint8_t*>(dev), bytes, s);
    }
    return hipMemcpyAsync(dev, pin, bytes, hipMemcpyHostToDevice, s);
}
inline hipError_t pipe_d2h(void* pin, const void* dev, size_t bytes, hipStream_t s, bool kernel = false) {
    if (kernel && bytes % 4u == 0) {
        void* pd = nullptr;
        const hipError_t e = hipHostGetDevicePointer(&pd, pin, 0);
        if (e != hipSuccess) return e;
        return dips::launch_copy_to_host(static_cast<const uint8_t*>(dev), static_cast<uint8_t*>(pd), bytes, s);
    }
    return hipMemcpyAsync(pin, dev, bytes, hipMemcpyDeviceToHost, s);
}

// Host copy over the persistent pool (copy_pool.h).
inline void staged_copy(uint8_t* dst, const uint8_t* src, size_t bytes) { pool_copy(dst, src, bytes); }

// Piece size of the per-frame transfers: small enough that the first DMA
// starts while the pool still copies the rest, large enough that a DMA
// command moves data most of the time.  4 MiB measured best for a 4K RGBA8
// frame (1 / 2 / 4 / 8 MiB: 463 / 497-549 / 548-554 / 478-502 frames/s of
// frame_callback); a frame below 4 MiB is cut into quarters (64-B multiples,
// at least 4 KiB) so that its copy and transfer still overlap.
inline size_t piece_bytes(size_t frame_bytes) {
    constexpr size_t kPiece = (size_t)4u << 20;
    if (frame_bytes >= kPiece) return kPiece;
    return std::max<size_t>(4096u, (frame_bytes / 4u + 63u) & ~(size_t)63u);
}

// One frame host -> device through the pinned buffer `pin` (>= bytes): the
// pool copies piece_bytes() pieces into `pin` and each piece is DMA'd on `s` as
// soon as it is staged, so the host copy and the PCIe transfer overlap.
// The caller makes sure no earlier transfer still reads `pin`.
inline hipError_t upload_via(void* dev, const uint8_t* host, size_t bytes, uint8_t* pin, hipStream_t s) {
    const size_t kPieceBytes = piece_bytes(bytes);
    const size_t n = (bytes + kPieceBytes - 1) / kPieceBytes;
    std::atomic<int> err{(int)hipSuccess};
    CopyPool::global().run(n, [&](size_t i) {
        const size_t o = i * kPieceBytes, len = std::min(kPieceBytes, bytes - o);
        host_copy(pin + o, host + o, len);
        const hipError_t e = hipMemcpyAsync(static_cast<uint8_t*>(dev) + o, pin + o, len, hipMemcpyHostToDevice, s);
        if (e != hipSuccess) err.store((int)e);
    }, true);
    return (hipError_t)err.load();
}

// Events marking the completion of each piece of a download.
struct PieceEvents {
    std::vector<hipEvent_t> ev;
    hipError_t ensure(size_t n) {
        while (ev.size() < n) {
            hipEvent_t e = nullptr;
            const hipError_t r = hipEventCreateWithFlags(&e, hipEventDisableTiming);
            if (r != hipSuccess) return r;
            ev.push_back(e);
        }
        return hipSuccess;
    }
    void release() {
        for (auto e : ev) (void)hipEventDestroy(e);
        ev.clear();
    }
};

// One frame device -> host through `pin` (>= bytes): the pieces are DMA'd
// in order on `s` (after the work already queued there) and the pool copies
// each one out as soon as its DMA has landed.  Returns when `host` holds
// the whole frame.
inline hipError_t download_via(uint8_t* host, const void* dev, size_t bytes, uint8_t* pin, hipStream_t s,
                               PieceEvents& pe) {
    const size_t kPieceBytes = piece_bytes(bytes);
    const size_t n = (bytes + kPieceBytes - 1) / kPieceBytes;
    hipError_t e = pe.ensure(n);
    if (e != hipSuccess) return e;
    for (size_t i = 0; i < n; ++i) {
        const size_t o = i * kPieceBytes, len = std::min(kPieceBytes, bytes - o);
        if ((e = hipMemcpyAsync(pin + o, static_cast<const uint8_t*>(dev) + o, len, hipMemcpyDeviceToHost, s)) !=
            hipSuccess)
            return e;
        if ((e = hipEventRecord(pe.ev[i], s)) != hipSuccess) return e;
    }
    std::atomic<int> err{(int)hipSuccess};
    CopyPool::global().run(n, [&](size_t i) {
        const hipError_t r = hipEventSynchronize(pe.ev[i]);
        if (r != hipSuccess) {
            err.store((int)r);
            return;
        }
        const size_t o = i * kPieceBytes;
        host_copy(host + o, pin + o, std::min(kPieceBytes, bytes - o));
    }, true);
    return (hipError_t)err.load();
}

// Byte pieces per stripe of the zero-copy pipeline (run_striped_frame_direct).
constexpr uint32_t kDirectSplit = 8u;

// Rows of the first stripe: a quarter stripe, so that the first kernel (whose
// PCIe reads and writes do not overlap another kernel's) starts and lands
// early.
inline uint32_t direct_first_rows(uint32_t rows) { return std::max(1u, rows / 4u); }

// Staging of one piece [o, o + len) of the RGBA8 frame: copied as it is
// (in_bytes 0) or packed into the kernel's input form at pin_in + o / 4 *
// in_bytes (in_bytes 1 / 2 per pixel: pack_frame, chroma channel ch)
inline void stage_piece(uint8_t* pin_in, const uint8_t* frame, size_t o, size_t len, int in_bytes, int ch) {
    if (!len) return;
    if (in_bytes)
        pack_frame(pin_in + o / 4u * (size_t)in_bytes, frame + o, len / 4u, in_bytes, ch, true);
    else
        host_copy(pin_in + o, frame + o, len);
}

// Where one per-frame call's time went (run_striped_frame_direct; the
// bench's per_frame_call record, dips_callback_phases).  Times in us from
// `t0` (the caller's start of the call); CPU sums over the pool's tasks.
struct CallPhases {
    double sync_us = 0;      // the start-of-call stream synchronisations (caller)
    double staged_us = 0;    // the last input piece staged (packed) into pinned memory
    double launched_us = 0;  // the last stripe's kernel launched
    double kernels_us = 0;   // the last copy-out task past its wait for its stripe's kernel
    double expand_us = 0;    // the first copy-out task started (all staging tasks taken: the
                             // pool's tasks run in order, staging first)
    double wall_us = 0;      // the call returned (caller)
    double pack_cpu_us = 0;  // sum over staging tasks
    double expand_cpu_us = 0;  // sum over copy-out tasks, excluding their waits
    double wait_cpu_us = 0;  // sum over copy-out tasks of the wait for their stripe's kernel
    double threads = 0;      // pool threads (workers + the caller)
    double stripes = 0;
};

// Copy-out of one piece [o, o + len) of the RGBA8 frame: from pin_out itself
// (key_bytes 0) or rebuilt from the per-pixel keys the kernel wrote there
// (key_bytes 1 / 2 per pixel, pin_out + o / 4 * key_bytes; expand_keys).
inline void copy_out_piece(uint8_t* out, const uint8_t* pin_out, size_t o, size_t len, int key_bytes) {
    if (!len) return;
    if (key_bytes)
        expand_keys(out + o, pin_out + o / 4u * (size_t)key_bytes, len / 4u, key_bytes, true);
    else
        host_copy(out + o, pin_out + o, len);
}

// Stripe / piece geometry of the zero-copy frame pipeline, fixed at staging
// time so that a later collect uses the same cut.
struct DirectGeom {
    uint32_t height = 0, rows = 1, first = 1, n_s = 0, k = kDirectSplit;
    size_t row = 0;
    void init(uint32_t h, size_t row_bytes) {
        height = h;
        row = row_bytes;
        rows = (uint32_t)std::max<size_t>(1, piece_bytes(row * h) / row);
        first = std::min(height, direct_first_rows(rows));
        n_s = 1u + (height - first + rows - 1) / rows;
        k = kDirectSplit;
    }
    uint32_t y0(uint32_t si) const { return si == 0 ? 0u : std::min(height, first + (si - 1) * rows); }
    uint32_t y1(uint32_t si) const { return si + 1 == n_s ? height : y0(si + 1); }
    // byte range [o, o + len) of piece j of stripe si (64-B aligned cuts)
    void piece(uint32_t si, uint32_t j, size_t& o, size_t& len) const {
        const size_t so = (size_t)y0(si) * row, slen = (size_t)(y1(si) - y0(si)) * row;
        const size_t p0 = std::min(slen, (slen * j / k) & ~(size_t)63);
        const size_t p1 = j + 1 == k ? slen : std::min(slen, (slen * (j + 1) / k) & ~(size_t)63);
        o = so + p0;
        len = p1 - p0;
    }
};

// One frame through a per-pixel kernel that reads its input from, and writes
// its output to, the pinned buffers themselves (zero-copy over PCIe, no DMA
// engine).  The frame is cut into row stripes of ~piece_bytes() (the first
// one a quarter of that) and each stripe into kDirectSplit byte pieces for
// the copy pool: the pool stages the pieces into `pin_in` in stripe order, the thread that stages a stripe's
// last piece launches launch(y0, y1, stream) for it (stripes in any order --
// rows are independent; even stripes on compute[0], odd ones on compute[1],
// so one stripe's PCIe reads run beside the previous one's writes), and the
// pieces of stripe s are copied from `pin_out` to `out` as soon as its
// kernel has finished.  Small pieces let several threads stage the first
// stripe and copy out the last one, the two exposed ends of the call.  The
// copy-out tasks come after every staging task and wait for their stripe's
// launch, so one worker or many run the same schedule.  The caller makes
// sure no earlier kernel still reads `pin_in` or writes `pin_out`.
template <typename Launch>
hipError_t run_striped_frame_direct(const uint8_t* frame, uint8_t* out, uint32_t height, size_t row,
                                    uint8_t* pin_in, const uint8_t* pin_out, const hipStream_t (&compute)[2],
                                    int device, PieceEvents& ev, Launch&& launch, int key_bytes = 0,
                                    int in_bytes = 0, int ch = 0, CallPhases* ph = nullptr,
                                    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now()) {
    DirectGeom g;
    g.init(height, row);
    const uint32_t n_s = g.n_s, k = g.k;
    const size_t n_t = (size_t)n_s * k;  // pieces per direction
    hipError_t e = ev.ensure(n_s);
    if (e != hipSuccess) return e;
    std::unique_ptr<std::atomic<int>[]> ready(new std::atomic<int>[n_s]);
    std::unique_ptr<std::atomic<uint32_t>[]> staged(new std::atomic<uint32_t>[n_s]);
    for (uint32_t i = 0; i < n_s; ++i) {
        ready[i].store(0, std::memory_order_relaxed);
        staged[i].store(0, std::memory_order_relaxed);
    }
    std::mutex launch_mu;
    std::atomic<int> err{(int)hipSuccess};
    using clk = std::chrono::steady_clock;
    // phase record: latest-event times as integer ns since t0 (atomic max),
    // CPU sums in ns
    std::atomic<int64_t> p_staged{0}, p_launched{0}, p_kernels{0}, p_pack{0}, p_expand{0}, p_wait{0};
    std::atomic<int64_t> p_exp0{INT64_MAX};
    auto ns_since_t0 = [&]() {
        return (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(clk::now() - t0).count();
    };
    auto amax = [](std::atomic<int64_t>& a, int64_t v) {
        int64_t cur = a.load(std::memory_order_relaxed);
        while (v > cur && !a.compare_exchange_weak(cur, v, std::memory_order_relaxed)) {
        }
    };
    CopyPool::global().run(2 * n_t, [&](size_t i) {
        const size_t pi = i < n_t ? i : i - n_t;
        const uint32_t si = (uint32_t)(pi / k), j = (uint32_t)(pi % k);
        size_t o, len;
        g.piece(si, j, o, len);
        if (i < n_t) {
            // a staging task that throws still releases its stripe's copy-out
            // tasks (they would wait for it forever); the pool rethrows
            try {
                const int64_t a0 = ph ? ns_since_t0() : 0;
                stage_piece(pin_in, frame, o, len, in_bytes, ch);
                if (ph) {
                    const int64_t a1 = ns_since_t0();
                    p_pack.fetch_add(a1 - a0, std::memory_order_relaxed);
                    amax(p_staged, a1);
                }
                if (staged[si].fetch_add(1, std::memory_order_acq_rel) + 1 != k) return;
                // the stripe's last piece: its kernel and event back to back on the stream
                hipError_t r;
                {
                    std::lock_guard<std::mutex> lk(launch_mu);
                    hipStream_t cs = compute[si & 1u];
                    r = hipSetDevice(device);
                    if (r == hipSuccess) r = launch(g.y0(si), g.y1(si), cs);
                    if (r == hipSuccess) r = hipEventRecord(ev.ev[si], cs);
                }
                if (r != hipSuccess) err.store((int)r);
                if (ph) amax(p_launched, ns_since_t0());
                ready[si].store(r == hipSuccess ? 1 : -1, std::memory_order_release);
            } catch (...) {
                ready[si].store(-1, std::memory_order_release);
                throw;
            }
            return;
        }
        const int64_t w0 = ph ? ns_since_t0() : 0;
        if (ph) {
            int64_t cur = p_exp0.load(std::memory_order_relaxed);
            while (w0 < cur && !p_exp0.compare_exchange_weak(cur, w0, std::memory_order_relaxed)) {
            }
        }
        int st;
        while ((st = ready[si].load(std::memory_order_acquire)) == 0) std::this_thread::yield();
        if (st < 0) return;
        const hipError_t r = hipEventSynchronize(ev.ev[si]);
        if (r != hipSuccess) {
            err.store((int)r);
            return;
        }
        const int64_t w1 = ph ? ns_since_t0() : 0;
        copy_out_piece(out, pin_out, o, len, key_bytes);
        if (ph) {
            p_wait.fetch_add(w1 - w0, std::memory_order_relaxed);
            p_expand.fetch_add(ns_since_t0() - w1, std::memory_order_relaxed);
            amax(p_kernels, w1);
        }
    }, true);
    if (ph) {
        ph->staged_us = p_staged.load() * 1e-3;
        ph->launched_us = p_launched.load() * 1e-3;
        ph->kernels_us = p_kernels.load() * 1e-3;
        ph->expand_us = p_exp0.load() == INT64_MAX ? 0.0 : p_exp0.load() * 1e-3;
        ph->pack_cpu_us = p_pack.load() * 1e-3;
        ph->expand_cpu_us = p_expand.load() * 1e-3;
        ph->wait_cpu_us = p_wait.load() * 1e-3;
        ph->threads = (double)CopyPool::global().threads();
        ph->stripes = (double)n_s;
    }
    return (hipError_t)err.load();
}

// First half of the zero-copy pipeline: the pool stages the frame's pieces
// into `pin_in` and the thread that stages a stripe's last piece launches
// launch(y0, y1, stream) for it and records the stripe's event (stripes
// alternating over compute[0] / compute[1]).  Returns when every stripe is
// staged and launched; the kernels may still run (and read `pin_in`).
template <typename Launch>
hipError_t direct_stage_launch(const uint8_t* frame, uint8_t* pin_in, const hipStream_t (&compute)[2], int device,
                               PieceEvents& ev, const DirectGeom& g, Launch&& launch, int in_bytes = 0, int ch = 0) {
    hipError_t e = ev.ensure(g.n_s);
    if (e != hipSuccess) return e;
    std::unique_ptr<std::atomic<uint32_t>[]> staged(new std::atomic<uint32_t>[g.n_s]);
    for (uint32_t i = 0; i < g.n_s; ++i) staged[i].store(0, std::memory_order_relaxed);
    std::mutex launch_mu;
    std::atomic<int> err{(int)hipSuccess};
    CopyPool::global().run((size_t)g.n_s * g.k, [&](size_t i) {
        const uint32_t si = (uint32_t)(i / g.k), j = (uint32_t)(i % g.k);
        size_t o, len;
        g.piece(si, j, o, len);
        stage_piece(pin_in, frame, o, len, in_bytes, ch);
        if (staged[si].fetch_add(1, std::memory_order_acq_rel) + 1 != g.k) return;
        std::lock_guard<std::mutex> lk(launch_mu);
        hipStream_t cs = compute[si & 1u];
        hipError_t r = hipSetDevice(device);
        if (r == hipSuccess) r = launch(g.y0(si), g.y1(si), cs);
        if (r == hipSuccess) r = hipEventRecord(ev.ev[si], cs);
        if (r != hipSuccess) err.store((int)r);
    }, true);
    return (hipError_t)err.load();
}

// Second half: the pool copies each stripe's pieces from `pin_out` to `out`
// as soon as the stripe's event (recorded by direct_stage_launch) has fired.
inline hipError_t direct_collect(uint8_t* out, const uint8_t* pin_out, PieceEvents& ev, const DirectGeom& g,
                                 int key_bytes = 0) {
    std::atomic<int> err{(int)hipSuccess};
    CopyPool::global().run((size_t)g.n_s * g.k, [&](size_t i) {
        const uint32_t si = (uint32_t)(i / g.k), j = (uint32_t)(i % g.k);
        const hipError_t r = hipEventSynchronize(ev.ev[si]);
        if (r != hipSuccess) {
            err.store((int)r);
            return;
        }
        size_t o, len;
        g.piece(si, j, o, len);
        copy_out_piece(out, pin_out, o, len, key_bytes);
    }, true);
    return (hipError_t)err.load();
}

// Frames per pipelined chunk of an n-frame batch: ~256 MiB (two chunks in
// flight per direction keep both PCIe directions and the kernel busy), and
// at most a quarter of the batch, so that a small batch still overlaps its
// transfers with the kernels.
inline uint64_t feed_chunk_frames(size_t frame_bytes, uint64_t n_frames) {
    const uint64_t budget = (256ull << 20) / (frame_bytes ? frame_bytes : 1);
    const uint64_t quarter = (n_frames + 3u) / 4u;
    return std::max<uint64_t>(1u, std::min(budget, quarter));
}

struct StreamPipe {
    HostPinned pin_in[2], pin_out[2];
    DevBuf dev_in[2], dev_out[2];
    hipStream_t up = nullptr, down = nullptr;
    hipEvent_t uploaded[2] = {nullptr, nullptr}, computed[2] = {nullptr, nullptr},
               downloaded[2] = {nullptr, nullptr};

    hipError_t init() {
        if (up) return hipSuccess;
        hipError_t e = hipStreamCreateWithFlags(&up, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&down, hipStreamNonBlocking);
        for (int i = 0; i < 2 && e == hipSuccess; ++i) {
            e = hipEventCreateWithFlags(&uploaded[i], hipEventDisableTiming);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&computed[i], hipEventDisableTiming);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&downloaded[i], hipEventDisableTiming);
        }
        return e;
    }
    void release() {
        if (up) (void)hipStreamSynchronize(up);
        if (down) (void)hipStreamSynchronize(down);
        for (int i = 0; i < 2; ++i) {
            pin_in[i].release();
            pin_out[i].release();
            dev_in[i].release();
            dev_out[i].release();
            if (uploaded[i]) (void)hipEventDestroy(uploaded[i]);
            if (computed[i]) (void)hipEventDestroy(computed[i]);
            if (downloaded[i]) (void)hipEventDestroy(downloaded[i]);
            uploaded[i] = computed[i] = downloaded[i] = nullptr;
        }
        if (up) (void)hipStreamDestroy(up);
        if (down) (void)hipStreamDestroy(down);
        up = down = nullptr;
    }
};

// Process n items of `ib` input and `ob` output bytes each from host `in` to
// host `out`, `chunk` items at a time: fn(dev_in, dev_out, count) enqueues the
// compute of one chunk on `compute` (chunks in order) and returns 0 or a
// negative status.  Returns hipSuccess, or the first HIP error (*fn_status
// receives a negative fn result).
template <typename Fn>
hipError_t run_stream_pipe(StreamPipe& p, hipStream_t compute, uint64_t n, size_t ib, size_t ob, uint64_t chunk,
                           const uint8_t* in, uint8_t* out, Fn&& fn, int* fn_status) {
    *fn_status = 0;
    hipError_t e = p.init();
    if (e != hipSuccess) return e;
    // a previous call that ended early (HIP error, negative fn status) may
    // have left DMAs in flight that read pin_in / write pin_out: drain both
    // copy streams before the staging buffers are reused
    if ((e = hipStreamSynchronize(p.up)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(p.down)) != hipSuccess) return e;
    if (chunk == 0 || chunk > n) chunk = n;
    for (int i = 0; i < 2; ++i) {
        if ((e = p.pin_in[i].ensure(ib * chunk)) != hipSuccess) return e;
        if ((e = p.pin_out[i].ensure(ob * chunk)) != hipSuccess) return e;
        if ((e = p.dev_in[i].ensure(ib * chunk)) != hipSuccess) return e;
        if ((e = p.dev_out[i].ensure(ob * chunk)) != hipSuccess) return e;
    }
    const uint64_t n_chunks = (n + chunk - 1) / chunk;
    auto count_of = [&](uint64_t k) { return (k + 1) * chunk <= n ? chunk : n - k * chunk; };
    for (uint64_t k = 0; k <= n_chunks; ++k) {
        if (k < n_chunks) {
            const int b = (int)(k & 1u);
            const uint64_t m = count_of(k);
            // pin_in[b] and dev_in[b] were last used by chunk k-2
            if (k >= 2 && (e = hipEventSynchronize(p.uploaded[b])) != hipSuccess) return e;
            staged_copy(p.pin_in[b].bytes(), in + k * chunk * ib, m * ib);
            if (k >= 2 && (e = hipStreamWaitEvent(p.up, p.computed[b], 0)) != hipSuccess) return e;
            if ((e = pipe_h2d(p.dev_in[b].p, p.pin_in[b].p, m * ib, p.up)) != hipSuccess)
                return e;
            if ((e = hipEventRecord(p.uploaded[b], p.up)) != hipSuccess) return e;
            // dev_out[b] was last read by chunk k-2's download
            if ((e = hipStreamWaitEvent(compute, p.uploaded[b], 0)) != hipSuccess) return e;
            if (k >= 2 && (e = hipStreamWaitEvent(compute, p.downloaded[b], 0)) != hipSuccess) return e;
            const int st = fn(p.dev_in[b].template as<uint8_t>(), p.dev_out[b].template as<uint8_t>(), m);
            if (st < 0) {
                *fn_status = st;
                // leave no DMA running on the staging buffers
                (void)hipStreamSynchronize(p.up);
                (void)hipStreamSynchronize(p.down);
                return hipSuccess;
            }
            if ((e = hipEventRecord(p.computed[b], compute)) != hipSuccess) return e;
            if ((e = hipStreamWaitEvent(p.down, p.computed[b], 0)) != hipSuccess) return e;
            if ((e = pipe_d2h(p.pin_out[b].p, p.dev_out[b].p, m * ob, p.down)) != hipSuccess)
                return e;
            if ((e = hipEventRecord(p.downloaded[b], p.down)) != hipSuccess) return e;
        }
        if (k >= 1) {  // chunk k-1's results to the caller while chunk k runs
            const int b = (int)((k - 1) & 1u);
            if ((e = hipEventSynchronize(p.downloaded[b])) != hipSuccess) return e;
            staged_copy(out + (k - 1) * chunk * ob, p.pin_out[b].bytes(), count_of(k - 1) * ob);
        }
    }
    return hipSuccess;
}

}  // namespace dips_host
