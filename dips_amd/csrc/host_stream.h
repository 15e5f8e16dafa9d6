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
// (a DMA engine).  Measured in one process (tools/nt_copy_ab.py --var
// DIPS_PIPE_KERNEL_COPY): the streamed series' uploads by kernel ran 1.00-1.15x
// the DMA rate (the kernel default there), the visual operators' two-way
// pipe 0.81-0.82x with a kernel upload (DMA kept).  DIPS_PIPE_KERNEL_COPY
// overrides every call site: "1" kernels both ways, "0" DMA both ways, "h" /
// "d" a kernel for host->device / device->host only.  Read per call.
inline bool pipe_kernel_copy(bool to_host, bool dflt) {
    const char* e = std::getenv("DIPS_PIPE_KERNEL_COPY");
    if (!e || !e[0]) return dflt;
    const char c = e[0];
    return c == '1' || (c == 'h' && !to_host) || (c == 'd' && to_host);
}
inline hipError_t pipe_h2d(void* dev, const void* pin, size_t bytes, hipStream_t s, bool kernel_default = false) {
    if (pipe_kernel_copy(false, kernel_default) && bytes % 4u == 0) {
        void* pd = nullptr;
        const hipError_t e = hipHostGetDevicePointer(&pd, const_cast<void*>(pin), 0);
        if (e != hipSuccess) return e;
        return dips::launch_copy_from_host(static_cast<const uint8_t*>(pd), static_cast<uint8_t*>(dev), bytes, s);
    }
    return hipMemcpyAsync(dev, pin, bytes, hipMemcpyHostToDevice, s);
}
inline hipError_t pipe_d2h(void* pin, const void* dev, size_t bytes, hipStream_t s, bool kernel_default = false) {
    if (pipe_kernel_copy(true, kernel_default) && bytes % 4u == 0) {
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
// frame_callback); DIPS_PIECE_BYTES overrides it.
inline size_t piece_bytes() {
    if (const char* e = std::getenv("DIPS_PIECE_BYTES")) {
        const unsigned long long b = std::strtoull(e, nullptr, 10);
        if (b >= 64) return (size_t)b;
    }
    return (size_t)4u << 20;
}

// One frame host -> device through the pinned buffer `pin` (>= bytes): the
// pool copies ~2 MiB pieces into `pin` and each piece is DMA'd on `s` as
// soon as it is staged, so the host copy and the PCIe transfer overlap.
// The caller makes sure no earlier transfer still reads `pin`.
inline hipError_t upload_via(void* dev, const uint8_t* host, size_t bytes, uint8_t* pin, hipStream_t s) {
    const bool nt = nt_copy();  // on the calling thread, never in the workers
    const size_t kPieceBytes = piece_bytes();
    const size_t n = (bytes + kPieceBytes - 1) / kPieceBytes;
    std::atomic<int> err{(int)hipSuccess};
    CopyPool::global().run(n, [&](size_t i) {
        const size_t o = i * kPieceBytes, len = std::min(kPieceBytes, bytes - o);
        host_copy(pin + o, host + o, len, nt);
        const hipError_t e = hipMemcpyAsync(static_cast<uint8_t*>(dev) + o, pin + o, len, hipMemcpyHostToDevice, s);
        if (e != hipSuccess) err.store((int)e);
    });
    return (hipError_t)err.load();
}

// The per-frame pipelines' waiting threads sleep instead of spinning
// (DIPS_CB_BLOCKING=1: blocking-sync stripe events and a condition variable
// for the stripe launches; A/B runs, tools/pfc_threads_ab.py).  Read when an
// event set is created and per call.
inline bool cb_blocking() {
    const char* e = std::getenv("DIPS_CB_BLOCKING");
    return e && e[0] == '1';
}

// Events marking the completion of each piece of a download.
struct PieceEvents {
    std::vector<hipEvent_t> ev;
    hipError_t ensure(size_t n) {
        const unsigned flags = hipEventDisableTiming | (cb_blocking() ? hipEventBlockingSync : 0u);
        while (ev.size() < n) {
            hipEvent_t e = nullptr;
            const hipError_t r = hipEventCreateWithFlags(&e, flags);
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
    const bool nt = nt_copy();  // on the calling thread, never in the workers
    const size_t kPieceBytes = piece_bytes();
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
        host_copy(host + o, pin + o, std::min(kPieceBytes, bytes - o), nt);
    });
    return (hipError_t)err.load();
}

// One frame through a per-pixel kernel in row stripes, both PCIe directions
// at once: stripe s is staged by the copy pool and DMA'd into `dev_in` on
// `up`; `launch(y0, y1)` enqueues the kernel of rows [y0, y1) on `compute`
// once that stripe has landed; the stripe of `dev_out` then comes back on
// `compute` and the pool copies it out as soon as its event fires.  The
// caller makes sure both streams are idle and `pin_in` / `pin_out` (frame
// size each) are free.
template <typename Launch>
hipError_t run_striped_frame(const uint8_t* frame, uint8_t* out, uint32_t height, size_t row, uint8_t* pin_in,
                             uint8_t* pin_out, uint8_t* dev_in, const uint8_t* dev_out, hipStream_t up,
                             hipStream_t compute, PieceEvents& up_ev, PieceEvents& down_ev, Launch&& launch) {
    const bool nt = nt_copy();  // on the calling thread, never in the workers
    const size_t fb = row * height;
    const uint32_t rows = (uint32_t)std::max<size_t>(1, piece_bytes() / row);
    const uint32_t n_s = (height + rows - 1) / rows;
    hipError_t e = up_ev.ensure(n_s);
    if (e == hipSuccess) e = down_ev.ensure(n_s);
    if (e != hipSuccess) return e;
    // DIPS_STRIPE_TRACE: per call, the host time (us from entry) at which each
    // stripe was staged / its DMA enqueued, the kernels enqueued, each
    // readback landed and was copied out (tools/nt_copy_ab.py --trace)
    static const bool trace = std::getenv("DIPS_STRIPE_TRACE") != nullptr;
    using clk = std::chrono::steady_clock;
    const auto tbeg = clk::now();
    std::vector<double> ts(trace ? 4 * n_s : 0);
    auto since = [&]() { return std::chrono::duration<double, std::micro>(clk::now() - tbeg).count(); };
    std::atomic<int> err{(int)hipSuccess};
    CopyPool::global().run(n_s, [&](size_t si) {
        const size_t o = si * rows * row, len = std::min<size_t>((size_t)rows * row, fb - o);
        host_copy(pin_in + o, frame + o, len, nt);
        if (trace) ts[4 * si] = since();
        hipError_t r = hipMemcpyAsync(dev_in + o, pin_in + o, len, hipMemcpyHostToDevice, up);
        if (r == hipSuccess) r = hipEventRecord(up_ev.ev[si], up);
        if (r != hipSuccess) err.store((int)r);
        if (trace) ts[4 * si + 1] = since();
    });
    if ((e = (hipError_t)err.load()) != hipSuccess) return e;
    for (uint32_t si = 0; si < n_s; ++si) {
        const uint32_t y0 = si * rows, y1 = std::min(height, y0 + rows);
        const size_t o = (size_t)y0 * row, len = (size_t)(y1 - y0) * row;
        if ((e = hipStreamWaitEvent(compute, up_ev.ev[si], 0)) != hipSuccess) return e;
        if ((e = launch(y0, y1)) != hipSuccess) return e;
        if ((e = hipMemcpyAsync(pin_out + o, dev_out + o, len, hipMemcpyDeviceToHost, compute)) != hipSuccess)
            return e;
        if ((e = hipEventRecord(down_ev.ev[si], compute)) != hipSuccess) return e;
    }
    const double t_enq = trace ? since() : 0.0;
    CopyPool::global().run(n_s, [&](size_t si) {
        const hipError_t r = hipEventSynchronize(down_ev.ev[si]);
        if (r != hipSuccess) {
            err.store((int)r);
            return;
        }
        if (trace) ts[4 * si + 2] = since();
        const size_t o = si * rows * row;
        host_copy(out + o, pin_out + o, std::min<size_t>((size_t)rows * row, fb - o), nt);
        if (trace) ts[4 * si + 3] = since();
    });
    if (trace) {
        std::fprintf(stderr, "stripes %u enqueued %.0f us:", n_s, t_enq);
        for (uint32_t si = 0; si < n_s; ++si)
            std::fprintf(stderr, " [%.0f %.0f %.0f %.0f]", ts[4 * si], ts[4 * si + 1], ts[4 * si + 2], ts[4 * si + 3]);
        std::fprintf(stderr, " end %.0f\n", since());
    }
    return (hipError_t)err.load();
}

// One frame through a per-pixel kernel that reads its input from, and writes
// its output to, the pinned buffers themselves (zero-copy over PCIe, no DMA
// engine).  The frame is cut into row stripes of ~piece_bytes() (the first
// one a quarter of that) and each stripe into `split` byte pieces for the
// copy pool: the pool stages the
// pieces into `pin_in` in stripe order, the thread that stages a stripe's
// last piece launches launch(y0, y1, stream) for it (stripes in any order --
// rows are independent; even stripes on compute[0], odd ones on compute[1],
// so one stripe's PCIe reads run beside the previous one's writes), and the
// pieces of stripe s are copied from `pin_out` to `out` as soon as its
// kernel has finished.  Small pieces let several threads stage the first
// stripe and copy out the last one, the two exposed ends of the call.  The
// copy-out tasks come after every staging task and wait for their stripe's
// launch, so one worker or many run the same schedule.  The caller makes
// sure no earlier kernel still reads `pin_in` or writes `pin_out`.
inline uint32_t direct_split() {
    if (const char* e = std::getenv("DIPS_DIRECT_SPLIT")) {
        const long v = std::strtol(e, nullptr, 10);
        if (v >= 1 && v <= 64) return (uint32_t)v;
    }
    return 8u;
}

// Rows of the first stripe: a quarter stripe, so that the first kernel (whose
// PCIe reads and writes do not overlap another kernel's) starts and lands
// early; DIPS_DIRECT_FIRST=0 makes it a full stripe.
inline uint32_t direct_first_rows(uint32_t rows) {
    const char* e = std::getenv("DIPS_DIRECT_FIRST");
    if (e && e[0] == '0') return rows;
    return std::max(1u, rows / 4u);
}

// copy-out of one piece [o, o + len) of the RGBA8 frame: from pin_out itself
// (key_bytes 0) or rebuilt from the per-pixel keys the kernel wrote there
// (key_bytes 1 / 2 per pixel, pin_out + o / 4 * key_bytes; expand_keys).
// staging of one piece [o, o + len) of the RGBA8 frame: copied as it is
// (in_bytes 0) or packed into the kernel's input form at pin_in + o / 4 *
// in_bytes (in_bytes 1 / 2 per pixel: pack_frame, chroma channel ch)
inline void stage_piece(uint8_t* pin_in, const uint8_t* frame, size_t o, size_t len, int in_bytes, int ch, bool nt) {
    if (!len) return;
    if (in_bytes)
        pack_frame(pin_in + o / 4u * (size_t)in_bytes, frame + o, len / 4u, in_bytes, ch, nt);
    else
        host_copy(pin_in + o, frame + o, len, nt);
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

inline void copy_out_piece(uint8_t* out, const uint8_t* pin_out, size_t o, size_t len, int key_bytes, bool nt) {
    if (!len) return;
    if (key_bytes)
        expand_keys(out + o, pin_out + o / 4u * (size_t)key_bytes, len / 4u, key_bytes, nt);
    else
        host_copy(out + o, pin_out + o, len, nt);
}

template <typename Launch>
hipError_t run_striped_frame_direct(const uint8_t* frame, uint8_t* out, uint32_t height, size_t row,
                                    uint8_t* pin_in, const uint8_t* pin_out, const hipStream_t (&compute)[2],
                                    int device, PieceEvents& ev, Launch&& launch, int key_bytes = 0,
                                    int in_bytes = 0, int ch = 0, CallPhases* ph = nullptr,
                                    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now()) {
    const bool nt = nt_copy();  // on the calling thread, never in the workers
    const uint32_t rows = (uint32_t)std::max<size_t>(1, piece_bytes() / row);
    const uint32_t first = std::min(height, direct_first_rows(rows));
    const uint32_t n_s = 1u + (height - first + rows - 1) / rows;
    auto stripe_y0 = [&](uint32_t si) { return si == 0 ? 0u : std::min(height, first + (si - 1) * rows); };
    const uint32_t k = direct_split();
    const size_t n_t = (size_t)n_s * k;  // pieces per direction
    hipError_t e = ev.ensure(n_s);
    if (e != hipSuccess) return e;
    std::unique_ptr<std::atomic<int>[]> ready(new std::atomic<int>[n_s]);
    std::unique_ptr<std::atomic<uint32_t>[]> staged(new std::atomic<uint32_t>[n_s]);
    for (uint32_t i = 0; i < n_s; ++i) {
        ready[i].store(0, std::memory_order_relaxed);
        staged[i].store(0, std::memory_order_relaxed);
    }
    std::mutex launch_mu, ready_mu;
    std::condition_variable ready_cv;
    const bool blocking = cb_blocking();
    std::atomic<int> err{(int)hipSuccess};
    static const bool trace = std::getenv("DIPS_STRIPE_TRACE") != nullptr;
    using clk = std::chrono::steady_clock;
    const auto tbeg = clk::now();
    std::vector<double> ts(trace ? 2 * n_s + n_t : 0);
    auto since = [&]() { return std::chrono::duration<double, std::micro>(clk::now() - tbeg).count(); };
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
        const uint32_t y0 = stripe_y0(si), y1 = si + 1 == n_s ? height : stripe_y0(si + 1);
        const size_t so = (size_t)y0 * row, slen = (size_t)(y1 - y0) * row;
        // piece j of the stripe: 64-B aligned cut points
        const size_t p0 = std::min(slen, (slen * j / k) & ~(size_t)63);
        const size_t p1 = j + 1 == k ? slen : std::min(slen, (slen * (j + 1) / k) & ~(size_t)63);
        const size_t o = so + p0, len = p1 - p0;
        if (i < n_t) {
            const int64_t a0 = ph ? ns_since_t0() : 0;
            if (frame) stage_piece(pin_in, frame, o, len, in_bytes, ch, nt);  // frame == nullptr: already staged
            if (ph) {
                const int64_t a1 = ns_since_t0();
                p_pack.fetch_add(a1 - a0, std::memory_order_relaxed);
                amax(p_staged, a1);
            }
            if (staged[si].fetch_add(1, std::memory_order_acq_rel) + 1 != k) return;
            // the stripe's last piece: its kernel and event back to back on the stream
            if (trace) ts[2 * si] = since();
            hipError_t r;
            {
                std::lock_guard<std::mutex> lk(launch_mu);
                hipStream_t cs = compute[si & 1u];
                r = hipSetDevice(device);
                if (r == hipSuccess) r = launch(y0, y1, cs);
                if (r == hipSuccess) r = hipEventRecord(ev.ev[si], cs);
            }
            if (r != hipSuccess) err.store((int)r);
            if (trace) ts[2 * si + 1] = since();
            if (ph) amax(p_launched, ns_since_t0());
            ready[si].store(r == hipSuccess ? 1 : -1, std::memory_order_release);
            if (blocking) {
                std::lock_guard<std::mutex> lk(ready_mu);
                ready_cv.notify_all();
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
        if (blocking) {
            std::unique_lock<std::mutex> lk(ready_mu);
            ready_cv.wait(lk, [&]() { return ready[si].load(std::memory_order_acquire) != 0; });
            st = ready[si].load(std::memory_order_acquire);
        } else {
            while ((st = ready[si].load(std::memory_order_acquire)) == 0) std::this_thread::yield();
        }
        if (st < 0) return;
        const hipError_t r = hipEventSynchronize(ev.ev[si]);
        if (r != hipSuccess) {
            err.store((int)r);
            return;
        }
        const int64_t w1 = ph ? ns_since_t0() : 0;
        copy_out_piece(out, pin_out, o, len, key_bytes, nt);
        if (ph) {
            p_wait.fetch_add(w1 - w0, std::memory_order_relaxed);
            p_expand.fetch_add(ns_since_t0() - w1, std::memory_order_relaxed);
            amax(p_kernels, w1);
        }
        if (trace) ts[2 * n_s + pi] = since();
    });
    if (trace) {
        std::fprintf(stderr, "direct stripes %u x %u pieces: [staged launched copied-out]", n_s, k);
        for (uint32_t si = 0; si < n_s; ++si) {
            double done = 0.0;
            for (uint32_t j = 0; j < k; ++j) done = std::max(done, ts[2 * n_s + (size_t)si * k + j]);
            std::fprintf(stderr, " [%.0f %.0f %.0f]", ts[2 * si], ts[2 * si + 1], done);
        }
        std::fprintf(stderr, " end %.0f\n", since());
    }
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

// The per-frame call through the DMA engines with the compact forms: the
// pool packs each piece of a stripe into `pin_in` (pack_frame: IN bytes per
// pixel), the thread that stages a stripe's last piece enqueues its H2D copy
// into `dev_in` on `up` and, on `compute` behind that copy, the stripe's
// kernel (launch(y0, y1, compute): dev_in -> dev_out keys in HBM) and the D2H
// copy of its keys into `pin_out`; the copy-out tasks expand each stripe's
// keys into `out` once its event fires.  Against the zero-copy form the
// PCIe transfers are done by the copy engines at their full rate (the
// kernels' system-scope loads of pinned memory reached ~31 GB/s) and the
// kernels touch only HBM.  Same pieces, phases and error handling as
// run_striped_frame_direct; the caller makes sure both streams are idle and
// the four buffers free.
template <typename Launch>
hipError_t run_striped_frame_dma_keys(const uint8_t* frame, uint8_t* out, uint32_t height, size_t row,
                                      uint8_t* pin_in, const uint8_t* pin_out, uint8_t* dev_in, uint8_t* dev_out,
                                      hipStream_t up, hipStream_t compute, int device, PieceEvents& up_ev,
                                      PieceEvents& ev, Launch&& launch, int key_bytes, int in_bytes, int ch,
                                      CallPhases* ph = nullptr,
                                      std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now()) {
    const bool nt = nt_copy();  // on the calling thread, never in the workers
    const uint32_t rows = (uint32_t)std::max<size_t>(1, piece_bytes() / row);
    const uint32_t first = std::min(height, direct_first_rows(rows));
    const uint32_t n_s = 1u + (height - first + rows - 1) / rows;
    auto stripe_y0 = [&](uint32_t si) { return si == 0 ? 0u : std::min(height, first + (si - 1) * rows); };
    const uint32_t k = direct_split();
    const size_t n_t = (size_t)n_s * k;
    hipError_t e = ev.ensure(n_s);
    if (e == hipSuccess) e = up_ev.ensure(n_s);
    if (e != hipSuccess) return e;
    std::unique_ptr<std::atomic<int>[]> ready(new std::atomic<int>[n_s]);
    std::unique_ptr<std::atomic<uint32_t>[]> staged(new std::atomic<uint32_t>[n_s]);
    for (uint32_t i = 0; i < n_s; ++i) {
        ready[i].store(0, std::memory_order_relaxed);
        staged[i].store(0, std::memory_order_relaxed);
    }
    std::mutex launch_mu, ready_mu;
    std::condition_variable ready_cv;
    const bool blocking = cb_blocking();
    std::atomic<int> err{(int)hipSuccess};
    using clk = std::chrono::steady_clock;
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
    const size_t ib = (size_t)in_bytes, kb = (size_t)key_bytes;
    CopyPool::global().run(2 * n_t, [&](size_t i) {
        const size_t pi = i < n_t ? i : i - n_t;
        const uint32_t si = (uint32_t)(pi / k), j = (uint32_t)(pi % k);
        const uint32_t y0 = stripe_y0(si), y1 = si + 1 == n_s ? height : stripe_y0(si + 1);
        const size_t so = (size_t)y0 * row, slen = (size_t)(y1 - y0) * row;
        const size_t p0 = std::min(slen, (slen * j / k) & ~(size_t)63);
        const size_t p1 = j + 1 == k ? slen : std::min(slen, (slen * (j + 1) / k) & ~(size_t)63);
        const size_t o = so + p0, len = p1 - p0;
        if (i < n_t) {
            const int64_t a0 = ph ? ns_since_t0() : 0;
            stage_piece(pin_in, frame, o, len, in_bytes, ch, nt);
            if (ph) {
                const int64_t a1 = ns_since_t0();
                p_pack.fetch_add(a1 - a0, std::memory_order_relaxed);
                amax(p_staged, a1);
            }
            if (staged[si].fetch_add(1, std::memory_order_acq_rel) + 1 != k) return;
            hipError_t r;
            {
                std::lock_guard<std::mutex> lk(launch_mu);
                const size_t io = so / 4u * ib, il = slen / 4u * ib;
                const size_t oo = so / 4u * kb, ol = slen / 4u * kb;
                r = hipSetDevice(device);
                if (r == hipSuccess) r = hipMemcpyAsync(dev_in + io, pin_in + io, il, hipMemcpyHostToDevice, up);
                if (r == hipSuccess) r = hipEventRecord(up_ev.ev[si], up);
                if (r == hipSuccess) r = hipStreamWaitEvent(compute, up_ev.ev[si], 0);
                if (r == hipSuccess) r = launch(y0, y1, compute);
                if (r == hipSuccess)
                    r = hipMemcpyAsync(const_cast<uint8_t*>(pin_out) + oo, dev_out + oo, ol, hipMemcpyDeviceToHost,
                                       compute);
                if (r == hipSuccess) r = hipEventRecord(ev.ev[si], compute);
            }
            if (r != hipSuccess) err.store((int)r);
            if (ph) amax(p_launched, ns_since_t0());
            ready[si].store(r == hipSuccess ? 1 : -1, std::memory_order_release);
            if (blocking) {
                std::lock_guard<std::mutex> lk(ready_mu);
                ready_cv.notify_all();
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
        if (blocking) {
            std::unique_lock<std::mutex> lk(ready_mu);
            ready_cv.wait(lk, [&]() { return ready[si].load(std::memory_order_acquire) != 0; });
            st = ready[si].load(std::memory_order_acquire);
        } else {
            while ((st = ready[si].load(std::memory_order_acquire)) == 0) std::this_thread::yield();
        }
        if (st < 0) return;
        const hipError_t r = hipEventSynchronize(ev.ev[si]);
        if (r != hipSuccess) {
            err.store((int)r);
            return;
        }
        const int64_t w1 = ph ? ns_since_t0() : 0;
        copy_out_piece(out, pin_out, o, len, key_bytes, nt);
        if (ph) {
            p_wait.fetch_add(w1 - w0, std::memory_order_relaxed);
            p_expand.fetch_add(ns_since_t0() - w1, std::memory_order_relaxed);
            amax(p_kernels, w1);
        }
    });
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

// Stripe / piece geometry of the zero-copy frame pipeline (as in
// run_striped_frame_direct), fixed at staging time so that a later collect
// uses the same cut.
struct DirectGeom {
    uint32_t height = 0, rows = 1, first = 1, n_s = 0, k = 1;
    size_t row = 0;
    void init(uint32_t h, size_t row_bytes) {
        height = h;
        row = row_bytes;
        rows = (uint32_t)std::max<size_t>(1, piece_bytes() / row);
        first = std::min(height, direct_first_rows(rows));
        n_s = 1u + (height - first + rows - 1) / rows;
        k = direct_split();
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

// First half of the zero-copy pipeline: the pool stages the frame's pieces
// into `pin_in` and the thread that stages a stripe's last piece launches
// launch(y0, y1, stream) for it and records the stripe's event (stripes
// alternating over compute[0] / compute[1]).  Returns when every stripe is
// staged and launched; the kernels may still run (and read `pin_in`).
template <typename Launch>
hipError_t direct_stage_launch(const uint8_t* frame, uint8_t* pin_in, const hipStream_t (&compute)[2], int device,
                               PieceEvents& ev, const DirectGeom& g, Launch&& launch, int in_bytes = 0, int ch = 0) {
    const bool nt = nt_copy();  // on the calling thread, never in the workers
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
        stage_piece(pin_in, frame, o, len, in_bytes, ch, nt);
        if (staged[si].fetch_add(1, std::memory_order_acq_rel) + 1 != g.k) return;
        std::lock_guard<std::mutex> lk(launch_mu);
        hipStream_t cs = compute[si & 1u];
        hipError_t r = hipSetDevice(device);
        if (r == hipSuccess) r = launch(g.y0(si), g.y1(si), cs);
        if (r == hipSuccess) r = hipEventRecord(ev.ev[si], cs);
        if (r != hipSuccess) err.store((int)r);
    });
    return (hipError_t)err.load();
}

// Second half: the pool copies each stripe's pieces from `pin_out` to `out`
// as soon as the stripe's event (recorded by direct_stage_launch) has fired.
inline hipError_t direct_collect(uint8_t* out, const uint8_t* pin_out, PieceEvents& ev, const DirectGeom& g,
                                 int key_bytes = 0) {
    const bool nt = nt_copy();  // on the calling thread, never in the workers
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
        copy_out_piece(out, pin_out, o, len, key_bytes, nt);
    });
    return (hipError_t)err.load();
}

// Frames per pipelined chunk: ~256 MiB (two chunks in flight per direction
// keep both PCIe directions and the kernel busy); DIPS_FEED_CHUNK_BYTES
// overrides the byte budget (the tests use it to force many ragged chunks
// at small frame sizes).
inline uint64_t feed_chunk_frames(size_t frame_bytes) {
    uint64_t budget = 256ull << 20;
    if (const char* e = std::getenv("DIPS_FEED_CHUNK_BYTES")) {
        const unsigned long long v = std::strtoull(e, nullptr, 10);
        if (v > 0) budget = v;
    }
    const uint64_t n = budget / (frame_bytes ? frame_bytes : 1);
    return n ? n : 1;
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
    static const bool trace = std::getenv("DIPS_PIPE_TRACE") != nullptr;
    using clk = std::chrono::steady_clock;
    auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    auto count_of = [&](uint64_t k) { return (k + 1) * chunk <= n ? chunk : n - k * chunk; };
    for (uint64_t k = 0; k <= n_chunks; ++k) {
        if (k < n_chunks) {
            const int b = (int)(k & 1u);
            const uint64_t m = count_of(k);
            // pin_in[b] and dev_in[b] were last used by chunk k-2
            const auto t0 = clk::now();
            if (k >= 2 && (e = hipEventSynchronize(p.uploaded[b])) != hipSuccess) return e;
            const auto t1 = clk::now();
            staged_copy(p.pin_in[b].bytes(), in + k * chunk * ib, m * ib);
            const auto t2 = clk::now();
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
            if (trace)
                std::fprintf(stderr, "pipe chunk %llu: wait_up %.2f copy_in %.2f enqueue %.2f ms\n",
                             (unsigned long long)k, ms(t0, t1), ms(t1, t2), ms(t2, clk::now()));
        }
        if (k >= 1) {  // chunk k-1's results to the caller while chunk k runs
            const int b = (int)((k - 1) & 1u);
            const auto t0 = clk::now();
            if ((e = hipEventSynchronize(p.downloaded[b])) != hipSuccess) return e;
            const auto t1 = clk::now();
            staged_copy(out + (k - 1) * chunk * ob, p.pin_out[b].bytes(), count_of(k - 1) * ob);
            if (trace)
                std::fprintf(stderr, "pipe chunk %llu: wait_down %.2f copy_out %.2f ms\n", (unsigned long long)(k - 1),
                             ms(t0, t1), ms(t1, clk::now()));
        }
    }
    return hipSuccess;
}

}  // namespace dips_host
