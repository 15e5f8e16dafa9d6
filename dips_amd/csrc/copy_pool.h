// copy_pool.h -- persistent host worker threads for the PCIe staging copies
// (internal to libdips_hip.so).
//
// A single host thread copies pageable memory at a fraction of the PCIe DMA
// rate, and creating threads per call costs tens of microseconds each, which
// is too much for the per-frame operators (one 4K frame = 33 MB, ~0.6 ms of
// DMA).  The pool keeps up to 7 workers parked on a condition variable;
// run(n, fn) executes fn(0..n-1) on the workers and the calling thread and
// returns when all are done.  One run at a time (a process-wide mutex): the
// handles are not internally synchronised, but different handles may be
// driven from different threads.  A child process created by fork() gets a
// fresh pool (the parent's workers do not exist there).
//
// Failure model: a worker that cannot be started (std::thread throws
// std::system_error on EAGAIN -- a thread or process limit) is simply not
// there: the pool runs with the workers it got, down to none, where the
// calling thread runs every task itself.  A task that throws does not end its
// worker: the first exception is kept and rethrown on the calling thread
// when the run is over, where the ABI guard (abi_guard.h) turns it into a
// status.
#pragma once

#include <immintrin.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <functional>
#include <mutex>
#include <system_error>
#include <thread>
#include <vector>

namespace dips_host {

class CopyPool {
   public:
    explicit CopyPool(unsigned workers) {
        th_.reserve(workers);  // emplace_back below never reallocates
        for (unsigned i = 0; i < workers; ++i) {
            try {
                th_.emplace_back([this]() { loop(); });
            } catch (const std::system_error&) {
                break;  // no more threads: keep the ones started
            }
        }
    }
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    CopyPool(const CopyPool&) = delete;
    CopyPool& operator=(const CopyPool&) = delete;

    unsigned threads() const { return (unsigned)th_.size() + 1u; }

    // fn(i) for every i in [0, n), spread over the workers and the caller.
    // With `spin`, the workers watch for the next run for kSpinUs after this
    // one before parking (the per-frame pipelines: back-to-back calls).
    void run(size_t n, const std::function<void(size_t)>& fn, bool spin = false) {
        if (n == 0) return;
        std::lock_guard<std::mutex> one_run(run_mu_);
        if (n == 1 || th_.empty()) {
            std::exception_ptr ex;  // the same semantics as with workers: every task runs
            for (size_t i = 0; i < n; ++i) {
                try {
                    fn(i);
                } catch (...) {
                    if (!ex) ex = std::current_exception();
                }
            }
            if (ex) std::rethrow_exception(ex);
            return;
        }
        {
            std::lock_guard<std::mutex> lk(mu_);
            fn_ = &fn;
            n_ = n;
            spin_ = spin;
            next_.store(0, std::memory_order_relaxed);
            busy_ = (unsigned)th_.size();
            ++gen_;
            gen_seen_.store(gen_, std::memory_order_release);
        }
        cv_.notify_all();
        drain(fn, n);
        std::exception_ptr ex;
        {
            std::unique_lock<std::mutex> lk(mu_);
            done_cv_.wait(lk, [this]() { return busy_ == 0; });
            fn_ = nullptr;
            std::swap(ex, ex_);
        }
        if (ex) std::rethrow_exception(ex);
    }

    // The process-wide pool: min(8, hardware threads) - 1 workers.
    static CopyPool& global() {
        static std::mutex mu;
        static CopyPool* pool = nullptr;
        static pid_t owner = 0;
        std::lock_guard<std::mutex> lk(mu);
        if (!pool || owner != getpid()) {
            // after fork() the parent's workers are gone: leak the copy the
            // child inherited and start a new one
            unsigned hw = std::thread::hardware_concurrency();
            hw = hw == 0 ? 1u : std::min(hw, 8u);
            // DIPS_COPY_THREADS (1..32) overrides the count, read once per process
            if (const char* e = std::getenv("DIPS_COPY_THREADS")) {
                const long v = std::strtol(e, nullptr, 10);
                if (v >= 1 && v <= 32) hw = (unsigned)v;
            }
            pool = new CopyPool(hw - 1u);
            owner = getpid();
        }
        return *pool;
    }

   private:
    void drain(const std::function<void(size_t)>& fn, size_t n) {
        for (size_t i = next_.fetch_add(1); i < n; i = next_.fetch_add(1)) {
            try {
                fn(i);
            } catch (...) {
                std::lock_guard<std::mutex> lk(mu_);
                if (!ex_) ex_ = std::current_exception();
            }
        }
    }
    void loop() {
        uint64_t seen = 0;
        bool spin = false;  // the last run asked for the spin
        // After a per-frame run, watch for the next one for 200 us before
        // parking on the condition variable: back-to-back per-frame calls then
        // find the workers awake on warm cores.  Measured over four alternated
        // rounds of 200 4K frame_callback calls (round 4,
        // profiles/r04/k/): 1,689-1,837 frames/s (p90 0.56-0.63 ms) against
        // 1,363-1,687 (p90 0.61-0.88 ms) parking at once; the pool's own
        // pack / expand thread time drops too (1.6-1.8 vs 1.9-2.5 ms per
        // call).  Costs <= 200 us of each worker's time per call when calls
        // are sparse; batch copies (pool_copy) never spin.
        // DIPS_POOL_SPIN_US overrides the 200 us (0: park at once).
        static const long spin_us = []() {
            const char* e = std::getenv("DIPS_POOL_SPIN_US");
            const long v = e ? std::strtol(e, nullptr, 10) : 200;
            return v > 0 && v <= 10000 ? v : 0L;
        }();
        for (;;) {
            const std::function<void(size_t)>* fn;
            size_t n;
            if (spin_us > 0 && spin) {
                const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(spin_us);
                while (gen_seen_.load(std::memory_order_acquire) == seen && std::chrono::steady_clock::now() < until)
                    _mm_pause();
            }
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&]() { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                fn = fn_;
                n = n_;
                spin = spin_;
            }
            drain(*fn, n);
            {
                std::lock_guard<std::mutex> lk(mu_);
                if (--busy_ == 0) done_cv_.notify_one();
            }
        }
    }

    std::vector<std::thread> th_;
    std::mutex run_mu_, mu_;
    std::condition_variable cv_, done_cv_;
    const std::function<void(size_t)>* fn_ = nullptr;
    size_t n_ = 0;
    bool spin_ = false;
    std::exception_ptr ex_;  // the run's first task exception (under mu_)
    std::atomic<size_t> next_{0};
    unsigned busy_ = 0;
    uint64_t gen_ = 0;
    std::atomic<uint64_t> gen_seen_{0};  // gen_, readable without the mutex (the spin before parking)
    bool stop_ = false;
};

// Streaming copy for the staging buffers: every byte is written once and the
// CPU does not read it back (the DMA engine does, or the caller much later),
// so non-temporal 32-B stores skip the read-for-ownership of each
// destination line and leave the caches alone.  The closing sfence makes the
// write-combined stores globally visible before the caller enqueues a DMA
// that reads them.
__attribute__((target("avx2"))) inline void stream_copy_avx2(uint8_t* d, const uint8_t* s, size_t n) {
    size_t head = (32u - ((uintptr_t)d & 31u)) & 31u;
    if (head > n) head = n;
    std::memcpy(d, s, head);
    size_t i = head;
    for (; i + 128 <= n; i += 128) {
        const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i));
        const __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i + 32));
        const __m256i c = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i + 64));
        const __m256i e = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i + 96));
        _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i), a);
        _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i + 32), b);
        _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i + 64), c);
        _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i + 96), e);
    }
    std::memcpy(d + i, s + i, n - i);
    _mm_sfence();
}

// The staging copy: streaming stores for pieces of >= 64 KiB on CPUs with
// AVX2, memcpy otherwise.
inline void host_copy(uint8_t* dst, const uint8_t* src, size_t bytes) {
    static const bool avx2 = __builtin_cpu_supports("avx2");
    if (avx2 && bytes >= (64u << 10))
        stream_copy_avx2(dst, src, bytes);
    else
        std::memcpy(dst, src, bytes);
}

// RGBA8 texels rebuilt from the per-pixel keys compat_main_host_kernel
// writes (out_key): one byte k -> (k, k, k, 255); two bytes (r, g) ->
// (r, g, min(r, g), 255).  `npx` pixels from `keys` to `dst` (4 npx bytes).
// With `nt`, 32-B streaming stores (the caller's output is written once).
__attribute__((target("avx2"))) inline void put32(uint8_t* d, __m256i v, bool nt) {
    if (nt && ((uintptr_t)d & 31u) == 0)
        _mm256_stream_si256(reinterpret_cast<__m256i*>(d), v);
    else
        _mm256_storeu_si256(reinterpret_cast<__m256i*>(d), v);
}

__attribute__((target("avx2"))) inline void expand_keys_avx2(uint8_t* dst, const uint8_t* keys, size_t npx,
                                                            int key_bytes, bool nt) {
    const __m256i alpha = _mm256_set1_epi32((int)0xFF000000u);
    size_t i = 0;
    if (key_bytes == 1) {
        // 16 keys -> 64 B: each 128-bit lane of a broadcast picks 4 keys
        const __m256i s0 = _mm256_setr_epi8(0, 0, 0, -1, 1, 1, 1, -1, 2, 2, 2, -1, 3, 3, 3, -1,  //
                                            4, 4, 4, -1, 5, 5, 5, -1, 6, 6, 6, -1, 7, 7, 7, -1);
        const __m256i s1 = _mm256_setr_epi8(8, 8, 8, -1, 9, 9, 9, -1, 10, 10, 10, -1, 11, 11, 11, -1,  //
                                            12, 12, 12, -1, 13, 13, 13, -1, 14, 14, 14, -1, 15, 15, 15, -1);
        for (; i + 16 <= npx; i += 16) {
            const __m256i k = _mm256_broadcastsi128_si256(_mm_loadu_si128(reinterpret_cast<const __m128i*>(keys + i)));
            put32(dst + 4 * i, _mm256_or_si256(_mm256_shuffle_epi8(k, s0), alpha), nt);
            put32(dst + 4 * (i + 8), _mm256_or_si256(_mm256_shuffle_epi8(k, s1), alpha), nt);
        }
        for (; i < npx; ++i) {
            const uint32_t k = keys[i];
            const uint32_t t = k | (k << 8) | (k << 16) | 0xFF000000u;
            std::memcpy(dst + 4 * i, &t, 4);
        }
    } else {
        // 8 (r, g) keys -> 32 B: min of (r, g, r, .) and (r, g, g, .) puts min(r, g) in B
        // (both 128-bit lanes hold their 4 keys in bytes 0..7)
        const __m256i sa = _mm256_setr_epi8(0, 1, 0, -1, 2, 3, 2, -1, 4, 5, 4, -1, 6, 7, 6, -1,  //
                                            0, 1, 0, -1, 2, 3, 2, -1, 4, 5, 4, -1, 6, 7, 6, -1);
        const __m256i sb = _mm256_setr_epi8(0, 1, 1, -1, 2, 3, 3, -1, 4, 5, 5, -1, 6, 7, 7, -1,  //
                                            0, 1, 1, -1, 2, 3, 3, -1, 4, 5, 5, -1, 6, 7, 7, -1);
        for (; i + 8 <= npx; i += 8) {
            // keys of pixels i..i+3 in the low lane, i+4..i+7 in the high lane
            const __m128i lo = _mm_loadl_epi64(reinterpret_cast<const __m128i*>(keys + 2 * i));
            const __m128i hi = _mm_loadl_epi64(reinterpret_cast<const __m128i*>(keys + 2 * i + 8));
            const __m256i k = _mm256_inserti128_si256(_mm256_castsi128_si256(lo), hi, 1);
            const __m256i v = _mm256_min_epu8(_mm256_shuffle_epi8(k, sa), _mm256_shuffle_epi8(k, sb));
            put32(dst + 4 * i, _mm256_or_si256(v, alpha), nt);
        }
        for (; i < npx; ++i) {
            const uint32_t r = keys[2 * i], g = keys[2 * i + 1];
            const uint32_t t = r | (g << 8) | ((r < g ? r : g) << 16) | 0xFF000000u;
            std::memcpy(dst + 4 * i, &t, 4);
        }
    }
    if (nt) _mm_sfence();
}

// The same without AVX2 (and the reference the CPU test checks the AVX2
// form against, tests/test_copy_pool_cpu.py).
inline void expand_keys_scalar(uint8_t* dst, const uint8_t* keys, size_t npx, int key_bytes) {
    for (size_t i = 0; i < npx; ++i) {
        const uint32_t r = keys[key_bytes * i], g = key_bytes == 1 ? r : keys[2 * i + 1];
        const uint32_t t = r | (g << 8) | ((r < g ? r : g) << 16) | 0xFF000000u;
        std::memcpy(dst + 4 * i, &t, 4);
    }
}

inline void expand_keys(uint8_t* dst, const uint8_t* keys, size_t npx, int key_bytes, bool nt) {
    static const bool avx2 = __builtin_cpu_supports("avx2");
    if (avx2)
        expand_keys_avx2(dst, keys, npx, key_bytes, nt);
    else
        expand_keys_scalar(dst, keys, npx, key_bytes);
}

// The per-frame zero-copy input in the form the kernel needs (compat_main_
// host_packed_kernel, in_key): the RGBA8 frame's per-pixel (max, min) of
// R, G, B (in_bytes 2, chroma None: get_intensity uses nothing else) or its
// one chroma channel ch = 0 / 1 / 2 (in_bytes 1), `npx` pixels from `src` to
// `dst` (npx * in_bytes bytes): half or a quarter of the frame's bytes over
// PCIe.
__attribute__((target("avx2"))) inline void pack_frame_avx2(uint8_t* dst, const uint8_t* src, size_t npx,
                                                           int in_bytes, int ch, bool nt) {
    size_t i = 0;
    if (in_bytes == 2) {
        // per 128-bit lane: R0..R3 | G0..G3 | B0..B3 of its 4 pixels
        const __m256i s = _mm256_setr_epi8(0, 4, 8, 12, 1, 5, 9, 13, 2, 6, 10, 14, -1, -1, -1, -1,  //
                                           0, 4, 8, 12, 1, 5, 9, 13, 2, 6, 10, 14, -1, -1, -1, -1);
        for (; i + 16 <= npx; i += 16) {
            __m256i o[2];
            for (int h = 0; h < 2; ++h) {
                const __m256i v = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + 4 * (i + 8 * h)));
                const __m256i t = _mm256_shuffle_epi8(v, s);
                const __m256i g = _mm256_srli_si256(t, 4), b = _mm256_srli_si256(t, 8);
                const __m256i mx = _mm256_max_epu8(_mm256_max_epu8(t, g), b);
                const __m256i mn = _mm256_min_epu8(_mm256_min_epu8(t, g), b);
                // (max, min) of pixels 0..3 in each lane's low 8 bytes; lanes -> qwords 0, 2
                o[h] = _mm256_permute4x64_epi64(_mm256_unpacklo_epi8(mx, mn), 0x08);
            }
            const __m256i w = _mm256_permute2x128_si256(o[0], o[1], 0x20);
            put32(dst + 2 * i, w, nt);
        }
        for (; i < npx; ++i) {
            const uint8_t r = src[4 * i], g = src[4 * i + 1], b = src[4 * i + 2];
            dst[2 * i] = std::max(std::max(r, g), b);
            dst[2 * i + 1] = std::min(std::min(r, g), b);
        }
    } else {
        // the channel's byte of each of the 4 pixels of a 128-bit lane
        const char c = (char)ch;
        const __m256i sel = _mm256_setr_epi8(c, (char)(c + 4), (char)(c + 8), (char)(c + 12), -1, -1, -1, -1, -1, -1, -1,
                                             -1, -1, -1, -1, -1, c, (char)(c + 4), (char)(c + 8), (char)(c + 12), -1, -1,
                                             -1, -1, -1, -1, -1, -1, -1, -1, -1, -1);
        const __m256i lanes = _mm256_setr_epi32(0, 4, 0, 0, 0, 0, 0, 0);
        for (; i + 8 <= npx; i += 8) {
            const __m256i v = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + 4 * i));
            const __m256i t = _mm256_permutevar8x32_epi32(_mm256_shuffle_epi8(v, sel), lanes);
            _mm_storel_epi64(reinterpret_cast<__m128i*>(dst + i), _mm256_castsi256_si128(t));
        }
        for (; i < npx; ++i) dst[i] = src[4 * i + ch];
    }
    if (nt) _mm_sfence();
}

// The same without AVX2 (and the CPU test's reference for the AVX2 form).
inline void pack_frame_scalar(uint8_t* dst, const uint8_t* src, size_t npx, int in_bytes, int ch) {
    for (size_t i = 0; i < npx; ++i) {
        const uint8_t r = src[4 * i], g = src[4 * i + 1], b = src[4 * i + 2];
        if (in_bytes == 2) {
            dst[2 * i] = std::max(std::max(r, g), b);
            dst[2 * i + 1] = std::min(std::min(r, g), b);
        } else {
            dst[i] = src[4 * i + ch];
        }
    }
}

inline void pack_frame(uint8_t* dst, const uint8_t* src, size_t npx, int in_bytes, int ch, bool nt) {
    static const bool avx2 = __builtin_cpu_supports("avx2");
    if (avx2)
        pack_frame_avx2(dst, src, npx, in_bytes, ch, nt);
    else
        pack_frame_scalar(dst, src, npx, in_bytes, ch);
}

// Host copy in ~4 MiB pieces over the pool.
inline void pool_copy(uint8_t* dst, const uint8_t* src, size_t bytes) {
    const size_t kPiece = 4u << 20;
    if (bytes < 2 * kPiece) {
        host_copy(dst, src, bytes);
        return;
    }
    const size_t n = (bytes + kPiece - 1) / kPiece;
    CopyPool::global().run(n, [&](size_t i) {
        const size_t o = i * kPiece;
        host_copy(dst + o, src + o, std::min(kPiece, bytes - o));
    });
}

}  // namespace dips_host
