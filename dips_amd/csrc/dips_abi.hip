// dips_abi.hip -- host side of include/dips_hip.h, part 1: the handle's
// lifecycle (ComputeState::new / Drop, dips/src/gpu/mod.rs:59-165), its
// stream, its errors and the kernel timing.  The dips-compat operator is in
// compat_abi.hip, the difference series in series_abi.hip; the handle and
// the shared helpers in dips_handle.h.  Every extern "C" body runs inside
// dips_abi::guard (abi_guard.h): no C++ exception leaves the library.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <mutex>
#include <new>
#include <string>

#include "dips_handle.h"

namespace {

std::mutex g_err_mu;
std::string g_create_err;

void set_create_err(const std::string& m) {
    std::lock_guard<std::mutex> lk(g_err_mu);
    g_create_err = m;
}

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

}  // namespace

namespace dips_abi {

void note_error(dips_handle* h, const char* msg) noexcept {
    if (!h) return;
    try {
        h->err = msg;
    } catch (...) {
    }
}

void note_error(CreateTag, const char* msg) noexcept {
    try {
        set_create_err(msg);
    } catch (...) {
    }
}

}  // namespace dips_abi

namespace dips_internal {

dips_status fail(dips_handle* h, dips_status st, const std::string& msg) {
    if (h) h->err = msg;
    return st;
}

dips_status hip_fail(dips_handle* h, hipError_t e, const char* what) {
    std::string m = std::string(what) + ": " + hipGetErrorString(e);
    return fail(h, e == hipErrorOutOfMemory ? DIPS_ERR_NOMEM : DIPS_ERR_HIP, m);
}

dips_status bind(dips_handle* h) {
    if (!h) return DIPS_ERR_INVALID;
    hipError_t e = hipSetDevice(h->device);
    if (e != hipSuccess) return hip_fail(h, e, "hipSetDevice");
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

}  // namespace dips_internal

using dips_abi::guard;
using namespace dips_internal;

namespace dips_abi {
int current_device() noexcept {
    int d = -1;
    return hipGetDevice(&d) == hipSuccess ? d : -1;
}
void set_device(int dev) noexcept { (void)hipSetDevice(dev); }
}  // namespace dips_abi

extern "C" {

int dips_abi_version(void) {
    return guard(nullptr, [&]() -> int { return DIPS_ABI_VERSION; });
}

dips_status dips_params_default(dips_params* p) {
    return guard(nullptr, [&]() -> dips_status {
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
    });
}

dips_status dips_create(const dips_params* params, int device, dips_handle** out) {
    return guard(dips_abi::CreateTag{}, [&]() -> dips_status {
        if (!out) return DIPS_ERR_INVALID;
        *out = nullptr;
        dips_params p;
        if (params) p = *params;
        else dips_params_default(&p);
        std::string why;
        if (validate_params(&p, &why) != DIPS_OK) {
            set_create_err(why);
            return DIPS_ERR_INVALID;
        }
        int count = 0;
        hipError_t e = hipGetDeviceCount(&count);
        if (e != hipSuccess || count <= 0 || device < 0 || device >= count) {
            set_create_err(std::string("no HIP device ") + std::to_string(device) + " (" +
                           (e == hipSuccess ? std::to_string(count) + " visible" : hipGetErrorString(e)) + ")");
            return DIPS_ERR_NODEVICE;
        }
        dips_handle* h = new (std::nothrow) dips_handle();
        if (!h) return DIPS_ERR_NOMEM;
        h->p = p;
        h->device = device;
        e = hipSetDevice(device);
        if (e == hipSuccess) e = hipDeviceGetAttribute(&h->cu_count, hipDeviceAttributeMultiprocessorCount, device);
        // blocking: ordered with stream 0 (see dips_set_stream)
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&h->own_stream, hipStreamDefault);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&h->copy_stream, hipStreamNonBlocking);
        for (int i = 0; i < 3 && e == hipSuccess; ++i) {
            e = hipEventCreateWithFlags(&h->copy_done[i], hipEventDisableTiming);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&h->kernel_done[i], hipEventDisableTiming);
        }
        if (e != hipSuccess) {
            set_create_err(std::string("HIP initialisation failed: ") + hipGetErrorString(e));
            dips_destroy(h);
            return DIPS_ERR_HIP;
        }
        h->stream = h->own_stream;
        *out = h;
        return DIPS_OK;
    });
}

void dips_destroy(dips_handle* h) {
    guard(h, [&]() -> void {
        if (!h) return;
        (void)hipSetDevice(h->device);
        if (h->stream) (void)hipStreamSynchronize(h->stream);
        if (h->copy_stream) (void)hipStreamSynchronize(h->copy_stream);
        if (h->comm_stream) (void)hipStreamSynchronize(h->comm_stream);
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
        h->gray_lut.release();
        h->start.release();
        h->out.release();
        h->io.release();
        h->shard_ref.release();
        h->shard_halo.release();
        h->shard_send.release();
        h->shard_recv.release();
        h->shard_send_frame.release();
        if (h->comm_stream) (void)hipStreamDestroy(h->comm_stream);
        if (h->shard_ev_in) (void)hipEventDestroy(h->shard_ev_in);
        if (h->shard_ev_halo) (void)hipEventDestroy(h->shard_ev_halo);
        if (h->switch_ev) (void)hipEventDestroy(h->switch_ev);
        if (h->join_ev) (void)hipEventDestroy(h->join_ev);
        if (h->own_stream) (void)hipStreamDestroy(h->own_stream);
        if (h->copy_stream) (void)hipStreamDestroy(h->copy_stream);
        delete h;
    });
}

const char* dips_last_error(const dips_handle* h) {
    return guard(h, [&]() -> const char* {
        if (h) return h->err.c_str();
        // this thread's copy: a failed dips_create on another thread may
        // replace the record while the caller still reads the message
        thread_local std::string copy;
        std::lock_guard<std::mutex> lk(g_err_mu);
        copy = g_create_err;
        return copy.c_str();
    });
}

dips_status dips_set_stream(dips_handle* h, void* stream) {
    return guard(h, [&]() -> dips_status {
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
    });
}

dips_status dips_synchronize(dips_handle* h) {
    return guard(h, [&]() -> dips_status {
        dips_status st = bind(h);
        if (st != DIPS_OK) return st;
        st = flush_pending(h);  // a deferred frame into its slot first
        if (st != DIPS_OK) return st;
        DIPS_HIP(h, hipStreamSynchronize(h->stream));
        return DIPS_OK;
    });
}

dips_status dips_kernel_time(dips_handle* h, double* total_ms, uint64_t* launches) {
    return guard(h, [&]() -> dips_status {
        dips_status st = bind(h);
        if (st != DIPS_OK) return st;
        for (auto& pr : h->ev_pending) {
            DIPS_HIP(h, hipEventSynchronize(pr.second));
            float ms = 0.0f;
            DIPS_HIP(h, hipEventElapsedTime(&ms, pr.first, pr.second));
            h->t_ms += ms;
            h->t_launches += 1;
            // keep the most recent kTimeKeep launches (drop the older half at the cap)
            if (h->t_each.size() >= dips_handle::kTimeKeep)
                h->t_each.erase(h->t_each.begin(), h->t_each.begin() + dips_handle::kTimeKeep / 2);
            h->t_each.push_back(ms);
            h->ev_free.push_back(pr.first);
            h->ev_free.push_back(pr.second);
        }
        h->ev_pending.clear();
        if (total_ms) *total_ms = h->t_ms;
        if (launches) *launches = h->t_launches;
        return DIPS_OK;
    });
}

dips_status dips_kernel_time_reset(dips_handle* h) {
    return guard(h, [&]() -> dips_status {
        dips_status st = dips_kernel_time(h, nullptr, nullptr);
        if (st != DIPS_OK) return st;
        h->t_ms = 0.0;
        h->t_launches = 0;
        h->t_each.clear();
        return DIPS_OK;
    });
}

dips_status dips_kernel_time_each(dips_handle* h, double* ms_each, uint64_t cap, uint64_t* launches) {
    return guard(h, [&]() -> dips_status {
        dips_status st = dips_kernel_time(h, nullptr, nullptr);
        if (st != DIPS_OK) return st;
        const uint64_t n = h->t_each.size();
        if (ms_each)
            for (uint64_t i = 0; i < n && i < cap; ++i) ms_each[i] = h->t_each[i];
        if (launches) *launches = n;
        return DIPS_OK;
    });
}

double dips_series_si(const dips_series_entry* e) {
    return guard(nullptr, [&]() -> double { return e ? std::ldexp((double)e->si_fixed, -32) : 0.0; });
}

}  // extern "C"
