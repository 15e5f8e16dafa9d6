// dips_handle.h -- the handle behind include/dips_hip.h's dips_* entry
// points and the helpers its three translation units share (internal to
// libdips_hip.so):
//   dips_abi.hip    lifecycle, streams, errors, kernel timing
//   compat_abi.hip  the dips-compat ComputeState (add_texture / dispatch /
//                   frame_callback and the batch form)
//   series_abi.hip  the north-star difference series and its measurement legs
//
// The handle plays the role of the reference's ComputeState
// (dips/src/gpu/mod.rs:39-56): it owns the HIP device binding, the stream,
// the temporal ring of the dips-compat path and the workspace of the batch
// series path.  Every entry point runs inside dips_abi::guard (abi_guard.h),
// returns a dips_status (or the documented int) and records a message for
// dips_last_error().
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <map>
#include <string>
#include <utility>
#include <vector>

#include "../../include/dips_hip.h"
#include "abi_guard.h"
#include "host_buffers.h"
#include "host_stream.h"

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
    dips_host::DevBuf partials, stage_frames, stage_ref, stage_series, stage_map;
    dips_host::DevBuf probe_out;  // sink of the read-ceiling kernels
    std::map<const void*, int> occupancy;

    // streamed feed
    dips_host::DevBuf ring[3];
    dips_host::DevBuf ring_ref;
    dips_host::HostPinned pinned[2];
    hipEvent_t copy_done[3] = {nullptr, nullptr, nullptr};
    hipEvent_t kernel_done[3] = {nullptr, nullptr, nullptr};

    // kernel timing (DIPS_FLAG_TIME_KERNEL): launches not yet read, the
    // totals since the last reset and the most recent kTimeKeep launches
    static constexpr size_t kTimeKeep = 65536;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pending;
    std::vector<hipEvent_t> ev_free;
    double t_ms = 0.0;
    uint64_t t_launches = 0;
    std::vector<double> t_each;

    // dips-compat ComputeState
    uint32_t width = 0, height = 0;
    int n_queued = 0;
    bool main_init = false;
    uint32_t ring_idx = 0;     // UCircularIndex (utils/indexing.rs:1-34)
    uint32_t uniform_idx = 0;  // starting_index uniform (bind_groups.rs:317-321)
    dips_host::DevBuf slots[4], raw, start, out;
    dips_host::HostPinned io;
    uint64_t added = 0;                   // frames added so far (global frame index of the next one)
    dips_host::DevBuf slots_alt[4];       // second ring for the multi-chunk batch kernel (swapped in after it)
    dips_host::DevBuf filtered;           // W > 1 batch: ring texels of a chunk of frames (compat_filter_frames)
    dips_host::StreamPipe pipe;           // host-pointer feed of dips_frame_callback_batch
    dips_host::PieceEvents pieces;        // per-piece completion of the per-frame readback
    dips_host::PieceEvents up_pieces;     // per-stripe upload completion (deferred W > 1 upload)
    dips_host::HostPinned io_out;         // readback staging of the striped frame_callback
    dips_host::CallPhases cb_phases;      // where the last zero-copy frame_callback's time went
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
    // T_d / T_c tables of the GRAY8 table kernel (series_gray.hip, layout 4:
    // layout 5's table and band word, then layout 2's kGrayLutAllocBytes
    // after it) for gray_lut_tau
    dips_host::DevBuf gray_lut;
    bool gray_lut_valid = false;
    float gray_lut_tau = 0.0f;
    dips_host::DevBuf cb_lut;  // epilogue table of compat_batch_lut_kernel (128 KiB)
    bool cb_lut_valid = false;
    uint32_t cb_lut_filter = 0, cb_lut_col = 0;
    float cb_lut_k = 0.0f;

    // frame-range sharding (shard_abi.hip): the broadcast reference, the
    // received halo frame, the padded send / gather buffers of the series,
    // the stream the halo exchange runs on beside the series launch
    dips_host::DevBuf shard_ref, shard_halo, shard_send, shard_recv;
    dips_host::DevBuf shard_send_frame;  // host-pointer calls: the last frame, sent as the next rank's halo
    hipStream_t comm_stream = nullptr;
    hipEvent_t shard_ev_in = nullptr, shard_ev_halo = nullptr;
    const uint8_t* shard_last_ref = nullptr;  // the reference of the last sharded call's first frame
    uint64_t shard_last_bytes = 0;

    bool crosscheck() const { return (p.flags & DIPS_FLAG_CROSSCHECK) != 0; }
};

namespace dips_internal {

dips_status fail(dips_handle* h, dips_status st, const std::string& msg);
dips_status hip_fail(dips_handle* h, hipError_t e, const char* what);
// hipSetDevice to the handle's device (DIPS_ERR_INVALID for a null handle)
dips_status bind(dips_handle* h);
// a timing event from the handle's free list, or a new one (nullptr on failure)
hipEvent_t take_event(dips_handle* h);
// the kernel's resident 256-thread blocks per CU, cached per handle
int occupancy_blocks(dips_handle* h, const void* kernel);
// a deferred frame's speculative kernels finished (compat_abi.hip)
dips_status flush_pending(dips_handle* h);
// the series of device frames, asynchronously on `s` (series_abi.hip)
dips_status run_series_device(dips_handle* h, uint32_t width, uint32_t height, const uint8_t* frames,
                              uint32_t n_frames, const uint8_t* ref0, dips_series_entry* series, uint8_t* map,
                              hipStream_t s);
// dips_compat_resume with the pointer kind given (compat_abi.hip)
dips_status compat_resume_impl(dips_handle* h, uint32_t width, uint32_t height, const uint8_t* start_rgba,
                               const uint8_t* halo, uint64_t t0, bool dev);
// the series of HOST frames through the pinned, side-stream feed
// (series_abi.hip); `ref_dev` a device reference of the first frame or NULL
dips_status run_series_streamed(dips_handle* h, uint32_t width, uint32_t height, const uint8_t* host_frames,
                                uint32_t n_frames, const uint8_t* ref_dev, dips_series_entry* series_dev,
                                uint32_t chunk_frames);
// waves of that launch for an aligned batch of this shape (0: not eligible),
// with or without the DIPS_SERIES_WAVES_PER_SIMD cap
uint64_t series_waves(dips_handle* h, uint32_t width, uint32_t height, uint32_t n_frames, bool env_cap);

}  // namespace dips_internal

#define DIPS_HIP(h, call)                                                     \
    do {                                                                      \
        hipError_t e_ = (call);                                               \
        if (e_ != hipSuccess) return dips_internal::hip_fail((h), e_, #call); \
    } while (0)
