//! Raw `extern "C"` declarations of `include/dips_hip.h`, one per entry point,
//! in header order.  `tests/test_rust_shim.py` parses this file and checks
//! every struct field and every signature against the header, and the
//! `const` blocks below assert the same sizes / offsets the header's
//! `DIPS_LAYOUT_ASSERT`s pin on the C side.
#![allow(non_camel_case_types)]

use core::ffi::{c_char, c_int, c_void};
use core::mem::{offset_of, size_of};

/// `dips_status`: 0 = OK, negative = error (DIPS_ERR_*).
pub type DipsStatus = c_int;

pub const DIPS_OK: DipsStatus = 0;
pub const DIPS_ERR_INVALID: DipsStatus = -1;
pub const DIPS_ERR_HIP: DipsStatus = -2;
pub const DIPS_ERR_STATE: DipsStatus = -3;
pub const DIPS_ERR_NOMEM: DipsStatus = -4;
pub const DIPS_ERR_CAPACITY: DipsStatus = -5;
pub const DIPS_ERR_NODEVICE: DipsStatus = -6;
pub const DIPS_ERR_INTERNAL: DipsStatus = -7;
pub const DIPS_ERR_COMM: DipsStatus = -8;

pub const DIPS_ABI_VERSION: c_int = 3;

pub const DIPS_FILTER_SIGMOID: u32 = 0;
pub const DIPS_FILTER_INVERSE_SIGMOID: u32 = 1;
pub const DIPS_FILTER_UNFILTERED: u32 = 255;
pub const DIPS_CHROMA_NONE: u32 = 0;
pub const DIPS_CHROMA_RED: u32 = 1;
pub const DIPS_CHROMA_GREEN: u32 = 2;
pub const DIPS_CHROMA_BLUE: u32 = 3;
pub const DIPS_FMT_GRAY8: u32 = 1;
pub const DIPS_FMT_RGB8: u32 = 3;
pub const DIPS_FMT_RGBA8: u32 = 4;
pub const DIPS_MODE_OVERALL: u32 = 0;
pub const DIPS_MODE_PER_FRAME: u32 = 1;
pub const DIPS_FLAG_DEVICE_PTRS: u32 = 0x1;
pub const DIPS_FLAG_TIME_KERNEL: u32 = 0x2;
pub const DIPS_FLAG_FORCE_GENERIC: u32 = 0x4;
pub const DIPS_FLAG_CROSSCHECK: u32 = 0x8;
pub const DIPS_FLAG_GRAY_BAND_TABLE: u32 = 0x10;
pub const DIPS_FLAG_GRAY_PAIR_TABLE: u32 = 0x20;
pub const DIPS_CALLBACK_PHASES: u32 = 11;
pub const DIPS_COMM_ID_BYTES: u32 = 128;
pub const DIPS_COMM_RCCL: c_int = 1;
pub const DIPS_COMM_LOOPBACK: c_int = 2;
pub const DIPS_COMM_HOST: c_int = 3;
pub const DIPS_SHARD_REF_RESIDENT: u32 = 0x1;

/// `dips_params`: ComputeState::new's arguments (dips/src/gpu/mod.rs:59-65,
/// DiPsProperties dips/src/lib.rs:63-86) + the batch series configuration.
#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct DipsParams {
    pub colorize: u8,
    pub spatial_window_size: i32,
    pub sensitivity: f32,
    pub filter_type: u32,
    pub chroma_filter: u32,
    pub mode: u32,
    pub format: u32,
    pub tau: f32,
    pub flags: u32,
}

/// `dips_series_entry`: one frame of the difference series.
#[repr(C)]
#[derive(Clone, Copy, Debug, Default, PartialEq, Eq)]
pub struct DipsSeriesEntry {
    pub sad: u64,
    pub sj: u64,
    pub count: u64,
    pub si_fixed: u64,
}

/// `dips_alt_params`: dips_alt's DiPsProperties
/// (dips_alt/src/dips_compute/mod.rs:167-186) + the texture count.
#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct DipsAltParams {
    pub colorize: u8,
    pub window_size: i32,
    pub sigmoid_horizontal_scalar: f32,
    pub filter_type: u32,
    pub chroma_filter: u32,
    pub num_textures: u32,
    pub flags: u32,
}

/// Opaque `dips_handle` / `dips_alt_handle`.
#[repr(C)]
pub struct DipsHandle {
    _p: [u8; 0],
}
#[repr(C)]
pub struct DipsAltHandle {
    _p: [u8; 0],
}

/// Opaque `dips_comm`: one rank's communicator of the sharded series.
#[repr(C)]
pub struct DipsComm {
    _p: [u8; 0],
}

/// `dips_comm_ops`: the caller's transport of DIPS_COMM_HOST (host buffers;
/// each returns 0 on success).
#[repr(C)]
#[derive(Clone, Copy)]
pub struct DipsCommOps {
    pub broadcast: Option<unsafe extern "C" fn(ctx: *mut c_void, buf: *mut c_void, bytes: usize, root: c_int) -> c_int>,
    pub sendrecv: Option<
        unsafe extern "C" fn(ctx: *mut c_void, send: *const c_void, to: c_int, recv: *mut c_void, from: c_int,
                             bytes: usize) -> c_int,
    >,
    pub gather: Option<
        unsafe extern "C" fn(ctx: *mut c_void, send: *const c_void, recv: *mut c_void, bytes: usize, root: c_int)
                             -> c_int,
    >,
}

// The same layout the header pins with DIPS_LAYOUT_ASSERT.
const _: () = {
    assert!(size_of::<DipsParams>() == 36);
    assert!(offset_of!(DipsParams, colorize) == 0);
    assert!(offset_of!(DipsParams, spatial_window_size) == 4);
    assert!(offset_of!(DipsParams, sensitivity) == 8);
    assert!(offset_of!(DipsParams, filter_type) == 12);
    assert!(offset_of!(DipsParams, chroma_filter) == 16);
    assert!(offset_of!(DipsParams, mode) == 20);
    assert!(offset_of!(DipsParams, format) == 24);
    assert!(offset_of!(DipsParams, tau) == 28);
    assert!(offset_of!(DipsParams, flags) == 32);
    assert!(size_of::<DipsSeriesEntry>() == 32);
    assert!(offset_of!(DipsSeriesEntry, sad) == 0);
    assert!(offset_of!(DipsSeriesEntry, sj) == 8);
    assert!(offset_of!(DipsSeriesEntry, count) == 16);
    assert!(offset_of!(DipsSeriesEntry, si_fixed) == 24);
    assert!(size_of::<DipsAltParams>() == 28);
    assert!(offset_of!(DipsAltParams, colorize) == 0);
    assert!(offset_of!(DipsAltParams, window_size) == 4);
    assert!(offset_of!(DipsAltParams, sigmoid_horizontal_scalar) == 8);
    assert!(offset_of!(DipsAltParams, filter_type) == 12);
    assert!(offset_of!(DipsAltParams, chroma_filter) == 16);
    assert!(offset_of!(DipsAltParams, num_textures) == 20);
    assert!(offset_of!(DipsAltParams, flags) == 24);
};

#[link(name = "dips_hip")]
extern "C" {
    // -- dips ComputeState (dips/src/gpu/mod.rs) + the difference series ----
    pub fn dips_params_default(p: *mut DipsParams) -> DipsStatus;
    pub fn dips_create(params: *const DipsParams, device: c_int, out: *mut *mut DipsHandle) -> DipsStatus;
    pub fn dips_destroy(h: *mut DipsHandle);
    pub fn dips_last_error(h: *const DipsHandle) -> *const c_char;
    pub fn dips_set_stream(h: *mut DipsHandle, stream: *mut c_void) -> DipsStatus;
    pub fn dips_synchronize(h: *mut DipsHandle) -> DipsStatus;
    pub fn dips_add_texture(h: *mut DipsHandle, width: u32, height: u32, frame_rgba: *const u8,
                            len: usize) -> DipsStatus;
    pub fn dips_dispatch(h: *mut DipsHandle, out_rgba: *mut u8, cap: usize) -> c_int;
    pub fn dips_frame_callback(h: *mut DipsHandle, width: u32, height: u32, frame_rgba: *const u8, len: usize,
                               out: *mut u8, cap: usize) -> c_int;
    pub fn dips_frame_callback_batch(h: *mut DipsHandle, width: u32, height: u32, frames: *const u8,
                                     n_frames: u32, out: *mut u8) -> DipsStatus;
    pub fn dips_callback_phases(h: *const DipsHandle, us: *mut f64, cap: u32, n: *mut u32) -> DipsStatus;
    pub fn dips_start_texture(h: *mut DipsHandle, out_rgba: *mut u8, cap: usize) -> c_int;
    pub fn dips_compat_resume(h: *mut DipsHandle, width: u32, height: u32, start_rgba: *const u8,
                              halo: *const u8, t0: u64) -> DipsStatus;
    pub fn dips_diff_series(h: *mut DipsHandle, width: u32, height: u32, frames: *const u8, n_frames: u32,
                            reference: *const u8, series: *mut DipsSeriesEntry, absdiff_map: *mut u8)
                            -> DipsStatus;
    pub fn dips_series_si(e: *const DipsSeriesEntry) -> f64;
    pub fn dips_diff_series_streamed(h: *mut DipsHandle, width: u32, height: u32, host_frames: *const u8,
                                     n_frames: u32, host_ref: *const u8, series: *mut DipsSeriesEntry,
                                     chunk_frames: u32) -> DipsStatus;
    pub fn dips_synth_frames(h: *mut DipsHandle, width: u32, height: u32, seed: u64, t0: u64, n_frames: u32,
                             dst: *mut u8) -> DipsStatus;
    pub fn dips_kernel_time(h: *mut DipsHandle, total_ms: *mut f64, launches: *mut u64) -> DipsStatus;
    pub fn dips_kernel_time_reset(h: *mut DipsHandle) -> DipsStatus;
    pub fn dips_kernel_time_each(h: *mut DipsHandle, ms_each: *mut f64, cap: u64, launches: *mut u64)
                                 -> DipsStatus;
    pub fn dips_series_geometry(h: *mut DipsHandle, width: u32, height: u32, n_frames: u32, waves: *mut u64,
                                tiles: *mut u64, partial_bytes: *mut u64) -> DipsStatus;
    pub fn dips_read_ceiling(h: *mut DipsHandle, dev_bytes: *const u8, bytes: u64, ms: *mut f64) -> DipsStatus;
    pub fn dips_read_ceiling_walk(h: *mut DipsHandle, dev_frames: *const u8, width: u32, height: u32,
                                  n_frames: u32, ms: *mut f64) -> DipsStatus;
    pub fn dips_abi_version() -> c_int;

    // -- frame-range sharding (no reference counterpart: dips/src/gpu/mod.rs:71-78
    //    asks for one adapter) ------------------------------------------------
    pub fn dips_comm_unique_id(id: *mut u8) -> DipsStatus;
    pub fn dips_comm_create(id: *const u8, nranks: c_int, rank: c_int, device: c_int, out: *mut *mut DipsComm)
                            -> DipsStatus;
    pub fn dips_comm_create_all(nranks: c_int, devices: *const c_int, comms: *mut *mut DipsComm) -> DipsStatus;
    pub fn dips_comm_create_loopback(nranks: c_int, device: c_int, comms: *mut *mut DipsComm) -> DipsStatus;
    pub fn dips_comm_create_host(ops: *const DipsCommOps, ctx: *mut c_void, nranks: c_int, rank: c_int,
                                 device: c_int, out: *mut *mut DipsComm) -> DipsStatus;
    pub fn dips_comm_destroy(comm: *mut DipsComm);
    pub fn dips_comm_last_error(comm: *const DipsComm) -> *const c_char;
    pub fn dips_comm_info(comm: *const DipsComm, kind: *mut c_int, nranks: *mut c_int, rank: *mut c_int)
                          -> DipsStatus;
    pub fn dips_shard_range(n_total: u64, nranks: c_int, rank: c_int, first: *mut u64, count: *mut u32)
                            -> DipsStatus;
    pub fn dips_shard_broadcast(h: *mut DipsHandle, comm: *mut DipsComm, width: u32, height: u32, frame: *const u8,
                                out: *mut u8) -> DipsStatus;
    pub fn dips_diff_series_sharded(h: *mut DipsHandle, comm: *mut DipsComm, width: u32, height: u32,
                                    frames: *const u8, n_local: u32, n_total: u64, reference: *const u8,
                                    shard_flags: u32, series_local: *mut DipsSeriesEntry,
                                    series_all: *mut DipsSeriesEntry) -> DipsStatus;
    pub fn dips_frame_callback_batch_sharded(h: *mut DipsHandle, comm: *mut DipsComm, width: u32, height: u32,
                                             frames: *const u8, n_local: u32, n_total: u64, out: *mut u8)
                                             -> DipsStatus;
    pub fn dips_shard_plan(h: *mut DipsHandle, comm: *const DipsComm, width: u32, height: u32, n_total: u64,
                           first: *mut u64, count: *mut u32, waves: *mut u64, waves_uncapped: *mut u64)
                           -> DipsStatus;
    pub fn dips_shard_reference(h: *mut DipsHandle, out: *mut u8, cap: usize) -> c_int;

    // -- dips_alt DiPsCompute (dips_alt/src/dips_compute/mod.rs) ----------------
    pub fn dips_alt_params_default(p: *mut DipsAltParams) -> DipsStatus;
    pub fn dips_alt_create(params: *const DipsAltParams, width: u32, height: u32, device: c_int,
                           out: *mut *mut DipsAltHandle) -> DipsStatus;
    pub fn dips_alt_destroy(h: *mut DipsAltHandle);
    pub fn dips_alt_last_error(h: *const DipsAltHandle) -> *const c_char;
    pub fn dips_alt_set_stream(h: *mut DipsAltHandle, stream: *mut c_void) -> DipsStatus;
    pub fn dips_alt_synchronize(h: *mut DipsAltHandle) -> DipsStatus;
    pub fn dips_alt_send_frame(h: *mut DipsAltHandle, frame_rgba: *const u8, len: usize, snapshot: c_int,
                               out_rgba: *mut u8, cap: usize) -> DipsStatus;
    pub fn dips_alt_send_frames(h: *mut DipsAltHandle, frames: *const u8, n_frames: u32,
                                snapshot_flags: *const u8, out: *mut u8) -> DipsStatus;
    pub fn dips_alt_run(h: *mut DipsAltHandle, frames: *const u8, n_frames: u32, refresh_markers: *const u64,
                        n_markers: u32, out: *mut u8) -> DipsStatus;
    pub fn dips_alt_run_sharded(h: *mut DipsAltHandle, comm: *mut DipsComm, frames: *const u8, n_local: u32,
                                n_total: u64, refresh_markers: *const u64, n_markers: u32, out: *mut u8)
                                -> DipsStatus;
    pub fn dips_alt_snapshot_texture(h: *mut DipsAltHandle, out_gray: *mut u8, cap: usize) -> DipsStatus;
    pub fn dips_alt_kernel_time(h: *mut DipsAltHandle, total_ms: *mut f64, launches: *mut u64) -> DipsStatus;
    pub fn dips_alt_kernel_time_reset(h: *mut DipsAltHandle) -> DipsStatus;
    pub fn dips_alt_lut_selfcheck(h: *mut DipsAltHandle, mismatches: *mut u64) -> DipsStatus;
    pub fn dips_alt_lut_index(l1: *mut u32, l1_cap: u32, diffs: *mut f32, slots: *mut u16, cap: u32,
                              n_diffs: *mut u32, l2_entries: *mut u32) -> DipsStatus;
}
