//! Safe Rust face of `libdips_hip.so`, the MI355X drop-in for the DiPs
//! crates' GPU operators.  The reference reaches its operator only through
//! `type CallbackFunction = fn(u32, u32, &[u8], &mut ComputeState) -> Vec<u8>`
//! (dips/src/lib.rs:23) and `ComputeState::{new, add_texture, dispatch}`
//! (dips/src/gpu/mod.rs:59, :170, :306; dips_opencv/src/gpu/mod.rs:59, :172,
//! :308).  This crate keeps those names, argument meanings and error
//! behaviour, so `dips/src/gpu/mod.rs` becomes `pub use dips_hip::ComputeState;`
//! and `frame_callback` (lib.rs:233-246) keeps working unchanged.  It adds the
//! north star's per-frame difference series (`DiffSeries`) and the dips_alt
//! operator (`DiPsCompute`, dips_alt/src/dips_compute/mod.rs:243-647).
//!
//! Every call goes through `ffi` (include/dips_hip.h); no CPU fallback
//! exists.  Failure contract: the library never unwinds into Rust (every C++
//! exception is caught at the boundary and returned as a status,
//! `DIPS_ERR_INTERNAL` / `DIPS_ERR_NOMEM`); this crate never unwinds into
//! the library.  The `try_*` methods return every failure as a `DipsError`;
//! the reference-shaped methods keep the reference's signatures and panic
//! where its wgpu path panics (a device error), so `None` from `dispatch`
//! means the warm-up only and `frame_callback` never passes the input
//! through on an error.

pub mod ffi;

use core::ffi::{c_int, CStr};
use core::ptr::{self, NonNull};
use std::fmt;

/// dips/src/lib.rs:25-41; `Into<f64>` gives the WGSL override id 3 code.
#[derive(Copy, Clone, Debug, PartialEq, Eq)]
pub enum DiPsFilter {
    Unfiltered,
    Sigmoid,
    InverseSigmoid,
}

impl From<DiPsFilter> for f64 {
    fn from(f: DiPsFilter) -> f64 {
        f.code() as f64
    }
}

impl DiPsFilter {
    pub fn code(self) -> u32 {
        match self {
            DiPsFilter::Unfiltered => ffi::DIPS_FILTER_UNFILTERED,
            DiPsFilter::Sigmoid => ffi::DIPS_FILTER_SIGMOID,
            DiPsFilter::InverseSigmoid => ffi::DIPS_FILTER_INVERSE_SIGMOID,
        }
    }
}

/// dips/src/lib.rs:43-61; `Into<f64>` gives the WGSL override id 4 code.
#[derive(Copy, Clone, Debug, PartialEq, Eq)]
pub enum ChromaFilter {
    None,
    Red,
    Green,
    Blue,
}

impl From<ChromaFilter> for f64 {
    fn from(c: ChromaFilter) -> f64 {
        c.code() as f64
    }
}

impl ChromaFilter {
    pub fn code(self) -> u32 {
        match self {
            ChromaFilter::None => ffi::DIPS_CHROMA_NONE,
            ChromaFilter::Red => ffi::DIPS_CHROMA_RED,
            ChromaFilter::Green => ffi::DIPS_CHROMA_GREEN,
            ChromaFilter::Blue => ffi::DIPS_CHROMA_BLUE,
        }
    }
}

/// A failed call: the status code and the library's message for it.
#[derive(Debug, Clone)]
pub struct DipsError {
    pub status: ffi::DipsStatus,
    pub message: String,
}

impl fmt::Display for DipsError {
    fn fmt(&self, f: &mut fmt::Formatter<'_>) -> fmt::Result {
        write!(f, "dips status {}: {}", self.status, self.message)
    }
}

impl std::error::Error for DipsError {}

fn message(p: *const core::ffi::c_char) -> String {
    if p.is_null() {
        return String::new();
    }
    // SAFETY: the library returns a NUL-terminated string it owns.
    unsafe { CStr::from_ptr(p) }.to_string_lossy().into_owned()
}

fn check(st: c_int, h: *const ffi::DipsHandle) -> Result<c_int, DipsError> {
    if st >= 0 {
        Ok(st)
    } else {
        // SAFETY: h is a live handle or null (the last creation error).
        Err(DipsError { status: st, message: message(unsafe { ffi::dips_last_error(h) }) })
    }
}

fn check_alt(st: c_int, h: *const ffi::DipsAltHandle) -> Result<c_int, DipsError> {
    if st >= 0 {
        Ok(st)
    } else {
        // SAFETY: as in `check`.
        Err(DipsError { status: st, message: message(unsafe { ffi::dips_alt_last_error(h) }) })
    }
}

/// The library this crate was written against (a stale or newer
/// `libdips_hip.so` is refused, not half-used).
fn check_abi() -> Result<(), DipsError> {
    // SAFETY: no arguments.
    let v = unsafe { ffi::dips_abi_version() };
    if v == ffi::DIPS_ABI_VERSION {
        Ok(())
    } else {
        Err(DipsError { status: ffi::DIPS_ERR_STATE,
                        message: format!("libdips_hip.so has ABI {v}, this crate expects {}", ffi::DIPS_ABI_VERSION) })
    }
}

fn create(p: &ffi::DipsParams, device: i32) -> Result<NonNull<ffi::DipsHandle>, DipsError> {
    check_abi()?;
    let mut h = ptr::null_mut();
    // SAFETY: p is a valid dips_params, h an out pointer.
    check(unsafe { ffi::dips_create(p, device, &mut h) }, ptr::null())?;
    NonNull::new(h).ok_or(DipsError { status: ffi::DIPS_ERR_STATE, message: "null handle".into() })
}

fn default_params() -> ffi::DipsParams {
    let mut p = ffi::DipsParams::default();
    // SAFETY: fills a caller-owned struct.
    unsafe { ffi::dips_params_default(&mut p) };
    p
}

/// Drop-in for `ComputeState` (dips/src/gpu/mod.rs): the 4-slot temporal
/// median, start texture, filter and visual epilogue on a HIP device.
pub struct ComputeState {
    h: NonNull<ffi::DipsHandle>,
    width: u32,
    height: u32,
}

// Used from the GStreamer streaming thread under the RwLock of
// dips/src/frame_extractor.rs:232: one call at a time, the handle may move.
unsafe impl Send for ComputeState {}

impl ComputeState {
    /// gpu/mod.rs:59-65.  The reference returns `anyhow::Result<Self>`; a
    /// `DipsError` converts with `?`.
    pub fn new(colorize: bool, spatial_window_size: i32, sensitivity: f32, filter_type: DiPsFilter,
               chroma_filter: ChromaFilter) -> Result<Self, DipsError> {
        Self::on_device(colorize, spatial_window_size, sensitivity, filter_type, chroma_filter, 0)
    }

    pub fn on_device(colorize: bool, spatial_window_size: i32, sensitivity: f32, filter_type: DiPsFilter,
                     chroma_filter: ChromaFilter, device: i32) -> Result<Self, DipsError> {
        let mut p = default_params();
        p.colorize = colorize as u8;
        p.spatial_window_size = spatial_window_size;
        p.sensitivity = sensitivity;
        p.filter_type = filter_type.code();
        p.chroma_filter = chroma_filter.code();
        p.format = ffi::DIPS_FMT_RGBA8; // the appsink caps (frame_extractor.rs:141-148)
        Ok(Self { h: create(&p, device)?, width: 0, height: 0 })
    }

    fn frame_bytes(&self) -> usize {
        self.width as usize * self.height as usize * 4
    }

    /// gpu/mod.rs:170-216.  Returns `()` like the reference, which swallows
    /// its errors (:189, :206); `try_add_texture` reports them.
    pub fn add_texture(&mut self, width: u32, height: u32, frame_data: &[u8]) {
        let _ = self.try_add_texture(width, height, frame_data);
    }

    pub fn try_add_texture(&mut self, width: u32, height: u32, frame_data: &[u8]) -> Result<(), DipsError> {
        // SAFETY: the frame is borrowed for the call only (read before return).
        let st = unsafe {
            ffi::dips_add_texture(self.h.as_ptr(), width, height, frame_data.as_ptr(), frame_data.len())
        };
        check(st, self.h.as_ptr())?;
        self.width = width;
        self.height = height;
        Ok(())
    }

    /// gpu/mod.rs:306-397: `Ok(None)` while the ring warms up (frames 0..2),
    /// `Ok(Some(frame))` after, `Err` on any failure.
    pub fn try_dispatch(&mut self) -> Result<Option<Vec<u8>>, DipsError> {
        let mut out = vec![0u8; self.frame_bytes()];
        // SAFETY: out has cap bytes.
        let r = unsafe { ffi::dips_dispatch(self.h.as_ptr(), out.as_mut_ptr(), out.len()) };
        match check(r, self.h.as_ptr())? {
            1 => Ok(Some(out)),
            _ => Ok(None),
        }
    }

    /// gpu/mod.rs:306-397 with the reference's signature: `None` only while
    /// the ring warms up (:394-396).  Panics on a device or argument error,
    /// as the reference's wgpu calls do; use `try_dispatch` to handle it.
    pub fn dispatch(&mut self) -> Option<Vec<u8>> {
        match self.try_dispatch() {
            Ok(v) => v,
            Err(e) => panic!("ComputeState::dispatch: {e}"),
        }
    }

    /// `frame_callback` (lib.rs:233-246) into a caller buffer (reused across
    /// frames: no allocation per call).  `Ok(true)` = dispatched output,
    /// `Ok(false)` = the input passed through (warm-up frames).
    pub fn frame_callback_into(&mut self, width: u32, height: u32, frame_data: &[u8], out: &mut [u8])
                               -> Result<bool, DipsError> {
        // SAFETY: both buffers are caller-owned for the call's duration.
        let r = unsafe {
            ffi::dips_frame_callback(self.h.as_ptr(), width, height, frame_data.as_ptr(), frame_data.len(),
                                     out.as_mut_ptr(), out.len())
        };
        let r = check(r, self.h.as_ptr())?;
        self.width = width;
        self.height = height;
        Ok(r == 1)
    }

    /// `n` consecutive frame_callback calls in one device pass: `frames` and
    /// `out` hold n RGBA8 frames back to back.
    pub fn frame_callback_batch(&mut self, width: u32, height: u32, frames: &[u8], out: &mut [u8])
                                -> Result<(), DipsError> {
        let fb = width as usize * height as usize * 4;
        if fb == 0 || frames.len() % fb != 0 || out.len() < frames.len() {
            return Err(DipsError { status: ffi::DIPS_ERR_INVALID, message: "frames/out not n RGBA8 frames".into() });
        }
        let n = frame_count(frames.len() / fb)?;
        // SAFETY: sizes checked above.
        let st = unsafe {
            ffi::dips_frame_callback_batch(self.h.as_ptr(), width, height, frames.as_ptr(), n, out.as_mut_ptr())
        };
        check(st, self.h.as_ptr())?;
        self.width = width;
        self.height = height;
        Ok(())
    }

    /// Where the last zero-copy `frame_callback` spent its time
    /// (dips_callback_phases: sync, staged, launched, kernels, wall, pack /
    /// expand / wait CPU sums in microseconds, pool threads, stripes, expand
    /// start).
    pub fn callback_phases(&self) -> Option<[f64; ffi::DIPS_CALLBACK_PHASES as usize]> {
        let mut v = [0f64; ffi::DIPS_CALLBACK_PHASES as usize];
        let mut n = 0u32;
        // SAFETY: v has cap entries.
        let st = unsafe { ffi::dips_callback_phases(self.h.as_ptr(), v.as_mut_ptr(), v.len() as u32, &mut n) };
        if st == ffi::DIPS_OK { Some(v) } else { None }
    }

    /// The start texture S (pre_compute_shader.wgsl:92-132): `Ok(None)`
    /// until the 4th frame has built it.
    pub fn try_start_texture(&mut self) -> Result<Option<Vec<u8>>, DipsError> {
        let mut out = vec![0u8; self.frame_bytes()];
        // SAFETY: out has cap bytes.
        let r = unsafe { ffi::dips_start_texture(self.h.as_ptr(), out.as_mut_ptr(), out.len()) };
        match check(r, self.h.as_ptr())? {
            1 => Ok(Some(out)),
            _ => Ok(None),
        }
    }

    /// `try_start_texture`, panicking on an error (`None`: not built yet).
    pub fn start_texture(&mut self) -> Option<Vec<u8>> {
        match self.try_start_texture() {
            Ok(v) => v,
            Err(e) => panic!("ComputeState::start_texture: {e}"),
        }
    }

    /// `frame_callback` over this rank's frames of a video sharded by frame
    /// range over `comm` (a fresh ComputeState on every rank): the outputs
    /// one ComputeState over all `n_total` frames gives them; the library
    /// broadcasts the start texture and passes each rank's last three frames
    /// to the next (every rank after the first starts at frame >= 7).
    pub fn frame_callback_batch_sharded(&mut self, comm: &mut Comm, width: u32, height: u32, frames: &[u8],
                                        n_total: u64, out: &mut [u8]) -> Result<(), DipsError> {
        let fb = width as usize * height as usize * 4;
        if fb == 0 || frames.len() % fb != 0 || out.len() < frames.len() {
            return Err(DipsError { status: ffi::DIPS_ERR_INVALID, message: "frames/out not n RGBA8 frames".into() });
        }
        let n = frame_count(frames.len() / fb)?;
        // SAFETY: sizes checked above; the call is collective over `comm`.
        let st = unsafe {
            ffi::dips_frame_callback_batch_sharded(self.h.as_ptr(), comm.c.as_ptr(), width, height, frames.as_ptr(),
                                                   n, n_total, out.as_mut_ptr())
        };
        check(st, self.h.as_ptr())?;
        self.width = width;
        self.height = height;
        Ok(())
    }

    /// Continue as if frame_callback had seen frames 0..t0-1 (t0 >= 7): the
    /// start texture of the process that saw frames 0..3 and the raw frames
    /// t0-3..t0-1 (frame-range sharding, one decoder per GPU).
    pub fn resume(&mut self, width: u32, height: u32, start: &[u8], halo: &[u8], t0: u64) -> Result<(), DipsError> {
        let fb = width as usize * height as usize * 4;
        if start.len() != fb || halo.len() != 3 * fb {
            return Err(DipsError { status: ffi::DIPS_ERR_INVALID, message: "start: 1 frame, halo: 3 frames".into() });
        }
        // SAFETY: sizes checked above.
        let st = unsafe {
            ffi::dips_compat_resume(self.h.as_ptr(), width, height, start.as_ptr(), halo.as_ptr(), t0)
        };
        check(st, self.h.as_ptr())?;
        self.width = width;
        self.height = height;
        Ok(())
    }
}

impl Drop for ComputeState {
    fn drop(&mut self) {
        // SAFETY: the handle is live and dropped once.
        unsafe { ffi::dips_destroy(self.h.as_ptr()) }
    }
}

/// dips/src/lib.rs:233-246, the `CallbackFunction` the GStreamer appsink
/// closure calls (frame_extractor.rs:232-240): add_texture, then dispatch
/// or the input passed through while the ring warms up.  One ABI call per
/// frame (dips_frame_callback overlaps the upload, the kernel and the
/// readback in row stripes).  An error panics, as the reference's wgpu path
/// does -- it is never disguised as the warm-up passthrough; callers that
/// handle errors use `ComputeState::frame_callback_into`.
pub fn frame_callback(width: u32, height: u32, frame_data: &[u8], compute: &mut ComputeState) -> Vec<u8> {
    let mut out = vec![0u8; frame_data.len()];
    match compute.frame_callback_into(width, height, frame_data, &mut out) {
        Ok(_) => out,
        Err(e) => panic!("frame_callback: {e}"),
    }
}

/// Pixel format of the series path.
#[derive(Copy, Clone, Debug, PartialEq, Eq)]
pub enum PixelFormat {
    Gray8,
    Rgb8,
    Rgba8,
}

impl PixelFormat {
    pub fn code(self) -> u32 {
        match self {
            PixelFormat::Gray8 => ffi::DIPS_FMT_GRAY8,
            PixelFormat::Rgb8 => ffi::DIPS_FMT_RGB8,
            PixelFormat::Rgba8 => ffi::DIPS_FMT_RGBA8,
        }
    }
    pub fn channels(self) -> usize {
        self.code() as usize
    }
}

/// README.md:7-11: against frame 0 (or a given reference) or the previous frame.
#[derive(Copy, Clone, Debug, PartialEq, Eq)]
pub enum Mode {
    Overall,
    PerFrame,
}

/// The per-frame difference series (north star): exact SAD and J sums, the
/// threshold count and the exact intensity sum of every frame.
pub struct DiffSeries {
    h: NonNull<ffi::DipsHandle>,
    format: PixelFormat,
}

unsafe impl Send for DiffSeries {}

impl DiffSeries {
    pub fn new(format: PixelFormat, mode: Mode, tau: f32, chroma_filter: ChromaFilter, device: i32)
               -> Result<Self, DipsError> {
        let mut p = default_params();
        p.format = format.code();
        p.mode = match mode {
            Mode::Overall => ffi::DIPS_MODE_OVERALL,
            Mode::PerFrame => ffi::DIPS_MODE_PER_FRAME,
        };
        p.tau = tau;
        p.chroma_filter = chroma_filter.code();
        Ok(Self { h: create(&p, device)?, format })
    }

    fn frame_bytes(&self, width: u32, height: u32) -> usize {
        width as usize * height as usize * self.format.channels()
    }

    fn frames_of(&self, width: u32, height: u32, frames: &[u8]) -> Result<u32, DipsError> {
        let fb = self.frame_bytes(width, height);
        if fb == 0 || frames.len() % fb != 0 {
            return Err(DipsError { status: ffi::DIPS_ERR_INVALID, message: "frames: n whole frames".into() });
        }
        frame_count(frames.len() / fb)
    }

    /// The C ABI takes no length for the reference and reads one whole frame
    /// from it: anything but exactly one frame is refused here.
    fn reference_ptr(&self, width: u32, height: u32, reference: Option<&[u8]>) -> Result<*const u8, DipsError> {
        match reference {
            None => Ok(ptr::null()),
            Some(r) if r.len() == self.frame_bytes(width, height) => Ok(r.as_ptr()),
            Some(_) => Err(DipsError { status: ffi::DIPS_ERR_INVALID, message: "reference: one whole frame".into() }),
        }
    }

    /// Series of host frames (staged through HBM); `reference` = None uses
    /// frame 0 ('overall') or each frame's predecessor ('per-frame').
    /// `absdiff_map`, if given, receives |F_t - R| (frames.len() bytes).
    pub fn run(&mut self, width: u32, height: u32, frames: &[u8], reference: Option<&[u8]>,
               absdiff_map: Option<&mut [u8]>) -> Result<Vec<ffi::DipsSeriesEntry>, DipsError> {
        let n = self.frames_of(width, height, frames)?;
        let ref_ptr = self.reference_ptr(width, height, reference)?;
        let mut series = vec![ffi::DipsSeriesEntry::default(); n as usize];
        let map_ptr = match absdiff_map {
            Some(m) if m.len() >= frames.len() => m.as_mut_ptr(),
            Some(_) => return Err(DipsError { status: ffi::DIPS_ERR_CAPACITY, message: "map too small".into() }),
            None => ptr::null_mut(),
        };
        // SAFETY: sizes checked; every buffer is caller-owned for the call.
        let st = unsafe {
            ffi::dips_diff_series(self.h.as_ptr(), width, height, frames.as_ptr(), n, ref_ptr, series.as_mut_ptr(),
                                  map_ptr)
        };
        check(st, self.h.as_ptr())?;
        Ok(series)
    }

    /// The same from pageable host memory through pinned staging and a side
    /// stream (the PCIe-bound end-to-end feed).
    pub fn run_streamed(&mut self, width: u32, height: u32, frames: &[u8], reference: Option<&[u8]>,
                        chunk_frames: u32) -> Result<Vec<ffi::DipsSeriesEntry>, DipsError> {
        let n = self.frames_of(width, height, frames)?;
        let ref_ptr = self.reference_ptr(width, height, reference)?;
        let mut series = vec![ffi::DipsSeriesEntry::default(); n as usize];
        // SAFETY: as in `run`.
        let st = unsafe {
            ffi::dips_diff_series_streamed(self.h.as_ptr(), width, height, frames.as_ptr(), n, ref_ptr,
                                           series.as_mut_ptr(), chunk_frames)
        };
        check(st, self.h.as_ptr())?;
        Ok(series)
    }
}

impl DiffSeries {
    /// Frame-range sharding over `comm` (dips_diff_series_sharded): this
    /// rank's host frames -- its `shard_range(n_total, ..)` -- give this
    /// rank's series entries and, on rank 0, the whole gathered series (the
    /// same as one `run` over all n_total frames).  `reference`: 'overall'
    /// rank 0's reference (None = its first frame), broadcast to every rank;
    /// 'per-frame' rank 0's predecessor of frame 0 (None = frame 0), the
    /// other ranks get theirs from rank r-1.  Every rank calls this with the
    /// same n_total, like a collective.
    pub fn run_sharded(&mut self, comm: &mut Comm, width: u32, height: u32, frames: &[u8], n_total: u64,
                       reference: Option<&[u8]>)
                       -> Result<(Vec<ffi::DipsSeriesEntry>, Option<Vec<ffi::DipsSeriesEntry>>), DipsError> {
        let n = self.frames_of(width, height, frames)?;
        let ref_ptr = self.reference_ptr(width, height, reference)?;
        let mut local = vec![ffi::DipsSeriesEntry::default(); n as usize];
        let mut all = if comm.rank == 0 {
            let total = usize::try_from(n_total)
                .map_err(|_| DipsError { status: ffi::DIPS_ERR_INVALID, message: "n_total too large".into() })?;
            Some(vec![ffi::DipsSeriesEntry::default(); total])
        } else {
            None
        };
        let all_ptr = all.as_mut().map_or(ptr::null_mut(), |v| v.as_mut_ptr());
        // SAFETY: sizes checked; every buffer is caller-owned for the call (host
        // pointers: the call returns with the results in them).
        let st = unsafe {
            ffi::dips_diff_series_sharded(self.h.as_ptr(), comm.c.as_ptr(), width, height, frames.as_ptr(), n,
                                          n_total, ref_ptr, 0, local.as_mut_ptr(), all_ptr)
        };
        check(st, self.h.as_ptr())?;
        Ok((local, all))
    }
}

/// One rank's communicator of the sharded series (dips_comm_*): RCCL over
/// xGMI across processes, or loopback ranks as threads of one process.
pub struct Comm {
    c: NonNull<ffi::DipsComm>,
    pub nranks: i32,
    pub rank: i32,
}

// A communicator is driven by one thread at a time and may move between them.
unsafe impl Send for Comm {}

fn check_comm(st: c_int, c: *const ffi::DipsComm) -> Result<c_int, DipsError> {
    if st >= 0 {
        Ok(st)
    } else {
        // SAFETY: c is a live communicator or null (the last creation error).
        Err(DipsError { status: st, message: message(unsafe { ffi::dips_comm_last_error(c) }) })
    }
}

impl Comm {
    fn wrap(c: *mut ffi::DipsComm) -> Result<Self, DipsError> {
        let c = NonNull::new(c).ok_or(DipsError { status: ffi::DIPS_ERR_STATE, message: "null communicator".into() })?;
        let (mut kind, mut nranks, mut rank) = (0, 0, 0);
        // SAFETY: c is live; the outputs are locals.
        check_comm(unsafe { ffi::dips_comm_info(c.as_ptr(), &mut kind, &mut nranks, &mut rank) }, c.as_ptr())?;
        Ok(Self { c, nranks, rank })
    }

    /// A new RCCL unique id: rank 0 makes it and hands it to every rank.
    pub fn unique_id() -> Result<[u8; ffi::DIPS_COMM_ID_BYTES as usize], DipsError> {
        check_abi()?;
        let mut id = [0u8; ffi::DIPS_COMM_ID_BYTES as usize];
        // SAFETY: id has DIPS_COMM_ID_BYTES bytes.
        check_comm(unsafe { ffi::dips_comm_unique_id(id.as_mut_ptr()) }, ptr::null())?;
        Ok(id)
    }

    /// Join the RCCL communicator `id` as `rank` of `nranks` on `device`.
    pub fn rccl(id: &[u8; ffi::DIPS_COMM_ID_BYTES as usize], nranks: i32, rank: i32, device: i32)
                -> Result<Self, DipsError> {
        check_abi()?;
        let mut c = ptr::null_mut();
        // SAFETY: id has DIPS_COMM_ID_BYTES bytes, c is an out pointer.
        check_comm(unsafe { ffi::dips_comm_create(id.as_ptr(), nranks, rank, device, &mut c) }, ptr::null())?;
        Self::wrap(c)
    }

    /// Every rank of an RCCL communicator in this process (ncclCommInitAll),
    /// rank r on `devices[r]`: one process driving every GPU of the node, one
    /// thread per rank.
    pub fn rccl_all(devices: &[i32]) -> Result<Vec<Self>, DipsError> {
        check_abi()?;
        let n = i32::try_from(devices.len())
            .map_err(|_| DipsError { status: ffi::DIPS_ERR_INVALID, message: "too many devices".into() })?;
        let mut cs = vec![ptr::null_mut(); devices.len()];
        // SAFETY: devices and cs both have n entries.
        check_comm(unsafe { ffi::dips_comm_create_all(n, devices.as_ptr(), cs.as_mut_ptr()) }, ptr::null())?;
        cs.into_iter().map(Self::wrap).collect()
    }

    /// `nranks` loopback ranks on `device`; each must be driven by its own
    /// thread (their collectives meet on the host).
    pub fn loopback(nranks: i32, device: i32) -> Result<Vec<Self>, DipsError> {
        check_abi()?;
        let count = usize::try_from(nranks)
            .map_err(|_| DipsError { status: ffi::DIPS_ERR_INVALID, message: "nranks < 0".into() })?;
        let mut cs = vec![ptr::null_mut(); count];
        // SAFETY: cs has nranks slots.
        check_comm(unsafe { ffi::dips_comm_create_loopback(nranks, device, cs.as_mut_ptr()) }, ptr::null())?;
        cs.into_iter().map(Self::wrap).collect()
    }
}

impl Drop for Comm {
    fn drop(&mut self) {
        // SAFETY: the communicator is live and dropped once.
        unsafe { ffi::dips_comm_destroy(self.c.as_ptr()) }
    }
}

/// Global frames [first, first + count) of `rank` of `nranks` over n_total.
pub fn shard_range(n_total: u64, nranks: i32, rank: i32) -> Result<(u64, u32), DipsError> {
    let (mut first, mut count) = (0u64, 0u32);
    // SAFETY: the outputs are locals.
    let st = unsafe { ffi::dips_shard_range(n_total, nranks, rank, &mut first, &mut count) };
    if st == ffi::DIPS_OK {
        Ok((first, count))
    } else {
        Err(DipsError { status: st, message: "rank outside [0, nranks)".into() })
    }
}

impl Drop for DiffSeries {
    fn drop(&mut self) {
        // SAFETY: the handle is live and dropped once.
        unsafe { ffi::dips_destroy(self.h.as_ptr()) }
    }
}

/// f64 intensity sum of a series entry (si_fixed * 2^-32).
pub fn series_si(e: &ffi::DipsSeriesEntry) -> f64 {
    // SAFETY: reads the entry only.
    unsafe { ffi::dips_series_si(e) }
}

/// dips_alt's DiPsProperties (dips_alt/src/dips_compute/mod.rs:151-234).
#[derive(Copy, Clone, Debug)]
pub struct AltProperties {
    pub colorize: bool,
    pub window_size: u32,
    pub sigmoid_horizontal_scalar: f32,
    pub filter_type: DiPsFilter,
    pub chroma_filter: ChromaFilter,
}

impl Default for AltProperties {
    /// mod.rs:176-186.
    fn default() -> Self {
        Self { colorize: true, window_size: 1, sigmoid_horizontal_scalar: 5.0, filter_type: DiPsFilter::Sigmoid,
               chroma_filter: ChromaFilter::None }
    }
}

/// Drop-in for dips_alt's `DiPsCompute` (mod.rs:243-647) without the
/// window surface (rendering is out of scope).
pub struct DiPsCompute {
    h: NonNull<ffi::DipsAltHandle>,
    bytes: usize,
}

unsafe impl Send for DiPsCompute {}

impl DiPsCompute {
    /// mod.rs:270-496.  The reference passes (rows, cols) in its
    /// `textures_width, textures_height` slots (lib.rs:596-603); kept here.
    pub fn new(num_textures: usize, textures_width: u32, textures_height: u32, props: AltProperties)
               -> Result<Self, DipsError> {
        let mut p = ffi::DipsAltParams::default();
        // SAFETY: fills a caller-owned struct.
        unsafe { ffi::dips_alt_params_default(&mut p) };
        p.colorize = props.colorize as u8;
        p.window_size = props.window_size as i32;
        p.sigmoid_horizontal_scalar = props.sigmoid_horizontal_scalar;
        p.filter_type = props.filter_type.code();
        p.chroma_filter = props.chroma_filter.code();
        p.num_textures = num_textures as u32;
        let (rows, cols) = (textures_width, textures_height);
        check_abi()?;
        let mut h = ptr::null_mut();
        // SAFETY: p valid, h an out pointer.
        check_alt(unsafe { ffi::dips_alt_create(&p, cols, rows, 0, &mut h) }, ptr::null())?;
        let h = NonNull::new(h).ok_or(DipsError { status: ffi::DIPS_ERR_STATE, message: "null handle".into() })?;
        Ok(Self { h, bytes: rows as usize * cols as usize * 4 })
    }

    /// mod.rs:498-646: the RGBA8 output texture of this frame.
    pub fn send_frame(&mut self, frame: &[u8], snapshot: Option<()>) -> Result<Vec<u8>, DipsError> {
        let mut out = vec![0u8; self.bytes];
        // SAFETY: out has cap bytes; the frame is read before return.
        let st = unsafe {
            ffi::dips_alt_send_frame(self.h.as_ptr(), frame.as_ptr(), frame.len(), snapshot.is_some() as c_int,
                                     out.as_mut_ptr(), out.len())
        };
        check_alt(st, self.h.as_ptr())?;
        Ok(out)
    }

    /// The frame loop of run_dips_on_file (lib.rs:588-683) over n frames
    /// back to back; the loop state persists across calls.
    pub fn run(&mut self, frames: &[u8], refresh_markers: &[u64], out: &mut [u8]) -> Result<(), DipsError> {
        if self.bytes == 0 || frames.len() % self.bytes != 0 || out.len() < frames.len() {
            return Err(DipsError { status: ffi::DIPS_ERR_INVALID, message: "frames/out not n frames".into() });
        }
        let n = frame_count(frames.len() / self.bytes)?;
        let n_markers = u32::try_from(refresh_markers.len())
            .map_err(|_| DipsError { status: ffi::DIPS_ERR_INVALID, message: "too many refresh markers".into() })?;
        // SAFETY: sizes checked above.
        let st = unsafe {
            ffi::dips_alt_run(self.h.as_ptr(), frames.as_ptr(), n,
                              if refresh_markers.is_empty() { ptr::null() } else { refresh_markers.as_ptr() },
                              n_markers, out.as_mut_ptr())
        };
        check_alt(st, self.h.as_ptr())?;
        Ok(())
    }

    /// This rank's frames of one run_dips_on_file loop over an n_total-frame
    /// video split by frame range over `comm` (shard_range); collective, on
    /// a fresh DiPsCompute of every rank.
    pub fn run_sharded(&mut self, comm: &mut Comm, frames: &[u8], n_total: u64, refresh_markers: &[u64],
                       out: &mut [u8]) -> Result<(), DipsError> {
        if self.bytes == 0 || frames.len() % self.bytes != 0 || out.len() < frames.len() {
            return Err(DipsError { status: ffi::DIPS_ERR_INVALID, message: "frames/out not n frames".into() });
        }
        let n = frame_count(frames.len() / self.bytes)?;
        let n_markers = u32::try_from(refresh_markers.len())
            .map_err(|_| DipsError { status: ffi::DIPS_ERR_INVALID, message: "too many refresh markers".into() })?;
        // SAFETY: sizes checked above; the call is collective over `comm`.
        let st = unsafe {
            ffi::dips_alt_run_sharded(self.h.as_ptr(), comm.c.as_ptr(), frames.as_ptr(), n, n_total,
                                      if refresh_markers.is_empty() { ptr::null() } else { refresh_markers.as_ptr() },
                                      n_markers, out.as_mut_ptr())
        };
        check_alt(st, self.h.as_ptr())?;
        Ok(())
    }
}

impl Drop for DiPsCompute {
    fn drop(&mut self) {
        // SAFETY: the handle is live and dropped once.
        unsafe { ffi::dips_alt_destroy(self.h.as_ptr()) }
    }
}

/// A frame count as the ABI's u32 (a batch of 2^32 or more frames is refused,
/// not truncated).
fn frame_count(n: usize) -> Result<u32, DipsError> {
    u32::try_from(n).map_err(|_| DipsError { status: ffi::DIPS_ERR_INVALID, message: "too many frames".into() })
}

/// The ABI version the library was built with (ffi::DIPS_ABI_VERSION expected).
pub fn abi_version() -> i32 {
    // SAFETY: no arguments.
    unsafe { ffi::dips_abi_version() }
}
