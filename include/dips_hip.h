/*
 * dips_hip.h -- C ABI of the MI355X-native DiPs frame-difference path.
 *
 * This is the drop-in boundary.  The reference crate (RubenMovsesyan/DiPs,
 * Rust) reaches its GPU operator only through
 *     type CallbackFunction = fn(u32, u32, &[u8], &mut ComputeState) -> Vec<u8>
 * (dips/src/lib.rs:23) and the three ComputeState methods new / add_texture /
 * dispatch (dips/src/gpu/mod.rs:59, :170, :306; identical copies in
 * dips_opencv/src/gpu/mod.rs:59, :172, :308).  Each entry point below names
 * the reference item it replaces.  Everything is plain C: pointers, sizes,
 * status codes.  No exception or panic crosses this boundary.
 *
 * Threading: a handle is not internally synchronised (the reference uses
 * ComputeState under an RwLock write guard, dips/src/frame_extractor.rs:232);
 * a handle may move between threads.  The caller owns every buffer.  Every
 * entry point leaves the calling thread's current HIP device as it found it
 * (work runs on the handle's device).
 */
#ifndef DIPS_HIP_H
#define DIPS_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DIPS_ABI_VERSION 3

typedef enum dips_status {
    DIPS_OK = 0,
    DIPS_ERR_INVALID = -1,  /* bad argument / shape / parameter */
    DIPS_ERR_HIP = -2,      /* HIP runtime error (see dips_last_error) */
    DIPS_ERR_STATE = -3,    /* call not valid in the handle's state */
    DIPS_ERR_NOMEM = -4,    /* device or host allocation failed */
    DIPS_ERR_CAPACITY = -5, /* caller's output buffer too small */
    DIPS_ERR_NODEVICE = -6, /* no HIP device / device index out of range */
    DIPS_ERR_INTERNAL = -7, /* a C++ exception inside the library, caught at the
                               boundary (see dips_last_error); the handle may
                               be left mid-call and should be destroyed */
    DIPS_ERR_COMM = -8      /* a communicator's transport failed (RCCL error,
                               a loopback rank that never arrived, a host
                               transport callback's non-zero return) */
} dips_status;

/* DiPsFilter -> override id 3 (dips/src/lib.rs:25-41, dips_shader.wgsl:20). */
#define DIPS_FILTER_SIGMOID 0u
#define DIPS_FILTER_INVERSE_SIGMOID 1u
#define DIPS_FILTER_UNFILTERED 255u
/* ChromaFilter -> override id 4 (dips/src/lib.rs:43-61, dips_shader.wgsl:21). */
#define DIPS_CHROMA_NONE 0u
#define DIPS_CHROMA_RED 1u
#define DIPS_CHROMA_GREEN 2u
#define DIPS_CHROMA_BLUE 3u

/* Pixel formats of the series path (the compat path is RGBA8 only, like the
 * reference's appsink caps, dips/src/frame_extractor.rs:141-148). */
#define DIPS_FMT_GRAY8 1u
#define DIPS_FMT_RGB8 3u
#define DIPS_FMT_RGBA8 4u

/* Reference choice of the series path (README.md:7-11). */
#define DIPS_MODE_OVERALL 0u   /* against frame 0 (or the given reference) */
#define DIPS_MODE_PER_FRAME 1u /* against the previous frame */

/* dips_params.flags */
#define DIPS_FLAG_DEVICE_PTRS 0x1u /* series pointers are device (HBM) pointers */
#define DIPS_FLAG_TIME_KERNEL 0x2u /* record hipEvents around the series kernel */
#define DIPS_FLAG_FORCE_GENERIC 0x4u /* use the generic (any-shape) series kernel */
/* Cross-check forms: the same results through the plain kernels instead of
 * the specialised ones -- GRAY8 series: the f32 kernel, not the table kernel;
 * RGB8 / RGBA8 series: the exact f64 intensity sum at every tau, not the
 * integer sum of tau >= 2^-5; dips-compat / dips_alt batches: the per-pixel
 * arithmetic epilogue, not the epilogue table; the per-frame calls: whole
 * RGBA8 frames through the DMA staging (add_texture + dispatch), not the
 * striped zero-copy pipeline with compact transfers.  For tests and
 * A/B checks; slower. */
#define DIPS_FLAG_CROSSCHECK 0x8u
/* GRAY8 series: pin the table kernel's layout instead of its per-workgroup
 * choice from the content it walks (series_gray.hip layout 4) -- the table
 * keyed by (a ^ b, a) with the band clamp (BAND: fastest on consecutive video
 * frames) or by (a, b) (PAIR: fastest on flat or i.i.d. random content).
 * Same results either way; both set = BAND. */
#define DIPS_FLAG_GRAY_BAND_TABLE 0x10u
#define DIPS_FLAG_GRAY_PAIR_TABLE 0x20u

/* Operator parameters.  The first five mirror ComputeState::new's arguments
 * (dips/src/gpu/mod.rs:59-65) and DiPsProperties (dips/src/lib.rs:63-86);
 * the rest configure the batch series path. */
typedef struct dips_params {
    uint8_t colorize;            /* override id 0; default 0 (lib.rs:80) */
    int32_t spatial_window_size; /* override id 1; 1..11; default 1 (lib.rs:81) */
    float sensitivity;           /* override id 2; default 5.0 (lib.rs:82) */
    uint32_t filter_type;        /* DIPS_FILTER_*; default UNFILTERED (lib.rs:83) */
    uint32_t chroma_filter;      /* DIPS_CHROMA_*; default NONE (lib.rs:84) */
    uint32_t mode;               /* DIPS_MODE_*; default OVERALL */
    uint32_t format;             /* DIPS_FMT_*; default RGB8 */
    float tau;                   /* intensity threshold, >= 0; default 0 */
    uint32_t flags;              /* DIPS_FLAG_* */
} dips_params;

/* One entry of the per-frame difference series.
 *   sad      = sum over pixels and channels of |F_t - R|          (exact)
 *   sj       = sum over pixels of |J_t - J_R|, J = max+min bytes   (exact)
 *   count    = number of pixels with dI > tau
 *   si_fixed = sum of dI over those pixels, scaled by 2^32         (exact)
 * dI = |I_t - I_R| in f32 with I = get_intensity (dips_shader.wgsl:64-82).
 * The f64 intensity sum is si_fixed * 2^-32 (dips_series_si). */
typedef struct dips_series_entry {
    uint64_t sad;
    uint64_t sj;
    uint64_t count;
    uint64_t si_fixed;
} dips_series_entry;

typedef struct dips_handle dips_handle;

/* Layouts pinned for foreign bindings: the Rust crate rust/dips-hip
 * (src/ffi.rs) asserts the same sizes and offsets on its #[repr(C)] twins. */
#ifdef __cplusplus
#define DIPS_LAYOUT_ASSERT(cond, msg) static_assert(cond, msg)
#else
#define DIPS_LAYOUT_ASSERT(cond, msg) _Static_assert(cond, msg)
#endif
DIPS_LAYOUT_ASSERT(sizeof(dips_params) == 36, "dips_params size");
DIPS_LAYOUT_ASSERT(offsetof(dips_params, colorize) == 0, "dips_params.colorize");
DIPS_LAYOUT_ASSERT(offsetof(dips_params, spatial_window_size) == 4, "dips_params.spatial_window_size");
DIPS_LAYOUT_ASSERT(offsetof(dips_params, sensitivity) == 8, "dips_params.sensitivity");
DIPS_LAYOUT_ASSERT(offsetof(dips_params, filter_type) == 12, "dips_params.filter_type");
DIPS_LAYOUT_ASSERT(offsetof(dips_params, chroma_filter) == 16, "dips_params.chroma_filter");
DIPS_LAYOUT_ASSERT(offsetof(dips_params, mode) == 20, "dips_params.mode");
DIPS_LAYOUT_ASSERT(offsetof(dips_params, format) == 24, "dips_params.format");
DIPS_LAYOUT_ASSERT(offsetof(dips_params, tau) == 28, "dips_params.tau");
DIPS_LAYOUT_ASSERT(offsetof(dips_params, flags) == 32, "dips_params.flags");
DIPS_LAYOUT_ASSERT(sizeof(dips_series_entry) == 32, "dips_series_entry size");
DIPS_LAYOUT_ASSERT(offsetof(dips_series_entry, sad) == 0, "dips_series_entry.sad");
DIPS_LAYOUT_ASSERT(offsetof(dips_series_entry, sj) == 8, "dips_series_entry.sj");
DIPS_LAYOUT_ASSERT(offsetof(dips_series_entry, count) == 16, "dips_series_entry.count");
DIPS_LAYOUT_ASSERT(offsetof(dips_series_entry, si_fixed) == 24, "dips_series_entry.si_fixed");

/* Fill `p` with DiPsProperties::new() defaults (dips/src/lib.rs:74-86). */
dips_status dips_params_default(dips_params *p);

/* Replaces ComputeState::new (dips/src/gpu/mod.rs:59-165): binds HIP device
 * `device`, validates the parameters, creates the stream and tables. */
dips_status dips_create(const dips_params *params, int device, dips_handle **out);

/* Replaces Drop of ComputeState. */
void dips_destroy(dips_handle *h);

/* Last error message for `h` (or the last creation failure if h == NULL). */
const char *dips_last_error(const dips_handle *h);

/* Run subsequent work on `stream` (a hipStream_t; NULL = the handle's own).
 * The handle's own stream is a blocking stream: its work is ordered with the
 * legacy default stream (stream 0) both ways, so a caller whose work runs on
 * stream 0 -- torch's default stream reports cuda_stream 0, which the Python
 * wrappers pass as NULL -- needs no extra synchronisation.  Switching streams orders the new stream after all work already issued on
 * the previous one (the handle's device scratch serves both), so the previous
 * stream must still exist at the switch; setting the current stream again is
 * free.  A caller that binds an external stream and may destroy it should
 * switch back to NULL before doing so (the Python wrappers do this after
 * every call: dips_amd._lib.on_stream). */
dips_status dips_set_stream(dips_handle *h, void *stream);

/* Block until all work issued through `h` has finished. */
dips_status dips_synchronize(dips_handle *h);

/* Replaces ComputeState::add_texture (dips/src/gpu/mod.rs:170-216): queue an
 * RGBA8 host frame (len = width*height*4, stride = width*4 as at
 * bind_groups.rs:264); the 4th frame builds the start texture and the
 * temporal ring, later frames replace the ring slot.  The frame is read
 * before the call returns (borrowed, as in the reference).  In steady state
 * (window 1, host pointers) the call also starts the compute of the
 * dispatch that normally follows on the staged frame; that dispatch then
 * only collects it, and any other call first lets it finish, keeping the
 * reference's state (DIPS_FLAG_CROSSCHECK turns this off). */
dips_status dips_add_texture(dips_handle *h, uint32_t width, uint32_t height,
                             const uint8_t *frame_rgba, size_t len);

/* Replaces ComputeState::dispatch (dips/src/gpu/mod.rs:306-397): returns 1
 * and writes width*height*4 RGBA8 bytes to `out` (Some), 0 while fewer than
 * four frames were added (None), or a negative dips_status. */
int dips_dispatch(dips_handle *h, uint8_t *out_rgba, size_t cap);

/* Replaces frame_callback (dips/src/lib.rs:233-246): add_texture, then
 * dispatch; if dispatch gives None the input is copied to `out`.  Returns 1
 * when `out` holds the visualisation, 0 when it holds the passthrough copy,
 * negative on error. */
int dips_frame_callback(dips_handle *h, uint32_t width, uint32_t height,
                        const uint8_t *frame_rgba, size_t len, uint8_t *out, size_t cap);

/* `n_frames` consecutive frame_callback calls (dips/src/lib.rs:233-246) in
 * one pass: frames and out are n_frames x width*height*4 RGBA8; out[t] is
 * the visualisation, or the passthrough copy for the stream's first three
 * frames.  The first frames of a stream (start texture, unquantised ring)
 * and spatial windows W > 1 run frame by frame; the steady state (W = 1,
 * from the stream's 8th frame) runs as one HBM-streaming kernel.  With
 * DIPS_FLAG_DEVICE_PTRS both are device pointers and the call is
 * asynchronous on the handle's stream; otherwise host pointers. */
dips_status dips_frame_callback_batch(dips_handle *h, uint32_t width, uint32_t height, const uint8_t *frames,
                                      uint32_t n_frames, uint8_t *out);

/* Where the last dips_frame_callback call that took the zero-copy striped
 * path (steady state, window 1, host pointers) spent its time -- the
 * per-phase record of the per-frame call pattern (dips/src/frame_extractor.rs:
 * 206-276 -> lib.rs:233-246 -> gpu/mod.rs:170-397, whose per-frame cost is
 * what this path replaces).  Writes up to `cap` values to `us`, *n = the
 * number available (DIPS_CALLBACK_PHASES), in this order:
 *   0 sync     us from the call's start to the end of its stream syncs
 *   1 staged   .. to the last input piece packed into pinned memory
 *   2 launched .. to the last stripe's kernel launch
 *   3 kernels  .. to the last output task past its wait for its stripe's
 *              kernel (output tasks start once every input piece is taken,
 *              so this is max(kernel done, output task start))
 *   4 wall     .. to the call's return
 *   5 pack_cpu, 6 expand_cpu, 7 wait_cpu: thread-time sums (us) of the copy
 *     pool's staging tasks, output tasks and their waits for the kernels
 *   8 threads  copy-pool threads (workers + the calling thread)
 *   9 stripes  row stripes the frame was cut into
 *  10 expand   us from the call's start to the first output task's start
 * DIPS_ERR_STATE if no such call has completed on `h`. */
#define DIPS_CALLBACK_PHASES 11u
dips_status dips_callback_phases(const dips_handle *h, double *us, uint32_t cap, uint32_t *n);

/* Copy the start texture (RGBA8 gray, pre_compute_shader.wgsl:92-132) built
 * at the 4th frame.  Returns 1 if available, 0 if not yet built. */
int dips_start_texture(dips_handle *h, uint8_t *out_rgba, size_t cap);

/* Frame-range sharding of the dips-compat path ("dips-compat
 * T=4 needs a 3-frame halo"): put the handle in the state ComputeState has
 * after frame_callback of global frames 0..t0-1 (dips/src/lib.rs:233-246;
 * ring and start texture of dips/src/gpu/mod.rs:170-216, bind_groups.rs:
 * 407-427), rebuilt from the start texture S (dips_start_texture of the
 * handle that saw frames 0..3) and the raw RGBA8 frames t0-3, t0-2, t0-1
 * (`halo`, 3 contiguous frames in that order; for spatial_window_size > 1
 * they are filtered into the ring as compute_main would have).  Requires
 * t0 >= 7.  Device pointers with DIPS_FLAG_DEVICE_PTRS
 * (asynchronous), host pointers otherwise. */
dips_status dips_compat_resume(dips_handle *h, uint32_t width, uint32_t height,
                               const uint8_t *start_rgba, const uint8_t *halo, uint64_t t0);

/* North-star batch path: the per-frame difference series of `n_frames`
 * contiguous frames (each width*height*C bytes, C from params.format).
 *   ref: overall mode -> the reference frame (NULL = frames[0]);
 *        per-frame mode -> the frame preceding frames[0] (NULL = frames[0]).
 *   series: n_frames entries (required).
 *   absdiff_map: optional n_frames*width*height*C bytes, |F_t - R| per byte.
 * With DIPS_FLAG_DEVICE_PTRS all four pointers are device pointers and the
 * call is asynchronous on the handle's stream; otherwise they are host
 * pointers and the call returns when the results are in host memory. */
dips_status dips_diff_series(dips_handle *h, uint32_t width, uint32_t height,
                             const uint8_t *frames, uint32_t n_frames,
                             const uint8_t *ref, dips_series_entry *series,
                             uint8_t *absdiff_map);

/* f64 intensity sum of one entry: si_fixed * 2^-32. */
double dips_series_si(const dips_series_entry *e);

/* Streaming front-end feed (next-1 of SURVEY.md s8f): frames in pageable or
 * pinned HOST memory are staged through pinned buffers and copied to HBM
 * with hipMemcpyAsync on a side stream, overlapping the series kernel of the
 * previous chunk.  Same semantics as dips_diff_series with host pointers;
 * `chunk_frames` = frames per DMA chunk (0 = automatic). */
dips_status dips_diff_series_streamed(dips_handle *h, uint32_t width, uint32_t height,
                                      const uint8_t *host_frames, uint32_t n_frames,
                                      const uint8_t *host_ref, dips_series_entry *series,
                                      uint32_t chunk_frames);

/* Synthetic frames (shared integer generator, bit-identical to the oracle),
 * global frame indices t0 .. t0+n_frames-1, written to DEVICE memory `dst`. */
dips_status dips_synth_frames(dips_handle *h, uint32_t width, uint32_t height,
                              uint64_t seed, uint64_t t0, uint32_t n_frames, uint8_t *dst);

/* Kernel timing (DIPS_FLAG_TIME_KERNEL): total milliseconds and launch count
 * of the series kernel since the last reset, from hipEvents recorded on the
 * launch stream.  Synchronises the handle's stream. */
dips_status dips_kernel_time(dips_handle *h, double *total_ms, uint64_t *launches);
dips_status dips_kernel_time_reset(dips_handle *h);
/* The same launches one by one: up to `cap` per-launch milliseconds (oldest
 * first) into ms_each, the number of launches held into *launches.  The
 * handle holds the launches since the last reset, at most the most recent
 * 65,536 (beyond that the older half is dropped; dips_kernel_time still
 * counts every launch). */
dips_status dips_kernel_time_each(dips_handle *h, double *ms_each, uint64_t cap, uint64_t *launches);

/* Geometry of the series kernel for a frame shape (for roofline accounting):
 * waves launched, tiles per frame, bytes of partial records per frame. */
dips_status dips_series_geometry(dips_handle *h, uint32_t width, uint32_t height,
                                 uint32_t n_frames, uint64_t *waves, uint64_t *tiles,
                                 uint64_t *partial_bytes);

/* Measured read ceiling: one read-only stream (non-temporal 16-byte loads,
 * grid-stride) over `bytes` of DEVICE memory, synchronous; *ms = its
 * hipEvent duration.  bench.py divides the series kernel's rate by it
 * ("% of a measured read-only-stream ceiling"). */
dips_status dips_read_ceiling(dips_handle *h, const uint8_t *dev_bytes, uint64_t bytes, double *ms);

/* The same with the RGB8 / RGBA8 series kernel's own access shape: its
 * persistent (tile, frame) schedule over n_frames DEVICE frames of
 * width x height (the handle's format and mode; the part-major schedule where
 * the series kernel runs it), 12- / 16-byte vecs, two frames of loads in
 * flight, no compute; *ms = the hipEvent duration. */
dips_status dips_read_ceiling_walk(dips_handle *h, const uint8_t *dev_frames, uint32_t width, uint32_t height,
                                   uint32_t n_frames, double *ms);

/* Library ABI version (DIPS_ABI_VERSION). */
int dips_abi_version(void);

/* ------------------------------------------------------------------------
 * Frame-range sharding of the difference series over one rank per GPU
 * (BASELINE.json north_star: "sharded by frame-range across
 * the 8 GPUs of one node with a single RCCL gather").  The reference is
 * single-device -- one wgpu adapter and queue (dips/src/gpu/mod.rs:66-98,
 * chosen at :71-78) driving frames strictly in order -- so these entry
 * points have no reference counterpart; they let a Rust (or C) host that
 * replaces dips/src/gpu/mod.rs:39-398 with this library use every GPU of a
 * node without any other runtime.
 *
 * Rank r of G owns the contiguous global frames [r*N/G, (r+1)*N/G)
 * (dips_shard_range).  The exchanges are:
 *   'overall':   the reference frame, broadcast from rank 0;
 *   'per-frame': the halo frame r*N/G - 1, sent by rank r-1 to rank r,
 *                overlapped with the series launch over the rank's own frames
 *                1..n-1 (which need no halo);
 *   both:        the per-frame series entries (32 B each), reassembled on
 *                rank 0 by ONE gather (ncclGather, rccl.h:745).
 * No collective touches the frame batch itself.
 *
 * A communicator is one of three transports behind one internal table:
 *   DIPS_COMM_RCCL      RCCL over xGMI (librccl), one process per GPU;
 *   DIPS_COMM_LOOPBACK  ranks as threads of one process on one device,
 *                       stream-ordered hipMemcpyAsync + events (tests, and a
 *                       host that shards one GPU between decoders);
 *   DIPS_COMM_HOST      the caller's own transport (MPI, a torch process
 *                       group, ...) through host-memory callbacks,
 *                       synchronous.
 * Collective contract (as RCCL's): every rank makes the same sequence of
 * sharded calls with the same n_total, mode and shard_flags; an argument
 * error one rank alone detects returns on that rank before any collective
 * and leaves the others waiting in theirs.
 * ------------------------------------------------------------------------ */
typedef struct dips_comm dips_comm;

#define DIPS_COMM_ID_BYTES 128u /* NCCL_UNIQUE_ID_BYTES (rccl.h:40) */
#define DIPS_COMM_RCCL 1
#define DIPS_COMM_LOOPBACK 2
#define DIPS_COMM_HOST 3

/* Caller-supplied transport of DIPS_COMM_HOST: every buffer is HOST memory
 * owned by the library for the call; each function returns 0 on success and
 * any other value on failure.  broadcast: `bytes` from rank `root` into
 * `buf` on every rank (in place).  sendrecv: send `bytes` of `send` to rank
 * `to` and receive `bytes` from rank `from` into `recv`, concurrently (either
 * side < 0: none).  gather: `bytes` of `send` from every rank into `recv` at
 * offset rank*bytes on rank `root` (`recv` NULL elsewhere). */
typedef struct dips_comm_ops {
    int (*broadcast)(void *ctx, void *buf, size_t bytes, int root);
    int (*sendrecv)(void *ctx, const void *send, int to, void *recv, int from, size_t bytes);
    int (*gather)(void *ctx, const void *send, void *recv, size_t bytes, int root);
} dips_comm_ops;

/* A new RCCL unique id (ncclGetUniqueId) into id[DIPS_COMM_ID_BYTES]; rank 0
 * makes it and the caller hands it to every rank out of band. */
dips_status dips_comm_unique_id(uint8_t *id);

/* Join the RCCL communicator `id` as `rank` of `nranks` on HIP device
 * `device` (ncclCommInitRank; blocks until every rank has joined). */
dips_status dips_comm_create(const uint8_t *id, int nranks, int rank, int device, dips_comm **out);

/* All `nranks` RCCL communicators of ONE process (ncclCommInitAll): rank r
 * on HIP device devices[r] (NULL: device r), comms[r] = rank r.  The host
 * that drives every GPU from one process -- the reference's single decoder
 * feeding a node -- runs each rank's calls on its own thread. */
dips_status dips_comm_create_all(int nranks, const int *devices, dips_comm **comms);

/* `nranks` loopback communicators on `device`; comms[r] = rank r; each must
 * be driven by its own thread (the collectives meet on the host). */
dips_status dips_comm_create_loopback(int nranks, int device, dips_comm **comms);

/* A communicator over the caller's transport `ops` (context `ctx`). */
dips_status dips_comm_create_host(const dips_comm_ops *ops, void *ctx, int nranks, int rank, int device,
                                  dips_comm **out);

/* Leave and free a communicator (ncclCommDestroy for RCCL). */
void dips_comm_destroy(dips_comm *comm);

/* Last error message of `comm` (or of the last failed creation if NULL). */
const char *dips_comm_last_error(const dips_comm *comm);

/* Transport (DIPS_COMM_*), size and rank of `comm`. */
dips_status dips_comm_info(const dips_comm *comm, int *kind, int *nranks, int *rank);

/* The frame range of `rank` of `nranks` over `n_total` frames: global
 * frames [*first, *first + *count), balanced to within one frame. */
dips_status dips_shard_range(uint64_t n_total, int nranks, int rank, uint64_t *first, uint32_t *count);

/* DIPS_SHARD_REF_RESIDENT: 'overall' mode, every rank passes in `ref`
 * its own copy of the reference (e.g. from dips_shard_broadcast), so the
 * call skips the broadcast. */
#define DIPS_SHARD_REF_RESIDENT 0x1u

/* Broadcast one frame (width*height*C bytes) from rank 0's `frame` into
 * `out` on every rank (on rank 0 `out` may equal `frame`).  Device pointers
 * with DIPS_FLAG_DEVICE_PTRS (asynchronous on the handle's stream), host
 * pointers otherwise. */
dips_status dips_shard_broadcast(dips_handle *h, dips_comm *comm, uint32_t width, uint32_t height,
                                 const uint8_t *frame, uint8_t *out);

/* The sharded series: this rank's `n_local` frames (its dips_shard_range of
 * n_total; every rank needs >= 1 frame, so n_total >= nranks), the same
 * semantics as one dips_diff_series over all n_total frames.
 *   ref:          'overall': on rank 0 the reference (NULL = its frames[0]),
 *                 broadcast to every rank; with DIPS_SHARD_REF_RESIDENT every
 *                 rank's own copy.  'per-frame': on rank 0 the frame before
 *                 global frame 0 (NULL = frame 0 itself); ignored elsewhere
 *                 (the halo comes from rank r-1).
 *   series_local: n_local entries, this rank's slice (required).
 *   series_all:   rank 0: n_total entries, the gathered series (required;
 *                 may begin at series_local); other ranks: ignored.
 * With DIPS_FLAG_DEVICE_PTRS every pointer is a device pointer and the call
 * is asynchronous on the handle's stream (RCCL / loopback); otherwise host
 * pointers: the exchange runs first, then the rank's frames go through the
 * pinned side-stream feed of dips_diff_series_streamed (no batch-sized HBM
 * staging), and the call returns with the results in host memory.  h's
 * device must be the communicator's. */
dips_status dips_diff_series_sharded(dips_handle *h, dips_comm *comm, uint32_t width, uint32_t height,
                                     const uint8_t *frames, uint32_t n_local, uint64_t n_total,
                                     const uint8_t *ref, uint32_t shard_flags, dips_series_entry *series_local,
                                     dips_series_entry *series_all);

/* The plan of that call on this rank, without running it: its frame range
 * and the waves of its main series launch (the one the halo transfer
 * overlaps: frames 1..n-1 on ranks > 0 in 'per-frame' mode, all frames
 * otherwise), with the DIPS_SERIES_WAVES_PER_SIMD deployment cap applied
 * (`waves`) and without it (`waves_uncapped`).  The launch itself runs the
 * full persistent grid: the halo's kernels are posted before it. */
dips_status dips_shard_plan(dips_handle *h, const dips_comm *comm, uint32_t width, uint32_t height,
                            uint64_t n_total, uint64_t *first, uint32_t *count, uint64_t *waves,
                            uint64_t *waves_uncapped);

/* The dips-compat ComputeState over frame ranges ("dips-compat
 * T=4 needs a 3-frame halo"): consecutive frame_callback calls of global
 * frames [first, first + n_local) (this rank's dips_shard_range of n_total)
 * on a FRESH handle of every rank, the outputs those frames get from one
 * ComputeState that saw every frame (dips/src/lib.rs:233-246,
 * dips/src/gpu/mod.rs:170-397).  Rank 0 runs frames 0..3 (passthrough, then
 * the start texture) and broadcasts the start texture; rank r sends its last
 * three frames to rank r+1 and resumes (dips_compat_resume) from the start
 * texture and the three frames it receives.  Every rank after the first must
 * start at global frame >= 7 and every rank but the last own >= 3 frames
 * (n_total >= 7 * nranks suffices); the check is the same on every rank.
 * out: n_local RGBA8 frames on this rank (no gather: the outputs are frames,
 * each rank's muxer takes its own).  Pointers as dips_frame_callback_batch. */
dips_status dips_frame_callback_batch_sharded(dips_handle *h, dips_comm *comm, uint32_t width, uint32_t height,
                                              const uint8_t *frames, uint32_t n_local, uint64_t n_total,
                                              uint8_t *out);

/* Copy the reference the last sharded call used for this rank's first frame
 * (the received halo, the broadcast reference, or rank 0's own) into `out`
 * (width*height*C bytes; device pointer with DIPS_FLAG_DEVICE_PTRS).
 * Returns 1 if copied, 0 before any sharded call. */
int dips_shard_reference(dips_handle *h, uint8_t *out, size_t cap);

/* ------------------------------------------------------------------------
 * dips_alt operator.  The dips_alt crate's GPU
 * operator is DiPsCompute (dips_alt/src/dips_compute/mod.rs:243-647):
 * new(num_textures, textures_width, textures_height, window, device, queue,
 * properties) and send_frame(frame, snapshot, surface) -> Vec<u8>, driven by
 * the frame loop of run_dips_on_file (dips_alt/src/lib.rs:554-690).  The
 * reference's constructor takes (rows, cols) in that order (lib.rs:596-603);
 * this ABI takes width = columns, height = rows.  Frames are RGBA8, stride
 * width*4 (mod.rs:510-521).
 * ------------------------------------------------------------------------ */

/* DiPsProperties of dips_alt (dips_alt/src/dips_compute/mod.rs:167-186) plus
 * the operator's texture count. */
typedef struct dips_alt_params {
    uint8_t colorize;                /* COLORIZE; default 1 (mod.rs:179) */
    int32_t window_size;             /* WINDOW_SIZE; 1..11; default 1 (mod.rs:180) */
    float sigmoid_horizontal_scalar; /* SIGMOID_HORIZONTAL_SCALAR; default 5.0 (mod.rs:181) */
    uint32_t filter_type;            /* DIPS_FILTER_SIGMOID (default) / _INVERSE_SIGMOID;
                                        any other code: no filter (shader default branch) */
    uint32_t chroma_filter;          /* DIPS_CHROMA_*: All = NONE (default), Red, Green, Blue */
    uint32_t num_textures;           /* NUM_TEXTURES, 1..16; default FRAME_COUNT = 2 (lib.rs:36) */
    uint32_t flags;                  /* DIPS_FLAG_DEVICE_PTRS, _TIME_KERNEL, _FORCE_GENERIC */
} dips_alt_params;

typedef struct dips_alt_handle dips_alt_handle;

DIPS_LAYOUT_ASSERT(sizeof(dips_alt_params) == 28, "dips_alt_params size");
DIPS_LAYOUT_ASSERT(offsetof(dips_alt_params, colorize) == 0, "dips_alt_params.colorize");
DIPS_LAYOUT_ASSERT(offsetof(dips_alt_params, window_size) == 4, "dips_alt_params.window_size");
DIPS_LAYOUT_ASSERT(offsetof(dips_alt_params, sigmoid_horizontal_scalar) == 8,
                   "dips_alt_params.sigmoid_horizontal_scalar");
DIPS_LAYOUT_ASSERT(offsetof(dips_alt_params, filter_type) == 12, "dips_alt_params.filter_type");
DIPS_LAYOUT_ASSERT(offsetof(dips_alt_params, chroma_filter) == 16, "dips_alt_params.chroma_filter");
DIPS_LAYOUT_ASSERT(offsetof(dips_alt_params, num_textures) == 20, "dips_alt_params.num_textures");
DIPS_LAYOUT_ASSERT(offsetof(dips_alt_params, flags) == 24, "dips_alt_params.flags");

/* Fill `p` with DiPsProperties::default() (mod.rs:176-186), num_textures 2. */
dips_status dips_alt_params_default(dips_alt_params *p);

/* Replaces DiPsCompute::new (dips_alt/src/dips_compute/mod.rs:270-496):
 * texture slots, snapshot texture and output, all zero-initialised. */
dips_status dips_alt_create(const dips_alt_params *params, uint32_t width, uint32_t height, int device,
                            dips_alt_handle **out);

/* Replaces Drop of DiPsCompute. */
void dips_alt_destroy(dips_alt_handle *h);

/* Last error message for `h` (or the last creation failure if h == NULL). */
const char *dips_alt_last_error(const dips_alt_handle *h);

/* Run subsequent work on `stream` (a hipStream_t; NULL = the handle's own);
 * ordered after the previous stream's work as dips_set_stream. */
dips_status dips_alt_set_stream(dips_alt_handle *h, void *stream);
dips_status dips_alt_synchronize(dips_alt_handle *h);

/* Replaces DiPsCompute::send_frame (mod.rs:498-646): writes the frame into
 * texture slot texture_index, advances it, runs pre_compute_main with the
 * snapshot uniform = (snapshot != 0) and copies the RGBA8 output texture
 * (width*height*4 bytes) to `out_rgba`.  Host pointers always. */
dips_status dips_alt_send_frame(dips_alt_handle *h, const uint8_t *frame_rgba, size_t len, int snapshot,
                                uint8_t *out_rgba, size_t cap);

/* `n_frames` consecutive send_frame calls in one pass: frames n_frames x
 * width*height*4, snapshot_flags (host, n_frames bytes, NULL = none) the
 * per-frame snapshot argument, out n_frames x width*height*4.  With
 * DIPS_FLAG_DEVICE_PTRS frames/out are device pointers and the call is
 * asynchronous on the handle's stream. */
dips_status dips_alt_send_frames(dips_alt_handle *h, const uint8_t *frames, uint32_t n_frames,
                                 const uint8_t *snapshot_flags, uint8_t *out);

/* The frame loop of run_dips_on_file (lib.rs:588-683) minus OpenCV decode /
 * encode: snapshot while index == FRAME_COUNT, index saturating, a refresh
 * marker equal to the running 1-based frame count resets index to 0.  The
 * loop state persists across calls, so a video may be fed in pieces. */
dips_status dips_alt_run(dips_alt_handle *h, const uint8_t *frames, uint32_t n_frames,
                         const uint64_t *refresh_markers, uint32_t n_markers, uint8_t *out);

/* The dips_alt run loop over frame ranges: this rank's frames [first,
 * first + n_local) of an n_total-frame video (its dips_shard_range), on a
 * FRESH handle of every rank, with the outputs one run_dips_on_file loop over
 * every frame gives them (the same refresh markers on every rank).  Rank r
 * replays, outputs discarded, the source frames of the last snapshot before
 * its first frame and the num_textures frames before it (fewer, after zero
 * frames, near the start), fetched point to point from the ranks that own
 * them, then runs its own frames; any split, ranks with no frame included.
 * Pointers as dips_alt_send_frames; synchronous. */
dips_status dips_alt_run_sharded(dips_alt_handle *h, dips_comm *comm, const uint8_t *frames, uint32_t n_local,
                                 uint64_t n_total, const uint64_t *refresh_markers, uint32_t n_markers, uint8_t *out);

/* Copy the snapshot texture's .r channel (width*height bytes, host). */
dips_status dips_alt_snapshot_texture(dips_alt_handle *h, uint8_t *out_gray, size_t cap);

/* Kernel timing of the batch kernel (DIPS_FLAG_TIME_KERNEL), as dips_kernel_time. */
dips_status dips_alt_kernel_time(dips_alt_handle *h, double *total_ms, uint64_t *launches);
dips_status dips_alt_kernel_time_reset(dips_alt_handle *h);

/* Self-check of the batch kernel's epilogue table (alt_lut.h) for the
 * handle's properties: every snapshot byte against every (max, min) byte
 * pair -- all pixel intensities of every chroma mode -- through the table and
 * through the specification's epilogue; *mismatches = the count of texels
 * that differ (0 expected).  Synchronous; for tests. */
dips_status dips_alt_lut_selfcheck(dips_alt_handle *h, uint64_t *mismatches);

/* The host-built index of that table (alt_lut.h), no device needed: the
 * level-1 entries {x, sh} of the 1,021 clusters (l1_cap >= 2042 words), the
 * distinct diff values and their level-2 slots (cap >= *n_diffs), and the
 * level-2 size.  Any output pointer may be NULL.  For tests. */
dips_status dips_alt_lut_index(uint32_t *l1, uint32_t l1_cap, float *diffs, uint16_t *slots, uint32_t cap,
                               uint32_t *n_diffs, uint32_t *l2_entries);

#ifdef __cplusplus
}
#endif
#endif /* DIPS_HIP_H */
