// dips_kernels.h -- kernel argument blocks and host launchers (internal).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dips_hip.h"

namespace dips {

// Unroll (vecs per lane) of the fast series kernel; a tile = 64 * U vecs.
// A dispatch holds fewer than 2^32 work-items (the grid size is a 32-bit
// count of work-items, not of workgroups): one-dimensional launches of
// 256-thread workgroups over n items must check n against this, or the grid
// wraps and the launch silently runs only the remainder.
constexpr bool fits_grid256(uint64_t n) { return n <= (1ull << 32) - 256u; }

constexpr int kUnrollRGB = 4;   // 1024 px / wave / frame for RGB8 and RGBA8
constexpr int kUnrollGray = 2;  // 2048 px / wave / frame for GRAY8
constexpr int kUnrollV2 = 4;    // series_v2_kernel RGBA8: 1024 px / wave / frame
constexpr int kUnrollV2Rgb = 5; // series_v2_kernel RGB8: 1280 px / wave / frame (12-B vecs: 5 x 64 x 12 < 4096)
template <int C>
constexpr int v2_unroll() { return C == 3 ? kUnrollV2Rgb : kUnrollV2; }
// series_gray_lut_kernel: 64 * 16 * U px / wave / frame (U = 4: 4K gray8
// 61.9-62.1 % of 8 TB/s vs 60.4-60.6 % at U = 2, profiles/r02_gray_lut_unroll.jsonl;
// confirmed in one process with the final kernel: U = 4 65.5-65.9 %, U = 3
// 64.9-65.7 %, U = 2 63.6-63.9 %, profiles/r02_gray_variant_ab.jsonl)
#ifndef DIPS_UNROLL_GRAY_LUT
#define DIPS_UNROLL_GRAY_LUT 4
#endif
constexpr int kUnrollGrayLut = DIPS_UNROLL_GRAY_LUT;
constexpr uint32_t kGrayLutWaves = 16;  // its waves per workgroup (one 1024-thread group per CU)
constexpr size_t kGrayLutBytes = 131072;  // its T_d / T_c tables
constexpr size_t kGrayLutAllocBytes = kGrayLutBytes + 256;  // + layout 5's band word (series_gray.hip)
// layout 4 (auto) keeps layout 5's table + band word and layout 2's after it
// Prefetch depth: frames of loads each wave keeps in flight.
#ifndef DIPS_DEPTH_RGB
#define DIPS_DEPTH_RGB 2
#endif
#ifndef DIPS_DEPTH_GRAY
#define DIPS_DEPTH_GRAY 2
#endif
constexpr int kDepthRGB = DIPS_DEPTH_RGB;
constexpr int kDepthGray = DIPS_DEPTH_GRAY;

struct SeriesArgs {
    const uint8_t* frames;   // n_frames * frame_bytes, contiguous
    const uint8_t* ref0;     // overall: reference; per-frame: predecessor of frame 0
    uint8_t* dmap;           // optional |F - R| map (same layout as frames)
    uint64_t* partials;      // [n_tiles][n_frames] x 16-byte records
    uint64_t items;          // n_tiles * n_frames
    uint32_t frame_bytes;    // frame stride in bytes (W * H * C; any alignment)
    uint32_t vec_bytes;      // bytes of whole vecs per frame (the descriptor range; the
                             // < pixels_per_vec trailing pixels go to the generic kernel)
    uint32_t n_frames;
    uint32_t n_tiles;
    uint32_t n_waves;
    float thr;               // threshold in kernel units: series_threshold()
    const void* lut;         // GRAY8 table kernel: T_d / T_c bytes (series_gray.hip), 128 KiB
    uint32_t part_frames;    // frames per part of the part-major schedule (series_v2 SCHED = 1)
    // GRAY8 table kernel, layout 4: each workgroup samples its waves' first
    // items and takes layout 5 when band >= probe_min / 1024 of the sampled
    // pixels and (band >= probe_hi / 1024 of them or the waves' byte spreads
    // average >= probe_spread), else layout 2 (probe_min 0: always 5, > 1024:
    // always 2 -- the pinned layouts)
    uint32_t probe_min;
    uint32_t probe_hi;
    uint32_t probe_spread;
    uint64_t* zero;          // when set: the kernel zeroes zero[0 .. zero_n) (the series, before its
    uint32_t zero_n;         // reduce's atomics; replaces a separate fill launch)
};

struct GenericArgs {
    const uint8_t* frames;
    const uint8_t* ref0;
    uint8_t* dmap;
    dips_series_entry* series;
    uint64_t frame_bytes;
    uint64_t n_px;
    uint64_t px0;            // first pixel of each frame to process (the fast kernel's ragged tail)
    uint32_t n_frames;
    uint32_t blocks_per_frame;
    uint32_t mode;
    uint32_t chroma;
    float tau;
};

struct SynthArgs {
    uint8_t* dst;
    uint64_t total_bytes;
    uint64_t frame_bytes;
    uint64_t seed;
    uint64_t t0;
    uint32_t channels;
    uint32_t width;
    uint32_t height;
    uint32_t radius;
};

struct CompatArgs {
    const uint8_t* raw;      // filter source (RGBA8) for the newest slot
    uint8_t* slots[4];       // temporal ring (RGBA8)
    const uint8_t* start;    // start texture (RGBA8 gray)
    uint8_t* out;            // visualisation (RGBA8)
    uint32_t width, height;
    uint32_t newest;         // starting_index uniform
    int32_t window;
    uint32_t chroma;
    uint32_t filter;
    float sensitivity;
    uint32_t colorize;
    uint32_t y0, y1;         // compat_main: rows [y0, y1) only (y1 = 0: all rows)
    uint32_t out_key;        // compat_main_host: 0 RGBA8 texels; 1 one byte (gray: R = G = B, A = 255);
                             // 2 two bytes R | G << 8 (colorized: B = min(R, G), A = 255) -- the host
                             // expands them (host_stream.h expand_keys)
    uint32_t in_key;         // compat_main_host: raw holds RGBA8 texels (0), or per pixel the chroma
                             // channel (1) / (max, min) of R, G, B (2) (copy_pool.h pack_frame);
                             // compat_main_host_packed_kernel, out_key 1 / 2 only
};

// dips ComputeState over a batch in steady state (compat_batch.hip).
struct CompatBatchArgs {
    const uint8_t* frames;   // n_frames x frame_bytes (RGBA8)
    uint8_t* out;            // n_frames x frame_bytes (RGBA8)
    const uint8_t* start;    // start texture (RGBA8 gray, R = S)
    const uint8_t* pre[3];   // ring slots of the frames before frames[0] (gray texels): t-1, t-2, t-3
    uint8_t* post[4];        // ring slots that receive frames n-1 .. n-4 as gray texels (null: none)
    uint32_t frame_bytes;
    uint32_t n_vec;          // 4-pixel vecs per frame
    uint32_t n_frames, chunk, n_chunks, n_tiles;
    float k;                 // sensitivity (SIGMOID_HORIZONTAL_SCALAR)
    float kneg_half;         // -k / 2
    const uint16_t* lut;     // epilogue table (compat_batch_lut_kernel): 65536 x (R | G << 8)
};
constexpr int kUnrollCompatBatch = 2;
// U vecs per lane and D frames of loads in flight per wave of the table
// kernel.  In one process over one batch (round 2,
// profiles/r02_compat_variant_ab.jsonl) U = 4, D = 3 ran 76.2 % of 8 TB/s
// read + write, against 72.4 % for U = 2, D = 2 (an earlier cross-process
// A/B had called U = 4 equal).  126 VGPRs: the 1024-thread workgroup's
// budget is 128, and D = 4 spills.
constexpr int kUnrollCompatLut = 4;
constexpr int kDepthCompatLut = 3;
constexpr uint32_t kCompatLutWaves = 16;  // waves per workgroup of compat_batch_lut_kernel (one per CU)
// the epilogue table of the current properties: lut[S * 256 + m]
hipError_t launch_compat_lut(uint16_t* lut, uint32_t filter, float k, bool colorize, hipStream_t s);
const void* compat_batch_lut_kernel_ptr(int chroma);
hipError_t launch_compat_batch_lut(const CompatBatchArgs& a, int chroma, uint32_t blocks, hipStream_t s);
const void* compat_batch_kernel_ptr(int chroma, int filter, bool colorize, bool fast);
hipError_t launch_compat_batch(const CompatBatchArgs& a, int chroma, int filter, bool colorize, bool fast,
                               uint32_t blocks, hipStream_t s);

// dips_alt DiPsCompute (alt_kernels.hip).
constexpr int kAltMaxTextures = 16;  // MAX_TEMPORAL_ARRAY_SIZE (dips_alt pre_compute_shader.wgsl:12)
constexpr int kUnrollAlt = 2;        // vecs (4 px) per lane of alt_batch_kernel
// vecs per lane / frames of loads in flight of its epilogue-table form.  In one process
// over one batch (round 2, profiles/r02_alt_variant_ab.jsonl):
// U = 4, D = 2 72.8 % of 8 TB/s read + write, U = 2, D = 2 72.1 %, the others
// 71.2-72.3 % (8 groups of 256 threads per CU already keep enough in flight).
constexpr int kUnrollAltLut = 4;
constexpr int kDepthAltLut = 2;

struct AltArgs {                     // one send_frame dispatch
    const uint8_t* slots[kAltMaxTextures];  // RGBA8 contents of the N texture slots
    uint8_t* snap;                   // snapshot texture, one byte (.r) per pixel
    uint8_t* out;                    // RGBA8 output texture
    uint32_t width, height;
    uint32_t n_tex;
    int32_t window;
    uint32_t chroma, filter;
    float scalar;
    uint32_t colorize;
    uint32_t snapshot;
    uint32_t y0, y1;                 // rows [y0, y1) only (y1 = 0: all rows)
};

struct AltBatchArgs {                // a run of frames, N = 2, W = 1
    const uint8_t* frames;           // n_frames x frame_bytes (RGBA8)
    const uint8_t* prev0;            // slot holding the frame before frames[0]
    const uint8_t* snap_in;          // snapshot bytes before the batch
    uint8_t* snap_out;               // snapshot bytes after the batch's last snapshot
    uint8_t* out;                    // n_frames x frame_bytes (RGBA8)
    const uint8_t* flags;            // device: n_frames snapshot flags
    const int32_t* chunk_snap;       // device: per chunk, last snapshot frame before it or -1
    uint32_t frame_bytes;
    uint32_t n_vec;                  // 4-pixel vecs per frame
    uint32_t n_frames, chunk, n_chunks, n_tiles;
    int32_t last_snap;               // last snapshot frame of the batch or -1
    float scalar;                    // SIGMOID_HORIZONTAL_SCALAR k
    float kneg_half;                 // -k / 2 (fast epilogue)
    const uint32_t* lut_l1;          // epilogue table (alt_lut.h): level-1 {x, sh} per cluster
    const uint16_t* lut_l2;          //   and the u16 texel entries (LUT kernel only)
};

hipError_t launch_alt_frame(const AltArgs& a, hipStream_t s);
// send_frame (W = 1) reading the new frame from pinned host memory `in`,
// storing it into `newest_slot` (= a.slots[newest]) and writing a.out (pinned
// host memory): the per-frame call's zero-copy form
hipError_t launch_alt_frame_host(const AltArgs& a, const uint8_t* in, uint8_t* newest_slot, uint32_t newest,
                                 hipStream_t s);

struct CopyFramesArgs {
    const uint8_t* src[2];
    uint8_t* dst[2];
    uint64_t n16;  // 16-byte words per frame (16-byte aligned frames)
};
hipError_t launch_copy_frames(const CopyFramesArgs& a, uint32_t count, hipStream_t s);
// fast: the branch-free epilogue (alt_fast_epilogue_ok)
// chroma -1: frames are prefiltered f32 I2s intensities (launch_alt_filter_frames)
const void* alt_batch_kernel_ptr(int chroma, int filter, bool colorize, bool fast);
// W > 1: the filtered intensity (I * 2^23, f32) of each pixel of n RGBA8
// frames, one f32 per pixel (the layout the batch kernel reads with chroma -1)
hipError_t launch_alt_filter_frames(const uint8_t* frames, float* dst, uint32_t width, uint32_t height, uint32_t n,
                                   int32_t window, uint32_t chroma, hipStream_t s);
hipError_t launch_alt_batch(const AltBatchArgs& a, int chroma, int filter, bool colorize, bool fast, uint32_t blocks,
                            hipStream_t s);
// the epilogue-table form (alt_lut.h): any filter / k / colour, same outputs
const void* alt_batch_lut_kernel_ptr(int chroma);
hipError_t launch_alt_batch_lut(const AltBatchArgs& a, int chroma, uint32_t blocks, hipStream_t s);
// lut_l2[slots[i]] = R | G << 8 of visual_epilogue(diffs[i], filter, k, colorize)
// exhaustive table check over every (S, max, min): mismatches added to *bad
hipError_t launch_alt_lut_check(const uint32_t* l1, const uint16_t* l2, uint32_t filter, float k, bool colorize,
                                unsigned long long* bad, hipStream_t s);
hipError_t launch_alt_lut_fill(uint16_t* lut_l2, const float* diffs, const uint16_t* slots, uint32_t n,
                               uint32_t filter, float k, bool colorize, hipStream_t s);
// the fast epilogue's preconditions (epilogue_fast.h): sigmoid with a scalar
// k of |k| <= 160 (0 or |k| >= 2^-60 so -k/2 is exact), or no filter
inline bool alt_fast_epilogue_ok(uint32_t filter, float k) {
    if (filter == 1u) return false;
    if (filter != 0u) return true;
    const float a = k < 0.0f ? -k : k;
    return a <= 160.0f && (a == 0.0f || a >= 0x1p-60f);
}

int pixels_per_vec(int channels);
int fast_unroll(int channels);
// isi (series_v2, RGB8 / RGBA8): 0 the exact f64 intensity sum, 1 the
// integer sum with a threshold select (ISI; needs tau >= 2^-5)
const void* series_fast_kernel_ptr(int channels, int chroma, bool per_frame, bool map, bool align = false,
                                   int isi = 0);
const void* series_v2_kernel_ptr(int channels, int chroma, bool per_frame, bool map, bool align = false,
                                 int isi = 0);
// whether tau admits the integer intensity sum of series_v2 (tau >= 2^-5)
bool series_v2_isi(float tau);
// threshold argument (SeriesArgs::thr) of the kernel series_fast_kernel_ptr picks
float series_threshold(int channels, float tau, int isi = 0);
hipError_t launch_series_fast(const SeriesArgs& a, int channels, int chroma, bool per_frame, bool map,
                              uint32_t blocks, hipStream_t s, bool align = false, int isi = 0);
// record layout: 0 RGB(A), 1 gray (series_fast_kernel), 2 gray table kernel (series_gray_lut_kernel)
hipError_t launch_series_reduce(const uint64_t* partials, uint32_t n_frames, uint32_t n_tiles, int layout,
                                dips_series_entry* series, hipStream_t s);
// GRAY8 table kernel: table layout 4, i.e. layout 5 (the u16 table keyed by
// (a ^ b, a) with the band clamp) or 2 (the u16 table keyed by (a, b),
// swizzled) per workgroup from a sample of its items
const void* series_gray_lut_kernel_ptr(bool per_frame, bool map);
// the tables of layout 4 (5, then 2 kGrayLutAllocBytes after it), or of one layout
hipError_t launch_gray_lut(uint8_t* tab, float tau, int layout, hipStream_t s);
hipError_t launch_series_gray_lut(const SeriesArgs& a, bool per_frame, bool map, uint32_t blocks, hipStream_t s);
hipError_t launch_series_generic(const GenericArgs& a, int channels, hipStream_t s);
hipError_t launch_synth(const SynthArgs& a, hipStream_t s);
hipError_t launch_read_ceiling(const uint8_t* p, uint64_t bytes, uint32_t* out, hipStream_t s);
// read-only walk in the RGB8 / RGBA8 series kernel's shape (vec_bytes 12 / 16, U = kUnrollV2Rgb / kUnrollV2)
hipError_t launch_read_walk(const SeriesArgs& a, int vec_bytes, uint32_t blocks, uint32_t* out, hipStream_t s);
hipError_t launch_compat_precompute(const CompatArgs& a, hipStream_t s);
hipError_t launch_compat_main(const CompatArgs& a, hipStream_t s);
// compat_main with raw / out in pinned host memory (zero-copy per-frame call)
// slot_mode 0: store the quantised gray texel into the newest slot
// (compute_main); 1: store the raw frame texel, 2: store nothing (the
// speculative dispatch of a deferred add_texture, W = 1 / W > 1)
hipError_t launch_compat_main_host(const CompatArgs& a, hipStream_t s, int slot_mode = 0);
// a raw ring slot into its gray texel q(get_intensity) in place
hipError_t launch_compat_quantise_slot(uint8_t* slot, uint64_t n_px, uint32_t chroma, hipStream_t s);
// bytes (a multiple of 4, 4-B aligned) between pinned host memory (its
// device-visible pointer) and HBM, by a kernel instead of a DMA engine
hipError_t launch_copy_from_host(const uint8_t* src, uint8_t* dst, uint64_t bytes, hipStream_t s);
hipError_t launch_copy_to_host(const uint8_t* src, uint8_t* dst, uint64_t bytes, hipStream_t s);
hipError_t launch_compat_gray(const uint8_t* src, uint8_t* dst, uint64_t n_px, uint32_t chroma, hipStream_t s);
// W > 1 steady state: the ring texel compute_main stores for each of n frames
// (gray q(spatial_median_filter(frame)), dips_shader.wgsl:120-170, 187), so
// that the batch kernel can run on the filtered frames.  frames, dst: n x
// width x height RGBA8.
hipError_t launch_compat_filter_frames(const uint8_t* frames, uint8_t* dst, uint32_t width, uint32_t height,
                                       uint32_t n, int32_t window, uint32_t chroma, hipStream_t s);

}  // namespace dips
