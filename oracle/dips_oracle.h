/*
 * dips_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the DiPs per-pixel frame-difference path, used as the
 * parity oracle for the HIP product in dips_amd/.  Only tests/, the smoke()
 * entry point and bench.py's cpu_baseline leg may load this library; the
 * product never links or calls it.
 *
 * Parity status: the reference (RubenMovsesyan/DiPs, Rust + WGSL through
 * wgpu 24 / naga 24.0.0) cannot be built in this image (no cargo/rustc, crates
 * not vendored) and ships no tests, fixtures or golden vectors (SURVEY.md
 * s4, s8c).  Its shader files are executed instead: oracle/wgsl_exec.py
 * interprets the reference's WGSL text, oracle/wgsl_ref.py restates the Rust
 * host side around it, and this oracle reproduces those outputs bit for bit
 * (tests/test_wgsl_pin.py, the wgsl_* fixtures; get_intensity over all 2^24
 * RGB triples).  The restatement is thereby pinned to the shader text; what
 * WGSL leaves to the backend is pinned as follows (the reference's bytes on
 * a given GPU depend on its driver for these, which nothing here can run):
 *   - naga bounds-check policy `Restrict` (Vulkan/DX12) for the
 *     out-of-bounds bubble-sort index (dips_shader.wgsl:198-203),
 *   - rgba8unorm load u(c) = c / 255.0f (IEEE division),
 *   - rgba8unorm store q(x) = rint(clamp(x,0,1) * 255.0f), round-half-even,
 *     NaN stored as 0,
 *   - exp/log: the deterministic f32 algorithms documented in DESIGN.md
 *     (the reference uses the GPU driver's exp/log, <= a few ulp away).
 */
#ifndef DIPS_ORACLE_H
#define DIPS_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* scalar helpers (exported so tests can pin them) */
float   dips_oracle_u(uint8_t c);          /* rgba8unorm load  */
uint8_t dips_oracle_q(float x);            /* rgba8unorm store */
float   dips_oracle_expf(float x);
float   dips_oracle_logf(float x);
float   dips_oracle_upper_median4(const float v[4]);

/* Difference series (north-star path).
 * channels: 1 (gray8), 3 (RGB8), 4 (RGBA8); chroma 0..3; mode 0 overall /
 * 1 per-frame.  out4[t*4 + {0,1,2,3}] = {SAD, SJ, count, SI_fixed}
 * (SI_fixed = sum of dI * 2^32, exact).  si_f64[t] = sequential double sum
 * of dI in pixel order.  dmap (optional) = |F_t - R| per byte.
 * Returns 0 on success, <0 on invalid arguments. */
int dips_oracle_series(int channels, int chroma, int mode, float tau,
                       uint32_t width, uint32_t height,
                       const uint8_t *frames, uint32_t n_frames,
                       const uint8_t *ref, uint64_t *out4, double *si_f64,
                       uint8_t *dmap);
/* Same, frames split over `nthreads` POSIX threads (CPU baseline). */
int dips_oracle_series_mt(int channels, int chroma, int mode, float tau,
                          uint32_t width, uint32_t height,
                          const uint8_t *frames, uint32_t n_frames,
                          const uint8_t *ref, uint64_t *out4, double *si_f64,
                          uint8_t *dmap, int nthreads);

/* Synthetic frame generator (global frame indices t0 .. t0+n-1). */
void dips_oracle_synth(int channels, uint32_t width, uint32_t height,
                       uint64_t seed, uint64_t t0, uint32_t n_frames,
                       uint8_t *out);

/* dips-compat ComputeState emulation (dips/src/gpu/mod.rs:39-398). */
typedef struct dips_oracle_cs dips_oracle_cs;
dips_oracle_cs *dips_oracle_cs_new(uint8_t colorize, int32_t window,
                                   float sensitivity, uint32_t filter,
                                   uint32_t chroma);
int  dips_oracle_cs_add_texture(dips_oracle_cs *cs, uint32_t width,
                                uint32_t height, const uint8_t *rgba);
int  dips_oracle_cs_dispatch(dips_oracle_cs *cs, uint8_t *out_rgba);
int  dips_oracle_cs_start_texture(const dips_oracle_cs *cs, uint8_t *out_rgba);
/* State after frames 0..t0-1 went through frame_callback (t0 >= 7), rebuilt
 * from the start texture and the raw frames t0-3, t0-2, t0-1 (`halo`, in
 * that order): the frame-range sharding of the dips-compat path. */
int  dips_oracle_cs_resume(dips_oracle_cs *cs, uint32_t width, uint32_t height,
                           const uint8_t *start_rgba, const uint8_t *halo, uint64_t t0);
void dips_oracle_cs_free(dips_oracle_cs *cs);

/* dips_alt DiPsCompute emulation (dips_alt/src/dips_compute/mod.rs:243-647,
 * shader dips_alt/src/dips_compute/shaders/pre_compute_shader.wgsl).
 * width = texture columns, height = rows; n_tex = num_textures (1..16). */
typedef struct dips_oracle_alt dips_oracle_alt;
dips_oracle_alt *dips_oracle_alt_new(uint32_t n_tex, uint32_t width, uint32_t height,
                                     uint8_t colorize, int32_t window, float scalar,
                                     uint32_t filter, uint32_t chroma);
float dips_oracle_alt_temporal(const float *v, uint32_t n);
int  dips_oracle_alt_send_frame(dips_oracle_alt *a, const uint8_t *rgba, int snapshot,
                                uint8_t *out_rgba);
int  dips_oracle_alt_run(dips_oracle_alt *a, const uint8_t *frames, uint32_t n_frames,
                         const uint64_t *markers, uint32_t n_markers, uint8_t *out);
void dips_oracle_alt_free(dips_oracle_alt *a);

#ifdef __cplusplus
}
#endif
#endif
