/*
 * dips_oracle.c -- TEST INFRASTRUCTURE ONLY (see dips_oracle.h).
 *
 * Plain-C, scalar restatement of the reference semantics.  Every function
 * cites the reference file:line it restates (paths relative to the
 * RubenMovsesyan/DiPs checkout).  Compile with -ffp-contract=off: the f32
 * expression order below is part of the specification.
 */
#include "dips_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ */
/* rgba8unorm conversions                                              */
/* ------------------------------------------------------------------ */

/* Texel load: textureLoad on rgba8unorm returns c/255 per channel
 * (dips/src/gpu/shaders/dips_shader.wgsl:124,138,192,213). */
float dips_oracle_u(uint8_t c) { return (float)c / 255.0f; }

/* Texel store: textureStore on rgba8unorm (dips_shader.wgsl:187,239;
 * pre_compute_shader.wgsl:131).  Pinned: clamp, x*255, round-half-even,
 * NaN -> 0. */
uint8_t dips_oracle_q(float x) {
    if (!(x > 0.0f)) return 0; /* also NaN */
    if (x > 1.0f) x = 1.0f;
    float y = x * 255.0f;
    return (uint8_t)rintf(y);
}

/* ------------------------------------------------------------------ */
/* Deterministic exp / log (spec in DESIGN.md "f32 transcendental      */
/* functions"); the reference calls WGSL exp()/log()                  */
/* (dips_shader.wgsl:111,117).                                         */
/* ------------------------------------------------------------------ */

static float o_bits_to_f(uint32_t b) { float f; memcpy(&f, &b, 4); return f; }
static uint32_t o_f_to_bits(float f) { uint32_t b; memcpy(&b, &f, 4); return b; }
static float o_pow2i(int n) { return o_bits_to_f((uint32_t)(n + 127) << 23); }

float dips_oracle_expf(float x) {
    if (x != x) return x;
    if (x > 88.72283935546875f) return INFINITY;
    if (x < -103.97208404541016f) return 0.0f;
    const float kf = rintf(x * 1.44269502162933349609375f);
    float r = x - kf * 0.693145751953125f;
    r = r - kf * 1.428606765330187045e-06f;
    float p = 1.3888889225e-3f;
    p = p * r + 8.3333337680e-3f;
    p = p * r + 4.1666667908e-2f;
    p = p * r + 1.6666667163e-1f;
    p = p * r + 0.5f;
    p = p * r + 1.0f;
    p = p * r + 1.0f;
    const int k = (int)kf;
    const int k1 = k / 2;
    const int k2 = k - k1;
    p = p * o_pow2i(k1);
    p = p * o_pow2i(k2);
    return p;
}

float dips_oracle_logf(float x) {
    if (x != x || x < 0.0f) return NAN;
    if (x == 0.0f) return -INFINITY;
    if (x == INFINITY) return INFINITY;
    uint32_t bits = o_f_to_bits(x);
    int e = 0;
    if (bits < 0x00800000u) { /* subnormal */
        x = x * 8388608.0f;
        bits = o_f_to_bits(x);
        e = -23;
    }
    e += (int)(bits >> 23) - 127;
    float m = o_bits_to_f((bits & 0x007FFFFFu) | 0x3F800000u);
    if (m > 1.41421353816986083984375f) { m = m * 0.5f; e += 1; }
    const float f = m - 1.0f;
    const float s = f / (2.0f + f);
    const float z = s * s;
    float t = 1.1111111194e-1f;
    t = t * z + 1.4285714924e-1f;
    t = t * z + 2.0000000298e-1f;
    t = t * z + 3.3333334327e-1f;
    t = t * z + 1.0f;
    const float lm = (2.0f * s) * t;
    const float ef = (float)e;
    return ef * 0.693145751953125f + (ef * 1.428606765330187045e-06f + lm);
}

/* ------------------------------------------------------------------ */
/* Intensity                                                           */
/* ------------------------------------------------------------------ */

/* get_intensity (dips_shader.wgsl:64-82, copy pre_compute_shader.wgsl:20-38)
 * on an RGB(A) texel given as bytes. */
static float o_intensity_rgb(uint8_t r, uint8_t g, uint8_t b, int chroma) {
    const float fr = dips_oracle_u(r), fg = dips_oracle_u(g), fb = dips_oracle_u(b);
    if (chroma == 1) return fr;
    if (chroma == 2) return fg;
    if (chroma == 3) return fb;
    float cmax = fmaxf(fr, fg);
    cmax = fmaxf(cmax, fb);
    float cmin = fminf(fr, fg);
    cmin = fminf(cmin, fb);
    return (cmax + cmin) / 2.0f;
}

/* get_intensity on a float texel (used on already-filtered values). */
static float o_intensity_f(float r, float g, float b, int chroma) {
    if (chroma == 1) return r;
    if (chroma == 2) return g;
    if (chroma == 3) return b;
    float cmax = fmaxf(fmaxf(r, g), b);
    float cmin = fminf(fminf(r, g), b);
    return (cmax + cmin) / 2.0f;
}

/* Pixel intensity and its integer twin J = max + min (SURVEY.md s8
 * "Canonical definitions").  Gray8 has r = g = b = v. */
static void o_pixel(const uint8_t *px, int channels, int chroma, float *I, int *J) {
    uint8_t r, g, b;
    if (channels == 1) { r = g = b = px[0]; }
    else { r = px[0]; g = px[1]; b = px[2]; }
    *I = o_intensity_rgb(r, g, b, chroma);
    if (chroma >= 1 && chroma <= 3) {
        const int c = chroma == 1 ? r : chroma == 2 ? g : b;
        *J = 2 * c;
    } else {
        int mx = r > g ? r : g; mx = mx > b ? mx : b;
        int mn = r < g ? r : g; mn = mn < b ? mn : b;
        *J = mx + mn;
    }
}

/* ------------------------------------------------------------------ */
/* Difference series                                                   */
/* ------------------------------------------------------------------ */

/* One frame F against reference R (north_star; R = frame 0 or the given
 * reference for 'overall', previous frame for 'per-frame', README.md:7-11). */
static void o_series_frame(int channels, int chroma, float tau, size_t npx,
                           const uint8_t *F, const uint8_t *R, uint64_t *out4,
                           double *si_f64, uint8_t *dmap) {
    uint64_t sad = 0, sj = 0, cnt = 0, sif = 0;
    double si = 0.0;
    for (size_t p = 0; p < npx; ++p) {
        const uint8_t *f = F + p * (size_t)channels;
        const uint8_t *r = R + p * (size_t)channels;
        for (int c = 0; c < channels; ++c) {
            const int d = f[c] > r[c] ? f[c] - r[c] : r[c] - f[c];
            sad += (uint64_t)d;
            if (dmap) dmap[p * (size_t)channels + c] = (uint8_t)d;
        }
        float If, Ir;
        int Jf, Jr;
        o_pixel(f, channels, chroma, &If, &Jf);
        o_pixel(r, channels, chroma, &Ir, &Jr);
        sj += (uint64_t)(Jf > Jr ? Jf - Jr : Jr - Jf);
        const float dI = fabsf(If - Ir);
        if (dI > tau) {
            cnt += 1;
            si += (double)dI;
            /* dI is a multiple of 2^-32 in [0,1]: dI * 2^32 is an exact integer */
            sif += (uint64_t)ldexp((double)dI, 32);
        }
    }
    out4[0] = sad;
    out4[1] = sj;
    out4[2] = cnt;
    out4[3] = sif;
    if (si_f64) *si_f64 = si;
}

static int o_check(int channels, int chroma, int mode, float tau, uint32_t w, uint32_t h) {
    if (channels != 1 && channels != 3 && channels != 4) return -1;
    if (chroma < 0 || chroma > 3) return -1;
    if (mode != 0 && mode != 1) return -1;
    if (!(tau >= 0.0f) || tau == INFINITY) return -1;
    if (w == 0 || h == 0) return -1;
    return 0;
}

int dips_oracle_series(int channels, int chroma, int mode, float tau,
                       uint32_t width, uint32_t height,
                       const uint8_t *frames, uint32_t n_frames,
                       const uint8_t *ref, uint64_t *out4, double *si_f64,
                       uint8_t *dmap) {
    if (o_check(channels, chroma, mode, tau, width, height)) return -1;
    if (n_frames == 0) return 0;
    const size_t npx = (size_t)width * height;
    const size_t fb = npx * (size_t)channels;
    for (uint32_t t = 0; t < n_frames; ++t) {
        const uint8_t *F = frames + (size_t)t * fb;
        const uint8_t *R;
        if (mode == 0) R = ref ? ref : frames;
        else R = t > 0 ? frames + (size_t)(t - 1) * fb : (ref ? ref : frames);
        o_series_frame(channels, chroma, tau, npx, F, R, out4 + 4 * (size_t)t,
                       si_f64 ? si_f64 + t : NULL, dmap ? dmap + (size_t)t * fb : NULL);
    }
    return 0;
}

typedef struct {
    int channels, chroma, mode;
    float tau;
    uint32_t width, height;
    const uint8_t *frames;
    uint32_t t0, t1;
    const uint8_t *ref;
    uint64_t *out4;
    double *si_f64;
    uint8_t *dmap;
} o_job;

static void *o_worker(void *arg) {
    o_job *j = (o_job *)arg;
    const size_t fb = (size_t)j->width * j->height * (size_t)j->channels;
    if (j->t1 <= j->t0) return NULL;
    const uint8_t *ref = j->ref;
    if (j->mode == 1 && j->t0 > 0) ref = j->frames + (size_t)(j->t0 - 1) * fb;
    dips_oracle_series(j->channels, j->chroma, j->mode, j->tau, j->width, j->height,
                       j->frames + (size_t)j->t0 * fb, j->t1 - j->t0,
                       (j->mode == 0 && !ref) ? j->frames : ref,
                       j->out4 + 4 * (size_t)j->t0, j->si_f64 ? j->si_f64 + j->t0 : NULL,
                       j->dmap ? j->dmap + (size_t)j->t0 * fb : NULL);
    return NULL;
}

int dips_oracle_series_mt(int channels, int chroma, int mode, float tau,
                          uint32_t width, uint32_t height,
                          const uint8_t *frames, uint32_t n_frames,
                          const uint8_t *ref, uint64_t *out4, double *si_f64,
                          uint8_t *dmap, int nthreads) {
    if (o_check(channels, chroma, mode, tau, width, height)) return -1;
    if (nthreads < 1) nthreads = 1;
    if ((uint32_t)nthreads > n_frames) nthreads = n_frames ? (int)n_frames : 1;
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    o_job *jobs = (o_job *)calloc((size_t)nthreads, sizeof(o_job));
    if (!th || !jobs) { free(th); free(jobs); return -2; }
    for (int k = 0; k < nthreads; ++k) {
        o_job *j = &jobs[k];
        j->channels = channels; j->chroma = chroma; j->mode = mode; j->tau = tau;
        j->width = width; j->height = height; j->frames = frames;
        j->t0 = (uint32_t)((uint64_t)n_frames * k / nthreads);
        j->t1 = (uint32_t)((uint64_t)n_frames * (k + 1) / nthreads);
        j->ref = ref; j->out4 = out4; j->si_f64 = si_f64; j->dmap = dmap;
        pthread_create(&th[k], NULL, o_worker, j);
    }
    for (int k = 0; k < nthreads; ++k) pthread_join(th[k], NULL);
    free(th);
    free(jobs);
    return 0;
}

/* ------------------------------------------------------------------ */
/* Synthetic generator (SURVEY.md s8d "Synthetic inputs")              */
/* ------------------------------------------------------------------ */

static uint64_t o_splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

void dips_oracle_synth(int channels, uint32_t width, uint32_t height,
                       uint64_t seed, uint64_t t0, uint32_t n_frames,
                       uint8_t *out) {
    const size_t fb = (size_t)width * height * (size_t)channels;
    const int64_t rad = height / 8 > 0 ? height / 8 : 1;
    for (uint32_t k = 0; k < n_frames; ++k) {
        const uint64_t t = t0 + k;
        const uint64_t fkey = o_splitmix64(seed + t);
        const int64_t cx = (int64_t)(((uint64_t)(width / 4) + 4u * t) % width);
        const int64_t cy = height / 2;
        uint8_t *F = out + (size_t)k * fb;
        for (uint32_t y = 0; y < height; ++y) {
            for (uint32_t x = 0; x < width; ++x) {
                const int64_t dx = (int64_t)x - cx, dy = (int64_t)y - cy;
                const int blob = (dx * dx + dy * dy <= rad * rad) ? 64 : 0;
                for (int c = 0; c < channels; ++c) {
                    const uint64_t idx = ((uint64_t)y * width + x) * (uint64_t)channels + (uint64_t)c;
                    const int base = (int)(o_splitmix64(seed ^ idx) & 0xFFu);
                    const uint64_t hsh = o_splitmix64(fkey ^ idx);
                    const int noise = (int)(((hsh >> 32) * 9u) >> 32) - 4;
                    int v = base + blob + noise;
                    v = v < 0 ? 0 : v > 255 ? 255 : v;
                    F[((size_t)y * width + x) * (size_t)channels + (size_t)c] = (uint8_t)v;
                }
            }
        }
    }
}

/* ------------------------------------------------------------------ */
/* dips-compat ComputeState                                            */
/* ------------------------------------------------------------------ */

#define O_T 4 /* TEMPORAL_BUFFER_SIZE, dips/src/gpu/bind_groups.rs:18 */

struct dips_oracle_cs {
    uint8_t colorize;
    int32_t window;
    float sensitivity;
    uint32_t filter, chroma;
    uint32_t width, height;
    int n_queued;           /* VecDeque length, dips/src/gpu/mod.rs:53,171-175 */
    uint8_t *queue[O_T];
    int pre_init, main_init; /* bind_groups.rs:43-96, 430-483 */
    uint8_t *start;          /* RGBA start texture (gray) */
    uint8_t *slots[O_T];     /* temporal_textures, RGBA */
    uint32_t ring_idx;       /* UCircularIndex, utils/indexing.rs:1-34 */
    uint32_t uniform_idx;    /* starting_index uniform, bind_groups.rs:317-321,420-424 */
    uint8_t *scratch;
};

dips_oracle_cs *dips_oracle_cs_new(uint8_t colorize, int32_t window, float sensitivity,
                                   uint32_t filter, uint32_t chroma) {
    if (window < 1 || window > 11 || chroma > 3) return NULL;
    dips_oracle_cs *cs = (dips_oracle_cs *)calloc(1, sizeof(*cs));
    if (!cs) return NULL;
    cs->colorize = colorize ? 1 : 0;
    cs->window = window;
    cs->sensitivity = sensitivity;
    cs->filter = filter;
    cs->chroma = chroma;
    return cs;
}

void dips_oracle_cs_free(dips_oracle_cs *cs) {
    if (!cs) return;
    for (int i = 0; i < O_T; ++i) { free(cs->queue[i]); free(cs->slots[i]); }
    free(cs->start);
    free(cs->scratch);
    free(cs);
}

/* spatial_median_filter (dips_shader.wgsl:120-170, pre_compute_shader.wgsl:40-90)
 * evaluated on an RGBA image `img` at (x,y); returns the filtered intensity.
 * Restates the exact quirks: only the (2h)^2 offsets in [-h,h) are filled,
 * the rest of the 121-entry array is zero, a bubble sort over indices
 * 0..W^2 (j+1 clamped to 120 by naga's Restrict policy), result index
 * W^2/2 + 1. */
static float o_spatial(const uint8_t *img, uint32_t w, uint32_t h, uint32_t x, uint32_t y,
                       int window, int chroma) {
    const uint8_t *px = img + ((size_t)y * w + x) * 4;
    if (window == 1) return o_intensity_rgb(px[0], px[1], px[2], chroma);
    float a[121];
    memset(a, 0, sizeof(a));
    const int hw = window / 2;
    for (int i = -hw; i < hw; ++i) {
        for (int j = -hw; j < hw; ++j) {
            float color;
            const int xi = (int)x + i, yj = (int)y + j;
            if (xi >= (int)w || yj >= (int)h || xi < 0 || yj < 0) color = 0.0f;
            else {
                const uint8_t *q = img + ((size_t)yj * w + (size_t)xi) * 4;
                color = o_intensity_rgb(q[0], q[1], q[2], chroma);
            }
            const int ai = i + hw, aj = j + hw;
            a[ai + window * aj] = color;
        }
    }
    const int ws2 = window * window;
    for (int i = 0; i < ws2; ++i) {
        int swapped = 0;
        for (int j = 0; j < ws2; ++j) {
            const int j1 = j + 1 > 120 ? 120 : j + 1;
            if (a[j] > a[j1]) {
                const float tmp = a[j];
                a[j] = a[j1];
                a[j1] = tmp;
                swapped = 1;
            }
        }
        if (!swapped) break;
    }
    int k = ws2 / 2 + 1;
    if (k > 120) k = 120;
    return a[k];
}

/* The 4-entry bubble sort of dips_shader.wgsl:196-211 and
 * pre_compute_shader.wgsl:111-126 with j+1 clamped to 3 (Restrict);
 * returns element [MEDIAN_ARRAY_SIZE/2] = [2]. */
float dips_oracle_upper_median4(const float v[4]) {
    float a[4] = {v[0], v[1], v[2], v[3]};
    for (int i = 0; i < 4; ++i) {
        int swapped = 0;
        for (int j = 0; j < 4; ++j) {
            const int j1 = j + 1 > 3 ? 3 : j + 1;
            if (a[j] > a[j1]) {
                const float tmp = a[j];
                a[j] = a[j1];
                a[j1] = tmp;
                swapped = 1;
            }
        }
        if (!swapped) break;
    }
    return a[2];
}

/* pre_compute_main (pre_compute_shader.wgsl:92-132) over frames 0..3. */
static void o_precompute(dips_oracle_cs *cs) {
    const uint32_t w = cs->width, h = cs->height;
    for (uint32_t y = 0; y < h; ++y) {
        for (uint32_t x = 0; x < w; ++x) {
            float m[4];
            for (int k = 0; k < 4; ++k) {
                const float f = o_spatial(cs->queue[k], w, h, x, y, cs->window, (int)cs->chroma);
                m[k] = o_intensity_f(f, f, f, (int)cs->chroma);
            }
            const uint8_t s = dips_oracle_q(dips_oracle_upper_median4(m));
            uint8_t *o = cs->start + ((size_t)y * w + x) * 4;
            o[0] = o[1] = o[2] = s;
            o[3] = 255;
        }
    }
}

int dips_oracle_cs_add_texture(dips_oracle_cs *cs, uint32_t width, uint32_t height,
                               const uint8_t *rgba) {
    /* ComputeState::add_texture, dips/src/gpu/mod.rs:170-216 */
    if (!cs || !rgba || width == 0 || height == 0) return -1;
    if (cs->n_queued > 0 && (width != cs->width || height != cs->height)) return -1;
    const size_t fb = (size_t)width * height * 4;
    cs->width = width;
    cs->height = height;
    uint8_t *copy = (uint8_t *)malloc(fb);
    if (!copy) return -2;
    memcpy(copy, rgba, fb); /* textures.push_back(frame_data.to_vec()) :171 */
    if (cs->n_queued == O_T) { /* pop_front when > TEMPORAL_BUFFER_SIZE :173-175 */
        free(cs->queue[0]);
        memmove(cs->queue, cs->queue + 1, (O_T - 1) * sizeof(uint8_t *));
        cs->queue[O_T - 1] = copy;
    } else {
        cs->queue[cs->n_queued++] = copy;
    }
    if (cs->n_queued != O_T) return 0;
    if (!cs->pre_init) { /* PreComputeBindGroups::initialize + run_precompute_pipeline :178-188 */
        cs->pre_init = 1;
        cs->start = (uint8_t *)malloc(fb);
        cs->scratch = (uint8_t *)malloc(fb);
        if (!cs->start || !cs->scratch) return -2;
        o_precompute(cs);
    }
    if (!cs->main_init) { /* MainComputeBindGroups::initialize, starting index 0 (bind_groups.rs:73) */
        cs->main_init = 1;
        for (int k = 0; k < O_T; ++k) {
            cs->slots[k] = (uint8_t *)malloc(fb);
            if (!cs->slots[k]) return -2;
            memcpy(cs->slots[k], cs->queue[k], fb);
        }
        cs->ring_idx = 0;
        cs->uniform_idx = 0;
    } else { /* update_temporal_texture, bind_groups.rs:407-427 */
        memcpy(cs->slots[cs->ring_idx], rgba, fb);
        cs->uniform_idx = cs->ring_idx;
        cs->ring_idx = (cs->ring_idx + 1) % O_T;
    }
    return 0;
}

int dips_oracle_cs_resume(dips_oracle_cs *cs, uint32_t width, uint32_t height, const uint8_t *start_rgba,
                          const uint8_t *halo, uint64_t t0) {
    /* After frame_callback of frames 0..t0-1 (t0 >= 7): pre/main bind groups
     * initialised, start texture S, ring index t0 mod 4, and slot (t0-1-j)
     * mod 4 holding frame t0-1-j as its own dispatch left it -- the gray
     * texel q(spatial_median_filter(frame)) (dips_shader.wgsl:187) -- for
     * j = 0, 1, 2.  The fourth slot is overwritten by the next add_texture
     * before anything reads it; the VecDeque is not read after init. */
    if (!cs || !start_rgba || !halo || width == 0 || height == 0 || t0 < 7) return -1;
    const size_t fb = (size_t)width * height * 4;
    for (int i = 0; i < O_T; ++i) { free(cs->queue[i]); free(cs->slots[i]); cs->queue[i] = cs->slots[i] = NULL; }
    free(cs->start);
    free(cs->scratch);
    cs->start = (uint8_t *)malloc(fb);
    cs->scratch = (uint8_t *)malloc(fb);
    if (!cs->start || !cs->scratch) return -2;
    for (int i = 0; i < O_T; ++i) {
        cs->queue[i] = (uint8_t *)calloc(1, fb);
        cs->slots[i] = (uint8_t *)calloc(1, fb);
        if (!cs->queue[i] || !cs->slots[i]) return -2;
    }
    cs->width = width;
    cs->height = height;
    cs->n_queued = O_T;
    cs->pre_init = cs->main_init = 1;
    memcpy(cs->start, start_rgba, fb);
    for (int j = 0; j < 3; ++j) {
        const uint8_t *raw = halo + (size_t)(2 - j) * fb; /* frame t0-1-j */
        uint8_t *sl = cs->slots[(t0 - 1 - (uint64_t)j) % O_T];
        for (uint32_t y = 0; y < height; ++y)
            for (uint32_t x = 0; x < width; ++x) {
                const size_t p = (size_t)y * width + x;
                const uint8_t q = dips_oracle_q(o_spatial(raw, width, height, x, y, cs->window, (int)cs->chroma));
                sl[p * 4 + 0] = sl[p * 4 + 1] = sl[p * 4 + 2] = q;
                sl[p * 4 + 3] = 255;
            }
    }
    cs->ring_idx = (uint32_t)(t0 % O_T);
    cs->uniform_idx = (uint32_t)((t0 - 1) % O_T);
    return 0;
}

static float o_sigmoid(float x, float k) {
    /* dips_shader.wgsl:108-112 */
    return 1.0f / (1.0f + dips_oracle_expf(-k * x)) - 0.5f;
}

static float o_inv_sigmoid(float x, float k) {
    /* dips_shader.wgsl:114-118 */
    return (-dips_oracle_logf((1.0f / (x + 0.5f)) - 1.0f)) / k;
}

/* hsl_to_rgb (dips_shader.wgsl:40-62) for the two hues diff_to_color uses. */
static void o_hsl(float hue, float s, float l, float rgb[3]) {
    const float chroma = s * (1.0f - fabsf(2.0f * l - 1.0f));
    const float hp = hue / 60.0f;
    const float x = chroma * (1.0f - fabsf(fmodf(hp, 2.0f) - 1.0f));
    const float m = l - chroma / 2.0f;
    if (hp >= 0.0f && hp < 1.0f) { rgb[0] = chroma + m; rgb[1] = x + m; rgb[2] = 0.0f + m; }
    else if (hp >= 1.0f && hp < 2.0f) { rgb[0] = x + m; rgb[1] = chroma + m; rgb[2] = 0.0f + m; }
    else if (hp >= 2.0f && hp < 3.0f) { rgb[0] = 0.0f + m; rgb[1] = chroma + m; rgb[2] = x + m; }
    else if (hp >= 3.0f && hp < 4.0f) { rgb[0] = 0.0f + m; rgb[1] = x + m; rgb[2] = chroma + m; }
    else if (hp >= 4.0f && hp < 5.0f) { rgb[0] = x + m; rgb[1] = 0.0f + m; rgb[2] = chroma + m; }
    else if (hp >= 5.0f && hp <= 6.0f) { rgb[0] = chroma + m; rgb[1] = 0.0f + m; rgb[2] = x + m; }
    else { rgb[0] = rgb[1] = rgb[2] = 0.0f + m; }
}

int dips_oracle_cs_dispatch(dips_oracle_cs *cs, uint8_t *out) {
    /* ComputeState::dispatch, dips/src/gpu/mod.rs:306-397; kernel compute_main
     * dips_shader.wgsl:172-240. */
    if (!cs || !cs->main_init) return 0; /* None while warming up (:394-396) */
    const uint32_t w = cs->width, h = cs->height;
    const size_t fb = (size_t)w * h * 4;
    const uint32_t u = cs->uniform_idx;
    /* Pinned race-free semantics: the filter of the newest slot
     * reads the slot as it was before this dispatch. */
    memcpy(cs->scratch, cs->slots[u], fb);
    for (uint32_t y = 0; y < h; ++y) {
        for (uint32_t x = 0; x < w; ++x) {
            const size_t p = (size_t)y * w + x;
            const float fi = o_spatial(cs->scratch, w, h, x, y, cs->window, (int)cs->chroma);
            const uint8_t qi = dips_oracle_q(fi);
            uint8_t *sl = cs->slots[u] + p * 4;
            sl[0] = sl[1] = sl[2] = qi;
            sl[3] = 255; /* vec4(I,I,I,1.0) stored, :125, :169 */
            float m[4];
            for (int i = 0; i < 4; ++i) {
                const uint8_t *t = cs->slots[i] + p * 4;
                m[i] = o_intensity_rgb(t[0], t[1], t[2], (int)cs->chroma);
            }
            const float original = dips_oracle_u(cs->start[p * 4 + 0]);
            float diff = original - dips_oracle_upper_median4(m);
            diff = diff * ((0.5f - -0.5f) / (1.0f - -1.0f)); /* map(), :97-105,217 */
            if (cs->filter == 0) diff = o_sigmoid(diff, cs->sensitivity);
            else if (cs->filter == 1) diff = o_inv_sigmoid(diff, cs->sensitivity);
            diff *= 5.0f; /* SENSITIVITY, :25,229 */
            float rgb[3];
            if (cs->colorize) {
                if (diff < 0.0f) o_hsl(0.0f, fabsf(diff), 0.5f, rgb);
                else o_hsl(120.0f, diff, 0.5f, rgb);
            } else {
                rgb[0] = rgb[1] = rgb[2] = 0.5f - diff;
            }
            uint8_t *o = out + p * 4;
            o[0] = dips_oracle_q(rgb[0]);
            o[1] = dips_oracle_q(rgb[1]);
            o[2] = dips_oracle_q(rgb[2]);
            o[3] = 255;
        }
    }
    return 1;
}

int dips_oracle_cs_start_texture(const dips_oracle_cs *cs, uint8_t *out) {
    if (!cs || !cs->pre_init) return 0;
    memcpy(out, cs->start, (size_t)cs->width * cs->height * 4);
    return 1;
}

/* ------------------------------------------------------------------ */
/* dips_alt DiPsCompute (next-4 of SURVEY.md s8f)                      */
/* ------------------------------------------------------------------ */

#define O_ALT_MAX_TEX 16 /* MAX_TEMPORAL_ARRAY_SIZE, dips_alt pre_compute_shader.wgsl:12 */

struct dips_oracle_alt {
    uint32_t n_tex;          /* num_textures, dips_alt/src/dips_compute/mod.rs:270-279 */
    uint32_t width, height;  /* texture extent (mod.rs:283-287: width = cols) */
    uint8_t colorize;
    int32_t window;
    float scalar;            /* SIGMOID_HORIZONTAL_SCALAR */
    uint32_t filter, chroma;
    uint8_t *slots[O_ALT_MAX_TEX]; /* input_textures, zero-initialised (wgpu) */
    uint8_t *snap;           /* snapshot_texture (.r channel), zero-initialised */
    uint32_t tex_idx;        /* texture_index: UCircularIndex(0, n), mod.rs:494 */
};

dips_oracle_alt *dips_oracle_alt_new(uint32_t n_tex, uint32_t width, uint32_t height,
                                     uint8_t colorize, int32_t window, float scalar,
                                     uint32_t filter, uint32_t chroma) {
    if (n_tex < 1 || n_tex > O_ALT_MAX_TEX || width == 0 || height == 0) return NULL;
    if (window < 1 || window > 11 || chroma > 3) return NULL;
    dips_oracle_alt *a = (dips_oracle_alt *)calloc(1, sizeof(*a));
    if (!a) return NULL;
    a->n_tex = n_tex;
    a->width = width;
    a->height = height;
    a->colorize = colorize ? 1 : 0;
    a->window = window;
    a->scalar = scalar;
    a->filter = filter;
    a->chroma = chroma;
    const size_t fb = (size_t)width * height * 4;
    for (uint32_t k = 0; k < n_tex; ++k) {
        a->slots[k] = (uint8_t *)calloc(fb, 1);
        if (!a->slots[k]) { dips_oracle_alt_free(a); return NULL; }
    }
    a->snap = (uint8_t *)calloc((size_t)width * height, 1);
    if (!a->snap) { dips_oracle_alt_free(a); return NULL; }
    return a;
}

void dips_oracle_alt_free(dips_oracle_alt *a) {
    if (!a) return;
    for (uint32_t k = 0; k < O_ALT_MAX_TEX; ++k) free(a->slots[k]);
    free(a->snap);
    free(a);
}

/* spatial_median_filter of dips_alt (dips_alt pre_compute_shader.wgsl:134-186):
 * the (2h)^2 offsets in [-h, h) are filled (out-of-frame = 0), the rest of the
 * 121-entry array is zero, a bubble sort over the first W^2 entries (all
 * indices in bounds for W <= 11, unlike dips' W^2 + 1), result [W^2/2 + 1]. */
static float o_alt_spatial(const uint8_t *img, uint32_t w, uint32_t h, uint32_t x, uint32_t y,
                           int window, int chroma) {
    const uint8_t *px = img + ((size_t)y * w + x) * 4;
    if (window == 1) return o_intensity_rgb(px[0], px[1], px[2], chroma); /* :135-139 */
    float a[121];
    memset(a, 0, sizeof(a));
    const int hw = window / 2;
    for (int i = -hw; i < hw; ++i) {
        for (int j = -hw; j < hw; ++j) {
            float color;
            const int xi = (int)x + i, yj = (int)y + j;
            if (xi >= (int)w || yj >= (int)h || xi < 0 || yj < 0) color = 0.0f;
            else {
                const uint8_t *q = img + ((size_t)yj * w + (size_t)xi) * 4;
                color = o_intensity_rgb(q[0], q[1], q[2], chroma);
            }
            a[(i + hw) + window * (j + hw)] = color;
        }
    }
    const int ws2 = window * window;
    for (int i = 0; i < ws2 - 1; ++i) {
        int swapped = 0;
        for (int j = 0; j < ws2 - 1; ++j) {
            if (a[j] > a[j + 1]) {
                const float tmp = a[j];
                a[j] = a[j + 1];
                a[j + 1] = tmp;
                swapped = 1;
            }
        }
        if (!swapped) break;
    }
    return a[ws2 / 2 + 1];
}

/* The temporal sort of dips_alt pre_compute_main (pre_compute_shader.wgsl:200,
 * 212-227, 232, 238): a 16-entry zero-initialised array holding the n
 * filtered values, n bubble passes over j < n comparing [j] and [j+1]
 * (index 16 clamped to 15 by naga's Restrict policy when n = 16), element
 * [n/2].  For n < 16 the sort covers one trailing zero. */
float dips_oracle_alt_temporal(const float *v, uint32_t n) {
    float a[O_ALT_MAX_TEX];
    memset(a, 0, sizeof(a));
    for (uint32_t i = 0; i < n; ++i) a[i] = v[i];
    for (uint32_t i = 0; i < n; ++i) {
        int swapped = 0;
        for (uint32_t j = 0; j < n; ++j) {
            const uint32_t j1 = j + 1 > O_ALT_MAX_TEX - 1 ? O_ALT_MAX_TEX - 1 : j + 1;
            if (a[j] > a[j1]) {
                const float tmp = a[j];
                a[j] = a[j1];
                a[j1] = tmp;
                swapped = 1;
            }
        }
        if (!swapped) break;
    }
    return a[n / 2];
}

/* DiPsCompute::send_frame (dips_alt/src/dips_compute/mod.rs:498-646) with the
 * compute pass pre_compute_main (pre_compute_shader.wgsl:188-263); returns the
 * RGBA8 output texture (width*height*4).  `snapshot` != 0 is the Some(())
 * case: the uniform is 1 for this dispatch only (mod.rs:525-528, 617-620). */
int dips_oracle_alt_send_frame(dips_oracle_alt *a, const uint8_t *rgba, int snapshot,
                               uint8_t *out) {
    if (!a || !rgba || !out) return -1;
    const uint32_t w = a->width, h = a->height;
    const size_t fb = (size_t)w * h * 4;
    memcpy(a->slots[a->tex_idx], rgba, fb);    /* queue.write_texture, :510-521 */
    a->tex_idx = (a->tex_idx + 1) % a->n_tex;  /* texture_index += 1, :523 */
    for (uint32_t y = 0; y < h; ++y) {
        for (uint32_t x = 0; x < w; ++x) {
            const size_t p = (size_t)y * w + x;
            float m[O_ALT_MAX_TEX];
            for (uint32_t k = 0; k < a->n_tex; ++k) /* array generator, dynamic_texture_array.rs:67-69 */
                m[k] = o_alt_spatial(a->slots[k], w, h, x, y, a->window, (int)a->chroma);
            const float med = dips_oracle_alt_temporal(m, a->n_tex);
            uint8_t *o = out + p * 4;
            if (snapshot) { /* :231-235 */
                const uint8_t s = dips_oracle_q(med);
                a->snap[p] = s;
                o[0] = o[1] = o[2] = s;
                o[3] = 255;
                continue;
            }
            const float original = dips_oracle_u(a->snap[p]); /* :237 */
            float diff = original - med;
            diff = diff * ((0.5f - -0.5f) / (1.0f - -1.0f)); /* map(), :100-108, 240 */
            if (a->filter == 0) diff = o_sigmoid(diff, a->scalar);
            else if (a->filter == 1) diff = o_inv_sigmoid(diff, a->scalar);
            diff *= 5.0f; /* DIFF_SCALE, :26, 252 */
            float rgb[3];
            if (a->colorize) {
                if (diff < 0.0f) o_hsl(0.0f, fabsf(diff), 0.5f, rgb);
                else o_hsl(120.0f, diff, 0.5f, rgb);
            } else {
                rgb[0] = rgb[1] = rgb[2] = 0.5f - diff;
            }
            o[0] = dips_oracle_q(rgb[0]);
            o[1] = dips_oracle_q(rgb[1]);
            o[2] = dips_oracle_q(rgb[2]);
            o[3] = 255;
        }
    }
    return 0;
}

/* The frame loop of run_dips_on_file (dips_alt/src/lib.rs:588-683) without
 * the OpenCV decode / encode: snapshot when index == FRAME_COUNT (2), index
 * saturates at FRAME_COUNT + 1, and a refresh marker equal to the 1-based
 * frame count resets index to 0.  Writes n_frames outputs. */
int dips_oracle_alt_run(dips_oracle_alt *a, const uint8_t *frames, uint32_t n_frames,
                        const uint64_t *markers, uint32_t n_markers, uint8_t *out) {
    if (!a) return -1;
    const size_t fb = (size_t)a->width * a->height * 4;
    uint64_t index = 0, overall = 0;
    for (uint32_t t = 0; t < n_frames; ++t) {
        int rc = dips_oracle_alt_send_frame(a, frames + (size_t)t * fb, index == 2, out + (size_t)t * fb);
        if (rc) return rc;
        if (index <= 2) index += 1;
        overall += 1;
        for (uint32_t k = 0; k < n_markers; ++k)
            if (markers[k] == overall) { index = 0; break; }
    }
    return 0;
}
