// read_walk_probe.hip -- read-only ceilings over the headline batch (5000
// 3840x2160 RGB8 frames, 124.4 GB resident in HBM) with three access shapes:
//   grid   -- the library's read_ceiling_kernel shape: grid-stride 16-B
//             non-temporal loads, 4 in flight per lane, 1024 blocks;
//   walk12 -- the series kernel's shape: persistent waves, a wave owns a
//             tile of 64 lanes x 4 vecs of 12 B and walks it through every
//             frame, two frames of loads in flight;
//   walk16 -- the same with 16-B vecs.
// Each is timed by hipEvents over 3 single launches and over one run of 10
// back-to-back launches (sustained).  The best is the read ceiling the series
// kernel is compared with.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/read_walk_probe tools/read_walk_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) {                                                              \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
            std::exit(1);                                                                    \
        }                                                                                    \
    } while (0)

typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes) {
    const uint64_t a = (uint64_t)(uintptr_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    void* base = (void*)(uintptr_t)(((uint64_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(base, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

__global__ __launch_bounds__(256) void grid_kernel(const u32x4* __restrict__ p, uint64_t n16, uint32_t* out) {
    constexpr int kUnr = 4;
    uint32_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * 256u * kUnr;
    for (uint64_t i = (uint64_t)blockIdx.x * 256u * kUnr + threadIdx.x; i < n16; i += stride) {
        u32x4 v[kUnr];
#pragma unroll
        for (int u = 0; u < kUnr; ++u) {
            const uint64_t j = i + (uint64_t)u * 256u;
            v[u] = j < n16 ? __builtin_nontemporal_load(p + j) : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < kUnr; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    if (acc == 0x9E3779B9u) out[0] = acc;
}

// items = n_tiles * n_frames split into one contiguous range per wave (the
// series kernel's schedule); 2 frames of loads in flight.
template <int VB>
__global__ __launch_bounds__(256) void walk_kernel(const uint8_t* frames, uint32_t fb, uint32_t n_frames,
                                                   uint32_t n_tiles, uint32_t n_waves, uint32_t* out) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
    if (wave >= n_waves) return;
    const uint64_t items = (uint64_t)n_tiles * n_frames;
    uint64_t i = (uint64_t)wave * items / n_waves;
    const uint64_t iend = (uint64_t)(wave + 1) * items / n_waves;
    uint32_t acc = 0;
    while (i < iend) {
        const uint32_t tile = (uint32_t)(i / n_frames);
        uint32_t t = (uint32_t)(i - (uint64_t)tile * n_frames);
        const uint64_t rem = iend - i;
        const uint32_t tend = (uint32_t)((uint64_t)n_frames < t + rem ? (uint64_t)n_frames : t + rem);
        i += tend - t;
        const uint32_t voff = (tile * 4u * 64u + lane) * VB;
        for (; t < tend; t += 2) {
            const uint32_t t1 = t + 1 < tend ? t + 1 : t;
            const __amdgpu_buffer_rsrc_t r0 = rsrc(frames + (uint64_t)t * fb, fb);
            const __amdgpu_buffer_rsrc_t r1 = rsrc(frames + (uint64_t)t1 * fb, fb);
            uint32_t x = 0;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if constexpr (VB == 12) {
                    const u32x3 a = __builtin_amdgcn_raw_buffer_load_b96(r0, voff + u * 64 * VB, 0, 2);
                    const u32x3 b = __builtin_amdgcn_raw_buffer_load_b96(r1, voff + u * 64 * VB, 0, 2);
                    x ^= a.x ^ a.y ^ a.z ^ b.x ^ b.y ^ b.z;
                } else {
                    const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(r0, voff + u * 64 * VB, 0, 2);
                    const u32x4 b = __builtin_amdgcn_raw_buffer_load_b128(r1, voff + u * 64 * VB, 0, 2);
                    x ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w;
                }
            }
            acc ^= x;
        }
    }
    if (acc == 0x9E3779B9u) out[0] = acc;
}

// lockstep walk: wave w owns tiles w, w + n_waves, ... and walks each through
// every frame; with n_waves = n_tiles all waves sweep the frames together.
template <int VB>
__global__ __launch_bounds__(256) void lockstep_kernel(const uint8_t* frames, uint32_t fb, uint32_t n_frames,
                                                       uint32_t n_tiles, uint32_t n_waves, uint32_t* out) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
    if (wave >= n_waves) return;
    uint32_t acc = 0;
    for (uint32_t tile = wave; tile < n_tiles; tile += n_waves) {
        const uint32_t voff = (tile * 4u * 64u + lane) * VB;
        for (uint32_t t = 0; t < n_frames; t += 2) {
            const uint32_t t1 = t + 1 < n_frames ? t + 1 : t;
            const __amdgpu_buffer_rsrc_t r0 = rsrc(frames + (uint64_t)t * fb, fb);
            const __amdgpu_buffer_rsrc_t r1 = rsrc(frames + (uint64_t)t1 * fb, fb);
            uint32_t x = 0;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if constexpr (VB == 12) {
                    const u32x3 a = __builtin_amdgcn_raw_buffer_load_b96(r0, voff + u * 64 * VB, 0, 2);
                    const u32x3 b = __builtin_amdgcn_raw_buffer_load_b96(r1, voff + u * 64 * VB, 0, 2);
                    x ^= a.x ^ a.y ^ a.z ^ b.x ^ b.y ^ b.z;
                } else {
                    const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(r0, voff + u * 64 * VB, 0, 2);
                    const u32x4 b = __builtin_amdgcn_raw_buffer_load_b128(r1, voff + u * 64 * VB, 0, 2);
                    x ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w;
                }
            }
            acc ^= x;
        }
    }
    if (acc == 0x9E3779B9u) out[0] = acc;
}

// The three load shapes of one tile (1024 RGB8 pixels = 3072 B per frame):
//   SHAPE 0 -- the series kernel's: 4 vecs of 12 B per lane, lane-interleaved
//              (one dwordx3 instruction reads 768 contiguous B);
//   SHAPE 1 -- each lane's 48 contiguous B (16 pixels) as 3 dwordx4 (an
//              instruction touches every third 16-B word of the 3072 B);
//   SHAPE 2 -- 3 dwordx4 lane-interleaved (an instruction reads 1024
//              contiguous B; pixels straddle lanes).
// SCHED 0 -- one contiguous (tile, frame) range per wave; SCHED 1 -- the
// part-major schedule (parts of L frames, items (part, tile) with stride
// n_waves), as series_v2_body.  Two frames of loads in flight.
template <int SHAPE, int SCHED>
__global__ __launch_bounds__(256) void shape_kernel(const uint8_t* frames, uint32_t fb, uint32_t n_frames,
                                                    uint32_t n_tiles, uint32_t n_waves, uint32_t plen,
                                                    uint32_t* out) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
    if (wave >= n_waves) return;
    const uint64_t items = (uint64_t)n_tiles * n_frames;
    uint64_t i = (uint64_t)wave * items / n_waves;
    const uint64_t iend = (uint64_t)(wave + 1) * items / n_waves;
    const uint64_t pitems = SCHED ? (uint64_t)((n_frames + plen - 1) / plen) * n_tiles : 0u;
    uint64_t it = wave;
    uint32_t acc = 0;
    while (true) {
        uint32_t tile, t, tend;
        if (SCHED == 0) {
            if (i >= iend) break;
            tile = (uint32_t)(i / n_frames);
            t = (uint32_t)(i - (uint64_t)tile * n_frames);
            const uint64_t rem = iend - i;
            tend = (uint32_t)((uint64_t)n_frames < t + rem ? (uint64_t)n_frames : t + rem);
            i += tend - t;
        } else {
            if (it >= pitems) break;
            const uint32_t part = (uint32_t)(it / n_tiles);
            tile = (uint32_t)(it - (uint64_t)part * n_tiles);
            t = part * plen;
            tend = min(n_frames, t + plen);
            it += n_waves;
        }
        const uint32_t base = tile * 3072u;
        for (; t < tend; t += 2) {
            const uint32_t t1 = t + 1 < tend ? t + 1 : t;
            const __amdgpu_buffer_rsrc_t r0 = rsrc(frames + (uint64_t)t * fb, fb);
            const __amdgpu_buffer_rsrc_t r1 = rsrc(frames + (uint64_t)t1 * fb, fb);
            uint32_t x = 0;
            if constexpr (SHAPE == 0) {
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const uint32_t o = base + (u * 64u + lane) * 12u;
                    const u32x3 a = __builtin_amdgcn_raw_buffer_load_b96(r0, o, 0, 2);
                    const u32x3 b = __builtin_amdgcn_raw_buffer_load_b96(r1, o, 0, 2);
                    x ^= a.x ^ a.y ^ a.z ^ b.x ^ b.y ^ b.z;
                }
            } else {
#pragma unroll
                for (int u = 0; u < 3; ++u) {
                    const uint32_t o = SHAPE == 1 ? base + lane * 48u + u * 16u : base + (u * 64u + lane) * 16u;
                    const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(r0, o, 0, 2);
                    const u32x4 b = __builtin_amdgcn_raw_buffer_load_b128(r1, o, 0, 2);
                    x ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w;
                }
            }
            acc ^= x;
        }
    }
    if (acc == 0x9E3779B9u) out[0] = acc;
}

int main(int argc, char** argv) {
    const uint32_t W = 3840, H = 2160, C = 3;
    const uint32_t nf = argc > 1 ? (uint32_t)std::atoi(argv[1]) : 5000;
    const uint64_t fb = (uint64_t)W * H * C;
    const uint64_t total = fb * nf;
    uint8_t* d = nullptr;
    uint32_t* o = nullptr;
    CK(hipMalloc(&d, total));
    CK(hipMalloc(&o, 256));
    CK(hipMemset(d, 7, total));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char* name, auto launch) {
        launch();
        CK(hipDeviceSynchronize());
        float best = 1e30f, sum = 0;
        for (int r = 0; r < 3; ++r) {
            CK(hipEventRecord(e0, 0));
            launch();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
            sum += ms;
        }
        CK(hipEventRecord(e0, 0));
        for (int r = 0; r < 10; ++r) launch();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms10;
        CK(hipEventElapsedTime(&ms10, e0, e1));
        ms10 /= 10;
        std::printf("{\"shape\": \"%s\", \"frames\": %u, \"bytes\": %llu, \"ms_mean3\": %.3f, \"GBps_mean3\": %.1f, "
                    "\"ms_sustained10\": %.3f, \"GBps_sustained10\": %.1f}\n",
                    name, nf, (unsigned long long)total, sum / 3, total / (sum / 3 * 1e-3) / 1e9, ms10,
                    total / (ms10 * 1e-3) / 1e9);
        std::fflush(stdout);
    };
    const bool all = argc > 2 && argv[2][0] == 'a';
    run("grid: 16-B nt loads, grid-stride, 1024 blocks (library read_ceiling_kernel)", [&] {
        hipLaunchKernelGGL(grid_kernel, dim3(1024), dim3(256), 0, 0, (const u32x4*)d, total / 16, o);
    });
    for (uint32_t wps : {5u, 8u}) {
        if (!all) break;
        const uint32_t n_tiles12 = (uint32_t)((fb / 12 + 255) / 256);
        const uint32_t waves = wps * 4 * cus;
        char name[160];
        std::snprintf(name, sizeof name, "walk12: series-kernel shape, 12-B vecs, %u waves/SIMD", wps);
        run(name, [&] {
            hipLaunchKernelGGL(walk_kernel<12>, dim3(waves / 4), dim3(256), 0, 0, d, (uint32_t)fb, nf, n_tiles12,
                               waves, o);
        });
        const uint32_t n_tiles16 = (uint32_t)((fb / 16 + 255) / 256);
        std::snprintf(name, sizeof name, "walk16: series-kernel shape, 16-B vecs, %u waves/SIMD", wps);
        run(name, [&] {
            hipLaunchKernelGGL(walk_kernel<16>, dim3(waves / 4), dim3(256), 0, 0, d, (uint32_t)fb, nf, n_tiles16,
                               waves, o);
        });
    }
    if (all) {
        const uint32_t n_tiles12 = (uint32_t)((fb / 12 + 255) / 256);
        for (uint32_t waves : {n_tiles12, n_tiles12 / 2, n_tiles12 / 3}) {
            char name[160];
            std::snprintf(name, sizeof name, "lockstep12: %u waves, %u tile(s) each, all frames in order", waves,
                          n_tiles12 / waves);
            run(name, [&] {
                hipLaunchKernelGGL(lockstep_kernel<12>, dim3((waves + 3) / 4), dim3(256), 0, 0, d, (uint32_t)fb, nf,
                                   n_tiles12, waves, o);
            });
        }
    }
    {
        // the three tile shapes, contiguous ranges and part-major (L = 1000,
        // the library's 4K choice), 5 waves/SIMD (the series kernel's);
        // alternated over two rounds in this one process
        const uint32_t n_tiles = (uint32_t)((fb / 12 + 255) / 256);
        const uint32_t slots = 5u * 4u * (uint32_t)cus;
        const uint32_t L = nf >= 1000 ? 1000u : nf;
        const uint64_t pitems = (uint64_t)((nf + L - 1) / L) * n_tiles;
        const uint32_t kk = (uint32_t)((pitems + slots - 1) / slots);
        const uint32_t pwaves = (uint32_t)((pitems + kk - 1) / kk);
        const char* shapes[3] = {"4 x dwordx3 lane-interleaved (series kernel)", "3 x dwordx4 lane-contiguous 48 B",
                                 "3 x dwordx4 lane-interleaved"};
        for (int round = 0; round < 2; ++round)
            for (int sh = 0; sh < 3; ++sh)
                for (int sc = 0; sc < 2; ++sc) {
                    char name[200];
                    std::snprintf(name, sizeof name, "tile shape %s, %s, round %d", shapes[sh],
                                  sc ? "part-major L=1000" : "contiguous ranges", round);
                    const uint32_t waves = sc ? pwaves : slots;
                    run(name, [&] {
                        const dim3 g((waves + 3) / 4), b(256);
                        if (sh == 0 && sc == 0) hipLaunchKernelGGL((shape_kernel<0, 0>), g, b, 0, 0, d, (uint32_t)fb, nf, n_tiles, waves, L, o);
                        if (sh == 0 && sc == 1) hipLaunchKernelGGL((shape_kernel<0, 1>), g, b, 0, 0, d, (uint32_t)fb, nf, n_tiles, waves, L, o);
                        if (sh == 1 && sc == 0) hipLaunchKernelGGL((shape_kernel<1, 0>), g, b, 0, 0, d, (uint32_t)fb, nf, n_tiles, waves, L, o);
                        if (sh == 1 && sc == 1) hipLaunchKernelGGL((shape_kernel<1, 1>), g, b, 0, 0, d, (uint32_t)fb, nf, n_tiles, waves, L, o);
                        if (sh == 2 && sc == 0) hipLaunchKernelGGL((shape_kernel<2, 0>), g, b, 0, 0, d, (uint32_t)fb, nf, n_tiles, waves, L, o);
                        if (sh == 2 && sc == 1) hipLaunchKernelGGL((shape_kernel<2, 1>), g, b, 0, 0, d, (uint32_t)fb, nf, n_tiles, waves, L, o);
                    });
                }
    }
    CK(hipFree(d));
    CK(hipFree(o));
    return 0;
}
