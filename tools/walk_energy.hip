// walk_energy.hip -- read schedules of the series path compared by time AND
// energy in one process over one buffer (tools/walk_energy.py samples the
// energy counter).  4K RGB8 frames, 12-B vecs, 64 lanes x 4 vecs per tile:
//   walk     -- the series kernel's schedule: one contiguous (tile, frame)
//               range per wave, so concurrent waves sit at unrelated frames;
//   parts    -- frames cut into parts of L; items (part, tile) part-major,
//               wave w takes items w, w + W, ...: all waves sweep the same
//               frames of adjacent tiles together (plus one reference frame
//               per item, the series kernel's reload);
//   grid     -- grid-stride 16-B reads (the library's read ceiling kernel);
//   series   -- the shipped series kernel (per-frame, tau 8/255).
// Usage: walk_energy <frames> <seconds per run> <rounds> <L>
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o build/walk_energy tools/walk_energy.hip
#include "../dips_amd/csrc/series_kernels.hip"
#include "../dips_amd/csrc/series_v2.hip"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace dips;

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

__global__ __launch_bounds__(256) void parts_kernel(const uint8_t* frames, uint32_t fb, uint32_t n_frames,
                                                    uint32_t n_tiles, uint32_t L, uint32_t n_waves, uint32_t* out) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
    if (wave >= n_waves) return;
    const uint32_t n_parts = (n_frames + L - 1) / L;
    const uint64_t items = (uint64_t)n_parts * n_tiles;
    uint32_t acc = 0;
    for (uint64_t it = wave; it < items; it += n_waves) {
        const uint32_t part = (uint32_t)(it / n_tiles), tile = (uint32_t)(it - (uint64_t)part * n_tiles);
        const uint32_t f0 = part * L, f1 = min(n_frames, f0 + L);
        const uint32_t voff = (tile * 4u * 64u + lane) * 12u;
        // the reference tile (frame f0 - 1), as the series kernel reloads it
        {
            const __amdgpu_buffer_rsrc_t rr = make_rsrc(frames + (uint64_t)(f0 ? f0 - 1 : 0) * fb, fb);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const u32x3 a = __builtin_amdgcn_raw_buffer_load_b96(rr, voff + u * 64 * 12, 0, 2);
                acc ^= a.x ^ a.y ^ a.z;
            }
        }
        for (uint32_t t = f0; t < f1; t += 2) {
            const uint32_t t1 = t + 1 < f1 ? t + 1 : t;
            const __amdgpu_buffer_rsrc_t r0 = make_rsrc(frames + (uint64_t)t * fb, fb);
            const __amdgpu_buffer_rsrc_t r1 = make_rsrc(frames + (uint64_t)t1 * fb, fb);
            uint32_t x = 0;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const u32x3 a = __builtin_amdgcn_raw_buffer_load_b96(r0, voff + u * 64 * 12, 0, 2);
                const u32x3 b = __builtin_amdgcn_raw_buffer_load_b96(r1, voff + u * 64 * 12, 0, 2);
                x ^= a.x ^ a.y ^ a.z ^ b.x ^ b.y ^ b.z;
            }
            acc ^= x;
        }
    }
    if (acc == 0x9E3779B9u) out[0] = acc;
}

int main(int argc, char** argv) {
    const uint32_t W = 3840, H = 2160, C = 3;
    const uint32_t F = argc > 1 ? (uint32_t)atoi(argv[1]) : 2000;
    const double secs = argc > 2 ? atof(argv[2]) : 4.0;
    const int rounds = argc > 3 ? atoi(argv[3]) : 2;
    const uint32_t L = argc > 4 ? (uint32_t)atoi(argv[4]) : 128;
    const uint64_t fb = (uint64_t)W * H * C, total = fb * F;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess) return 1;
    uint8_t* frames = nullptr;
    if (hipMalloc(&frames, total) != hipSuccess) return 1;
    SynthArgs sa{};
    sa.dst = frames; sa.total_bytes = total; sa.frame_bytes = fb; sa.seed = 0xD1B5; sa.t0 = 0;
    sa.channels = C; sa.width = W; sa.height = H; sa.radius = H / 8;
    if (launch_synth(sa, 0) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return 1;
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)&series_v2_kernel<3, 0, kUnrollV2, true, false>,
                                                     256, 0) != hipSuccess)
        return 1;
    const uint64_t nvec = fb / 12, tiles = (nvec + 64ull * kUnrollV2 - 1) / (64ull * kUnrollV2);
    SeriesArgs a{};
    a.frames = frames; a.ref0 = frames;
    a.frame_bytes = (uint32_t)fb; a.vec_bytes = (uint32_t)fb; a.n_frames = F;
    a.n_tiles = (uint32_t)tiles; a.items = tiles * F;
    a.n_waves = (uint32_t)std::min<uint64_t>(a.items, (uint64_t)occ * cus * 4);
    a.thr = series_threshold(3, 8.0f / 255.0f);
    uint64_t* partials = nullptr;
    dips_series_entry* series = nullptr;
    uint32_t* sink = nullptr;
    if (hipMalloc(&partials, a.items * 16 + 4096) != hipSuccess) return 1;
    if (hipMalloc(&series, sizeof(dips_series_entry) * F) != hipSuccess) return 1;
    if (hipMalloc(&sink, 4096) != hipSuccess) return 1;
    a.partials = partials;
    const uint32_t blocks = (a.n_waves + 3) / 4;
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return 1;
    const char* names[] = {"walk", "parts", "grid", "series"};
    for (int r = 0; r < rounds; ++r) {
        for (int what = 0; what < 4; ++what) {
            std::vector<float> ms;
            const double t0 = now();
            while (now() - t0 < secs) {
                if (what == 3) (void)hipMemsetAsync(series, 0, sizeof(dips_series_entry) * F, 0);
                if (hipEventRecord(e0, 0) != hipSuccess) return 1;
                hipError_t e = hipSuccess;
                if (what == 0) {
                    e = launch_read_walk(a, 12, blocks, sink, 0);
                } else if (what == 1) {
                    hipLaunchKernelGGL(parts_kernel, dim3(blocks), dim3(256), 0, 0, frames, (uint32_t)fb, F,
                                       (uint32_t)tiles, L, a.n_waves, sink);
                    e = hipGetLastError();
                } else if (what == 2) {
                    e = launch_read_ceiling(frames, total, sink, 0);
                } else {
                    hipLaunchKernelGGL((series_v2_kernel<3, 0, kUnrollV2, true, false>), dim3(blocks), dim3(256), 0, 0, a);
                    e = launch_series_reduce(partials, F, a.n_tiles, 0, series, 0);
                }
                if (e != hipSuccess) return 1;
                if (hipEventRecord(e1, 0) != hipSuccess || hipEventSynchronize(e1) != hipSuccess) return 1;
                float t = 0;
                (void)hipEventElapsedTime(&t, e0, e1);
                ms.push_back(t);
            }
            const double t1 = now();
            std::sort(ms.begin(), ms.end());
            const double med = ms[ms.size() / 2];
            printf("run\t%d\t%s\t%.6f\t%.6f\t%.4f\t%.4f\t%u\n", r, names[what], t0, t1, med,
                   (double)total / (med / 1e3) / 8e12, F);
            fflush(stdout);
            const double g = now();
            while (now() - g < 1.0) {}
        }
    }
    return 0;
}
