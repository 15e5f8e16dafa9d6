// alloc_probe.hip -- does the series kernel's rate depend on where its frame
// buffer landed?  Allocates several frame buffers in one process (hipMalloc
// "m" or hipExtMallocWithFlags(hipDeviceMallocContiguous) "c"), fills each with
// the same synthetic frames, and times the series kernel (4K RGB8, per-frame,
// tau 8/255) over each buffer in alternated rounds.
// Usage: alloc_probe <frames> <seconds per run> <rounds> <m,m,c,...>
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o build/alloc_probe tools/alloc_probe.hip
#include "../dips_amd/csrc/series_kernels.hip"
#include "../dips_amd/csrc/series_v2.hip"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

using namespace dips;

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
    const uint32_t W = 3840, H = 2160, C = 3;
    const uint32_t F = argc > 1 ? (uint32_t)atoi(argv[1]) : 2000;
    const double secs = argc > 2 ? atof(argv[2]) : 2.0;
    const int rounds = argc > 3 ? atoi(argv[3]) : 2;
    const std::string kinds = argc > 4 ? argv[4] : "m,m,m";
    const uint64_t fb = (uint64_t)W * H * C, total = fb * F;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess) return 1;
    std::vector<uint8_t*> bufs;
    std::vector<char> kind;
    for (char k : kinds) {
        if (k == ',') continue;
        uint8_t* p = nullptr;
        hipError_t e = k == 'c' ? hipExtMallocWithFlags((void**)&p, total, hipDeviceMallocContiguous)
                                : hipMalloc(&p, total);
        if (e != hipSuccess) {
            printf("alloc\t%c\tfailed\t%s\n", k, hipGetErrorString(e));
            continue;
        }
        bufs.push_back(p);
        kind.push_back(k);
        SynthArgs sa{};
        sa.dst = p; sa.total_bytes = total; sa.frame_bytes = fb; sa.seed = 0xD1B5; sa.t0 = 0;
        sa.channels = C; sa.width = W; sa.height = H; sa.radius = H / 8;
        if (launch_synth(sa, 0) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return 1;
    }
    if (bufs.empty()) return 1;
    const void* kp = (const void*)&series_v2_kernel<3, 0, kUnrollV2, true, false>;
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kp, 256, 0) != hipSuccess) return 1;
    const uint64_t nvec = fb / 12, tiles = (nvec + 64ull * kUnrollV2 - 1) / (64ull * kUnrollV2);
    uint64_t* partials = nullptr;
    dips_series_entry* series = nullptr;
    SeriesArgs a{};
    a.frame_bytes = (uint32_t)fb; a.vec_bytes = (uint32_t)fb; a.n_frames = F;
    a.n_tiles = (uint32_t)tiles; a.items = tiles * F;
    a.n_waves = (uint32_t)std::min<uint64_t>(a.items, (uint64_t)occ * cus * 4);
    a.thr = series_threshold(3, 8.0f / 255.0f);
    if (hipMalloc(&partials, a.items * 16 + 4096) != hipSuccess) return 1;
    if (hipMalloc(&series, sizeof(dips_series_entry) * F) != hipSuccess) return 1;
    a.partials = partials;
    uint32_t* sink = nullptr;
    if (hipMalloc(&sink, 4096) != hipSuccess) return 1;
    const uint32_t blocks = (a.n_waves + 3) / 4;
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return 1;
    for (int r = 0; r < rounds; ++r) {
        for (size_t b = 0; b < bufs.size(); ++b) {
            a.frames = bufs[b];
            a.ref0 = bufs[b];
            for (int what = 0; what < 3; ++what) {  // series, read walk (same shape), grid-stride read
                std::vector<float> ms;
                const double t0 = now();
                while (now() - t0 < (what == 0 ? secs : secs / 2)) {
                    (void)hipMemsetAsync(series, 0, sizeof(dips_series_entry) * F, 0);
                    if (hipEventRecord(e0, 0) != hipSuccess) return 1;
                    if (what == 0) {
                        hipLaunchKernelGGL((series_v2_kernel<3, 0, kUnrollV2, true, false>), dim3(blocks), dim3(256),
                                           0, 0, a);
                        if (launch_series_reduce(partials, F, a.n_tiles, 0, series, 0) != hipSuccess) return 1;
                    } else if (what == 1) {
                        if (launch_read_walk(a, 12, blocks, sink, 0) != hipSuccess) return 1;
                    } else {
                        if (launch_read_ceiling(bufs[b], total, sink, 0) != hipSuccess) return 1;
                    }
                    if (hipEventRecord(e1, 0) != hipSuccess || hipEventSynchronize(e1) != hipSuccess) return 1;
                    float t = 0;
                    (void)hipEventElapsedTime(&t, e0, e1);
                    ms.push_back(t);
                }
                const double t1 = now();
                std::sort(ms.begin(), ms.end());
                const double med = ms[ms.size() / 2];
                printf("run\t%d\t%zu\t%c\t%s\t%p\t%.6f\t%.6f\t%.4f\t%.4f\n", r, b, kind[b],
                       what == 0 ? "series" : (what == 1 ? "walk" : "grid"), (void*)bufs[b], t0, t1, med,
                       (double)total / (med / 1e3) / 8e12);
                fflush(stdout);
            }
        }
    }
    for (auto p : bufs) (void)hipFree(p);
    return 0;
}
