// sched_ab.hip -- schedule A/B of the series kernel in ONE process over ONE
// frame buffer: the shipped contiguous (tile, frame) range per wave against
// the part-major schedule (series_v2_body SCHED = 1) at several part
// lengths L.  4K RGB8, per-frame, tau 8/255; series checked equal.
// Prints "run <round> <name> <t0> <t1> <median ms> <frac of 8 TB/s> <frames>"
// (tools/walk_energy.py --bin build/sched_ab adds the energy per frame).
// Usage: sched_ab <frames> <seconds per run> <rounds> <L,L,...>
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o build/sched_ab tools/sched_ab.hip
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

__global__ __launch_bounds__(256, (v2_min_waves<3, kUnrollV2, true, false>())) void parts_series(SeriesArgs a) {
    series_v2_body<3, 0, kUnrollV2, true, false, kAuxNT, kAuxNT, 1>(a);
}

int main(int argc, char** argv) {
    const uint32_t W = 3840, H = 2160, C = 3;
    const uint32_t F = argc > 1 ? (uint32_t)atoi(argv[1]) : 2000;
    const double secs = argc > 2 ? atof(argv[2]) : 3.0;
    const int rounds = argc > 3 ? atoi(argv[3]) : 2;
    std::vector<uint32_t> Ls = {0};
    if (argc > 4)
        for (char* q = argv[4]; *q;) {
            Ls.push_back((uint32_t)strtoul(q, &q, 10));
            if (*q == ',') ++q;
        }
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
    if (hipMalloc(&partials, a.items * 16 + 4096) != hipSuccess) return 1;
    if (hipMalloc(&series, sizeof(dips_series_entry) * F) != hipSuccess) return 1;
    a.partials = partials;
    const uint32_t blocks = (a.n_waves + 3) / 4;
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return 1;
    std::vector<dips_series_entry> ref(F), h(F);
    bool have_ref = false;
    for (int r = 0; r < rounds; ++r) {
        for (uint32_t L : Ls) {
            SeriesArgs args = a;
            args.part_frames = L;
            std::vector<float> ms;
            const double t0 = now();
            while (now() - t0 < secs) {
                (void)hipMemsetAsync(series, 0, sizeof(dips_series_entry) * F, 0);
                if (hipEventRecord(e0, 0) != hipSuccess) return 1;
                if (L == 0)
                    hipLaunchKernelGGL((series_v2_kernel<3, 0, kUnrollV2, true, false>), dim3(blocks), dim3(256), 0, 0,
                                       args);
                else
                    hipLaunchKernelGGL(parts_series, dim3(blocks), dim3(256), 0, 0, args);
                if (launch_series_reduce(partials, F, a.n_tiles, 0, series, 0) != hipSuccess) return 1;
                if (hipEventRecord(e1, 0) != hipSuccess || hipEventSynchronize(e1) != hipSuccess) return 1;
                float t = 0;
                (void)hipEventElapsedTime(&t, e0, e1);
                ms.push_back(t);
            }
            const double t1 = now();
            if (hipMemcpy(h.data(), series, sizeof(dips_series_entry) * F, hipMemcpyDeviceToHost) != hipSuccess) return 1;
            if (!have_ref) { ref = h; have_ref = true; }
            bool same = true;
            for (uint32_t t = 0; t < F; ++t)
                same = same && h[t].sad == ref[t].sad && h[t].sj == ref[t].sj && h[t].count == ref[t].count &&
                       h[t].si_fixed == ref[t].si_fixed;
            std::sort(ms.begin(), ms.end());
            const double med = ms[ms.size() / 2];
            std::string name = L == 0 ? "contiguous" : "parts" + std::to_string(L);
            printf("run\t%d\t%s%s\t%.6f\t%.6f\t%.4f\t%.4f\t%u\n", r, name.c_str(), same ? "" : "-DIFF", t0, t1, med,
                   (double)total / (med / 1e3) / 8e12, F);
            fflush(stdout);
            const double g = now();
            while (now() - g < 1.0) {}
        }
    }
    return 0;
}
