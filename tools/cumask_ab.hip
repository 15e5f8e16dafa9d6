// cumask_ab.hip -- the headline series kernel (4K RGB8, per-frame, tau 8/255,
// integer SI) on streams restricted to a fraction of the CUs
// (hipExtStreamCreateWithCUMask), in ONE process over ONE frame buffer,
// alternated over rounds: does leaving CUs idle (clock-gated) lower the
// package power enough that the rest run faster under the power limit?
// The persistent grid fills the enabled CUs at the kernel's occupancy.
// Output lines "run <round> <name> <t0> <t1> <median ms> <frac of 8 TB/s>
// <frames>" for tools/walk_energy.py (--bin build/cumask_ab), which adds the
// SMU energy of each window.
// Usage: cumask_ab <frames> <seconds per run> <rounds>
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o build/cumask_ab tools/cumask_ab.hip
#include "../dips_amd/csrc/series_kernels.hip"
#include "../dips_amd/csrc/series_v2.hip"

#include <hip/hip_ext.h>

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

struct Variant {
    const char* name;
    int keep_of_8;  // CUs kept in every group of 8 consecutive mask bits
};

int main(int argc, char** argv) {
    const uint32_t W = 3840, H = 2160, C = 3;
    const uint32_t F = argc > 1 ? (uint32_t)atoi(argv[1]) : 2000;
    const double secs = argc > 2 ? atof(argv[2]) : 3.0;
    const int rounds = argc > 3 ? atoi(argv[3]) : 2;
    const uint64_t fb = (uint64_t)W * H * C, total = fb * F;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess) return 1;
    uint8_t* frames = nullptr;
    if (hipMalloc(&frames, total) != hipSuccess) return 1;
    SynthArgs sa{};
    sa.dst = frames; sa.total_bytes = total; sa.frame_bytes = fb; sa.seed = 0xD1B5; sa.t0 = 0;
    sa.channels = C; sa.width = W; sa.height = H; sa.radius = H / 8;
    if (launch_synth(sa, 0) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return 1;
    const void* k = series_v2_kernel_ptr(3, 0, true, false, false, 1);
    int occ = 0;
    if (!k || hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k, 256, 0) != hipSuccess || occ < 1) return 1;
    const uint64_t nvec = fb / 12, tiles = (nvec + 64ull * kUnrollV2 - 1) / (64ull * kUnrollV2);
    uint64_t* partials = nullptr;
    dips_series_entry* series = nullptr;
    SeriesArgs a{};
    a.frames = frames; a.ref0 = frames;
    a.frame_bytes = (uint32_t)fb; a.vec_bytes = (uint32_t)fb; a.n_frames = F;
    a.n_tiles = (uint32_t)tiles; a.items = tiles * F;
    a.thr = series_threshold(3, 8.0f / 255.0f, 1);
    if (hipMalloc(&partials, a.items * 16 + 4096) != hipSuccess) return 1;
    if (hipMalloc(&series, sizeof(dips_series_entry) * F) != hipSuccess) return 1;
    a.partials = partials;
    // CU masks: keep k of every 8 consecutive mask bits (balanced over the
    // XCDs whether the mask's bits run XCD by XCD or interleave them)
    const std::vector<Variant> vs = {{"all", 8}, {"7/8", 7}, {"3/4", 6}, {"5/8", 5}, {"1/2", 4}};
    const uint32_t words = (uint32_t)((cus + 31) / 32);
    std::vector<hipStream_t> streams;
    std::vector<uint32_t> active;
    for (const Variant& v : vs) {
        std::vector<uint32_t> mask(words, 0u);
        uint32_t n = 0;
        for (int i = 0; i < cus; ++i)
            if ((i % 8) < v.keep_of_8) {
                mask[i / 32] |= 1u << (i % 32);
                ++n;
            }
        hipStream_t s = nullptr;
        if (hipExtStreamCreateWithCUMask(&s, words, mask.data()) != hipSuccess) return 1;
        streams.push_back(s);
        active.push_back(n);
    }
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return 1;
    std::vector<dips_series_entry> ref(F), h(F);
    for (int r = 0; r < rounds; ++r) {
        for (size_t vi = 0; vi < vs.size(); ++vi) {
            const size_t i = (r % 2 == 0) ? vi : vs.size() - 1 - vi;
            hipStream_t s = streams[i];
            SeriesArgs args = a;
            args.n_waves = (uint32_t)std::min<uint64_t>(a.items, (uint64_t)occ * active[i] * 4);
            const uint32_t blocks = (args.n_waves + 3) / 4;
            std::vector<float> ms;
            const double t0 = now();
            while (now() - t0 < secs) {
                (void)hipMemsetAsync(series, 0, sizeof(dips_series_entry) * F, s);
                if (hipEventRecord(e0, s) != hipSuccess) return 1;
                void* params[] = {&args};
                if (hipLaunchKernel(k, dim3(blocks), dim3(256), params, 0, s) != hipSuccess) return 1;
                if (hipEventRecord(e1, s) != hipSuccess) return 1;
                if (launch_series_reduce(partials, F, a.n_tiles, 0, series, s) != hipSuccess) return 1;
                if (hipStreamSynchronize(s) != hipSuccess) return 1;
                float t = 0;
                (void)hipEventElapsedTime(&t, e0, e1);
                ms.push_back(t);
            }
            const double t1 = now();
            if (hipMemcpy(h.data(), series, sizeof(dips_series_entry) * F, hipMemcpyDeviceToHost) != hipSuccess) return 1;
            if (r == 0 && vi == 0) ref = h;
            const bool same = std::equal(h.begin(), h.end(), ref.begin(), [](const dips_series_entry& x,
                                                                           const dips_series_entry& y) {
                return x.sad == y.sad && x.sj == y.sj && x.count == y.count && x.si_fixed == y.si_fixed;
            });
            std::sort(ms.begin(), ms.end());
            const double med = ms[ms.size() / 2];
            printf("run\t%d\t%s(%u CUs)%s\t%.6f\t%.6f\t%.4f\t%.4f\t%u\n", r, vs[i].name, active[i], same ? "" : " DIFF",
                   t0, t1, med, (double)total / (med / 1e3) / 8e12, F);
            fflush(stdout);
        }
    }
    return 0;
}
