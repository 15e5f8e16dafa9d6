// policy_probe.hip -- the series kernel (4K RGB8, per-frame, tau 8/255)
// back to back for a fixed time with the frame loads' cache-policy bits set
// at build time (-DDIPS_LOAD_AUX=<aux>: gfx950 sc0 = 1, nt = 2, sc1 = 16),
// for tools/policy_energy.py, which samples the energy counter meanwhile.
// Prints "run <aux> <t0> <t1> <launches> <frames> <median ms>" (steady clock).
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -DDIPS_LOAD_AUX=2 -o build/policy_2 tools/policy_probe.hip
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

int main(int argc, char** argv) {
    const uint32_t W = 3840, H = 2160, C = 3;
    const uint32_t F = argc > 1 ? (uint32_t)atoi(argv[1]) : 2000;
    const double secs = argc > 2 ? atof(argv[2]) : 5.0;
    const uint64_t fb = (uint64_t)W * H * C, total = fb * F;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess) return 1;
    uint8_t* frames = nullptr;
    uint64_t* partials = nullptr;
    dips_series_entry* series = nullptr;
    // optional: byte offsets of the frames base inside a larger allocation
    // (argv[3], comma list), each timed for `secs` in this one process
    std::vector<uint64_t> offs = {0};
    if (argc > 3) {
        offs.clear();
        for (char* q = argv[3]; *q;) {
            offs.push_back(strtoull(q, &q, 10));
            if (*q == ',') ++q;
        }
    }
    const uint64_t max_off = *std::max_element(offs.begin(), offs.end());
    uint8_t* base = nullptr;
    if (hipMalloc(&base, total + max_off + 4096) != hipSuccess) return 1;
    frames = base;
    SynthArgs sa{};
    sa.dst = frames; sa.total_bytes = total; sa.frame_bytes = fb; sa.seed = 0xD1B5; sa.t0 = 0;
    sa.channels = C; sa.width = W; sa.height = H; sa.radius = H / 8;
    if (launch_synth(sa, 0) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return 1;
    const void* k = (const void*)&series_v2_kernel<3, 0, kUnrollV2, true, false>;
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k, 256, 0) != hipSuccess) return 1;
    const uint64_t nvec = fb / 12, tiles = (nvec + 64ull * kUnrollV2 - 1) / (64ull * kUnrollV2);
    SeriesArgs a{};
    a.frames = frames; a.ref0 = frames; a.frame_bytes = (uint32_t)fb; a.vec_bytes = (uint32_t)fb; a.n_frames = F;
    a.n_tiles = (uint32_t)tiles; a.items = tiles * F;
    a.n_waves = (uint32_t)std::min<uint64_t>(a.items, (uint64_t)occ * cus * 4);
    a.thr = series_threshold(3, 8.0f / 255.0f);
    if (hipMalloc(&partials, a.items * 16 + 4096) != hipSuccess) return 1;
    if (hipMalloc(&series, sizeof(dips_series_entry) * F) != hipSuccess) return 1;
    a.partials = partials;
    const uint32_t blocks = (a.n_waves + 3) / 4;
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return 1;
    auto run = [&]() {
        (void)hipMemsetAsync(series, 0, sizeof(dips_series_entry) * F, 0);
        hipLaunchKernelGGL((series_v2_kernel<3, 0, kUnrollV2, true, false>), dim3(blocks), dim3(256), 0, 0, a);
        return launch_series_reduce(partials, F, a.n_tiles, 0, series, 0);
    };
    for (uint64_t off : offs) {
    if (off != 0 || offs.size() > 1) {
        // regenerate the frames at this offset (same contents)
        frames = base + off;
        sa.dst = frames;
        if (launch_synth(sa, 0) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return 1;
        a.frames = frames; a.ref0 = frames;
    }
    if (run() != hipSuccess || hipDeviceSynchronize() != hipSuccess) return 1;
    std::vector<float> ms;
    long launches = 0;
    const double t0 = now();
    while (now() - t0 < secs) {
        if (hipEventRecord(e0, 0) != hipSuccess || run() != hipSuccess || hipEventRecord(e1, 0) != hipSuccess) return 1;
        if (hipEventSynchronize(e1) != hipSuccess) return 1;
        float t = 0;
        (void)hipEventElapsedTime(&t, e0, e1);
        ms.push_back(t);
        ++launches;
    }
    const double t1 = now();
    std::sort(ms.begin(), ms.end());
    // checksum of the series so that the variants can be compared
    std::vector<dips_series_entry> h(F);
    if (hipMemcpy(h.data(), series, sizeof(dips_series_entry) * F, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    uint64_t ck = 0;
    for (const auto& e : h) ck = ck * 1000003ull + e.sad + 7 * e.sj + 13 * e.count + 17 * e.si_fixed;
    printf("run\t%d\t%.6f\t%.6f\t%ld\t%u\t%.4f\t%016llx\t%llu\t%p\n", DIPS_LOAD_AUX, t0, t1, launches, F,
           ms[ms.size() / 2], (unsigned long long)ck, (unsigned long long)off, (void*)frames);
    fflush(stdout);
    }
    return 0;
}
