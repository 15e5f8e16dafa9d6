// alloc_policy_ab.hip -- the headline series kernel (4K RGB8, per-frame,
// tau 8/255, integer SI) over frame buffers allocated with different memory
// types (hipExtMallocWithFlags: default coarse-grained, fine-grained,
// uncached, contiguous), in ONE process, alternated over rounds: does a
// memory type that skips the caches read the frames for less energy, and so
// faster under the package power limit?  Same frames in every buffer (one
// synthesis, copied); the series of every run is compared with the first.
// Output lines "run <round> <name> <t0> <t1> <median ms> <frac of 8 TB/s>
// <frames>" for tools/walk_energy.py (--bin build/alloc_policy_ab), which
// adds the SMU energy of each window.
// Usage: alloc_policy_ab <frames> <seconds per run> <rounds> [kinds, e.g.
// default,finegrained,default,finegrained: repeated kinds separate the memory
// type from where a buffer happens to land; "padN" allocates N GiB that is
// not measured, before the next buffer)] [L,L,...: also the part-major
// schedule (series_v2_body SCHED = 1) with parts of L frames, per buffer]
// [waves of the part-major runs: e.g. 4050 = 32,400 items of L = 1250 / 8]
// (an L written with a trailing x, e.g. 1000x, runs the part-major schedule
// in 1024-thread workgroups)
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o build/alloc_policy_ab tools/alloc_policy_ab.hip
#include "../dips_amd/csrc/series_kernels.hip"
#include "../dips_amd/csrc/series_v2.hip"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

using namespace dips;

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

__global__ __launch_bounds__(256, (v2_min_waves<3, kUnrollV2Rgb, true, false, false>())) void parts_isi(SeriesArgs a) {
    series_v2_body<3, 0, kUnrollV2Rgb, true, false, kAuxNT, kAuxNT, 1, false, 1>(a);
}
// the same in 1024-thread workgroups: the 16 waves of a CU (at 4 per SIMD)
// take 16 adjacent tiles, 61 KB of each frame, instead of 4 groups of 4
__global__ __launch_bounds__(1024, (v2_min_waves<3, kUnrollV2Rgb, true, false, false>())) void parts_isi_wg16(SeriesArgs a) {
    series_v2_body<3, 0, kUnrollV2Rgb, true, false, kAuxNT, kAuxNT, 1, false, 1, 16>(a);
}

struct Kind {
    const char* name;
    unsigned flags;
};

int main(int argc, char** argv) {
    const uint32_t W = 3840, H = 2160, C = 3;
    const uint32_t F = argc > 1 ? (uint32_t)atoi(argv[1]) : 2000;
    const double secs = argc > 2 ? atof(argv[2]) : 3.0;
    const int rounds = argc > 3 ? atoi(argv[3]) : 2;
    const uint64_t fb = (uint64_t)W * H * C, total = fb * F;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess) return 1;
    const std::vector<Kind> all = {{"default", hipDeviceMallocDefault},
                                   {"finegrained", hipDeviceMallocFinegrained},
                                   {"uncached", hipDeviceMallocUncached},
                                   {"contiguous", hipDeviceMallocContiguous}};
    std::vector<Kind> kinds;
    {
        const std::string list = argc > 4 ? argv[4] : "default,finegrained,uncached,contiguous";
        size_t pos = 0;
        while (pos <= list.size()) {
            const size_t e = std::min(list.find(',', pos), list.size());
            const std::string name = list.substr(pos, e - pos);
            for (const Kind& kd : all)
                if (name == kd.name) kinds.push_back(kd);
            if (name.rfind("pad", 0) == 0) kinds.push_back({strdup(name.c_str()), 0x80000000u});
            pos = e + 1;
        }
    }
    std::vector<uint8_t*> bufs;
    std::vector<size_t> ok;
    for (size_t i = 0; i < kinds.size(); ++i) {
        void* p = nullptr;
        if (kinds[i].flags == 0x80000000u) {  // pad: N GiB, not measured
            const size_t n = (size_t)atoi(kinds[i].name + 3) << 30;
            if (hipMalloc(&p, n) != hipSuccess) return 1;
            fprintf(stderr, "%s at %p\n", kinds[i].name, p);
            bufs.push_back(nullptr);
            continue;
        }
        if (hipExtMallocWithFlags(&p, total, kinds[i].flags) != hipSuccess || !p) {
            fprintf(stderr, "%s: allocation failed, skipped\n", kinds[i].name);
            (void)hipGetLastError();
            bufs.push_back(nullptr);
            continue;
        }
        bufs.push_back(static_cast<uint8_t*>(p));
        ok.push_back(i);
        fprintf(stderr, "%s#%zu at %p\n", kinds[i].name, i, p);
    }
    if (ok.empty() || bufs[ok[0]] == nullptr) return 1;
    SynthArgs sa{};
    sa.dst = bufs[ok[0]]; sa.total_bytes = total; sa.frame_bytes = fb; sa.seed = 0xD1B5; sa.t0 = 0;
    sa.channels = C; sa.width = W; sa.height = H; sa.radius = H / 8;
    if (launch_synth(sa, 0) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return 1;
    for (size_t j = 1; j < ok.size(); ++j)
        if (hipMemcpy(bufs[ok[j]], bufs[ok[0]], total, hipMemcpyDeviceToDevice) != hipSuccess) return 1;
    std::vector<uint32_t> Ls = {0};  // 0: the shipped schedule
    std::vector<bool> xcd = {false};
    if (argc > 5)
        for (char* q = argv[5]; *q;) {
            Ls.push_back((uint32_t)strtoul(q, &q, 10));
            xcd.push_back(*q == 'x');
            if (*q == 'x') ++q;
            if (*q == ',') ++q;
        }
    const void* k0 = series_v2_kernel_ptr(3, 0, true, false, false, 1);

    int occ = 0;
    if (!k0 || hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k0, 256, 0) != hipSuccess || occ < 1) return 1;
    const uint64_t nvec = fb / 12, tiles = (nvec + 64ull * kUnrollV2Rgb - 1) / (64ull * kUnrollV2Rgb);
    uint64_t* partials = nullptr;
    dips_series_entry* series = nullptr;
    SeriesArgs a{};
    a.frame_bytes = (uint32_t)fb; a.vec_bytes = (uint32_t)fb; a.n_frames = F;
    a.n_tiles = (uint32_t)tiles; a.items = tiles * F;
    a.n_waves = (uint32_t)std::min<uint64_t>(a.items, (uint64_t)occ * cus * 4);
    a.thr = series_threshold(3, 8.0f / 255.0f, 1);
    if (hipMalloc(&partials, a.items * 16 + 4096) != hipSuccess) return 1;
    if (hipMalloc(&series, sizeof(dips_series_entry) * F) != hipSuccess) return 1;
    a.partials = partials;

    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return 1;
    std::vector<dips_series_entry> ref(F), h(F);
    bool have_ref = false;
    for (int r = 0; r < rounds; ++r) {
        for (size_t vj = 0; vj < ok.size() * Ls.size(); ++vj) {
            const size_t vv = (r % 2 == 0) ? vj : ok.size() * Ls.size() - 1 - vj;
            const size_t i = ok[vv / Ls.size()];
            const uint32_t L = Ls[vv % Ls.size()];
            (void)0;
            const bool X = xcd[vv % Ls.size()];
            const void* k = L == 0 ? k0 : (X ? (const void*)&parts_isi_wg16 : (const void*)&parts_isi);
            SeriesArgs args = a;
            args.frames = bufs[i];
            args.ref0 = bufs[i];
            args.part_frames = L;
            if (L != 0 && argc > 6) args.n_waves = (uint32_t)atoi(argv[6]);
            const uint32_t wpb = X ? 16u : 4u;  // waves per workgroup
            const uint32_t blocks = (args.n_waves + wpb - 1) / wpb;
            std::vector<float> ms;
            const double t0 = now();
            while (now() - t0 < secs) {
                (void)hipMemsetAsync(series, 0, sizeof(dips_series_entry) * F, 0);
                if (hipEventRecord(e0, 0) != hipSuccess) return 1;
                void* params[] = {&args};
                if (hipLaunchKernel(k, dim3(blocks), dim3(wpb * 64u), params, 0, 0) != hipSuccess) return 1;
                if (hipEventRecord(e1, 0) != hipSuccess) return 1;
                if (launch_series_reduce(partials, F, a.n_tiles, 0, series, 0) != hipSuccess) return 1;
                if (hipDeviceSynchronize() != hipSuccess) return 1;
                float t = 0;
                (void)hipEventElapsedTime(&t, e0, e1);
                ms.push_back(t);
            }
            const double t1 = now();
            if (hipMemcpy(h.data(), series, sizeof(dips_series_entry) * F, hipMemcpyDeviceToHost) != hipSuccess) return 1;
            if (!have_ref) {
                ref = h;
                have_ref = true;
            }
            const bool same = std::equal(h.begin(), h.end(), ref.begin(), [](const dips_series_entry& x,
                                                                           const dips_series_entry& y) {
                return x.sad == y.sad && x.sj == y.sj && x.count == y.count && x.si_fixed == y.si_fixed;
            });
            std::sort(ms.begin(), ms.end());
            const double med = ms[ms.size() / 2];
            printf("run\t%d\t%s#%zu/%s%u%s%s\t%.6f\t%.6f\t%.4f\t%.4f\t%u\n", r, kinds[i].name, i, L ? "P" : "S", L,
                   X ? "x" : "", same ? "" : " DIFF", t0, t1, med,
                   (double)total / (med / 1e3) / 8e12, F);
            fflush(stdout);
        }
    }
    return 0;
}
