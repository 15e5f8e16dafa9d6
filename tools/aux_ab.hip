// aux_ab.hip -- frame-load cache policy A/B of the series kernel inside ONE
// process over ONE frame buffer (a buffer's placement alone moves the rate by
// a few %, tools/alloc_probe.hip, so variants are compared on the same
// buffer, alternated over rounds).  4K RGB8, per-frame, tau 8/255.
// Usage: aux_ab <frames> <seconds per run> <rounds>
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o build/aux_ab tools/aux_ab.hip
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

template <int AUX, int SAUX, bool MAP>
__global__ __launch_bounds__(256, (v2_min_waves<3, kUnrollV2, true, MAP>())) void probe_kernel(SeriesArgs a) {
    series_v2_body<3, 0, kUnrollV2, true, MAP, AUX, SAUX>(a);
}

struct V {
    int aux;
    const void* k;
};

int main(int argc, char** argv) {
    const uint32_t W = 3840, H = 2160, C = 3;
    const uint32_t F = argc > 1 ? (uint32_t)atoi(argv[1]) : 2000;
    const double secs = argc > 2 ? atof(argv[2]) : 2.0;
    const int rounds = argc > 3 ? atoi(argv[3]) : 3;
    const uint64_t fb = (uint64_t)W * H * C, total = fb * F;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess) return 1;
    uint8_t* frames = nullptr;
    if (hipMalloc(&frames, total) != hipSuccess) return 1;
    SynthArgs sa{};
    sa.dst = frames; sa.total_bytes = total; sa.frame_bytes = fb; sa.seed = 0xD1B5; sa.t0 = 0;
    sa.channels = C; sa.width = W; sa.height = H; sa.radius = H / 8;
    if (launch_synth(sa, 0) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return 1;
    // mode "load": the frame-load policy; mode "map": the map-store policy
    // of the MAP variant (frame loads nt)
    const bool map = argc > 4 && std::string(argv[4]) == "map";
    const std::vector<V> vload = {{2, (const void*)&probe_kernel<2, 2, false>},
                                  {0, (const void*)&probe_kernel<0, 2, false>},
                                  {1, (const void*)&probe_kernel<1, 2, false>},
                                  {3, (const void*)&probe_kernel<3, 2, false>},
                                  {16, (const void*)&probe_kernel<16, 2, false>},
                                  {18, (const void*)&probe_kernel<18, 2, false>}};
    const std::vector<V> vmap = {{2, (const void*)&probe_kernel<2, 2, true>},
                                 {0, (const void*)&probe_kernel<2, 0, true>},
                                 {1, (const void*)&probe_kernel<2, 1, true>},
                                 {3, (const void*)&probe_kernel<2, 3, true>},
                                 {16, (const void*)&probe_kernel<2, 16, true>},
                                 {17, (const void*)&probe_kernel<2, 17, true>},
                                 {18, (const void*)&probe_kernel<2, 18, true>},
                                 {19, (const void*)&probe_kernel<2, 19, true>}};
    const std::vector<V>& vs = map ? vmap : vload;
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, vs[0].k, 256, 0) != hipSuccess) return 1;
    const uint64_t nvec = fb / 12, tiles = (nvec + 64ull * kUnrollV2 - 1) / (64ull * kUnrollV2);
    uint64_t* partials = nullptr;
    dips_series_entry* series = nullptr;
    SeriesArgs a{};
    a.frames = frames; a.ref0 = frames;
    a.frame_bytes = (uint32_t)fb; a.vec_bytes = (uint32_t)fb; a.n_frames = F;
    a.n_tiles = (uint32_t)tiles; a.items = tiles * F;
    a.n_waves = (uint32_t)std::min<uint64_t>(a.items, (uint64_t)occ * cus * 4);
    a.thr = series_threshold(3, 8.0f / 255.0f);
    if (hipMalloc(&partials, a.items * 16 + 4096) != hipSuccess) return 1;
    if (hipMalloc(&series, sizeof(dips_series_entry) * F) != hipSuccess) return 1;
    a.partials = partials;
    if (map) {
        uint8_t* dmap = nullptr;
        if (hipMalloc(&dmap, total) != hipSuccess) return 1;
        a.dmap = dmap;
    }
    const uint32_t blocks = (a.n_waves + 3) / 4;
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return 1;
    std::vector<dips_series_entry> ref(F), h(F);
    for (int r = 0; r < rounds; ++r) {
        for (const V& v : vs) {
            std::vector<float> ms;
            const double t0 = now();
            while (now() - t0 < secs) {
                (void)hipMemsetAsync(series, 0, sizeof(dips_series_entry) * F, 0);
                if (hipEventRecord(e0, 0) != hipSuccess) return 1;
                SeriesArgs args = a;
                void* params[] = {&args};
                if (hipLaunchKernel(v.k, dim3(blocks), dim3(256), params, 0, 0) != hipSuccess) return 1;
                if (launch_series_reduce(partials, F, a.n_tiles, 0, series, 0) != hipSuccess) return 1;
                if (hipEventRecord(e1, 0) != hipSuccess || hipEventSynchronize(e1) != hipSuccess) return 1;
                float t = 0;
                (void)hipEventElapsedTime(&t, e0, e1);
                ms.push_back(t);
            }
            const double t1 = now();
            if (hipMemcpy(h.data(), series, sizeof(dips_series_entry) * F, hipMemcpyDeviceToHost) != hipSuccess) return 1;
            if (r == 0 && &v == &vs[0]) ref = h;
            const bool same = std::equal(h.begin(), h.end(), ref.begin(), [](const dips_series_entry& x,
                                                                           const dips_series_entry& y) {
                return x.sad == y.sad && x.sj == y.sj && x.count == y.count && x.si_fixed == y.si_fixed;
            });
            std::sort(ms.begin(), ms.end());
            const double med = ms[ms.size() / 2];
            printf("run\t%d\t%d\t%.6f\t%.6f\t%.4f\t%.4f\t%s\t%s\n", r, v.aux, t0, t1, med,
                   (map ? 2.0 : 1.0) * (double)total / (med / 1e3) / 8e12, same ? "same" : "DIFF", map ? "map" : "load");
            fflush(stdout);
        }
    }
    return 0;
}
