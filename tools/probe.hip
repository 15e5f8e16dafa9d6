// probe.hip -- standalone HBM / kernel-variant probe for the series path.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o build/probe tools/probe.hip
// Run on the GPU box: build/probe [frames]
//
// Variants are timed interleaved in one process (cdna_hip_programming.md
// §5.4 rule 24): median of R rounds per variant, GB/s of frame bytes.
#include "../dips_amd/csrc/series_kernels.hip"
#include "../dips_amd/csrc/series_v2.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

using namespace dips;

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e = (x);                                                                \
        if (e != hipSuccess) {                                                             \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

// Plain streaming read: grid-stride, 16 B per lane, UNR loads in flight.
template <int UNR>
__global__ __launch_bounds__(256) void read_stream(const u32x4* __restrict__ p, uint64_t n16, uint32_t* out) {
    uint32_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * 256u * UNR;
    for (uint64_t i = (uint64_t)blockIdx.x * 256u * UNR + threadIdx.x; i < n16; i += stride) {
        u32x4 v[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            const uint64_t j = i + (uint64_t)u * 256u;
            v[u] = j < n16 ? __builtin_nontemporal_load(p + j) : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < UNR; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// The series kernel's access pattern with no compute: tile-resident waves
// walking frames, U vec loads per lane per frame (dwordx3 or x4).
template <int VB, int U, bool PREFETCH>
__global__ __launch_bounds__(256) void walk_probe(SeriesArgs a, uint32_t* out) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
    if (wave >= a.n_waves) return;
    const uint32_t fb = a.frame_bytes;
    uint32_t acc = 0;
    uint64_t i = (uint64_t)wave * a.items / a.n_waves;
    const uint64_t iend = (uint64_t)(wave + 1) * a.items / a.n_waves;
    while (i < iend) {
        const uint32_t tile = (uint32_t)(i / a.n_frames);
        uint32_t t = (uint32_t)(i - (uint64_t)tile * a.n_frames);
        const uint64_t remaining = iend - i;
        const uint32_t tend = (uint32_t)((uint64_t)a.n_frames < t + remaining ? (uint64_t)a.n_frames : t + remaining);
        i += tend - t;
        uint32_t voff[U];
#pragma unroll
        for (int u = 0; u < U; ++u) voff[u] = ((tile * U + u) * 64u + lane) * (uint32_t)VB;
        for (; t < tend; ++t) {
            const __amdgpu_buffer_rsrc_t r = make_rsrc(a.frames + (uint64_t)t * fb, fb);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if constexpr (VB == 12) {
                    const u32x3 x = __builtin_amdgcn_raw_buffer_load_b96(r, voff[u], 0, kAuxNT);
                    acc ^= x.x ^ x.y ^ x.z;
                } else {
                    const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(r, voff[u], 0, kAuxNT);
                    acc ^= x.x ^ x.y ^ x.z ^ x.w;
                }
            }
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}


struct Timer {
    hipEvent_t a, b;
    Timer() { CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); }
};

int main(int argc, char** argv) {
    const uint32_t W = 3840, H = 2160, C = 3;
    const uint32_t F = argc > 1 ? (uint32_t)atoi(argv[1]) : 1000;
    const int R = argc > 2 ? atoi(argv[2]) : 5;
    const uint64_t fb = (uint64_t)W * H * C;
    const uint64_t total = fb * F;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint8_t* frames;
    CK(hipMalloc(&frames, total + 4096));
    uint32_t* out;
    CK(hipMalloc(&out, 4096));
    uint64_t* partials;
    SynthArgs sa{};
    sa.dst = frames; sa.total_bytes = total; sa.frame_bytes = fb; sa.seed = 0xD1B5; sa.t0 = 0;
    sa.channels = C; sa.width = W; sa.height = H; sa.radius = H / 8;
    CK(launch_synth(sa, 0));
    CK(hipDeviceSynchronize());
    dips_series_entry* series;
    CK(hipMalloc(&series, sizeof(dips_series_entry) * F));

    struct Variant {
        std::string name;
        std::function<void()> run;
        std::vector<float> ms;
        std::string group;  // variants of one group must give identical series
    };
    std::vector<Variant> vs;

    // geometry helper for tile-walk kernels
    auto geom = [&](int VB, int U, const void* kern, SeriesArgs& a, uint32_t& blocks, int& occ) {
        const uint64_t nvec = fb / VB;
        const uint64_t tiles = (nvec + 64ull * U - 1) / (64ull * U);
        occ = 0;
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, 256, 0));
        const uint64_t items = tiles * F;
        const uint64_t resident = (uint64_t)occ * cus * 4;
        a = SeriesArgs{};
        a.frames = frames; a.ref0 = frames; a.frame_bytes = (uint32_t)fb; a.vec_bytes = (uint32_t)fb; a.n_frames = F;
        a.n_tiles = (uint32_t)tiles; a.items = items; a.n_waves = (uint32_t)std::min<uint64_t>(items, resident);
        if (const char* ew = getenv("PROBE_WAVES")) a.n_waves = (uint32_t)std::min<uint64_t>(items, strtoull(ew, nullptr, 10));
        a.thr = 2.0f * 8.0f / 255.0f;
        blocks = (a.n_waves + 3) / 4;
    };

    for (int g : {1024}) {
        vs.push_back({"read_stream<4> grid=" + std::to_string(g), [=]() {
                          hipLaunchKernelGGL(read_stream<4>, dim3(g), dim3(256), 0, 0,
                                             (const u32x4*)frames, total / 16, out);
                      }, {}});
    }
    vs.push_back({"read_stream<8> grid=2048", [=]() {
                      hipLaunchKernelGGL(read_stream<8>, dim3(2048), dim3(256), 0, 0, (const u32x4*)frames, total / 16, out);
                  }, {}});

#define WALK(VB, U)                                                                                   \
    {                                                                                                 \
        SeriesArgs a; uint32_t blocks; int occ;                                                       \
        geom(VB, U, (const void*)&walk_probe<VB, U, false>, a, blocks, occ);                          \
        vs.push_back({"walk<" #VB "," #U "> occ=" + std::to_string(occ) + " waves=" + std::to_string(a.n_waves), \
                      [=]() { hipLaunchKernelGGL((walk_probe<VB, U, false>), dim3(blocks), dim3(256), 0, 0, a, out); }, {}}); \
    }
    WALK(12, 4)

    // kernels: series_fast_kernel (previous RGB kernel) and series_v2_kernel
    CK(hipMalloc(&partials, (uint64_t)F * 16200 * 16 + 4096));
#define SERIES(U, D, PF)                                                                              \
    {                                                                                                 \
        SeriesArgs a; uint32_t blocks; int occ;                                                       \
        const void* k = (const void*)&series_fast_kernel<3, 0, U, D, PF, false>;                      \
        geom(12, U, k, a, blocks, occ);                                                               \
        a.partials = partials;                                                                        \
        vs.push_back({"series<U=" #U ",D=" #D ",PF=" #PF "> occ=" + std::to_string(occ) + " waves=" +  \
                          std::to_string(a.n_waves),                                                  \
                      [=]() { hipLaunchKernelGGL((series_fast_kernel<3, 0, U, D, PF, false>), dim3(blocks), dim3(256), 0, 0, a); \
                              CK(launch_series_reduce(partials, F, a.n_tiles, 0, series, 0)); }, {}, "PF=" #PF " tau=8.0f"}); \
    }
#define SERIES_V2U(PF, U) SERIES_V2X(PF, U, 8.0f)
#define SERIES_V2X(PF, U, TAU255)                                                                             \
    {                                                                                                 \
        SeriesArgs a; uint32_t blocks; int occ;                                                       \
        const void* k = (const void*)&series_v2_kernel<3, 0, U, PF, false>;                           \
        geom(12, U, k, a, blocks, occ);                                                               \
        a.partials = partials;                                                                        \
        a.thr = series_threshold(3, TAU255 / 255.0f);                                                 \
        vs.push_back({"v2<U=" #U ",PF=" #PF "> tau=" #TAU255 "/255 occ=" + std::to_string(occ) + " waves=" + std::to_string(a.n_waves), \
                      [=]() { hipLaunchKernelGGL((series_v2_kernel<3, 0, U, PF, false>), dim3(blocks), dim3(256), 0, 0, a); \
                              CK(launch_series_reduce(partials, F, a.n_tiles, 0, series, 0)); }, {}, "PF=" #PF " tau=" #TAU255}); \
    }
#define SERIES_V2(PF) SERIES_V2U(PF, kUnrollV2)
    SERIES(4, 2, true)
    SERIES_V2(true)
    SERIES(4, 2, false)
    SERIES_V2(false)
    SERIES_V2X(true, kUnrollV2, 0.0f)
    SERIES_V2U(true, 2)
    SERIES_V2U(true, 3)

    if (argc > 3) {  // substring filter on variant names
        std::vector<Variant> keep;
        for (auto& v : vs)
            if (v.name.find(argv[3]) != std::string::npos) keep.push_back(v);
        vs.swap(keep);
    }
    // parity: every variant's series (last run) against the first variant of
    // the same mode (names containing PF=true / PF=false)
    std::vector<dips_series_entry> host(F);
    auto run_series = [&](Variant& v) {
        CK(hipMemset(series, 0, sizeof(dips_series_entry) * F));
        v.run();
        CK(hipDeviceSynchronize());
        std::vector<dips_series_entry> h(F);
        CK(hipMemcpy(h.data(), series, sizeof(dips_series_entry) * F, hipMemcpyDeviceToHost));
        return h;
    };
    std::vector<std::string> groups;
    for (auto& v : vs)
        if (!v.group.empty() && std::find(groups.begin(), groups.end(), v.group) == groups.end()) groups.push_back(v.group);
    for (const auto& grp : groups) {
        std::vector<dips_series_entry> ref;
        std::string refname;
        for (auto& v : vs) {
            if (v.group != grp) continue;
            auto h = run_series(v);
            if (ref.empty()) { ref = h; refname = v.name; continue; }
            const bool same = memcmp(ref.data(), h.data(), sizeof(dips_series_entry) * F) == 0;
            printf("parity %-30s vs %-30s : %s\n", v.name.c_str(), refname.c_str(), same ? "IDENTICAL" : "MISMATCH");
            if (!same)
                for (uint32_t t = 0; t < F; ++t)
                    if (memcmp(&ref[t], &h[t], sizeof(dips_series_entry))) {
                        printf("  frame %u: %llu %llu %llu %llu vs %llu %llu %llu %llu\n", t,
                               (unsigned long long)ref[t].sad, (unsigned long long)ref[t].sj,
                               (unsigned long long)ref[t].count, (unsigned long long)ref[t].si_fixed,
                               (unsigned long long)h[t].sad, (unsigned long long)h[t].sj,
                               (unsigned long long)h[t].count, (unsigned long long)h[t].si_fixed);
                        break;
                    }
        }
    }
    Timer tm;
    for (int r = 0; r < R; ++r) {
        for (auto& v : vs) {
            CK(hipEventRecord(tm.a, 0));
            v.run();
            CK(hipEventRecord(tm.b, 0));
            CK(hipEventSynchronize(tm.b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, tm.a, tm.b));
            v.ms.push_back(ms);
        }
    }
    printf("frames=%u frame_bytes=%llu total=%.2f GB cus=%d rounds=%d\n", F, (unsigned long long)fb, total / 1e9, cus, R);
    for (auto& v : vs) {
        std::sort(v.ms.begin(), v.ms.end());
        const float med = v.ms[v.ms.size() / 2], mn = v.ms[0];
        printf("%-48s median %8.3f ms  min %8.3f ms  -> %7.1f GB/s (best %7.1f)\n", v.name.c_str(), med, mn,
               total / (med / 1e3) / 1e9, total / (mn / 1e3) / 1e9);
    }
    return 0;
}
