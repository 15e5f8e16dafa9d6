// altprobe.hip -- timing probe of the dips_alt batch kernel variants against a
// plain read+write stream of the same bytes (interleaved rounds, median).
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o build/altprobe tools/altprobe.hip
// Run on the GPU box: build/altprobe [frames]
#include "../dips_amd/csrc/alt_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
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

// read 16 B, write 16 B per lane: the copy ceiling of the alt stream
__global__ __launch_bounds__(256) void copy_stream(const u32x4* __restrict__ src, u32x4* __restrict__ dst, uint64_t n16) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256u) {
        u32x4 v = __builtin_nontemporal_load(src + i);
        v.x ^= 0x01010101u;
        __builtin_nontemporal_store(v, dst + i);
    }
}

template <int U>
static void setup(AltBatchArgs& a, uint32_t n, uint32_t n_vec, int resident, std::vector<int32_t>& cs) {
    const uint64_t n_tiles = (n_vec + 64u * U - 1) / (64u * U);
    uint64_t n_chunks = (resident + n_tiles - 1) / n_tiles;
    n_chunks = std::min<uint64_t>(n_chunks, (n + 15u) / 16u);
    n_chunks = std::max<uint64_t>(n_chunks, 1);
    const uint32_t chunk = (uint32_t)((n + n_chunks - 1) / n_chunks);
    n_chunks = (n + chunk - 1) / chunk;
    a.n_tiles = (uint32_t)n_tiles;
    a.n_chunks = (uint32_t)n_chunks;
    a.chunk = chunk;
    cs.assign(n_chunks, -1);
    for (uint32_t c = 0; c < n_chunks; ++c) cs[c] = c * chunk > 2 ? 2 : -1;
}

int main(int argc, char** argv) {
    const uint32_t F = argc > 1 ? (uint32_t)atoi(argv[1]) : 500;
    const uint32_t W = 3840, H = 2160;
    const uint64_t fb = (uint64_t)W * H * 4;
    const uint32_t n_vec = W * H / 4;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint8_t *frames, *out, *prev0, *snap_in, *snap_out, *flags;
    int32_t* cs_dev;
    CK(hipMalloc(&frames, fb * F));
    CK(hipMalloc(&out, fb * F));
    CK(hipMalloc(&prev0, fb));
    CK(hipMalloc(&snap_in, W * H));
    CK(hipMalloc(&snap_out, W * H));
    CK(hipMalloc(&flags, F));
    CK(hipMalloc(&cs_dev, 4096 * 4));
    CK(hipMemset(prev0, 0, fb));
    CK(hipMemset(snap_in, 0, W * H));
    CK(hipMemset(flags, 0, F));
    CK(hipMemset(flags + 2, 1, 1));
    // synthetic frames (same generator as the library)
    SynthArgs sa{};
    sa.dst = frames;
    sa.channels = 4;
    sa.width = W;
    sa.height = H;
    sa.frame_bytes = fb;
    sa.total_bytes = fb * F;
    sa.seed = 0xD1B5;
    sa.t0 = 0;
    sa.radius = H / 8;
    CK(launch_synth(sa, 0));
    CK(hipDeviceSynchronize());

    struct Variant {
        std::string name;
        std::function<void()> run;
    };
    std::vector<Variant> vs;
    vs.push_back({"copy_stream (read+write 16B/lane)", [&]() {
                      hipLaunchKernelGGL(copy_stream, dim3(8192), dim3(256), 0, 0, (const u32x4*)frames, (u32x4*)out,
                                         fb * F / 16);
                  }});
    auto add = [&](const char* name, const void* k, int U, auto setup_fn) {
        int nb = 0;
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, 256, 0));
        AltBatchArgs a{};
        a.frames = frames;
        a.prev0 = prev0;
        a.snap_in = snap_in;
        a.snap_out = snap_out;
        a.out = out;
        a.flags = flags;
        a.chunk_snap = cs_dev;
        a.frame_bytes = (uint32_t)fb;
        a.n_vec = n_vec;
        a.n_frames = F;
        a.last_snap = 2;
        a.scalar = 5.0f;
        a.kneg_half = -2.5f;
        std::vector<int32_t> cs;
        setup_fn(a, F, n_vec, nb * 4 * cus, cs);
        char nm[160];
        snprintf(nm, sizeof nm, "%s occ=%d tiles=%u chunks=%u", name, nb * 4, a.n_tiles, a.n_chunks);
        vs.push_back({nm, [=]() {
                          CK(hipMemcpy(cs_dev, cs.data(), cs.size() * 4, hipMemcpyHostToDevice));
                          AltBatchArgs b = a;
                          void* params[] = {&b};
                          const uint32_t blocks = (a.n_tiles * a.n_chunks + 3) / 4;
                          CK(hipLaunchKernel(k, dim3(blocks), dim3(256), params, 0, 0));
                      }});
        (void)U;
    };
    add("alt<U=1>", (const void*)&alt_batch_kernel<0, 0, 1, true, 1>, 1, setup<1>);
    add("alt<U=2>", (const void*)&alt_batch_kernel<0, 0, 1, true, 2>, 2, setup<2>);
    add("alt<U=4>", (const void*)&alt_batch_kernel<0, 0, 1, true, 4>, 4, setup<4>);
    add("alt<U=2> unfiltered", (const void*)&alt_batch_kernel<0, 255, 1, true, 2>, 2, setup<2>);
    add("alt<U=2> spec epilogue", (const void*)&alt_batch_kernel<0, 0, 1, false, 2>, 2, setup<2>);

    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int R = 5;
    std::vector<std::vector<float>> ms(vs.size());
    for (auto& v : vs) v.run();  // warm
    CK(hipDeviceSynchronize());
    for (int r = 0; r < R; ++r) {
        for (size_t i = 0; i < vs.size(); ++i) {
            CK(hipEventRecord(e0, 0));
            vs[i].run();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            ms[i].push_back(t);
        }
    }
    printf("frames=%u 4K RGBA8, bytes moved per launch (read+write) = %.2f GB, cus=%d, rounds=%d\n", F,
           2.0 * fb * F / 1e9, cus, R);
    for (size_t i = 0; i < vs.size(); ++i) {
        auto m = ms[i];
        std::sort(m.begin(), m.end());
        const double med = m[m.size() / 2];
        printf("%-58s median %8.3f ms  min %8.3f ms -> %7.1f GB/s  %8.0f frames/s\n", vs[i].name.c_str(), med, m[0],
               2.0 * fb * F / (med / 1e3) / 1e9, F / (med / 1e3));
    }
    return 0;
}
