// zc_probe.hip -- the per-frame call's GPU side in isolation: how fast a
// kernel moves one 4K frame's packed input (2 B/px, 16.6 MB) from pinned host
// memory and its keys (1 B/px, 8.3 MB) back, with no host thread competing
// for memory bandwidth, against the copy engines (hipMemcpyAsync) moving the
// same bytes.  Read widths of 4 / 8 / 16 B per thread (system-scope loads, as
// compat_main_host_packed_kernel), key stores of the matching 2 / 4 / 8 B;
// one kernel over the frame and the same cut into 9 stripes on two streams
// (the pipeline's shape).  hipEvent times, median of 20.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/zc_probe tools/zc_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

// W bytes of packed input per thread (W / 2 pixels), W / 2 key bytes out.
template <int W>
__global__ __launch_bounds__(256) void zc_kernel(const uint8_t* in, uint8_t* out, uint64_t px0, uint64_t px1) {
    constexpr int P = W / 2;  // pixels per thread
    const uint64_t p = px0 + (uint64_t)P * ((uint64_t)blockIdx.x * 256u + threadIdx.x);
    if (p + P > px1) return;
    uint64_t keys = 0;
    if constexpr (W == 4) {
        const uint32_t w = __hip_atomic_load(reinterpret_cast<const uint32_t*>(in + 2 * p), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_SYSTEM);
        keys = ((w & 0xFFu) + ((w >> 8) & 0xFFu)) / 2u | ((((w >> 16) & 0xFFu) + (w >> 24)) / 2u) << 8;
        __hip_atomic_store(reinterpret_cast<uint16_t*>(out + p), (uint16_t)keys, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    } else if constexpr (W == 8) {
        const uint64_t w = __hip_atomic_load(reinterpret_cast<const uint64_t*>(in + 2 * p), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_SYSTEM);
        for (int g = 0; g < 4; ++g) keys |= (((w >> (16 * g)) & 0xFFu) + ((w >> (16 * g + 8)) & 0xFFu)) / 2u << (8 * g);
        __hip_atomic_store(reinterpret_cast<uint32_t*>(out + p), (uint32_t)keys, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    } else {
        const uint64_t w0 = __hip_atomic_load(reinterpret_cast<const uint64_t*>(in + 2 * p), __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_SYSTEM);
        const uint64_t w1 = __hip_atomic_load(reinterpret_cast<const uint64_t*>(in + 2 * p + 8), __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_SYSTEM);
        for (int g = 0; g < 4; ++g) keys |= (((w0 >> (16 * g)) & 0xFFu) + ((w0 >> (16 * g + 8)) & 0xFFu)) / 2u << (8 * g);
        for (int g = 0; g < 4; ++g)
            keys |= (uint64_t)((((w1 >> (16 * g)) & 0xFFu) + ((w1 >> (16 * g + 8)) & 0xFFu)) / 2u) << (8 * g + 32);
        __hip_atomic_store(reinterpret_cast<uint64_t*>(out + p), keys, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

int main() {
    const uint64_t npx = 3840ull * 2160ull;
    uint8_t *pin_in = nullptr, *pin_out = nullptr, *dev_in = nullptr, *dev_out = nullptr;
    CK(hipHostMalloc(&pin_in, npx * 2, hipHostMallocDefault));
    CK(hipHostMalloc(&pin_out, npx, hipHostMallocDefault));
    CK(hipMalloc(&dev_in, npx * 2));
    CK(hipMalloc(&dev_out, npx));
    for (uint64_t i = 0; i < npx * 2; ++i) pin_in[i] = (uint8_t)(i * 2654435761u >> 13);
    void *din = nullptr, *dout = nullptr;
    CK(hipHostGetDevicePointer(&din, pin_in, 0));
    CK(hipHostGetDevicePointer(&dout, pin_out, 0));
    hipStream_t s[2];
    CK(hipStreamCreateWithFlags(&s[0], hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s[1], hipStreamNonBlocking));
    hipEvent_t e0, e1, j1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventCreateWithFlags(&j1, hipEventDisableTiming));
    auto timeit = [&](const char* name, auto body) {
        body();
        CK(hipDeviceSynchronize());
        std::vector<float> t;
        for (int r = 0; r < 20; ++r) {
            CK(hipEventRecord(e0, s[0]));
            CK(hipStreamWaitEvent(s[1], e0, 0));
            body();
            CK(hipEventRecord(j1, s[1]));
            CK(hipStreamWaitEvent(s[0], j1, 0));
            CK(hipEventRecord(e1, s[0]));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        const double ms = t[t.size() / 2];
        std::printf("{\"case\": \"%s\", \"ms_median\": %.4f, \"in_GBps\": %.1f, \"out_GBps\": %.1f}\n", name, ms,
                    npx * 2 / (ms * 1e-3) / 1e9, npx / (ms * 1e-3) / 1e9);
        std::fflush(stdout);
    };
    const uint32_t stripes = 9;
    auto zc = [&](auto kern, int P, bool striped) {
        const uint32_t ns = striped ? stripes : 1;
        for (uint32_t k = 0; k < ns; ++k) {
            const uint64_t a = npx * k / ns / 8 * 8, b = npx * (k + 1) / ns / 8 * 8;
            const uint64_t threads = (b - a) / P;
            hipLaunchKernelGGL(kern, dim3((uint32_t)((threads + 255) / 256)), dim3(256), 0, s[k & 1],
                               (const uint8_t*)din, (uint8_t*)dout, a, b);
        }
    };
    for (int round = 0; round < 2; ++round) {
        timeit("zero-copy kernel, 4 B in / 2 B out per thread, whole frame", [&] { zc(zc_kernel<4>, 2, false); });
        timeit("zero-copy kernel, 8 B in / 4 B out per thread, whole frame", [&] { zc(zc_kernel<8>, 4, false); });
        timeit("zero-copy kernel, 16 B in / 8 B out per thread, whole frame", [&] { zc(zc_kernel<16>, 8, false); });
        timeit("zero-copy kernel, 4 B in / 2 B out, 9 stripes on 2 streams", [&] { zc(zc_kernel<4>, 2, true); });
        timeit("zero-copy kernel, 8 B in / 4 B out, 9 stripes on 2 streams", [&] { zc(zc_kernel<8>, 4, true); });
        timeit("zero-copy kernel, 16 B in / 8 B out, 9 stripes on 2 streams", [&] { zc(zc_kernel<16>, 8, true); });
        timeit("copy engines: H2D 16.6 MB then D2H 8.3 MB, one stream", [&] {
            CK(hipMemcpyAsync(dev_in, pin_in, npx * 2, hipMemcpyHostToDevice, s[0]));
            CK(hipMemcpyAsync(pin_out, dev_out, npx, hipMemcpyDeviceToHost, s[0]));
        });
        timeit("copy engines: H2D 16.6 MB and D2H 8.3 MB on two streams", [&] {
            CK(hipMemcpyAsync(dev_in, pin_in, npx * 2, hipMemcpyHostToDevice, s[0]));
            CK(hipMemcpyAsync(pin_out, dev_out, npx, hipMemcpyDeviceToHost, s[1]));
        });
        timeit("copy engines: 9 stripes, H2D on one stream, D2H on the other", [&] {
            for (uint32_t k = 0; k < stripes; ++k) {
                const uint64_t a = npx * k / stripes, b = npx * (k + 1) / stripes;
                CK(hipMemcpyAsync(dev_in + 2 * a, pin_in + 2 * a, 2 * (b - a), hipMemcpyHostToDevice, s[0]));
                CK(hipMemcpyAsync(pin_out + a, dev_out + a, b - a, hipMemcpyDeviceToHost, s[1]));
            }
        });
    }
    return 0;
}
