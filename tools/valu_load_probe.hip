// valu_load_probe.hip -- how much VALU work per byte a full-rate HBM stream
// carries before the package power limit takes bandwidth away.
//
// The grid-stride read of read_ceiling_kernel (non-temporal 16-B loads, 4 in
// flight per lane, 4 waves per SIMD) with K dependent v_fma_f32 per loaded
// dword on a value derived from the dword (16 independent chains per lane),
// folded into one result per thread.  K = 0 is the plain read.  For RGB8
// frames a dword is 4/3 pixel, so K fma per dword = 0.75 K VALU ops per
// pixel (+ the 2 ops per dword that make the value); the series kernel
// issues ~12.75 per pixel in its pixel loop (13.65 in all at U = 5).  Driven by tools/valu_load_probe.py, which reads
// power, PPT residency and clocks around each K.
//
// Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC -cuid=valu_load_probe \
//          -o tools/libvalu_load_probe.so tools/valu_load_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int K>
__global__ __launch_bounds__(256) void valu_load_kernel(const u32x4* __restrict__ p, uint64_t n16, float c1,
                                                        float c2, float* __restrict__ out) {
    constexpr int kUnr = 4;
    float acc = 0.0f;
    const uint64_t stride = (uint64_t)gridDim.x * 256u * kUnr;
    for (uint64_t i = (uint64_t)blockIdx.x * 256u * kUnr + threadIdx.x; i < n16; i += stride) {
        u32x4 v[kUnr];
#pragma unroll
        for (int u = 0; u < kUnr; ++u) {
            const uint64_t j = i + (uint64_t)u * 256u;
            v[u] = j < n16 ? __builtin_nontemporal_load(p + j) : u32x4{0, 0, 0, 0};
        }
        float x[kUnr * 4];
#pragma unroll
        for (int u = 0; u < kUnr; ++u) {
            x[4 * u + 0] = __uint_as_float((v[u].x & 0x007FFFFFu) | 0x3F800000u);
            x[4 * u + 1] = __uint_as_float((v[u].y & 0x007FFFFFu) | 0x3F800000u);
            x[4 * u + 2] = __uint_as_float((v[u].z & 0x007FFFFFu) | 0x3F800000u);
            x[4 * u + 3] = __uint_as_float((v[u].w & 0x007FFFFFu) | 0x3F800000u);
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
#pragma unroll
            for (int q = 0; q < kUnr * 4; ++q) x[q] = __builtin_fmaf(x[q], c1, c2);
        }
#pragma unroll
        for (int q = 0; q < kUnr * 4; ++q) acc += x[q];
    }
    // one store per thread, taken only for an impossible sum (keeps the work)
    if (acc == -1.0f) out[blockIdx.x * 256u + threadIdx.x] = acc;
}

extern "C" int valu_load_launch(const void* p, uint64_t bytes, int k, void* out, void* stream) {
    const uint64_t n16 = bytes / 16u;
    const dim3 grid(1024), block(256);
    const hipStream_t s = static_cast<hipStream_t>(stream);
    const auto* src = static_cast<const u32x4*>(p);
    float* o = static_cast<float*>(out);
    const float c1 = 0.999999f, c2 = 1e-7f;
    switch (k) {
#define VLP(K) \
    case K: hipLaunchKernelGGL(valu_load_kernel<K>, grid, block, 0, s, src, n16, c1, c2, o); break;
        VLP(0) VLP(1) VLP(2) VLP(4) VLP(6) VLP(8) VLP(10) VLP(12) VLP(16) VLP(20) VLP(24)
#undef VLP
        default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
