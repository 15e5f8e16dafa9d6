// unaligned_probe.hip -- do raw buffer loads/stores of 12 and 16 bytes at
// byte-unaligned addresses return / write the right bytes on gfx950 (the
// HSA runtime's alignment mode), and what do they cost when streaming?
// Decides whether the series kernels can take unaligned frame batches
// (frame_bytes % 4 != 0, or a batch at an odd address) without a fallback.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/unaligned_probe tools/unaligned_probe.hip
// Run on the GPU box: tools/unaligned_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                \
        }                                                                                \
    } while (0)

typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes) {
    const uint64_t a = (uint64_t)(uintptr_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    void* base = (void*)(uintptr_t)(((uint64_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(base, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// out[lane] = 12 (VB=12) or 16 bytes loaded at base + off0 + lane*VB, for a
// descriptor whose base is `src + s` (s = 0..3) and a range `range` bytes.
template <int VB>
__global__ void load_kernel(const uint8_t* src, uint32_t s, uint32_t off0, uint32_t range, uint32_t* out) {
    const __amdgpu_buffer_rsrc_t r = rsrc(src + s, range);
    const uint32_t off = off0 + threadIdx.x * VB;
    if constexpr (VB == 12) {
        const u32x3 x = __builtin_amdgcn_raw_buffer_load_b96(r, off, 0, 2);
        out[threadIdx.x * 3 + 0] = x.x;
        out[threadIdx.x * 3 + 1] = x.y;
        out[threadIdx.x * 3 + 2] = x.z;
    } else {
        const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 2);
        out[threadIdx.x * 4 + 0] = x.x;
        out[threadIdx.x * 4 + 1] = x.y;
        out[threadIdx.x * 4 + 2] = x.z;
        out[threadIdx.x * 4 + 3] = x.w;
    }
}

template <int VB>
__global__ void store_kernel(uint8_t* dst, uint32_t s, uint32_t range) {
    const __amdgpu_buffer_rsrc_t r = rsrc(dst + s, range);
    const uint32_t off = threadIdx.x * VB;
    uint32_t w[4];
    for (int k = 0; k < 4; ++k) {
        const uint32_t b = off + 4 * k;
        w[k] = ((b + 1) & 0xFF) | (((b + 2) & 0xFF) << 8) | (((b + 3) & 0xFF) << 16) | (((b + 4) & 0xFF) << 24);
    }
    if constexpr (VB == 12) {
        u32x3 x;
        x.x = w[0]; x.y = w[1]; x.z = w[2];
        __builtin_amdgcn_raw_buffer_store_b96(x, r, off, 0, 2);
    } else {
        u32x4 x;
        x.x = w[0]; x.y = w[1]; x.z = w[2]; x.w = w[3];
        __builtin_amdgcn_raw_buffer_store_b128(x, r, off, 0, 2);
    }
}

// Streaming read of n_frames frames of fb bytes starting at src + s, 12-byte
// vecs, 4 vecs per lane per frame (the series kernel's access shape).
__global__ __launch_bounds__(256) void stream_kernel(const uint8_t* src, uint32_t s, uint64_t fb, uint32_t n_frames,
                                                     uint32_t n_tiles, uint32_t* out) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = blockIdx.x * 4u + (threadIdx.x >> 6);
    const uint32_t n_waves = gridDim.x * 4u;
    uint32_t acc = 0;
    for (uint32_t tile = wave; tile < n_tiles; tile += n_waves) {
        for (uint32_t t = 0; t < n_frames; ++t) {
            const __amdgpu_buffer_rsrc_t r = rsrc(src + s + (uint64_t)t * fb, (uint32_t)fb);
            u32x3 x[4];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                x[u] = __builtin_amdgcn_raw_buffer_load_b96(r, ((tile * 4u + u) * 64u + lane) * 12u, 0, 2);
#pragma unroll
            for (int u = 0; u < 4; ++u) acc ^= x[u].x ^ x[u].y ^ x[u].z;
        }
    }
    if (acc == 0x9E3779B9u) out[0] = acc;
}

int main() {
    const size_t N = 1 << 20;
    std::vector<uint8_t> h(N);
    for (size_t i = 0; i < N; ++i) h[i] = (uint8_t)((i * 2654435761u) >> 13);
    uint8_t* d = nullptr;
    uint32_t* o = nullptr;
    CK(hipMalloc(&d, N));
    CK(hipMalloc(&o, 64 * 16));
    CK(hipMemcpy(d, h.data(), N, hipMemcpyHostToDevice));
    int bad_load = 0, bad_tail = 0, bad_store = 0;
    for (int vb : {12, 16}) {
        for (uint32_t s = 0; s < 4; ++s) {
            for (uint32_t off0 : {0u, 1u, 2u, 3u, 4096u + 3u}) {
                const uint32_t range = 64 * vb + off0;  // full range
                CK(hipMemset(o, 0xEE, 64 * 16));
                if (vb == 12) hipLaunchKernelGGL(load_kernel<12>, dim3(1), dim3(64), 0, 0, d, s, off0, range, o);
                else hipLaunchKernelGGL(load_kernel<16>, dim3(1), dim3(64), 0, 0, d, s, off0, range, o);
                CK(hipDeviceSynchronize());
                std::vector<uint8_t> got(64 * vb);
                CK(hipMemcpy(got.data(), o, 64 * vb, hipMemcpyDeviceToHost));
                if (std::memcmp(got.data(), h.data() + s + off0, 64 * vb) != 0) {
                    ++bad_load;
                    std::printf("LOAD MISMATCH vb=%d s=%u off0=%u first bytes got %02x %02x %02x want %02x %02x %02x\n",
                                vb, s, off0, got[0], got[1], got[2], h[s + off0], h[s + off0 + 1], h[s + off0 + 2]);
                }
            }
            // range ending inside the last lane's vec: which bytes come back?
            for (uint32_t cut = 1; cut < (uint32_t)vb; ++cut) {
                const uint32_t range = 63 * vb + cut;
                CK(hipMemset(o, 0xEE, 64 * 16));
                if (vb == 12) hipLaunchKernelGGL(load_kernel<12>, dim3(1), dim3(64), 0, 0, d, s, 0u, range, o);
                else hipLaunchKernelGGL(load_kernel<16>, dim3(1), dim3(64), 0, 0, d, s, 0u, range, o);
                CK(hipDeviceSynchronize());
                std::vector<uint8_t> got(64 * vb);
                CK(hipMemcpy(got.data(), o, 64 * vb, hipMemcpyDeviceToHost));
                char pat[17] = {0};
                for (int b = 0; b < vb; ++b) {
                    const uint8_t g = got[63 * vb + b], w = h[s + 63 * vb + b];
                    pat[b] = g == w ? (g == 0 ? 'z' : 'v') : (g == 0 ? '0' : 'x');
                }
                const bool in_ok = std::memcmp(got.data(), h.data() + s, 63 * vb) == 0;
                if (!in_ok) ++bad_tail;
                std::printf("tail vb=%d s=%u range_end_in_vec=%2u last vec bytes [%s] (v=valid 0=zeroed x=other)%s\n", vb,
                            s, cut, pat, in_ok ? "" : " EARLIER LANES WRONG");
            }
            // unaligned stores
            CK(hipMemset(d, 0, 4096));
            if (vb == 12) hipLaunchKernelGGL(store_kernel<12>, dim3(1), dim3(64), 0, 0, d, s, 64u * 12u);
            else hipLaunchKernelGGL(store_kernel<16>, dim3(1), dim3(64), 0, 0, d, s, 64u * 16u);
            CK(hipDeviceSynchronize());
            std::vector<uint8_t> got(4096);
            CK(hipMemcpy(got.data(), d, 4096, hipMemcpyDeviceToHost));
            for (uint32_t b = 0; b < 64u * vb; ++b)
                if (got[s + b] != (uint8_t)((b + 1) & 0xFF)) {
                    ++bad_store;
                    std::printf("STORE MISMATCH vb=%d s=%u byte %u got %u\n", vb, s, b, got[s + b]);
                    break;
                }
            for (uint32_t b = 0; b < s; ++b)
                if (got[b] != 0) { ++bad_store; std::printf("STORE CLOBBER before vb=%d s=%u\n", vb, s); break; }
            for (uint32_t b = s + 64u * vb; b < 4096; ++b)
                if (got[b] != 0) { ++bad_store; std::printf("STORE CLOBBER after vb=%d s=%u byte %u\n", vb, s, b); break; }
            CK(hipMemcpy(d, h.data(), 4096, hipMemcpyHostToDevice));
        }
    }
    std::printf("unaligned loads: %s (%d bad); stores: %s (%d bad); tail cases with wrong in-range lanes: %d\n",
                bad_load ? "WRONG" : "exact", bad_load, bad_store ? "WRONG" : "exact", bad_store, bad_tail);
    CK(hipFree(d));

    // streaming cost: 400 frames of 1920x1080 RGB8 from an aligned and an
    // unaligned base, and frame stride fb + 1 (every frame a different shift)
    const uint64_t fb = 1920ull * 1080 * 3;
    const uint32_t nf = 400;
    uint8_t* big = nullptr;
    CK(hipMalloc(&big, (fb + 1) * nf + 64));
    CK(hipMemset(big, 1, (fb + 1) * nf + 64));
    const uint32_t n_tiles = (uint32_t)((fb / 12 + 255) / 256);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int rep = 0; rep < 3; ++rep) {
        for (auto cfg : {std::make_pair(0u, fb), std::make_pair(1u, fb), std::make_pair(0u, fb + 1),
                         std::make_pair(2u, fb + 1)}) {
            hipLaunchKernelGGL(stream_kernel, dim3(1280), dim3(256), 0, 0, big, cfg.first, cfg.second, nf, n_tiles, o);
            CK(hipEventRecord(e0, 0));
            for (int k = 0; k < 5; ++k)
                hipLaunchKernelGGL(stream_kernel, dim3(1280), dim3(256), 0, 0, big, cfg.first, cfg.second, nf, n_tiles,
                                   o);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ms /= 5;
            std::printf("stream rep %d base+%u stride %llu: %.3f ms, %.1f GB/s\n", rep, cfg.first,
                        (unsigned long long)cfg.second, ms, (double)fb * nf / (ms * 1e-3) / 1e9);
        }
    }
    CK(hipFree(big));
    CK(hipFree(o));
    return 0;
}
