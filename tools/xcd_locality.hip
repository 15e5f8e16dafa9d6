// xcd_locality.hip -- is HBM read bandwidth XCD-local at some interleave
// granularity?  A 16 GiB buffer is cut into chunks of 2^shift bytes; with
// offset d, the workgroups on XCD x (hardware XCC id, s_getreg) read only the
// chunks c with c % 8 == (x + d) % 8, each chunk once (non-temporal 16-B
// loads).  Every d reads the same bytes with the same access shape; if the
// memory interleave gave each XCD nearer stacks at this granularity, one d
// (and for a plain modulo interleave, one d per granularity) would run
// faster.  Prints GB/s per (shift, d), alternated over rounds.
// Usage: xcd_locality [rounds]
// Build: hipcc --offload-arch=gfx950 -O3 -o build/xcd_locality tools/xcd_locality.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t xcc_id() {
    uint32_t r;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(r));
    return r;
}

// blocks_per_xcd blocks per XCD (grid = 8 * blocks_per_xcd, dealt round
// robin, so block b's slot on its XCD is b / 8)
__global__ __launch_bounds__(256) void locality_kernel(const u32x4* __restrict__ p, uint64_t n_chunks, uint32_t shift,
                                                       uint32_t d, uint32_t blocks_per_xcd, uint32_t* __restrict__ out) {
    const uint32_t x = xcc_id();
    const uint32_t slot = blocks_per_xcd > 0 ? (blockIdx.x / 8u) % blocks_per_xcd : 0u;
    const uint64_t chunk_vecs = (1ull << shift) / 16u;
    const uint32_t want = (x + d) & 7u;
    uint32_t acc = 0;
    // chunks want, want + 8, ... taken by this XCD's blocks in turn
    for (uint64_t c = want + 8ull * slot; c < n_chunks; c += 8ull * blocks_per_xcd) {
        const u32x4* q = p + c * chunk_vecs;
        for (uint64_t v = threadIdx.x; v < chunk_vecs; v += 256u) {
            const u32x4 w = __builtin_nontemporal_load(q + v);
            acc ^= w.x ^ w.y ^ w.z ^ w.w;
        }
    }
    if (acc == 0x9E3779B9u) out[0] = acc;
}

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 2;
    const uint64_t bytes = 16ull << 30;
    uint8_t* buf = nullptr;
    uint32_t* out = nullptr;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    if (hipMemset(buf, 0x5A, bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return 1;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess) return 1;
    const uint32_t blocks_per_xcd = (uint32_t)(cus / 8) * 4u;  // 4 groups of 256 per CU
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return 1;
    const std::vector<uint32_t> shifts = {8, 10, 12, 14, 16, 21};
    for (int r = 0; r < rounds; ++r) {
        for (uint32_t shift : shifts) {
            const uint64_t n_chunks = bytes >> shift;
            for (uint32_t d = 0; d < 8; ++d) {
                std::vector<float> ms;
                for (int rep = 0; rep < 4; ++rep) {
                    if (hipEventRecord(e0, 0) != hipSuccess) return 1;
                    hipLaunchKernelGGL(locality_kernel, dim3(8 * blocks_per_xcd), dim3(256), 0, 0,
                                       reinterpret_cast<const u32x4*>(buf), n_chunks, shift, d, blocks_per_xcd, out);
                    if (hipEventRecord(e1, 0) != hipSuccess || hipEventSynchronize(e1) != hipSuccess) return 1;
                    float t = 0;
                    (void)hipEventElapsedTime(&t, e0, e1);
                    ms.push_back(t);
                }
                std::sort(ms.begin(), ms.end());
                // each d reads 1/8 of the chunks per XCD x 8 XCDs = the whole buffer
                printf("{\"round\": %d, \"chunk_bytes\": %llu, \"d\": %u, \"ms\": %.4f, \"GBps\": %.1f}\n", r,
                       1ull << shift, d, ms[1], (double)bytes / (ms[1] / 1e3) / 1e9);
                fflush(stdout);
            }
        }
    }
    return 0;
}
