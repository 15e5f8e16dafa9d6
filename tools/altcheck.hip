// altcheck.hip -- exhaustive device check of dips_amd/csrc/epilogue_fast.h
// against the specification functions of dips_math.h (which the CPU oracle
// states identically).  Build: hipcc --offload-arch=gfx950 -O3
// -ffp-contract=off -std=c++17 -o build/altcheck tools/altcheck.hip; run on the
// GPU box: build/altcheck
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../dips_amd/csrc/epilogue_fast.h"

using namespace dips;

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e = (x);                                                                \
        if (e != hipSuccess) {                                                             \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

struct Result {
    unsigned long long bad;
    unsigned int first;
    unsigned int pad;
};

__device__ void report(Result* r, uint32_t bits) {
    atomicAdd(&r->bad, 1ull);
    atomicMin(&r->first, bits);
}

// bit patterns [lo, hi) of f32 values
__global__ void k_recip(uint32_t lo, uint32_t hi, Result* r) {
    for (uint64_t b = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < hi;
         b += (uint64_t)gridDim.x * blockDim.x) {
        const float y = __uint_as_float((uint32_t)b);
        if (__float_as_uint(recip_ge1(y)) != __float_as_uint(__fdiv_rn(1.0f, y))) report(r, (uint32_t)b);
    }
}

__global__ void k_exp(uint32_t lo, uint32_t hi, Result* r) {
    for (uint64_t b = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < hi;
         b += (uint64_t)gridDim.x * blockDim.x) {
        const float x = __uint_as_float((uint32_t)b);
        if (__float_as_uint(exp_small(x)) != __float_as_uint(det_expf(x))) report(r, (uint32_t)b);
    }
}

__global__ void k_q(Result* r) {
    for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < (1ull << 32);
         b += (uint64_t)gridDim.x * blockDim.x) {
        const float x = __uint_as_float((uint32_t)b);
        if (x != x) continue;  // the fast path never sees a NaN
        if ((q_bits(x) & 0xFFu) != unorm_store(x)) report(r, (uint32_t)b);
    }
}

template <int FILT, bool COL>
__global__ void k_epi(uint32_t lo, uint32_t hi, float k, Result* r) {
    const float knh = -k * 0.5f;
    for (uint64_t b = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < hi;
         b += (uint64_t)gridDim.x * blockDim.x) {
        const float d = __uint_as_float((uint32_t)b);
        if (epilogue_fast<FILT, COL>(d, knh) != visual_epilogue(d, (uint32_t)FILT, k, COL)) report(r, (uint32_t)b);
    }
}

static uint32_t fbits(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
}

static int run(const char* what, void (*launch)(Result*), Result* d) {
    CK(hipMemset(d, 0, sizeof(Result)));
    Result init{0, 0xFFFFFFFFu, 0};
    CK(hipMemcpy(d, &init, sizeof(Result), hipMemcpyHostToDevice));
    launch(d);
    CK(hipGetLastError());
    Result h;
    CK(hipMemcpy(&h, d, sizeof(Result), hipMemcpyDeviceToHost));
    float f;
    memcpy(&f, &h.first, 4);
    printf("%-44s mismatches %llu%s", what, h.bad, h.bad ? "" : "\n");
    if (h.bad) printf("  first bits 0x%08x (%a)\n", h.first, f);
    fflush(stdout);
    return h.bad ? 1 : 0;
}

static const dim3 G(8192), B(256);
static float g_k;
static uint32_t g_lo, g_hi;

int main() {
    Result* d;
    CK(hipMalloc(&d, sizeof(Result)));
    int bad = 0;
    bad += run("recip_ge1 == 1/y, y in [1, 2^117)", [](Result* r) {
        hipLaunchKernelGGL(k_recip, G, B, 0, 0, fbits(1.0f), fbits(0x1p117f), r);
    }, d);
    bad += run("exp_small == det_expf, x in [0, 80]", [](Result* r) {
        hipLaunchKernelGGL(k_exp, G, B, 0, 0, 0u, fbits(80.0f) + 1u, r);
    }, d);
    bad += run("exp_small == det_expf, x in [-80, -0]", [](Result* r) {
        hipLaunchKernelGGL(k_exp, G, B, 0, 0, 0x80000000u, fbits(-80.0f) + 1u, r);
    }, d);
    bad += run("q_bits == unorm_store, all non-NaN f32", [](Result* r) { hipLaunchKernelGGL(k_q, G, B, 0, 0, r); }, d);
    const float ks[] = {1.0f, 2.5f, 5.0f, 7.3f, 10.0f, 160.0f};
    char name[128];
    for (int sign = 0; sign < 2; ++sign) {
        g_lo = sign ? 0x80000000u : 0u;
        g_hi = sign ? fbits(-1.0f) + 1u : fbits(1.0f) + 1u;
        const char* sg = sign ? "[-1, -0]" : "[0, 1]";
        for (float k : ks) {
            g_k = k;
            snprintf(name, sizeof name, "sigmoid gray   k=%g diff in %s", k, sg);
            bad += run(name, [](Result* r) { hipLaunchKernelGGL((k_epi<0, false>), G, B, 0, 0, g_lo, g_hi, g_k, r); }, d);
            snprintf(name, sizeof name, "sigmoid colour k=%g diff in %s", k, sg);
            bad += run(name, [](Result* r) { hipLaunchKernelGGL((k_epi<0, true>), G, B, 0, 0, g_lo, g_hi, g_k, r); }, d);
        }
        snprintf(name, sizeof name, "unfiltered gray   diff in %s", sg);
        bad += run(name, [](Result* r) { hipLaunchKernelGGL((k_epi<255, false>), G, B, 0, 0, g_lo, g_hi, 1.0f, r); }, d);
        snprintf(name, sizeof name, "unfiltered colour diff in %s", sg);
        bad += run(name, [](Result* r) { hipLaunchKernelGGL((k_epi<255, true>), G, B, 0, 0, g_lo, g_hi, 1.0f, r); }, d);
    }
    printf(bad ? "ALTCHECK FAILED (%d checks)\n" : "ALTCHECK OK\n", bad);
    CK(hipFree(d));
    return bad ? 1 : 0;
}
