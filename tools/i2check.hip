// i2check.hip -- exhaustive device check of series_v2's intensity formula:
// derive_v2<3, 0> on every RGB8 triple (2^24 pixels) must give
// I2s = (u(max) + u(min)) * 2^22 exactly (u(c) = c/255 in f32), and the
// chroma variants 2 u(channel) * 2^22 on every byte.
#include "../dips_amd/csrc/series_v2.hip"
#include <cstdio>
#include <cstring>
#include <vector>
using namespace dips;

template <int CH>
__global__ void i2_all(const uint32_t* px, float* out, uint32_t nvec) {
    const uint32_t v = blockIdx.x * 256u + threadIdx.x;
    if (v >= nvec) return;
    uint32_t d[3] = {px[3 * v], px[3 * v + 1], px[3 * v + 2]};
    St2 s;
    derive_v2<3, CH>(d, s);
    out[4 * v + 0] = s.i[0].x;
    out[4 * v + 1] = s.i[0].y;
    out[4 * v + 2] = s.i[1].x;
    out[4 * v + 3] = s.i[1].y;
}

int main() {
    const uint32_t npx = 1u << 24, nvec = npx / 4;
    std::vector<uint8_t> bytes((size_t)npx * 3);
    for (uint32_t p = 0; p < npx; ++p) {
        bytes[3 * (size_t)p] = (uint8_t)(p >> 16);
        bytes[3 * (size_t)p + 1] = (uint8_t)(p >> 8);
        bytes[3 * (size_t)p + 2] = (uint8_t)p;
    }
    float u[256];
    for (int c = 0; c < 256; ++c) u[c] = (float)c / 255.0f;
    uint32_t* dpx;
    float* dout;
    (void)hipMalloc(&dpx, bytes.size());
    (void)hipMalloc(&dout, (size_t)npx * 4);
    (void)hipMemcpy(dpx, bytes.data(), bytes.size(), hipMemcpyHostToDevice);
    std::vector<float> got(npx);
    long total_bad = 0;
    for (int ch = 0; ch < 4; ++ch) {
        switch (ch) {
            case 0: hipLaunchKernelGGL(i2_all<0>, dim3(nvec / 256), dim3(256), 0, 0, dpx, dout, nvec); break;
            case 1: hipLaunchKernelGGL(i2_all<1>, dim3(nvec / 256), dim3(256), 0, 0, dpx, dout, nvec); break;
            case 2: hipLaunchKernelGGL(i2_all<2>, dim3(nvec / 256), dim3(256), 0, 0, dpx, dout, nvec); break;
            default: hipLaunchKernelGGL(i2_all<3>, dim3(nvec / 256), dim3(256), 0, 0, dpx, dout, nvec); break;
        }
        (void)hipMemcpy(got.data(), dout, (size_t)npx * 4, hipMemcpyDeviceToHost);
        long bad = 0;
        for (uint32_t p = 0; p < npx; ++p) {
            const uint8_t r = bytes[3 * (size_t)p], g = bytes[3 * (size_t)p + 1], b = bytes[3 * (size_t)p + 2];
            float want;
            if (ch == 0) {
                const uint8_t mx = r > g ? (r > b ? r : b) : (g > b ? g : b);
                const uint8_t mn = r < g ? (r < b ? r : b) : (g < b ? g : b);
                want = (u[mx] + u[mn]) * 4194304.0f;
            } else {
                const uint8_t c = ch == 1 ? r : (ch == 2 ? g : b);
                want = (u[c] + u[c]) * 4194304.0f;
            }
            if (std::memcmp(&got[p], &want, 4)) {
                if (bad < 5) printf("chroma %d px (%u,%u,%u): want %.9g got %.9g\n", ch, r, g, b, want, got[p]);
                ++bad;
            }
        }
        printf("i2check chroma %d: %ld mismatches of %u pixels\n", ch, bad, npx);
        total_bad += bad;
    }
    return total_bad != 0;
}
