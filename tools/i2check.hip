// i2check.hip -- exhaustive device check of series_v2's intensity formula:
// for every (max, min) byte pair, derive_v2 on an RGB8 pixel (max, min, min)
// must give I2s = (u(max) + u(min)) * 2^22 exactly (u(c) = c/255 in f32).
#include "../dips_amd/csrc/series_v2.hip"
#include <cstdio>
#include <cstring>
#include <vector>
using namespace dips;

__global__ void i2_all(const uint32_t* px, float* out, uint32_t nvec) {
    const uint32_t v = blockIdx.x * 256u + threadIdx.x;
    if (v >= nvec) return;
    uint32_t d[3] = {px[3 * v], px[3 * v + 1], px[3 * v + 2]};
    St2 s;
    derive_v2<3, 0>(d, s);
    out[4 * v + 0] = s.i[0].x;
    out[4 * v + 1] = s.i[0].y;
    out[4 * v + 2] = s.i[1].x;
    out[4 * v + 3] = s.i[1].y;
}

int main() {
    std::vector<uint8_t> bytes;
    std::vector<float> want;
    for (uint32_t mx = 0; mx < 256; ++mx)
        for (uint32_t mn = 0; mn <= mx; ++mn) {
            bytes.push_back((uint8_t)mx);
            bytes.push_back((uint8_t)mn);
            bytes.push_back((uint8_t)mn);
            const float u = (float)mx / 255.0f, w = (float)mn / 255.0f;
            want.push_back((u + w) * 4194304.0f);
        }
    while (want.size() % 4) {  // pad to whole vecs with black pixels
        bytes.insert(bytes.end(), {0, 0, 0});
        want.push_back(0.0f);
    }
    const uint32_t nvec = (uint32_t)want.size() / 4;
    uint32_t* dpx;
    float* dout;
    (void)hipMalloc(&dpx, bytes.size());
    (void)hipMalloc(&dout, want.size() * 4);
    (void)hipMemcpy(dpx, bytes.data(), bytes.size(), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(i2_all, dim3((nvec + 255) / 256), dim3(256), 0, 0, dpx, dout, nvec);
    std::vector<float> got(want.size());
    (void)hipMemcpy(got.data(), dout, got.size() * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (size_t i = 0; i < want.size(); ++i)
        if (std::memcmp(&got[i], &want[i], 4)) {
            if (bad < 8) printf("px %zu (%u,%u): want %.9g got %.9g\n", i, bytes[3 * i], bytes[3 * i + 1], want[i], got[i]);
            ++bad;
        }
    printf("i2check: %d mismatches of %zu pixels (all max >= min byte pairs)\n", bad, want.size());
    return bad != 0;
}
