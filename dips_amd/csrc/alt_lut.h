// alt_lut.h -- the dips_alt epilogue as a table (alt_batch_kernel, LUT form).
//
// In the dips_alt batch the epilogue's argument is
//     diff = u(S) - I           (pre_compute_shader.wgsl:237-241)
// with S the snapshot byte and I a pixel intensity (the temporal min of two
// intensities, or the prefiltered window value, is one of them), and every
// pixel intensity is (u(max) + u(min)) / 2 for some byte pair (a single
// channel c is the pair (c, c); 0 is (0, 0)).  Those are 638 distinct f32
// values, so diff takes only 2,993 distinct f32 values, and the RGBA output
// is a function of diff alone.  The table maps each of them to R | G << 8 of
// the specification's texel (B = min(R, G), A = 255: compat_batch.hip
// lut_texel), through an exact two-level index:
//   level 1: the cluster n = rint(510 * diff) in [-510, 510] (one v_fma_f32
//            with the 1.5 * 2^23 round-to-integer offset), 8 bytes per
//            cluster: {x, sh};
//   level 2: byte address ((bits(diff) >> sh) << 1) + x, where sh is the
//            smallest right shift that keeps the cluster's members apart and
//            x folds the cluster's base and its offset in the u16 table.
// The index depends only on the value set (built once per process, host
// arithmetic identical to the device's: IEEE f32 division, subtraction and
// fmaf); the u16 contents depend on (filter, k, colorize) and are filled by
// alt_lut_fill_kernel from the spec epilogue.  tests/test_gpu_alt.py checks
// the LUT kernel against the arithmetic one and the oracle, and
// dips_alt_lut_selfcheck evaluates the whole (S, max, min) space on device.
#pragma once

#include <stdint.h>

#include <vector>

namespace dips {

constexpr int kAltLutClusters = 1021;      // n = -510 .. 510
// u16 entries (5,822 used).  LDS per workgroup 8,168 + 11,776 = 19,944 B:
// eight 256-thread groups per CU fit the 160 KiB with room to spare (at
// 20,456 B the eighth group filled it to the last 192 B).
constexpr int kAltLutL2Max = 5888;
constexpr float kAltLutRound = 12582912.0f;  // 1.5 * 2^23
// byte address of the level-1 entry: (bits(fma(diff, 510, 1.5 * 2^23)) << 3) - kAltLutL1Bias
constexpr uint32_t kAltLutL1Bias = (0x4B400000u - 510u) << 3;

struct AltLutIndex {
    uint32_t l1[2 * kAltLutClusters];  // per cluster {x, sh}
    std::vector<float> diffs;          // the distinct diff values
    std::vector<uint16_t> slots;       // their level-2 entry
    uint32_t l2_entries = 0;
};

// Built on first use (thread-safe).
const AltLutIndex& alt_lut_index();

}  // namespace dips
