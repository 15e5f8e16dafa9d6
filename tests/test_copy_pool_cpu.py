"""CPU check of the copy pool's per-pixel packers (dips_amd/csrc/copy_pool.h,
ADVICE r3): the AVX2 forms of pack_frame ((max, min) of R, G, B, or one
chroma channel, per RGBA8 pixel) and expand_keys (1-B gray / 2-B colour keys
back to RGBA8 texels) against their scalar forms, for pixel counts that are
and are not multiples of the vector widths, both store kinds (streaming and
plain), and misaligned destinations.  A small C++ harness is compiled with
g++ against the header itself; no GPU and no HIP runtime are involved."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

HARNESS = r'''
#include "copy_pool.h"
#include <cstdio>
#include <random>
#include <vector>
using namespace dips_host;
int main() {
    if (!__builtin_cpu_supports("avx2")) { std::puts("SKIP no avx2"); return 0; }
    std::mt19937 rng(1234);
    long bad = 0, cases = 0;
    for (size_t npx : {0ul, 1ul, 7ul, 8ul, 15ul, 16ul, 17ul, 31ul, 33ul, 1000ul, 4093ul}) {
        for (size_t off : {0ul, 1ul, 3ul, 32ul}) {
            std::vector<uint8_t> src(4 * npx + 64), keys(2 * npx + 64);
            for (auto& b : src) b = (uint8_t)rng();
            for (auto& b : keys) b = (uint8_t)rng();
            for (bool nt : {false, true}) {
                for (int ib : {1, 2}) for (int ch = 0; ch < (ib == 1 ? 3 : 1); ++ch) {
                    std::vector<uint8_t> a(2 * npx + 64, 0xAA), b(2 * npx + 64, 0xAA);
                    pack_frame_avx2(a.data() + off, src.data() + 3, npx, ib, ch, nt);
                    pack_frame_scalar(b.data() + off, src.data() + 3, npx, ib, ch);
                    bad += a != b; ++cases;
                }
                for (int kb : {1, 2}) {
                    std::vector<uint8_t> a(4 * npx + 64, 0xAA), b(4 * npx + 64, 0xAA);
                    expand_keys_avx2(a.data() + off, keys.data() + 1, npx, kb, nt);
                    expand_keys_scalar(b.data() + off, keys.data() + 1, npx, kb);
                    bad += a != b; ++cases;
                }
            }
        }
    }
    std::printf("cases %ld bad %ld\n", cases, bad);
    return bad != 0;
}
'''


def test_avx2_packers_equal_scalar(tmp_path):
    src = tmp_path / "h.cpp"
    src.write_text(HARNESS)
    exe = tmp_path / "h"
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", "-I", os.path.join(ROOT, "dips_amd", "csrc"),
                    str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    if out.stdout.startswith("SKIP"):
        pytest.skip(out.stdout.strip())
    assert out.returncode == 0, out.stdout + out.stderr
    assert "bad 0" in out.stdout


POOL_HARNESS = r'''
#include "copy_pool.h"
#include <atomic>
#include <cstdio>
#include <thread>
#include <vector>
using namespace dips_host;
int main() {
    // back-to-back runs of varying size on one pool, each task bumping its own
    // slot: every slot of every run exactly once, nothing after run() returns
    CopyPool pool(7);
    long bad = 0;
    for (int r = 0; r < 20000; ++r) {
        const size_t n = 1 + (size_t)(r * 7919) % 37;
        std::vector<std::atomic<int>> hits(n);
        for (auto& h : hits) h.store(0);
        pool.run(n, [&](size_t i) {
            if (i % 5 == 0) std::this_thread::yield();
            hits[i].fetch_add(1);
        });
        for (size_t i = 0; i < n; ++i) bad += hits[i].load() != 1;
    }
    std::printf("bad %ld\n", bad);
    return bad != 0;
}
'''


@pytest.mark.parametrize("tsan", [False, True])
def test_pool_runs_every_task_once(tmp_path, tsan):
    """CopyPool::run: 20,000 back-to-back runs of 1-37 tasks on one pool,
    every task exactly once per run, none after the run returned (its slots
    live on the caller's stack); also under ThreadSanitizer."""
    src = tmp_path / "p.cpp"
    src.write_text(POOL_HARNESS)
    exe = tmp_path / "p"
    flags = ["-O1", "-g", "-fsanitize=thread"] if tsan else ["-O2"]
    r = subprocess.run(["g++", *flags, "-std=c++17", "-pthread", "-I", os.path.join(ROOT, "dips_amd", "csrc"),
                        str(src), "-o", str(exe)], capture_output=True, text=True)
    if tsan and r.returncode != 0:
        pytest.skip("no ThreadSanitizer runtime: " + r.stderr[-200:])
    assert r.returncode == 0, r.stderr
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1")
    out = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=300)
    if tsan and "FATAL: ThreadSanitizer" in out.stderr:
        pytest.skip("ThreadSanitizer cannot run here: " + out.stderr[-200:])
    assert out.returncode == 0, out.stdout + out.stderr[-3000:]
    assert "bad 0" in out.stdout
