"""CPU checks of the C ABI's failure contract (no exception
or panic crosses the ABI):

* every function include/dips_hip.h declares is defined in dips_amd/csrc as
  `{ return dips_abi::guard(where, [&]() -> T { ... }); }` (abi_guard.h) --
  the whole body inside the guard, nothing before or after it;
* the copy pool (copy_pool.h) keeps working when the system refuses its
  worker threads (std::thread throws std::system_error on EAGAIN): under an
  address-space limit that leaves room for only a few thread stacks, or none,
  and under `prlimit --nproc` where that binds (not as root), every task of
  every run completes; a task that throws has its exception rethrown on the
  calling thread once the run is over, and the pool runs the next job;
* abi_guard.h's guard itself turns std::bad_alloc, std::exception and
  foreign exceptions into the documented statuses and messages.
The harnesses are compiled with g++ against the headers; no GPU, no HIP
runtime."""
import os
import re
import shutil
import subprocess

import pytest

from dips_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "dips_amd", "csrc")


def _sources():
    out = {}
    for fn in sorted(os.listdir(CSRC)):
        if fn.endswith((".hip", ".h", ".cpp")):
            with open(os.path.join(CSRC, fn)) as f:
                out[fn] = f.read()
    return out


def _strip_comments(s):
    s = re.sub(r"/\*.*?\*/", " ", s, flags=re.S)
    return re.sub(r"//[^\n]*", " ", s)


def _match_brace(s, i, open_c="{", close_c="}"):
    """Index just past the bracket matching s[i] (string literals skipped)."""
    depth, k, n = 0, i, len(s)
    while k < n:
        c = s[k]
        if c == '"':
            k += 1
            while s[k] != '"':
                k += 2 if s[k] == "\\" else 1
        elif c == "'":
            k += 1
            while s[k] != "'":
                k += 2 if s[k] == "\\" else 1
        elif c == open_c:
            depth += 1
        elif c == close_c:
            depth -= 1
            if depth == 0:
                return k + 1
        k += 1
    raise AssertionError("unbalanced")


def _definitions(name, sources):
    """(file, body) of every definition of function `name` at file scope."""
    found = []
    for fn, text in sources.items():
        t = _strip_comments(text)
        for m in re.finditer(r"^[A-Za-z_][\w \*]*?\b%s\s*\(" % re.escape(name), t, flags=re.M):
            p_end = _match_brace(t, m.end() - 1, "(", ")")
            rest = t[p_end:]
            k = len(rest) - len(rest.lstrip())
            if not rest[k:].startswith("{"):
                continue  # a declaration or a call
            b_end = _match_brace(t, p_end + k)
            found.append((fn, t[p_end + k:b_end]))
    return found


GUARDED = re.compile(r"^\{\s*(?:return\s+)?guard\(\s*([^,]+?)\s*,\s*\[&\]\(\)\s*->\s*[\w\s\*]+?\{(.*)\}\s*\)\s*;\s*\}$",
                     re.S)


def test_every_exported_function_body_is_inside_the_guard():
    sources = _sources()
    names = _lib.header_functions()
    assert len(names) >= 38
    for name in names:
        defs = _definitions(name, sources)
        assert len(defs) == 1, (name, [d[0] for d in defs])
        fn, body = defs[0]
        m = GUARDED.match(body.strip())
        assert m, f"{fn}: {name} is not written as {{ return guard(where, [&]() -> T {{ ... }}); }}"
        where = m.group(1)
        # the error goes to the handle argument, or (creation / handle-free
        # functions) to the process-wide record or nowhere
        assert where in ("h", "comm", "nullptr", "dips_abi::CreateTag{}", "dips_abi::AltCreateTag{}",
                         "dips_abi::CommCreateTag{}"), (name, where)
        if where in ("dips_abi::CreateTag{}", "dips_abi::AltCreateTag{}"):
            assert name in ("dips_create", "dips_alt_create"), name
        if where == "dips_abi::CommCreateTag{}":
            assert name.startswith(("dips_comm_create", "dips_comm_unique_id")), name
    # the guard's translation units use the guard from abi_guard.h
    for fn in ("dips_abi.hip", "compat_abi.hip", "series_abi.hip", "alt_abi.hip", "shard_abi.hip"):
        assert "using dips_abi::guard;" in sources[fn], fn


def test_no_exported_function_outside_the_header():
    """Every extern "C" function defined in the library is one the header
    declares (so the check above covers all of them)."""
    sources = _sources()
    declared = set(_lib.header_functions())
    for fn, text in sources.items():
        t = _strip_comments(text)
        for m in re.finditer(r'extern "C"\s*\{', t):
            block = t[m.end() - 1:_match_brace(t, m.end() - 1)]
            for d in re.finditer(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(dips_[a-z_0-9]+)\s*\(", block, flags=re.M):
                assert d.group(1) in declared, (fn, d.group(1))


_GUARD_HARNESS = r'''
#include "abi_guard.h"
#include <cstdio>
#include <cstring>
#include <new>
#include <stdexcept>
#include <string>
struct dips_handle { std::string err; };
struct dips_alt_handle { std::string err; };
namespace dips_abi {
void note_error(dips_handle* h, const char* m) noexcept { if (h) h->err = m; }
void note_error(dips_alt_handle* h, const char* m) noexcept { if (h) h->err = m; }
static std::string g_create;
void note_error(CreateTag, const char* m) noexcept { g_create = m; }
void note_error(AltCreateTag, const char* m) noexcept { g_create = m; }
// the HIP device of the calling thread, simulated
static int g_dev = 1, g_dev_reads = 0;
int current_device() noexcept { ++g_dev_reads; return g_dev; }
void set_device(int d) noexcept { g_dev = d; }
}
using dips_abi::guard;
int main() {
    int bad = 0;
    dips_handle h;
    bad += guard(&h, [&]() -> dips_status { throw std::bad_alloc(); }) != DIPS_ERR_NOMEM;
    bad += h.err.find("bad_alloc") == std::string::npos;
    bad += guard(&h, [&]() -> int { throw std::runtime_error("boom"); }) != DIPS_ERR_INTERNAL;
    bad += h.err != "boom";
    bad += guard(&h, [&]() -> int { throw 42; }) != DIPS_ERR_INTERNAL;
    bad += h.err.find("unknown") == std::string::npos;
    bad += guard(dips_abi::CreateTag{}, [&]() -> dips_status { throw std::logic_error("create"); }) != DIPS_ERR_INTERNAL;
    bad += dips_abi::g_create != "create";
    const double d = guard(nullptr, [&]() -> double { throw std::bad_alloc(); });
    bad += d == d;  // NaN
    const char* s = guard(static_cast<const dips_handle*>(&h), [&]() -> const char* { throw 1; });
    bad += s == nullptr || std::strlen(s) == 0;
    bool ran = false;
    guard(&h, [&]() -> void { ran = true; throw std::runtime_error("void"); });
    bad += !ran || h.err != "void";
    bad += guard(&h, [&]() -> int { return 7; }) != 7;
    // the caller's device is put back, also when the body throws; host-only
    // functions (nullptr) never read it
    dips_abi::g_dev = 1;
    bad += guard(&h, [&]() -> int { dips_abi::g_dev = 3; return 0; }) != 0;
    bad += dips_abi::g_dev != 1;
    guard(&h, [&]() -> void { dips_abi::g_dev = 2; throw std::runtime_error("x"); });
    bad += dips_abi::g_dev != 1;
    const int reads = dips_abi::g_dev_reads;
    (void)guard(nullptr, [&]() -> int { return 0; });
    bad += dips_abi::g_dev_reads != reads;
    std::printf("bad %d\n", bad);
    return bad != 0;
}
'''


def test_guard_maps_exceptions_to_statuses(tmp_path):
    src = tmp_path / "g.cpp"
    src.write_text(_GUARD_HARNESS)
    exe = tmp_path / "g"
    subprocess.run(["g++", "-O1", "-std=c++17", "-I", CSRC, "-I", os.path.join(ROOT, "include"), str(src), "-o",
                    str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "bad 0" in r.stdout, r.stdout + r.stderr


_POOL_LIMIT_HARNESS = r'''
#include "copy_pool.h"
#include <sys/resource.h>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <stdexcept>
#include <string>
#include <vector>
using namespace dips_host;
// bytes of address space in use now (VmSize)
static size_t vm_bytes() {
    std::ifstream f("/proc/self/status");
    std::string k;
    size_t v = 0;
    while (f >> k) {
        if (k == "VmSize:") { f >> v; return v * 1024; }
    }
    return 0;
}
int main(int argc, char** argv) {
    const unsigned want = 7;
    const long room = std::atol(argv[1]);  // thread stacks of room: -1 = no AS limit (nproc mode)
    if (room >= 0) {
        struct rlimit rl;
        getrlimit(RLIMIT_STACK, &rl);
        const size_t stack = rl.rlim_cur == RLIM_INFINITY ? (8u << 20) : rl.rlim_cur;
        // space for `room` thread stacks (+ guard pages and slack), not more
        const size_t lim = vm_bytes() + (size_t)room * (stack + (1u << 20)) + (4u << 20);
        rl.rlim_cur = rl.rlim_max = lim;
        if (setrlimit(RLIMIT_AS, &rl) != 0) { std::puts("SKIP setrlimit"); return 0; }
    }
    long bad = 0;
    CopyPool pool(want);
    const unsigned got = pool.threads() - 1;
    for (int r = 0; r < 3000; ++r) {
        const size_t n = 1 + (size_t)(r * 7919) % 37;
        std::vector<std::atomic<int>> hits(n);
        for (auto& x : hits) x.store(0);
        pool.run(n, [&](size_t i) { hits[i].fetch_add(1); }, (r & 1) != 0);
        for (size_t i = 0; i < n; ++i) bad += hits[i].load() != 1;
    }
    // a task that throws: every other task still runs once, the exception
    // reaches the caller after the run, and the pool takes the next run
    for (int r = 0; r < 200; ++r) {
        std::vector<std::atomic<int>> hits(16);
        for (auto& x : hits) x.store(0);
        bool caught = false;
        try {
            pool.run(16, [&](size_t i) {
                hits[i].fetch_add(1);
                if (i == (size_t)(r % 16)) throw std::runtime_error("task");
            });
        } catch (const std::runtime_error&) {
            caught = true;
        }
        bad += !caught;
        for (auto& x : hits) bad += x.load() != 1;
    }
    std::printf("workers %u of %u bad %ld\n", got, want, bad);
    return bad != 0;
}
'''


def _build_pool_harness(tmp_path):
    src = tmp_path / "pl.cpp"
    src.write_text(_POOL_LIMIT_HARNESS)
    exe = tmp_path / "pl"
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", "-I", CSRC, str(src), "-o", str(exe)], check=True)
    return exe


@pytest.mark.parametrize("room", [0, 2])
def test_pool_survives_thread_creation_failure(tmp_path, room):
    """Under an address-space limit that leaves room for `room` thread stacks
    (std::thread then throws std::system_error), CopyPool starts the workers
    it can -- none, or a few of the 7 asked for -- and every task of every run
    still completes exactly once (the calling thread drains alone at 0)."""
    exe = _build_pool_harness(tmp_path)
    r = subprocess.run([str(exe), str(room)], capture_output=True, text=True, timeout=120)
    if r.stdout.startswith("SKIP"):
        pytest.skip(r.stdout.strip())
    assert r.returncode == 0, r.stdout + r.stderr
    m = re.search(r"workers (\d+) of 7 bad 0", r.stdout)
    assert m, r.stdout
    assert int(m.group(1)) <= room  # the limit did bind: fewer workers than asked


def test_pool_under_prlimit_nproc(tmp_path):
    """The same under `prlimit --nproc` (the thread / process limit of a GPU
    box's process guard).  RLIMIT_NPROC does not bind root, so as root this
    only checks that the run completes."""
    if shutil.which("prlimit") is None:
        pytest.skip("no prlimit")
    exe = _build_pool_harness(tmp_path)
    nproc = 1 if os.geteuid() != 0 else 2
    r = subprocess.run(["prlimit", f"--nproc={nproc}", str(exe), "-1"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    m = re.search(r"workers (\d+) of 7 bad 0", r.stdout)
    assert m, r.stdout
    if os.geteuid() != 0:
        assert int(m.group(1)) < 7
