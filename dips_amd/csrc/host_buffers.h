// host_buffers.h -- device / pinned-host buffers owned by the C-ABI handles
// (internal to libdips_hip.so).
#pragma once

#include <hip/hip_runtime.h>

#include <sys/mman.h>

#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <cstring>

namespace dips_host {

// Grow-only device allocation.
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t n) {
        if (n <= cap) return hipSuccess;
        if (p) {
            hipError_t e = hipFree(p);
            p = nullptr;
            cap = 0;
            if (e != hipSuccess) return e;
        }
        hipError_t e = hipMalloc(&p, n);
        if (e == hipSuccess) cap = n;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    template <typename T> T* as() const { return static_cast<T*>(p); }
};

// Whether pinned staging buffers are built from 2 MiB transparent huge pages
// (DIPS_PIN_HUGE=1: anonymous mmap, madvise(MADV_HUGEPAGE), then
// hipHostRegister) instead of hipHostMalloc.  Read by the allocating call.
inline bool pin_huge() {
    const char* e = std::getenv("DIPS_PIN_HUGE");
    return e && e[0] == '1';
}

// Grow-only pinned host allocation (DMA staging, and the zero-copy buffers the
// per-frame kernels read and write over PCIe).
struct HostPinned {
    void* p = nullptr;
    size_t cap = 0;
    void* map = nullptr;  // huge-page form: the mmap'd range behind p
    size_t map_len = 0;
    hipError_t ensure(size_t n) {
        if (n <= cap) return hipSuccess;
        release();
        if (pin_huge()) return ensure_huge(n);
        hipError_t e = hipHostMalloc(&p, n, hipHostMallocDefault);
        if (e == hipSuccess) cap = n;
        return e;
    }
    hipError_t ensure_huge(size_t n) {
        constexpr size_t kHuge = 2u << 20;
        const size_t sz = (n + kHuge - 1) & ~(kHuge - 1);
        void* m = mmap(nullptr, sz + kHuge, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (m == MAP_FAILED) return hipErrorOutOfMemory;
        uint8_t* q = reinterpret_cast<uint8_t*>(((uintptr_t)m + kHuge - 1) & ~(uintptr_t)(kHuge - 1));
        (void)madvise(q, sz, MADV_HUGEPAGE);
        std::memset(q, 0, sz);  // fault the pages in (as huge pages where the kernel has them)
        const hipError_t e = hipHostRegister(q, sz, hipHostRegisterMapped | hipHostRegisterPortable);
        if (e != hipSuccess) {
            munmap(m, sz + kHuge);
            return e;
        }
        map = m;
        map_len = sz + kHuge;
        p = q;
        cap = n;
        return hipSuccess;
    }
    void release() {
        if (map) {
            // unmap only what the runtime let go of: if the unregister fails
            // the pages may still be mapped for the device, so the range is
            // leaked rather than returned to the OS under a live mapping
            if (hipHostUnregister(p) == hipSuccess) munmap(map, map_len);
            map = nullptr;
            map_len = 0;
        } else if (p) {
            (void)hipHostFree(p);
        }
        p = nullptr;
        cap = 0;
    }
    uint8_t* bytes() const { return static_cast<uint8_t*>(p); }
};

}  // namespace dips_host
