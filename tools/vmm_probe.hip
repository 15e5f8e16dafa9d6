// vmm_probe.hip -- frame buffers through the HIP virtual-memory API, to see
// whether how a 124 GB buffer is backed and mapped (physical chunk size,
// virtual alignment) decides the 2.5-3 point placement spread of the
// headline (tools/placement_probe.py).  A buffer is a virtual range
// reserved with the given alignment and backed by physical allocations of
// `chunk` bytes (hipMemCreate), mapped back to back and made read/write for
// the device.  Driven by tools/placement_probe.py --vmm.
//
// Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC -cuid=vmm_probe \
//          -o tools/libvmm_probe.so tools/vmm_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

namespace {
struct Buf {
    void* va = nullptr;
    size_t size = 0;
    std::vector<hipMemGenericAllocationHandle_t> handles;
};
std::vector<Buf> g_bufs;
}  // namespace

extern "C" {

// granularity (recommended) of device allocations on `device`, bytes
size_t vmm_granularity(int device) {
    hipMemAllocationProp prop{};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = device;
    size_t g = 0;
    if (hipMemGetAllocationGranularity(&g, &prop, hipMemAllocationGranularityRecommended) != hipSuccess) return 0;
    return g;
}

// returns an id >= 0 and the device pointer in *out, or a negative hipError_t
int vmm_alloc(int device, size_t size, size_t va_align, size_t chunk, void** out) {
    const size_t g = vmm_granularity(device);
    if (g == 0) return -1000;
    if (chunk % g || size % chunk) return -1001;
    Buf b;
    b.size = size;
    hipError_t e = hipMemAddressReserve(&b.va, size, va_align, nullptr, 0);
    if (e != hipSuccess) return -(int)e;
    hipMemAllocationProp prop{};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = device;
    for (size_t off = 0; off < size; off += chunk) {
        hipMemGenericAllocationHandle_t h;
        e = hipMemCreate(&h, chunk, &prop, 0);
        if (e != hipSuccess) return -(int)e;
        b.handles.push_back(h);
        e = hipMemMap(static_cast<char*>(b.va) + off, chunk, 0, h, 0);
        if (e != hipSuccess) return -(int)e;
    }
    hipMemAccessDesc acc{};
    acc.location.type = hipMemLocationTypeDevice;
    acc.location.id = device;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    e = hipMemSetAccess(b.va, size, &acc, 1);
    if (e != hipSuccess) return -(int)e;
    *out = b.va;
    g_bufs.push_back(b);
    return (int)g_bufs.size() - 1;
}

int vmm_free(int id) {
    if (id < 0 || id >= (int)g_bufs.size() || !g_bufs[id].va) return -1;
    Buf& b = g_bufs[id];
    (void)hipDeviceSynchronize();
    (void)hipMemUnmap(b.va, b.size);
    for (auto h : b.handles) (void)hipMemRelease(h);
    (void)hipMemAddressFree(b.va, b.size);
    b.va = nullptr;
    b.handles.clear();
    return 0;
}
}
