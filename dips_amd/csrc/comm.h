// comm.h -- the transport table behind the dips_comm* of include/dips_hip.h
// (internal to libdips_hip.so).  shard_abi.hip implements it three times
// (RCCL, loopback threads, the caller's host callbacks) and runs the sharded
// series / ComputeState calls over it; alt_abi.hip runs the sharded dips_alt
// loop over the same table.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <string>

#include "../../include/dips_hip.h"

// ---------------------------------------------------------------------------
// The transport table
// ---------------------------------------------------------------------------
struct dips_comm {
    int kind = 0, nranks = 1, rank = 0, device = 0;
    std::string err;
    virtual ~dips_comm() = default;
    // `bytes` of `send` on rank `root` into `recv` on every rank
    virtual dips_status broadcast(const void* send, void* recv, size_t bytes, int root, hipStream_t s) = 0;
    // send `bytes` of `send` to rank `to`, receive `bytes` from rank `from`
    // into `recv`, concurrently (either side < 0: none)
    virtual dips_status exchange(const void* send, int to, void* recv, int from, size_t bytes, hipStream_t s) = 0;
    // `bytes` of `send` from every rank into `recv` + rank*bytes on `root`
    virtual dips_status gather(const void* send, void* recv, size_t bytes, int root, hipStream_t s) = 0;
    // true: the collectives complete inside the call on the host (the
    // series launch goes first so that the exchange overlaps it)
    virtual bool host_synchronous() const { return false; }

    dips_status failc(dips_status st, const std::string& m) {
        err = m;
        return st;
    }
    dips_status hipc(hipError_t e, const char* what) {
        if (e == hipSuccess) return DIPS_OK;
        return failc(DIPS_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
    }
};

#define COMM_HIP(c, call)                                         \
    do {                                                          \
        dips_status s_ = (c)->hipc((call), #call);                \
        if (s_ != DIPS_OK) return s_;                             \
    } while (0)

