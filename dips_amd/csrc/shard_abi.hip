// shard_abi.hip -- host side of include/dips_hip.h, part 5: frame-range
// sharding of the difference series over one rank per GPU (SURVEY.md s8e;
// north_star: "sharded by frame-range across the 8 GPUs of one node with a
// single RCCL gather over xGMI").  The reference has no counterpart: it
// drives one wgpu adapter and queue (dips/src/gpu/mod.rs:66-98, the adapter
// request at :71-78) with frames strictly in order.
//
// Rank r of G owns the global frames [r*N/G, (r+1)*N/G).  One sharded call
// is, on every rank:
//   'overall':   ncclBroadcast of the reference from rank 0 (or none with
//                DIPS_SHARD_REF_RESIDENT), the series launch over the rank's
//                frames;
//   'per-frame': rank r sends its last frame to r+1 and receives r-1's
//                (ncclSend / ncclRecv in one group) on a side stream, posted
//                before the series launch over its frames 1..n-1 (each
//                against its own predecessor), so the transfer's kernels are
//                resident first and the full persistent grid fills the rest
//                (a grid capped to leave them room measured worse:
//                profiles/r06/halo_contention/); frame 0 against the halo
//                once it has landed;
//   both:        one ncclGather of the padded per-rank series (32 B a frame)
//                onto rank 0, trimmed into place there.
// Everything is stream-ordered on the handle's stream: the call returns
// after enqueueing (device pointers), as dips_diff_series does.
//
// The collectives go through a small transport table (struct dips_comm):
// RCCL; a loopback of ranks as threads on one device (hipMemcpyAsync
// between the ranks' buffers, ordered by events, the ranks meeting on the
// host); and the caller's own transport through host callbacks.  Every
// extern "C" body runs inside dips_abi::guard (abi_guard.h).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <condition_variable>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "comm.h"
#include "dips_handle.h"

using dips_abi::guard;
using namespace dips_internal;

namespace {

std::mutex g_comm_err_mu;
std::string g_comm_create_err;

void set_comm_create_err(const std::string& m) {
    std::lock_guard<std::mutex> lk(g_comm_err_mu);
    g_comm_create_err = m;
}

// -- RCCL over xGMI ---------------------------------------------------------
struct RcclComm final : dips_comm {
    ncclComm_t c = nullptr;

    ~RcclComm() override {
        if (c) {
            (void)hipSetDevice(device);
            (void)ncclCommDestroy(c);
        }
    }

    dips_status nccl(ncclResult_t r, const char* what) {
        if (r == ncclSuccess) return DIPS_OK;
        const char* last = ncclGetLastError(c);
        return failc(DIPS_ERR_COMM, std::string(what) + ": " + ncclGetErrorString(r) +
                                        (last && *last ? std::string(" (") + last + ")" : std::string()));
    }

    dips_status broadcast(const void* send, void* recv, size_t bytes, int root, hipStream_t s) override {
        return nccl(ncclBroadcast(rank == root ? send : nullptr, recv, bytes, ncclUint8, root, c, s), "ncclBroadcast");
    }

    dips_status exchange(const void* send, int to, void* recv, int from, size_t bytes, hipStream_t s) override {
        if (to < 0 && from < 0) return DIPS_OK;
        dips_status st = nccl(ncclGroupStart(), "ncclGroupStart");
        if (st != DIPS_OK) return st;
        if (to >= 0) st = nccl(ncclSend(send, bytes, ncclUint8, to, c, s), "ncclSend");
        if (st == DIPS_OK && from >= 0) st = nccl(ncclRecv(recv, bytes, ncclUint8, from, c, s), "ncclRecv");
        // the group is closed whatever happened inside it
        const dips_status end = nccl(ncclGroupEnd(), "ncclGroupEnd");
        return st != DIPS_OK ? st : end;
    }

    dips_status gather(const void* send, void* recv, size_t bytes, int root, hipStream_t s) override {
        return nccl(ncclGather(send, rank == root ? recv : nullptr, bytes, ncclUint8, root, c, s), "ncclGather");
    }
};

// -- loopback: ranks as threads on one device -------------------------------
constexpr int kLoopTimeoutS = 60;  // a rank that never reaches a collective

struct LoopGroup {
    struct Post {
        const void* send = nullptr;
        void* recv = nullptr;
        size_t bytes = 0;
        int to = -1;
        hipEvent_t ready = nullptr;  // recorded after the rank's prior work on its stream
        hipEvent_t done = nullptr;   // recorded after the rank's copies of this collective
    };
    int n = 0;
    std::mutex mu;
    std::condition_variable cv;
    int waiting = 0;
    uint64_t gen = 0;
    bool broken = false;
    std::vector<Post> posts[2];  // collective k uses posts[k & 1] (see LoopComm::collective)

    // all n ranks arrive, or none proceeds (timeout, or a rank that failed)
    bool barrier() {
        std::unique_lock<std::mutex> lk(mu);
        if (broken) return false;
        const uint64_t g = gen;
        if (++waiting == n) {
            waiting = 0;
            ++gen;
            cv.notify_all();
            return true;
        }
        const bool met = cv.wait_for(lk, std::chrono::seconds(kLoopTimeoutS), [&] { return gen != g || broken; });
        if (!met || broken) {
            broken = true;
            cv.notify_all();
            return false;
        }
        return true;
    }

    void fail() {
        std::lock_guard<std::mutex> lk(mu);
        broken = true;
        cv.notify_all();
    }
};

struct LoopComm final : dips_comm {
    std::shared_ptr<LoopGroup> g;
    uint64_t seq = 0;
    hipEvent_t ready[2] = {nullptr, nullptr};
    hipEvent_t done[2] = {nullptr, nullptr};

    ~LoopComm() override {
        (void)hipSetDevice(device);
        for (int i = 0; i < 2; ++i) {
            if (ready[i]) (void)hipEventDestroy(ready[i]);
            if (done[i]) (void)hipEventDestroy(done[i]);
        }
    }

    // Post this rank's buffers, meet, enqueue this rank's copies (`copy`,
    // reading the others' posts), meet again, enqueue the waits that keep
    // this rank's buffers unchanged until the others' copies of them are done
    // (`hold`).  Posts alternate between two slots: a rank can post collective
    // k+2 only after every rank has posted k+1, i.e. finished reading k.
    template <typename Copy, typename Hold>
    dips_status collective(LoopGroup::Post mine, hipStream_t s, Copy&& copy, Hold&& hold) {
        const int slot = (int)(seq++ & 1u);
        auto broken = [&](dips_status st) {
            g->fail();
            return st;
        };
        if (hipc(hipEventRecord(ready[slot], s), "hipEventRecord") != DIPS_OK) return broken(DIPS_ERR_HIP);
        mine.ready = ready[slot];
        mine.done = done[slot];
        {
            std::lock_guard<std::mutex> lk(g->mu);
            g->posts[slot][rank] = mine;
        }
        if (!g->barrier())
            return failc(DIPS_ERR_COMM, "loopback: a rank did not reach the collective (timeout or failure)");
        std::vector<LoopGroup::Post> all;
        {
            std::lock_guard<std::mutex> lk(g->mu);
            all = g->posts[slot];
        }
        dips_status st = copy(all);
        if (st == DIPS_OK) st = hipc(hipEventRecord(done[slot], s), "hipEventRecord");
        if (st != DIPS_OK) return broken(st);
        if (!g->barrier())
            return failc(DIPS_ERR_COMM, "loopback: a rank did not finish the collective (timeout or failure)");
        st = hold(all);
        return st != DIPS_OK ? broken(st) : DIPS_OK;
    }

    dips_status wait_for(hipStream_t s, hipEvent_t e) { return hipc(hipStreamWaitEvent(s, e, 0), "hipStreamWaitEvent"); }

    dips_status copy_from(hipStream_t s, void* dst, const LoopGroup::Post& p, const void* src, size_t bytes) {
        dips_status st = wait_for(s, p.ready);
        if (st != DIPS_OK) return st;
        return hipc(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s), "hipMemcpyAsync");
    }

    dips_status broadcast(const void* send, void* recv, size_t bytes, int root, hipStream_t s) override {
        LoopGroup::Post mine;
        mine.send = send;
        mine.recv = recv;
        mine.bytes = bytes;
        return collective(
            mine, s,
            [&](std::vector<LoopGroup::Post>& all) -> dips_status {
                if (all[root].bytes != bytes) return failc(DIPS_ERR_COMM, "loopback broadcast: sizes differ");
                if (rank == root)
                    return send == recv ? DIPS_OK
                                        : hipc(hipMemcpyAsync(recv, send, bytes, hipMemcpyDeviceToDevice, s),
                                               "hipMemcpyAsync");
                return copy_from(s, recv, all[root], all[root].send, bytes);
            },
            [&](std::vector<LoopGroup::Post>& all) -> dips_status {
                if (rank != root) return DIPS_OK;
                for (int r = 0; r < nranks; ++r)
                    if (r != root && wait_for(s, all[r].done) != DIPS_OK) return DIPS_ERR_HIP;
                return DIPS_OK;
            });
    }

    dips_status exchange(const void* send, int to, void* recv, int from, size_t bytes, hipStream_t s) override {
        LoopGroup::Post mine;
        mine.send = send;
        mine.recv = recv;
        mine.bytes = bytes;
        mine.to = to;
        return collective(
            mine, s,
            [&](std::vector<LoopGroup::Post>& all) -> dips_status {
                if (from < 0) return DIPS_OK;
                if (all[from].to != rank || all[from].bytes != bytes)
                    return failc(DIPS_ERR_COMM, "loopback exchange: rank " + std::to_string(from) +
                                                    " does not send " + std::to_string(bytes) + " B to rank " +
                                                    std::to_string(rank));
                return copy_from(s, recv, all[from], all[from].send, bytes);
            },
            [&](std::vector<LoopGroup::Post>& all) -> dips_status {
                return to >= 0 ? wait_for(s, all[to].done) : DIPS_OK;
            });
    }

    dips_status gather(const void* send, void* recv, size_t bytes, int root, hipStream_t s) override {
        LoopGroup::Post mine;
        mine.send = send;
        mine.recv = recv;
        mine.bytes = bytes;
        return collective(
            mine, s,
            [&](std::vector<LoopGroup::Post>& all) -> dips_status {
                if (rank != root) return DIPS_OK;
                uint8_t* dst = static_cast<uint8_t*>(recv);
                for (int r = 0; r < nranks; ++r) {
                    if (all[r].bytes != bytes) return failc(DIPS_ERR_COMM, "loopback gather: sizes differ");
                    uint8_t* at = dst + (size_t)r * bytes;
                    if (r == root) {
                        if (send != at) {
                            dips_status st =
                                hipc(hipMemcpyAsync(at, send, bytes, hipMemcpyDeviceToDevice, s), "hipMemcpyAsync");
                            if (st != DIPS_OK) return st;
                        }
                    } else {
                        dips_status st = copy_from(s, at, all[r], all[r].send, bytes);
                        if (st != DIPS_OK) return st;
                    }
                }
                return DIPS_OK;
            },
            [&](std::vector<LoopGroup::Post>& all) -> dips_status {
                return rank == root ? DIPS_OK : wait_for(s, all[root].done);
            });
    }
};

// -- the caller's transport over host memory --------------------------------
struct HostComm final : dips_comm {
    dips_comm_ops ops{};
    void* ctx = nullptr;
    dips_host::HostPinned a, b;

    ~HostComm() override {
        (void)hipSetDevice(device);
        a.release();
        b.release();
    }

    bool host_synchronous() const override { return true; }

    dips_status callback(int rc, const char* what) {
        return rc == 0 ? DIPS_OK
                       : failc(DIPS_ERR_COMM, std::string("host transport ") + what + " returned " + std::to_string(rc));
    }

    dips_status broadcast(const void* send, void* recv, size_t bytes, int root, hipStream_t s) override {
        COMM_HIP(this, a.ensure(bytes));
        COMM_HIP(this, hipStreamSynchronize(s));
        if (rank == root) {
            COMM_HIP(this, hipMemcpyAsync(a.p, send, bytes, hipMemcpyDeviceToHost, s));
            COMM_HIP(this, hipStreamSynchronize(s));
        }
        dips_status st = callback(ops.broadcast(ctx, a.p, bytes, root), "broadcast");
        if (st != DIPS_OK) return st;
        COMM_HIP(this, hipMemcpyAsync(recv, a.p, bytes, hipMemcpyHostToDevice, s));
        COMM_HIP(this, hipStreamSynchronize(s));
        return DIPS_OK;
    }

    dips_status exchange(const void* send, int to, void* recv, int from, size_t bytes, hipStream_t s) override {
        if (to < 0 && from < 0) return DIPS_OK;
        COMM_HIP(this, a.ensure(bytes));
        COMM_HIP(this, b.ensure(bytes));
        COMM_HIP(this, hipStreamSynchronize(s));
        if (to >= 0) {
            COMM_HIP(this, hipMemcpyAsync(a.p, send, bytes, hipMemcpyDeviceToHost, s));
            COMM_HIP(this, hipStreamSynchronize(s));
        }
        dips_status st = callback(ops.sendrecv(ctx, to >= 0 ? a.p : nullptr, to, from >= 0 ? b.p : nullptr, from, bytes),
                                  "sendrecv");
        if (st != DIPS_OK) return st;
        if (from >= 0) {
            COMM_HIP(this, hipMemcpyAsync(recv, b.p, bytes, hipMemcpyHostToDevice, s));
            COMM_HIP(this, hipStreamSynchronize(s));
        }
        return DIPS_OK;
    }

    dips_status gather(const void* send, void* recv, size_t bytes, int root, hipStream_t s) override {
        COMM_HIP(this, a.ensure(bytes));
        if (rank == root) COMM_HIP(this, b.ensure(bytes * (size_t)nranks));
        COMM_HIP(this, hipStreamSynchronize(s));
        COMM_HIP(this, hipMemcpyAsync(a.p, send, bytes, hipMemcpyDeviceToHost, s));
        COMM_HIP(this, hipStreamSynchronize(s));
        dips_status st = callback(ops.gather(ctx, a.p, rank == root ? b.p : nullptr, bytes, root), "gather");
        if (st != DIPS_OK) return st;
        if (rank == root) {
            COMM_HIP(this, hipMemcpyAsync(recv, b.p, bytes * (size_t)nranks, hipMemcpyHostToDevice, s));
            COMM_HIP(this, hipStreamSynchronize(s));
        }
        return DIPS_OK;
    }
};

// ---------------------------------------------------------------------------
// Helpers of the sharded call
// ---------------------------------------------------------------------------

// Global frames [first, first + count) of `rank` (balanced to within one).
bool shard_range(uint64_t n_total, int nranks, int rank, uint64_t* first, uint64_t* count) {
    if (nranks < 1 || rank < 0 || rank >= nranks) return false;
    const unsigned __int128 n = n_total;
    const uint64_t a = (uint64_t)(n * (unsigned)rank / (unsigned)nranks);
    const uint64_t b = (uint64_t)(n * (unsigned)(rank + 1) / (unsigned)nranks);
    *first = a;
    *count = b - a;
    return true;
}

dips_status device_ok(int device, std::string* why) {
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess || count <= 0 || device < 0 || device >= count) {
        *why = std::string("no HIP device ") + std::to_string(device) + " (" +
               (e == hipSuccess ? std::to_string(count) + " visible" : hipGetErrorString(e)) + ")";
        return DIPS_ERR_NODEVICE;
    }
    return DIPS_OK;
}

// A transport failure, reported on the handle (with the communicator's
// message) and returned.
dips_status comm_fail(dips_handle* h, const dips_comm* c, dips_status st) {
    return fail(h, st, "communicator (rank " + std::to_string(c->rank) + " of " + std::to_string(c->nranks) +
                           "): " + c->err);
}

#define DIPS_COMM(h, c, call)                                   \
    do {                                                        \
        dips_status s_ = (call);                                \
        if (s_ != DIPS_OK) return comm_fail((h), (c), s_);      \
    } while (0)

dips_status ensure_comm_stream(dips_handle* h) {
    if (!h->comm_stream) DIPS_HIP(h, hipStreamCreateWithFlags(&h->comm_stream, hipStreamNonBlocking));
    if (!h->shard_ev_in) DIPS_HIP(h, hipEventCreateWithFlags(&h->shard_ev_in, hipEventDisableTiming));
    if (!h->shard_ev_halo) DIPS_HIP(h, hipEventCreateWithFlags(&h->shard_ev_halo, hipEventDisableTiming));
    return DIPS_OK;
}

// The validation every rank does identically before any collective.
struct ShardArgs {
    uint64_t first = 0, count = 0, max_n = 0;
    size_t fb = 0;
};

dips_status check_shard(dips_handle* h, const dips_comm* comm, uint32_t width, uint32_t height, uint64_t n_total,
                        ShardArgs* a) {
    if (!comm) return fail(h, DIPS_ERR_INVALID, "sharded: null communicator");
    if (comm->device != h->device)
        return fail(h, DIPS_ERR_INVALID, "sharded: the handle is on device " + std::to_string(h->device) +
                                             ", the communicator on device " + std::to_string(comm->device));
    if (width == 0 || height == 0) return fail(h, DIPS_ERR_INVALID, "sharded: empty frame shape");
    if (n_total < (uint64_t)comm->nranks)
        return fail(h, DIPS_ERR_INVALID, "sharded: every rank needs at least one frame (n_total " +
                                             std::to_string(n_total) + " < nranks " + std::to_string(comm->nranks) +
                                             ")");
    shard_range(n_total, comm->nranks, comm->rank, &a->first, &a->count);
    a->max_n = (n_total + (uint64_t)comm->nranks - 1) / (uint64_t)comm->nranks;
    if (a->max_n >= (1ull << 31)) return fail(h, DIPS_ERR_INVALID, "sharded: more than 2^31 frames per rank");
    a->fb = (size_t)width * height * (size_t)h->p.format;
    return DIPS_OK;
}

}  // namespace

namespace dips_abi {

void note_error(dips_comm* c, const char* msg) noexcept {
    if (!c) return;
    try {
        c->err = msg;
    } catch (...) {
    }
}

void note_error(CommCreateTag, const char* msg) noexcept {
    try {
        set_comm_create_err(msg);
    } catch (...) {
    }
}

}  // namespace dips_abi

extern "C" {

dips_status dips_comm_unique_id(uint8_t* id) {
    return guard(dips_abi::CommCreateTag{}, [&]() -> dips_status {
        if (!id) return DIPS_ERR_INVALID;
        ncclUniqueId u;
        const ncclResult_t r = ncclGetUniqueId(&u);
        if (r != ncclSuccess) {
            set_comm_create_err(std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
            return DIPS_ERR_COMM;
        }
        static_assert(sizeof(u) == DIPS_COMM_ID_BYTES, "ncclUniqueId size");
        std::memcpy(id, &u, sizeof(u));
        return DIPS_OK;
    });
}

dips_status dips_comm_create(const uint8_t* id, int nranks, int rank, int device, dips_comm** out) {
    return guard(dips_abi::CommCreateTag{}, [&]() -> dips_status {
        if (!out) return DIPS_ERR_INVALID;
        *out = nullptr;
        if (!id || nranks < 1 || rank < 0 || rank >= nranks) {
            set_comm_create_err("comm_create: null id or rank outside [0, nranks)");
            return DIPS_ERR_INVALID;
        }
        std::string why;
        if (device_ok(device, &why) != DIPS_OK) {
            set_comm_create_err(why);
            return DIPS_ERR_NODEVICE;
        }
        hipError_t e = hipSetDevice(device);
        if (e != hipSuccess) {
            set_comm_create_err(std::string("hipSetDevice: ") + hipGetErrorString(e));
            return DIPS_ERR_HIP;
        }
        std::unique_ptr<RcclComm> c(new RcclComm());
        c->kind = DIPS_COMM_RCCL;
        c->nranks = nranks;
        c->rank = rank;
        c->device = device;
        ncclUniqueId u;
        std::memcpy(&u, id, sizeof(u));
        const ncclResult_t r = ncclCommInitRank(&c->c, nranks, u, rank);
        if (r != ncclSuccess) {
            const char* last = ncclGetLastError(nullptr);
            set_comm_create_err(std::string("ncclCommInitRank: ") + ncclGetErrorString(r) +
                                (last && *last ? std::string(" (") + last + ")" : std::string()));
            c->c = nullptr;
            return DIPS_ERR_COMM;
        }
        *out = c.release();
        return DIPS_OK;
    });
}

dips_status dips_comm_create_all(int nranks, const int* devices, dips_comm** comms) {
    return guard(dips_abi::CommCreateTag{}, [&]() -> dips_status {
        if (!comms || nranks < 1 || nranks > 1024) {
            set_comm_create_err("comm_create_all: null output or nranks outside [1, 1024]");
            return DIPS_ERR_INVALID;
        }
        for (int r = 0; r < nranks; ++r) comms[r] = nullptr;
        std::vector<int> devs(nranks);
        for (int r = 0; r < nranks; ++r) {
            devs[r] = devices ? devices[r] : r;
            std::string why;
            if (device_ok(devs[r], &why) != DIPS_OK) {
                set_comm_create_err(why);
                return DIPS_ERR_NODEVICE;
            }
        }
        std::vector<ncclComm_t> raw(nranks, nullptr);
        const ncclResult_t res = ncclCommInitAll(raw.data(), nranks, devs.data());
        if (res != ncclSuccess) {
            const char* last = ncclGetLastError(nullptr);
            set_comm_create_err(std::string("ncclCommInitAll: ") + ncclGetErrorString(res) +
                                (last && *last ? std::string(" (") + last + ")" : std::string()));
            return DIPS_ERR_COMM;
        }
        std::vector<std::unique_ptr<RcclComm>> made;
        for (int r = 0; r < nranks; ++r) {
            std::unique_ptr<RcclComm> c(new RcclComm());
            c->kind = DIPS_COMM_RCCL;
            c->nranks = nranks;
            c->rank = r;
            c->device = devs[r];
            c->c = raw[r];
            made.push_back(std::move(c));
        }
        for (int r = 0; r < nranks; ++r) comms[r] = made[r].release();
        return DIPS_OK;
    });
}

dips_status dips_comm_create_loopback(int nranks, int device, dips_comm** comms) {
    return guard(dips_abi::CommCreateTag{}, [&]() -> dips_status {
        if (!comms || nranks < 1 || nranks > 1024) {
            set_comm_create_err("comm_create_loopback: null output or nranks outside [1, 1024]");
            return DIPS_ERR_INVALID;
        }
        for (int r = 0; r < nranks; ++r) comms[r] = nullptr;
        std::string why;
        if (device_ok(device, &why) != DIPS_OK) {
            set_comm_create_err(why);
            return DIPS_ERR_NODEVICE;
        }
        hipError_t e = hipSetDevice(device);
        auto g = std::make_shared<LoopGroup>();
        g->n = nranks;
        g->posts[0].resize(nranks);
        g->posts[1].resize(nranks);
        std::vector<std::unique_ptr<LoopComm>> made;
        for (int r = 0; r < nranks && e == hipSuccess; ++r) {
            std::unique_ptr<LoopComm> c(new LoopComm());
            c->kind = DIPS_COMM_LOOPBACK;
            c->nranks = nranks;
            c->rank = r;
            c->device = device;
            c->g = g;
            for (int i = 0; i < 2 && e == hipSuccess; ++i) {
                e = hipEventCreateWithFlags(&c->ready[i], hipEventDisableTiming);
                if (e == hipSuccess) e = hipEventCreateWithFlags(&c->done[i], hipEventDisableTiming);
            }
            made.push_back(std::move(c));
        }
        if (e != hipSuccess) {
            set_comm_create_err(std::string("comm_create_loopback: ") + hipGetErrorString(e));
            return DIPS_ERR_HIP;
        }
        for (int r = 0; r < nranks; ++r) comms[r] = made[r].release();
        return DIPS_OK;
    });
}

dips_status dips_comm_create_host(const dips_comm_ops* ops, void* ctx, int nranks, int rank, int device,
                                  dips_comm** out) {
    return guard(dips_abi::CommCreateTag{}, [&]() -> dips_status {
        if (!out) return DIPS_ERR_INVALID;
        *out = nullptr;
        if (!ops || !ops->broadcast || !ops->sendrecv || !ops->gather || nranks < 1 || rank < 0 ||
            rank >= nranks) {
            set_comm_create_err("comm_create_host: every callback is required and rank must lie in [0, nranks)");
            return DIPS_ERR_INVALID;
        }
        std::string why;
        if (device_ok(device, &why) != DIPS_OK) {
            set_comm_create_err(why);
            return DIPS_ERR_NODEVICE;
        }
        std::unique_ptr<HostComm> c(new HostComm());
        c->kind = DIPS_COMM_HOST;
        c->nranks = nranks;
        c->rank = rank;
        c->device = device;
        c->ops = *ops;
        c->ctx = ctx;
        *out = c.release();
        return DIPS_OK;
    });
}

void dips_comm_destroy(dips_comm* comm) {
    guard(comm, [&]() -> void { delete comm; });
}

const char* dips_comm_last_error(const dips_comm* comm) {
    return guard(comm, [&]() -> const char* {
        if (comm) return comm->err.c_str();
        // this thread's copy (see dips_last_error)
        thread_local std::string copy;
        std::lock_guard<std::mutex> lk(g_comm_err_mu);
        copy = g_comm_create_err;
        return copy.c_str();
    });
}

dips_status dips_comm_info(const dips_comm* comm, int* kind, int* nranks, int* rank) {
    return guard(comm, [&]() -> dips_status {
        if (!comm) return DIPS_ERR_INVALID;
        if (kind) *kind = comm->kind;
        if (nranks) *nranks = comm->nranks;
        if (rank) *rank = comm->rank;
        return DIPS_OK;
    });
}

dips_status dips_shard_range(uint64_t n_total, int nranks, int rank, uint64_t* first, uint32_t* count) {
    return guard(nullptr, [&]() -> dips_status {
        uint64_t a = 0, n = 0;
        if (!shard_range(n_total, nranks, rank, &a, &n) || n >= (1ull << 32)) return DIPS_ERR_INVALID;
        if (first) *first = a;
        if (count) *count = (uint32_t)n;
        return DIPS_OK;
    });
}

dips_status dips_shard_broadcast(dips_handle* h, dips_comm* comm, uint32_t width, uint32_t height,
                                 const uint8_t* frame, uint8_t* out) {
    return guard(h, [&]() -> dips_status {
        dips_status st = bind(h);
        if (st != DIPS_OK) return st;
        if (!comm) return fail(h, DIPS_ERR_INVALID, "shard_broadcast: null communicator");
        if (comm->device != h->device) return fail(h, DIPS_ERR_INVALID, "shard_broadcast: device mismatch");
        if (!out || width == 0 || height == 0 || (comm->rank == 0 && !frame))
            return fail(h, DIPS_ERR_INVALID, "shard_broadcast: null or empty argument");
        const size_t fb = (size_t)width * height * (size_t)h->p.format;
        hipStream_t s = h->stream;
        if (h->p.flags & DIPS_FLAG_DEVICE_PTRS) {
            DIPS_COMM(h, comm, comm->broadcast(frame, out, fb, 0, s));
            return DIPS_OK;
        }
        DIPS_HIP(h, h->shard_ref.ensure(fb));
        if (comm->rank == 0) DIPS_HIP(h, hipMemcpyAsync(h->shard_ref.p, frame, fb, hipMemcpyHostToDevice, s));
        DIPS_COMM(h, comm, comm->broadcast(h->shard_ref.p, h->shard_ref.p, fb, 0, s));
        DIPS_HIP(h, hipMemcpyAsync(out, h->shard_ref.p, fb, hipMemcpyDeviceToHost, s));
        DIPS_HIP(h, hipStreamSynchronize(s));
        return DIPS_OK;
    });
}

dips_status dips_diff_series_sharded(dips_handle* h, dips_comm* comm, uint32_t width, uint32_t height,
                                     const uint8_t* frames, uint32_t n_local, uint64_t n_total, const uint8_t* ref,
                                     uint32_t shard_flags, dips_series_entry* series_local,
                                     dips_series_entry* series_all) {
    return guard(h, [&]() -> dips_status {
        dips_status st = bind(h);
        if (st != DIPS_OK) return st;
        ShardArgs a;
        st = check_shard(h, comm, width, height, n_total, &a);
        if (st != DIPS_OK) return st;
        const int G = comm->nranks, r = comm->rank;
        const bool pf = h->p.mode == DIPS_MODE_PER_FRAME;
        const bool resident = (shard_flags & DIPS_SHARD_REF_RESIDENT) != 0;
        if (shard_flags & ~DIPS_SHARD_REF_RESIDENT) return fail(h, DIPS_ERR_INVALID, "sharded: unknown shard_flags");
        if ((uint64_t)n_local != a.count)
            return fail(h, DIPS_ERR_INVALID, "sharded: rank " + std::to_string(r) + " owns " + std::to_string(a.count) +
                                                 " frames [" + std::to_string(a.first) + ", " +
                                                 std::to_string(a.first + a.count) + ") of " + std::to_string(n_total) +
                                                 ", n_local is " + std::to_string(n_local));
        if (!frames || !series_local || (r == 0 && !series_all))
            return fail(h, DIPS_ERR_INVALID, "sharded: null frames or series (series_all is required on rank 0)");
        if (!pf && resident && !ref)
            return fail(h, DIPS_ERR_INVALID, "sharded: DIPS_SHARD_REF_RESIDENT needs every rank's reference");
        const size_t fb = a.fb, eb = sizeof(dips_series_entry);
        const uint32_t n = n_local;
        const bool dev = (h->p.flags & DIPS_FLAG_DEVICE_PTRS) != 0;
        hipStream_t s = h->stream;

        // device views of the reference and the outputs (host pointers: the
        // series in HBM until the end, the frames through the streamed feed)
        const uint8_t* fr = frames;
        const uint8_t* rf = ref;
        dips_series_entry* sl = series_local;
        dips_series_entry* sa = series_all;
        if (!dev) {
            if (ref && (resident || r == 0)) {
                DIPS_HIP(h, h->stage_ref.ensure(fb));
                DIPS_HIP(h, hipMemcpyAsync(h->stage_ref.p, ref, fb, hipMemcpyHostToDevice, s));
                rf = h->stage_ref.as<uint8_t>();
            } else {
                rf = nullptr;
            }
            DIPS_HIP(h, h->stage_series.ensure(eb * ((size_t)n + (r == 0 ? (size_t)n_total : 0u))));
            sl = h->stage_series.as<dips_series_entry>();
            sa = r == 0 ? sl + n : nullptr;
        }

        if (!dev) {
            // 1h. host frames: the reference / halo exchange first, then the
            // rank's frames through the pinned side-stream feed
            // (run_series_streamed: PCIe-bound, ~55 GB/s per GPU, no batch-sized
            // HBM staging)
            const uint8_t* r0 = nullptr;
            if (!pf) {
                if (resident) {
                    r0 = rf;
                } else {
                    DIPS_HIP(h, h->shard_ref.ensure(fb));
                    if (r == 0)
                        DIPS_HIP(h, hipMemcpyAsync(h->shard_ref.p, rf ? rf : frames, fb,
                                                   rf ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, s));
                    DIPS_COMM(h, comm, comm->broadcast(h->shard_ref.p, h->shard_ref.p, fb, 0, s));
                    r0 = h->shard_ref.as<uint8_t>();
                }
            } else {
                const bool halo_in = r > 0, send_out = r + 1 < G;
                if (G > 1) {
                    st = ensure_comm_stream(h);
                    if (st != DIPS_OK) return st;
                    if (send_out) {
                        DIPS_HIP(h, h->shard_send_frame.ensure(fb));
                        DIPS_HIP(h, hipMemcpyAsync(h->shard_send_frame.p, frames + (size_t)(n - 1) * fb, fb,
                                                   hipMemcpyHostToDevice, s));
                    }
                    if (halo_in) DIPS_HIP(h, h->shard_halo.ensure(fb));
                    DIPS_HIP(h, hipEventRecord(h->shard_ev_in, s));
                    DIPS_HIP(h, hipStreamWaitEvent(h->comm_stream, h->shard_ev_in, 0));
                    DIPS_COMM(h, comm, comm->exchange(send_out ? h->shard_send_frame.p : nullptr, send_out ? r + 1 : -1,
                                                      halo_in ? h->shard_halo.p : nullptr, halo_in ? r - 1 : -1, fb,
                                                      h->comm_stream));
                    DIPS_HIP(h, hipEventRecord(h->shard_ev_halo, h->comm_stream));
                    DIPS_HIP(h, hipStreamWaitEvent(s, h->shard_ev_halo, 0));
                }
                if (halo_in) {
                    r0 = h->shard_halo.as<uint8_t>();
                } else if (rf) {
                    r0 = rf;
                } else {  // frame 0 against itself; staged so that dips_shard_reference can return it
                    DIPS_HIP(h, h->stage_ref.ensure(fb));
                    DIPS_HIP(h, hipMemcpyAsync(h->stage_ref.p, frames, fb, hipMemcpyHostToDevice, s));
                    r0 = h->stage_ref.as<uint8_t>();
                }
            }
            st = run_series_streamed(h, width, height, frames, n, r0, sl, 0);
            if (st != DIPS_OK) return st;
            h->shard_last_ref = r0;
            h->shard_last_bytes = fb;
        } else {
            // 1d. device frames
            const uint8_t* r0 = nullptr;  // the reference of the rank's first frame
            if (!pf) {
                if (resident) {
                    r0 = rf;
                } else {
                    DIPS_HIP(h, h->shard_ref.ensure(fb));
                    const uint8_t* src = r == 0 ? (rf ? rf : fr) : nullptr;
                    DIPS_COMM(h, comm, comm->broadcast(src, h->shard_ref.p, fb, 0, s));
                    r0 = h->shard_ref.as<uint8_t>();
                }
                st = run_series_device(h, width, height, fr, n, r0, sl, nullptr, s);
                if (st != DIPS_OK) return st;
            } else {
                // 'per-frame': the halo (global frame first-1) from rank r-1 and
                // this rank's last frame to rank r+1, on the side stream, beside
                // the launch that needs no halo -- every frame on rank 0, frames
                // 1..n-1 (each against its predecessor) elsewhere; then frame 0
                // against the halo once it has landed
                const bool halo_in = r > 0, send_out = r + 1 < G;
                const bool sync = G > 1 && comm->host_synchronous();
                uint8_t* halo = nullptr;
                if (G > 1) {
                    st = ensure_comm_stream(h);
                    if (st != DIPS_OK) return st;
                    // the frames are ready once the work issued before this call is
                    DIPS_HIP(h, hipEventRecord(h->shard_ev_in, s));
                    DIPS_HIP(h, hipStreamWaitEvent(h->comm_stream, h->shard_ev_in, 0));
                }
                if (halo_in) {
                    DIPS_HIP(h, h->shard_halo.ensure(fb));
                    halo = h->shard_halo.as<uint8_t>();
                }
                auto post = [&]() -> dips_status {
                    DIPS_COMM(h, comm, comm->exchange(fr + (size_t)(n - 1) * fb, send_out ? r + 1 : -1, halo,
                                                      halo_in ? r - 1 : -1, fb, h->comm_stream));
                    DIPS_HIP(h, hipEventRecord(h->shard_ev_halo, h->comm_stream));
                    return DIPS_OK;
                };
                if (G > 1 && !sync) {  // stream-ordered: its kernels start first
                    st = post();
                    if (st != DIPS_OK) return st;
                }
                const uint32_t n_main = halo_in ? n - 1 : n;
                if (n_main > 0) {
                    st = run_series_device(h, width, height, halo_in ? fr + fb : fr, n_main, halo_in ? fr : (rf ? rf : fr),
                                           halo_in ? sl + 1 : sl, nullptr, s);
                    if (st != DIPS_OK) return st;
                }
                if (sync) {  // completes on this thread while the launch runs
                    st = post();
                    if (st != DIPS_OK) return st;
                }
                // the halo has landed, and the frame sent may change again
                if (G > 1) DIPS_HIP(h, hipStreamWaitEvent(s, h->shard_ev_halo, 0));
                if (halo_in) {
                    st = run_series_device(h, width, height, fr, 1, halo, sl, nullptr, s);
                    if (st != DIPS_OK) return st;
                    r0 = halo;
                } else {
                    r0 = rf ? rf : fr;
                }
            }
            h->shard_last_ref = r0;
            h->shard_last_bytes = fb;
        }

        // 2. one gather of the series onto rank 0 (padded to the largest
        // shard; trimmed into place unless every shard has max_n frames)
        if (G == 1) {
            if (sa != sl) DIPS_HIP(h, hipMemcpyAsync(sa, sl, eb * n, hipMemcpyDeviceToDevice, s));
        } else {
            const size_t seg = eb * (size_t)a.max_n;
            const void* send = sl;
            if ((uint64_t)n < a.max_n) {
                DIPS_HIP(h, h->shard_send.ensure(seg));
                DIPS_HIP(h, hipMemsetAsync(h->shard_send.p, 0, seg, s));
                DIPS_HIP(h, hipMemcpyAsync(h->shard_send.p, sl, eb * n, hipMemcpyDeviceToDevice, s));
                send = h->shard_send.p;
            }
            const bool direct = n_total == (uint64_t)G * a.max_n;
            void* recv = nullptr;
            if (r == 0) {
                if (direct) {
                    recv = sa;
                } else {
                    DIPS_HIP(h, h->shard_recv.ensure(seg * (size_t)G));
                    recv = h->shard_recv.p;
                }
            }
            DIPS_COMM(h, comm, comm->gather(send, recv, seg, 0, s));
            if (r == 0 && !direct) {
                for (int k = 0; k < G; ++k) {
                    uint64_t f = 0, c = 0;
                    shard_range(n_total, G, k, &f, &c);
                    DIPS_HIP(h, hipMemcpyAsync(sa + f, static_cast<uint8_t*>(recv) + seg * (size_t)k, eb * c,
                                               hipMemcpyDeviceToDevice, s));
                }
            }
        }
        if (!dev) {
            DIPS_HIP(h, hipMemcpyAsync(series_local, sl, eb * n, hipMemcpyDeviceToHost, s));
            if (r == 0) DIPS_HIP(h, hipMemcpyAsync(series_all, sa, eb * n_total, hipMemcpyDeviceToHost, s));
            DIPS_HIP(h, hipStreamSynchronize(s));
        }
        return DIPS_OK;
    });
}

dips_status dips_frame_callback_batch_sharded(dips_handle* h, dips_comm* comm, uint32_t width, uint32_t height,
                                              const uint8_t* frames, uint32_t n_local, uint64_t n_total,
                                              uint8_t* out) {
    return guard(h, [&]() -> dips_status {
        dips_status st = bind(h);
        if (st != DIPS_OK) return st;
        if (!comm) return fail(h, DIPS_ERR_INVALID, "compat sharded: null communicator");
        if (comm->device != h->device) return fail(h, DIPS_ERR_INVALID, "compat sharded: device mismatch");
        if (width == 0 || height == 0) return fail(h, DIPS_ERR_INVALID, "compat sharded: empty frame shape");
        const int G = comm->nranks, r = comm->rank;
        // the layout rule, checked for every rank on every rank (the same
        // answer everywhere: no rank is left in a collective)
        for (int k = 0; k < G; ++k) {
            uint64_t f = 0, c = 0;
            shard_range(n_total, G, k, &f, &c);
            if (k > 0 && f < 7)
                return fail(h, DIPS_ERR_INVALID, "compat sharded: rank " + std::to_string(k) + " would start at frame " +
                                                     std::to_string(f) + " (< 7; n_total >= 7 * nranks suffices)");
            if (k + 1 < G && c < 3) return fail(h, DIPS_ERR_INVALID, "compat sharded: every rank but the last needs >= 3 frames");
        }
        uint64_t first = 0, count = 0;
        shard_range(n_total, G, r, &first, &count);
        if ((uint64_t)n_local != count)
            return fail(h, DIPS_ERR_INVALID, "compat sharded: rank " + std::to_string(r) + " owns " +
                                                 std::to_string(count) + " frames, n_local is " + std::to_string(n_local));
        if (n_local == 0) return DIPS_OK;
        if (!frames || !out) return fail(h, DIPS_ERR_INVALID, "compat sharded: null frames or output");
        if (h->added != 0 || h->main_init)
            return fail(h, DIPS_ERR_STATE, "compat sharded: the handle must be fresh (no frame added yet)");
        if (G == 1) return dips_frame_callback_batch(h, width, height, frames, n_local, out);
        const size_t fb = (size_t)width * height * 4u;
        const uint32_t n = n_local;
        const bool dev = (h->p.flags & DIPS_FLAG_DEVICE_PTRS) != 0;
        const bool halo_in = r > 0, send_out = r + 1 < G;
        hipStream_t s = h->stream;
        st = ensure_comm_stream(h);
        if (st != DIPS_OK) return st;

        // 1. the 3-frame halo: this rank's last three frames to r+1, r-1's
        // into shard_halo, on the side stream
        const uint8_t* send3 = nullptr;
        if (send_out) {
            send3 = frames + (size_t)(n - 3) * fb;
            if (!dev) {
                DIPS_HIP(h, h->shard_send_frame.ensure(3 * fb));
                DIPS_HIP(h, hipMemcpyAsync(h->shard_send_frame.p, send3, 3 * fb, hipMemcpyHostToDevice, s));
                send3 = h->shard_send_frame.as<uint8_t>();
            }
        }
        if (halo_in) DIPS_HIP(h, h->shard_halo.ensure(3 * fb));
        DIPS_HIP(h, hipEventRecord(h->shard_ev_in, s));
        DIPS_HIP(h, hipStreamWaitEvent(h->comm_stream, h->shard_ev_in, 0));
        DIPS_COMM(h, comm, comm->exchange(send3, send_out ? r + 1 : -1, halo_in ? h->shard_halo.p : nullptr,
                                          halo_in ? r - 1 : -1, 3 * fb, h->comm_stream));
        DIPS_HIP(h, hipEventRecord(h->shard_ev_halo, h->comm_stream));
        // the communicator's next operation (the broadcast) after this one on
        // every rank, and the sent frames unchanged until it is done
        DIPS_HIP(h, hipStreamWaitEvent(s, h->shard_ev_halo, 0));

        // 2. the start texture from rank 0, which builds it on frames 0..3
        if (r == 0) {
            st = dips_frame_callback_batch(h, width, height, frames, n < 4 ? n : 4u, out);
            if (st != DIPS_OK) return st;
        } else {
            DIPS_HIP(h, h->shard_ref.ensure(fb));
        }
        DIPS_HIP(h, h->start.ensure(fb));
        DIPS_COMM(h, comm, comm->broadcast(r == 0 ? h->start.p : nullptr, r == 0 ? h->start.p : h->shard_ref.p, fb, 0, s));

        // 3. the rank's frames: rank 0 goes on from frame 4, the others
        // resume at their first frame from S and the halo
        if (r == 0) {
            if (n > 4) return dips_frame_callback_batch(h, width, height, frames + 4 * fb, n - 4, out + 4 * fb);
            return DIPS_OK;
        }
        st = compat_resume_impl(h, width, height, h->shard_ref.as<uint8_t>(), h->shard_halo.as<uint8_t>(), first, true);
        if (st != DIPS_OK) return st;
        return dips_frame_callback_batch(h, width, height, frames, n, out);
    });
}

dips_status dips_shard_plan(dips_handle* h, const dips_comm* comm, uint32_t width, uint32_t height,
                            uint64_t n_total, uint64_t* first, uint32_t* count, uint64_t* waves,
                            uint64_t* waves_uncapped) {
    return guard(h, [&]() -> dips_status {
        dips_status st = bind(h);
        if (st != DIPS_OK) return st;
        ShardArgs a;
        st = check_shard(h, comm, width, height, n_total, &a);
        if (st != DIPS_OK) return st;
        // the launch the halo transfer overlaps ('per-frame'): frames 1..n-1
        // on ranks > 0, all frames on rank 0
        const bool pf = h->p.mode == DIPS_MODE_PER_FRAME;
        const uint32_t n_main = (uint32_t)(pf && comm->rank > 0 ? a.count - 1 : a.count);
        if (first) *first = a.first;
        if (count) *count = (uint32_t)a.count;
        if (waves) *waves = n_main ? series_waves(h, width, height, n_main, true) : 0;
        if (waves_uncapped) *waves_uncapped = n_main ? series_waves(h, width, height, n_main, false) : 0;
        return DIPS_OK;
    });
}

int dips_shard_reference(dips_handle* h, uint8_t* out, size_t cap) {
    return guard(h, [&]() -> int {
        dips_status st = bind(h);
        if (st != DIPS_OK) return st;
        if (!h->shard_last_ref) return 0;
        if (!out) return fail(h, DIPS_ERR_INVALID, "shard_reference: null output");
        if (cap < h->shard_last_bytes) return fail(h, DIPS_ERR_CAPACITY, "shard_reference: output too small");
        if (h->p.flags & DIPS_FLAG_DEVICE_PTRS) {
            DIPS_HIP(h, hipMemcpyAsync(out, h->shard_last_ref, h->shard_last_bytes, hipMemcpyDeviceToDevice,
                                       h->stream));
        } else {
            DIPS_HIP(h, hipMemcpyAsync(out, h->shard_last_ref, h->shard_last_bytes, hipMemcpyDeviceToHost,
                                       h->stream));
            DIPS_HIP(h, hipStreamSynchronize(h->stream));
        }
        return 1;
    });
}

}  // extern "C"
