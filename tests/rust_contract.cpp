// rust_contract.cpp -- the call sequences of rust/dips-hip/src/lib.rs executed
// through the C ABI (there is no cargo in this image, so the crate itself
// cannot be built).  Each method below restates one crate method: the same
// FFI calls in the same order, the same argument checks before the call and
// the same status handling after it (`check` -> Err(DipsError), the
// panicking reference-shaped forms -> a thrown Panic).  tests/test_rust_shim.py
// maps every crate method to its row here; tests/test_rust_contract.py runs the
// scenarios (CPU: the no-device rows; GPU: all) and reads one line per row:
//   ROW <name> ok          or   ROW <name> FAIL <why>
// Reference surface: dips/src/gpu/mod.rs:59-65, :170-216, :306-397 and
// dips/src/lib.rs:23, :233-246.
#include <array>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <optional>
#include <string>
#include <thread>
#include <vector>

#include "dips_hip.h"

namespace {

struct DipsError {
    int status = 0;
    std::string message;
};

template <typename T>
struct Result {
    bool ok = false;
    T value{};
    DipsError err;
    static Result Ok(T v) {
        Result r;
        r.ok = true;
        r.value = std::move(v);
        return r;
    }
    static Result Err(DipsError e) {
        Result r;
        r.err = std::move(e);
        return r;
    }
};

struct Panic {
    std::string what;
};

std::string message(const char* p) { return p ? std::string(p) : std::string(); }

// lib.rs `check`: st >= 0 -> Ok(st); else Err with dips_last_error(h)
Result<int> check(int st, const dips_handle* h) {
    if (st >= 0) return Result<int>::Ok(st);
    return Result<int>::Err({st, message(dips_last_error(h))});
}

Result<int> check_alt(int st, const dips_alt_handle* h) {
    if (st >= 0) return Result<int>::Ok(st);
    return Result<int>::Err({st, message(dips_alt_last_error(h))});
}

Result<int> check_comm(int st, const dips_comm* c) {
    if (st >= 0) return Result<int>::Ok(st);
    return Result<int>::Err({st, message(dips_comm_last_error(c))});
}

// lib.rs `check_abi`
Result<int> check_abi() {
    const int v = dips_abi_version();
    if (v == DIPS_ABI_VERSION) return Result<int>::Ok(0);
    return Result<int>::Err({DIPS_ERR_STATE, "libdips_hip.so has ABI " + std::to_string(v)});
}

// lib.rs `create`
Result<dips_handle*> create(const dips_params& p, int device) {
    auto a = check_abi();
    if (!a.ok) return Result<dips_handle*>::Err(a.err);
    dips_handle* h = nullptr;
    auto c = check(dips_create(&p, device, &h), nullptr);
    if (!c.ok) return Result<dips_handle*>::Err(c.err);
    if (!h) return Result<dips_handle*>::Err({DIPS_ERR_STATE, "null handle"});
    return Result<dips_handle*>::Ok(h);
}

dips_params default_params() {
    dips_params p;
    dips_params_default(&p);
    return p;
}

// lib.rs `ComputeState`
struct ComputeState {
    dips_handle* h = nullptr;
    uint32_t width = 0, height = 0;

    static Result<ComputeState*> on_device(bool colorize, int32_t window, float sensitivity, uint32_t filter,
                                           uint32_t chroma, int device) {
        dips_params p = default_params();
        p.colorize = colorize ? 1 : 0;
        p.spatial_window_size = window;
        p.sensitivity = sensitivity;
        p.filter_type = filter;
        p.chroma_filter = chroma;
        p.format = DIPS_FMT_RGBA8;
        auto h = create(p, device);
        if (!h.ok) return Result<ComputeState*>::Err(h.err);
        auto* cs = new ComputeState();
        cs->h = h.value;
        return Result<ComputeState*>::Ok(cs);
    }
    ~ComputeState() { dips_destroy(h); }
    size_t frame_bytes() const { return (size_t)width * height * 4; }

    Result<int> try_add_texture(uint32_t w, uint32_t hh, const std::vector<uint8_t>& frame) {
        auto r = check(dips_add_texture(h, w, hh, frame.data(), frame.size()), h);
        if (!r.ok) return r;
        width = w;
        height = hh;
        return Result<int>::Ok(0);
    }
    void add_texture(uint32_t w, uint32_t hh, const std::vector<uint8_t>& frame) { (void)try_add_texture(w, hh, frame); }

    Result<std::optional<std::vector<uint8_t>>> try_dispatch() {
        using R = Result<std::optional<std::vector<uint8_t>>>;
        std::vector<uint8_t> out(frame_bytes());
        const int r = dips_dispatch(h, out.data(), out.size());
        auto c = check(r, h);
        if (!c.ok) return R::Err(c.err);
        if (c.value == 1) return R::Ok(std::optional<std::vector<uint8_t>>(std::move(out)));
        return R::Ok(std::nullopt);
    }
    std::optional<std::vector<uint8_t>> dispatch() {
        auto r = try_dispatch();
        if (!r.ok) throw Panic{"ComputeState::dispatch: " + r.err.message};
        return r.value;
    }

    Result<bool> frame_callback_into(uint32_t w, uint32_t hh, const std::vector<uint8_t>& frame,
                                     std::vector<uint8_t>& out) {
        const int r = dips_frame_callback(h, w, hh, frame.data(), frame.size(), out.data(), out.size());
        auto c = check(r, h);
        if (!c.ok) return Result<bool>::Err(c.err);
        width = w;
        height = hh;
        return Result<bool>::Ok(c.value == 1);
    }

    Result<int> frame_callback_batch(uint32_t w, uint32_t hh, const std::vector<uint8_t>& frames,
                                     std::vector<uint8_t>& out) {
        const size_t fb = (size_t)w * hh * 4;
        if (fb == 0 || frames.size() % fb != 0 || out.size() < frames.size())
            return Result<int>::Err({DIPS_ERR_INVALID, "frames/out not n RGBA8 frames"});
        auto c = check(dips_frame_callback_batch(h, w, hh, frames.data(), (uint32_t)(frames.size() / fb), out.data()),
                       h);
        if (!c.ok) return c;
        width = w;
        height = hh;
        return Result<int>::Ok(0);
    }

    Result<int> frame_callback_batch_sharded(struct Comm& comm, uint32_t w, uint32_t hh,
                                             const std::vector<uint8_t>& frames, uint64_t n_total,
                                             std::vector<uint8_t>& out);

    std::optional<std::vector<double>> callback_phases() const {
        std::vector<double> v(DIPS_CALLBACK_PHASES);
        uint32_t n = 0;
        const int st = dips_callback_phases(h, v.data(), (uint32_t)v.size(), &n);
        if (st == DIPS_OK) return v;
        return std::nullopt;
    }

    Result<int> resume(uint32_t w, uint32_t hh, const std::vector<uint8_t>& start, const std::vector<uint8_t>& halo,
                       uint64_t t0) {
        const size_t fb = (size_t)w * hh * 4;
        if (start.size() != fb || halo.size() != 3 * fb)
            return Result<int>::Err({DIPS_ERR_INVALID, "start: 1 frame, halo: 3 frames"});
        auto c = check(dips_compat_resume(h, w, hh, start.data(), halo.data(), t0), h);
        if (!c.ok) return c;
        width = w;
        height = hh;
        return Result<int>::Ok(0);
    }

    Result<std::optional<std::vector<uint8_t>>> try_start_texture() {
        using R = Result<std::optional<std::vector<uint8_t>>>;
        std::vector<uint8_t> out(frame_bytes());
        auto c = check(dips_start_texture(h, out.data(), out.size()), h);
        if (!c.ok) return R::Err(c.err);
        if (c.value == 1) return R::Ok(std::optional<std::vector<uint8_t>>(std::move(out)));
        return R::Ok(std::nullopt);
    }
};

// lib.rs `ComputeState::start_texture`: try_start_texture, panicking on an error
std::optional<std::vector<uint8_t>> start_texture(ComputeState& cs) {
    auto r = cs.try_start_texture();
    if (!r.ok) throw Panic{"ComputeState::start_texture: " + r.err.message};
    return r.value;
}

// lib.rs `frame_callback` (dips/src/lib.rs:233-246): panics on an error
std::vector<uint8_t> frame_callback(uint32_t w, uint32_t hh, const std::vector<uint8_t>& frame, ComputeState& cs) {
    std::vector<uint8_t> out(frame.size());
    auto r = cs.frame_callback_into(w, hh, frame, out);
    if (!r.ok) throw Panic{"frame_callback: " + r.err.message};
    return out;
}

// lib.rs `Comm`
struct Comm {
    dips_comm* c = nullptr;
    int nranks = 0, rank = 0;
    ~Comm() { dips_comm_destroy(c); }
    static Result<std::array<uint8_t, DIPS_COMM_ID_BYTES>> unique_id() {
        using R = Result<std::array<uint8_t, DIPS_COMM_ID_BYTES>>;
        auto a = check_abi();
        if (!a.ok) return R::Err(a.err);
        std::array<uint8_t, DIPS_COMM_ID_BYTES> id{};
        auto c = check_comm(dips_comm_unique_id(id.data()), nullptr);
        if (!c.ok) return R::Err(c.err);
        return R::Ok(id);
    }
    static Result<Comm*> rccl(const std::array<uint8_t, DIPS_COMM_ID_BYTES>& id, int nranks, int rank, int device) {
        auto a = check_abi();
        if (!a.ok) return Result<Comm*>::Err(a.err);
        dips_comm* c = nullptr;
        auto r = check_comm(dips_comm_create(id.data(), nranks, rank, device, &c), nullptr);
        if (!r.ok) return Result<Comm*>::Err(r.err);
        auto* w = new Comm();
        w->c = c;
        int kind = 0;
        auto i = check_comm(dips_comm_info(c, &kind, &w->nranks, &w->rank), c);
        if (!i.ok) {
            delete w;
            return Result<Comm*>::Err(i.err);
        }
        return Result<Comm*>::Ok(w);
    }
    static Result<std::vector<Comm*>> rccl_all(const std::vector<int>& devices) {
        using R = Result<std::vector<Comm*>>;
        auto a = check_abi();
        if (!a.ok) return R::Err(a.err);
        std::vector<dips_comm*> cs(devices.size(), nullptr);
        auto r = check_comm(dips_comm_create_all((int)devices.size(), devices.data(), cs.data()), nullptr);
        if (!r.ok) return R::Err(r.err);
        std::vector<Comm*> out;
        for (auto* c : cs) {
            auto* w = new Comm();
            w->c = c;
            int kind = 0;
            auto i = check_comm(dips_comm_info(c, &kind, &w->nranks, &w->rank), c);
            if (!i.ok) return R::Err(i.err);
            out.push_back(w);
        }
        return R::Ok(out);
    }
    static Result<std::vector<Comm*>> loopback(int nranks, int device) {
        using R = Result<std::vector<Comm*>>;
        auto a = check_abi();
        if (!a.ok) return R::Err(a.err);
        if (nranks < 0) return R::Err({DIPS_ERR_INVALID, "nranks < 0"});
        std::vector<dips_comm*> cs(nranks, nullptr);
        auto r = check_comm(dips_comm_create_loopback(nranks, device, cs.data()), nullptr);
        if (!r.ok) return R::Err(r.err);
        std::vector<Comm*> out;
        for (auto* c : cs) {
            auto* w = new Comm();
            w->c = c;
            int kind = 0;
            auto i = check_comm(dips_comm_info(c, &kind, &w->nranks, &w->rank), c);
            if (!i.ok) return R::Err(i.err);
            out.push_back(w);
        }
        return R::Ok(out);
    }
};

// lib.rs `ComputeState::frame_callback_batch_sharded`
Result<int> ComputeState::frame_callback_batch_sharded(Comm& comm, uint32_t w, uint32_t hh,
                                                       const std::vector<uint8_t>& frames, uint64_t n_total,
                                                       std::vector<uint8_t>& out) {
    const size_t fb = (size_t)w * hh * 4;
    if (fb == 0 || frames.size() % fb != 0 || out.size() < frames.size())
        return Result<int>::Err({DIPS_ERR_INVALID, "frames/out not n RGBA8 frames"});
    auto c = check(dips_frame_callback_batch_sharded(h, comm.c, w, hh, frames.data(), (uint32_t)(frames.size() / fb),
                                                     n_total, out.data()),
                   h);
    if (!c.ok) return c;
    width = w;
    height = hh;
    return Result<int>::Ok(0);
}

// lib.rs `shard_range`
Result<std::pair<uint64_t, uint32_t>> shard_range(uint64_t n_total, int nranks, int rank) {
    uint64_t first = 0;
    uint32_t count = 0;
    const int st = dips_shard_range(n_total, nranks, rank, &first, &count);
    if (st == DIPS_OK) return Result<std::pair<uint64_t, uint32_t>>::Ok({first, count});
    return Result<std::pair<uint64_t, uint32_t>>::Err({st, "rank outside [0, nranks)"});
}

// lib.rs `DiffSeries`
struct DiffSeries {
    dips_handle* h = nullptr;
    uint32_t channels = 3;
    static Result<DiffSeries*> create_(uint32_t format, uint32_t mode, float tau, int device) {
        dips_params p = default_params();
        p.format = format;
        p.mode = mode;
        p.tau = tau;
        auto h = create(p, device);
        if (!h.ok) return Result<DiffSeries*>::Err(h.err);
        auto* d = new DiffSeries();
        d->h = h.value;
        d->channels = format;
        return Result<DiffSeries*>::Ok(d);
    }
    ~DiffSeries() { dips_destroy(h); }
    size_t frame_bytes(uint32_t w, uint32_t hh) const { return (size_t)w * hh * channels; }
    Result<uint32_t> frames_of(uint32_t w, uint32_t hh, const std::vector<uint8_t>& frames) const {
        const size_t fb = frame_bytes(w, hh);
        if (fb == 0 || frames.size() % fb != 0) return Result<uint32_t>::Err({DIPS_ERR_INVALID, "frames: n whole frames"});
        return Result<uint32_t>::Ok((uint32_t)(frames.size() / fb));
    }
    Result<const uint8_t*> reference_ptr(uint32_t w, uint32_t hh, const std::vector<uint8_t>* ref) const {
        if (!ref) return Result<const uint8_t*>::Ok(nullptr);
        if (ref->size() == frame_bytes(w, hh)) return Result<const uint8_t*>::Ok(ref->data());
        return Result<const uint8_t*>::Err({DIPS_ERR_INVALID, "reference: one whole frame"});
    }
    Result<std::vector<dips_series_entry>> run(uint32_t w, uint32_t hh, const std::vector<uint8_t>& frames,
                                               const std::vector<uint8_t>* ref, std::vector<uint8_t>* map) {
        using R = Result<std::vector<dips_series_entry>>;
        auto n = frames_of(w, hh, frames);
        if (!n.ok) return R::Err(n.err);
        auto rp = reference_ptr(w, hh, ref);
        if (!rp.ok) return R::Err(rp.err);
        std::vector<dips_series_entry> series(n.value);
        uint8_t* mp = nullptr;
        if (map) {
            if (map->size() < frames.size()) return R::Err({DIPS_ERR_CAPACITY, "map too small"});
            mp = map->data();
        }
        auto c = check(dips_diff_series(h, w, hh, frames.data(), n.value, rp.value, series.data(), mp), h);
        if (!c.ok) return R::Err(c.err);
        return R::Ok(series);
    }
    Result<std::vector<dips_series_entry>> run_streamed(uint32_t w, uint32_t hh, const std::vector<uint8_t>& frames,
                                                        uint32_t chunk) {
        using R = Result<std::vector<dips_series_entry>>;
        auto n = frames_of(w, hh, frames);
        if (!n.ok) return R::Err(n.err);
        std::vector<dips_series_entry> series(n.value);
        auto c = check(dips_diff_series_streamed(h, w, hh, frames.data(), n.value, nullptr, series.data(), chunk), h);
        if (!c.ok) return R::Err(c.err);
        return R::Ok(series);
    }
    Result<std::pair<std::vector<dips_series_entry>, std::vector<dips_series_entry>>> run_sharded(
        Comm& comm, uint32_t w, uint32_t hh, const uint8_t* frames, size_t len, uint64_t n_total) {
        using P = std::pair<std::vector<dips_series_entry>, std::vector<dips_series_entry>>;
        using R = Result<P>;
        const size_t fb = frame_bytes(w, hh);
        if (fb == 0 || len % fb != 0) return R::Err({DIPS_ERR_INVALID, "frames: n whole frames"});
        const uint32_t n = (uint32_t)(len / fb);
        std::vector<dips_series_entry> local(n), all;
        if (comm.rank == 0) all.resize(n_total);
        auto c = check(dips_diff_series_sharded(h, comm.c, w, hh, frames, n, n_total, nullptr, 0, local.data(),
                                                comm.rank == 0 ? all.data() : nullptr),
                       h);
        if (!c.ok) return R::Err(c.err);
        return R::Ok(P(std::move(local), std::move(all)));
    }
};

// lib.rs `DiPsCompute` (dips_alt): new(num_textures, rows, cols, props) -> dips_alt_create(cols, rows)
struct DiPsCompute {
    dips_alt_handle* h = nullptr;
    size_t bytes = 0;
    static Result<DiPsCompute*> create_(uint32_t num_textures, uint32_t rows, uint32_t cols) {
        dips_alt_params p;
        dips_alt_params_default(&p);
        p.num_textures = num_textures;
        auto a = check_abi();
        if (!a.ok) return Result<DiPsCompute*>::Err(a.err);
        dips_alt_handle* h = nullptr;
        auto c = check_alt(dips_alt_create(&p, cols, rows, 0, &h), nullptr);
        if (!c.ok) return Result<DiPsCompute*>::Err(c.err);
        auto* d = new DiPsCompute();
        d->h = h;
        d->bytes = (size_t)rows * cols * 4;
        return Result<DiPsCompute*>::Ok(d);
    }
    ~DiPsCompute() { dips_alt_destroy(h); }
    Result<std::vector<uint8_t>> send_frame(const std::vector<uint8_t>& frame, bool snapshot) {
        std::vector<uint8_t> out(bytes);
        auto c = check_alt(dips_alt_send_frame(h, frame.data(), frame.size(), snapshot ? 1 : 0, out.data(), out.size()),
                           h);
        if (!c.ok) return Result<std::vector<uint8_t>>::Err(c.err);
        return Result<std::vector<uint8_t>>::Ok(out);
    }
    Result<int> run(const std::vector<uint8_t>& frames, const std::vector<uint64_t>& markers,
                    std::vector<uint8_t>& out) {
        if (bytes == 0 || frames.size() % bytes != 0 || out.size() < frames.size())
            return Result<int>::Err({DIPS_ERR_INVALID, "frames/out not n frames"});
        return check_alt(dips_alt_run(h, frames.data(), (uint32_t)(frames.size() / bytes),
                                      markers.empty() ? nullptr : markers.data(), (uint32_t)markers.size(),
                                      out.data()),
                         h);
    }
    // lib.rs `DiPsCompute::run_sharded`
    Result<int> run_sharded(struct Comm& comm, const std::vector<uint8_t>& frames, uint64_t n_total,
                            const std::vector<uint64_t>& markers, std::vector<uint8_t>& out);
};

Result<int> DiPsCompute::run_sharded(Comm& comm, const std::vector<uint8_t>& frames, uint64_t n_total,
                                     const std::vector<uint64_t>& markers, std::vector<uint8_t>& out) {
    if (bytes == 0 || frames.size() % bytes != 0 || out.size() < frames.size())
        return Result<int>::Err({DIPS_ERR_INVALID, "frames/out not n frames"});
    return check_alt(dips_alt_run_sharded(h, comm.c, frames.data(), (uint32_t)(frames.size() / bytes), n_total,
                                          markers.empty() ? nullptr : markers.data(), (uint32_t)markers.size(),
                                          out.data()),
                     h);
}

// ---------------------------------------------------------------------------
int failures = 0;

void row(const char* name, bool ok, const std::string& why = "") {
    if (ok) {
        std::printf("ROW %s ok\n", name);
    } else {
        std::printf("ROW %s FAIL %s\n", name, why.c_str());
        ++failures;
    }
}

bool has(const std::string& s, const char* sub) { return s.find(sub) != std::string::npos; }

std::vector<uint8_t> frame_rgba(uint32_t w, uint32_t h, uint32_t seed) {
    std::vector<uint8_t> f((size_t)w * h * 4);
    uint32_t x = seed * 2654435761u + 12345u;
    for (auto& b : f) {
        x ^= x << 13;
        x ^= x >> 17;
        x ^= x << 5;
        b = (uint8_t)(x >> 24);
    }
    return f;
}

bool same(const std::vector<dips_series_entry>& a, const std::vector<dips_series_entry>& b) {
    return a.size() == b.size() && std::memcmp(a.data(), b.data(), a.size() * sizeof(dips_series_entry)) == 0;
}

void no_device_rows() {
    auto cs = ComputeState::on_device(false, 1, 5.0f, DIPS_FILTER_UNFILTERED, DIPS_CHROMA_NONE, 0);
    row("new", !cs.ok && cs.err.status == DIPS_ERR_NODEVICE && has(cs.err.message, "no HIP device"),
        cs.ok ? "created without a device" : cs.err.message);
    auto lb = Comm::loopback(2, 0);
    row("comm_loopback", !lb.ok && lb.err.status == DIPS_ERR_NODEVICE && has(lb.err.message, "no HIP device"),
        lb.ok ? "created without a device" : lb.err.message);
    auto ds = DiffSeries::create_(DIPS_FMT_RGB8, DIPS_MODE_PER_FRAME, 0.0f, 0);
    row("diff_series_new", !ds.ok && ds.err.status == DIPS_ERR_NODEVICE, ds.ok ? "created" : ds.err.message);
    auto alt = DiPsCompute::create_(2, 16, 24);
    row("dips_compute_new", !alt.ok && alt.err.status == DIPS_ERR_NODEVICE, alt.ok ? "created" : alt.err.message);
}

void device_rows() {
    const uint32_t W = 64, H = 40;
    // ComputeState::new (gpu/mod.rs:59-65), then the warm-up: dispatch gives
    // None (status 0, gpu/mod.rs:394-396) before the 4th frame
    auto made = ComputeState::on_device(false, 1, 5.0f, DIPS_FILTER_UNFILTERED, DIPS_CHROMA_NONE, 0);
    row("new", made.ok, made.ok ? "" : made.err.message);
    if (!made.ok) return;
    ComputeState& cs = *made.value;
    {
        auto d = cs.try_dispatch();
        bool ok = d.ok && !d.value.has_value();
        for (uint32_t t = 0; t < 3 && ok; ++t) {
            auto a = cs.try_add_texture(W, H, frame_rgba(W, H, t));
            auto d2 = cs.try_dispatch();
            ok = a.ok && d2.ok && !d2.value.has_value();
        }
        row("try_dispatch_warmup", ok);
    }
    {
        auto a = cs.try_add_texture(W, H, frame_rgba(W, H, 3));
        auto d = cs.try_dispatch();
        row("try_dispatch_some", a.ok && d.ok && d.value.has_value() && d.value->size() == (size_t)W * H * 4);
        auto st = cs.try_start_texture();
        row("try_start_texture", st.ok && st.value.has_value());
    }
    {
        // add_texture swallows its error (gpu/mod.rs:189, :206); try_ reports it
        auto bad = frame_rgba(W, H, 9);
        bad.pop_back();
        cs.add_texture(W, H, bad);  // no panic, no state change
        auto r = cs.try_add_texture(W, H, bad);
        row("try_add_texture_error", !r.ok && r.err.status == DIPS_ERR_INVALID && has(r.err.message, "len"),
            r.ok ? "accepted a short frame" : r.err.message);
    }
    {
        // a size change: < 0 with the message, the output untouched, and the
        // panicking frame_callback does not pass the input through
        std::vector<uint8_t> out((size_t)(W + 8) * H * 4, 0xAB);
        auto r = cs.frame_callback_into(W + 8, H, frame_rgba(W + 8, H, 5), out);
        bool untouched = true;
        for (auto b : out) untouched = untouched && b == 0xAB;
        row("frame_callback_into_size_change",
            !r.ok && r.err.status == DIPS_ERR_INVALID && has(r.err.message, "size changed") && untouched &&
                has(message(dips_last_error(cs.h)), "size changed"),
            r.ok ? "accepted" : r.err.message);
        bool panicked = false;
        try {
            (void)frame_callback(W + 8, H, frame_rgba(W + 8, H, 5), cs);
        } catch (const Panic& p) {
            panicked = has(p.what, "size changed");
        }
        row("frame_callback_panics", panicked);
        // the handle still works at its own size
        std::vector<uint8_t> ok_out((size_t)W * H * 4);
        auto r2 = cs.frame_callback_into(W, H, frame_rgba(W, H, 6), ok_out);
        row("frame_callback_into_ok", r2.ok && r2.value);
    }
    {
        // a negative status of dispatch reaches the panicking form: an output
        // smaller than the frame (the crate sizes it from the last frame)
        const uint32_t keep = cs.width;
        cs.width = W / 2;
        auto r = cs.try_dispatch();
        bool panicked = false;
        try {
            (void)cs.dispatch();
        } catch (const Panic& p) {
            panicked = has(p.what, "smaller");
        }
        cs.width = keep;
        row("try_dispatch_error", !r.ok && r.err.status == DIPS_ERR_CAPACITY && has(r.err.message, "smaller"),
            r.ok ? "accepted" : r.err.message);
        row("dispatch_panics", panicked);
    }
    delete made.value;

    {
        // frame_callback_batch == frame_callback one by one; callback_phases
        // only after a zero-copy call; start_texture (panicking form) is None
        // before the 4th frame; resume continues a stream mid-way (t0 >= 7)
        const uint32_t n = 10;
        std::vector<uint8_t> all;
        std::vector<std::vector<uint8_t>> one_by_one;
        auto a = ComputeState::on_device(false, 1, 5.0f, DIPS_FILTER_UNFILTERED, DIPS_CHROMA_NONE, 0);
        auto b = ComputeState::on_device(false, 1, 5.0f, DIPS_FILTER_UNFILTERED, DIPS_CHROMA_NONE, 0);
        auto c = ComputeState::on_device(false, 1, 5.0f, DIPS_FILTER_UNFILTERED, DIPS_CHROMA_NONE, 0);
        if (!a.ok || !b.ok || !c.ok) {
            row("frame_callback_batch", false, "create failed");
            return;
        }
        row("callback_phases", !a.value->callback_phases().has_value());
        bool no_start = false;
        try {
            no_start = !start_texture(*a.value).has_value();
        } catch (const Panic&) {
        }
        row("start_texture", no_start);
        for (uint32_t t = 0; t < n; ++t) {
            auto f = frame_rgba(W, H, 40 + t);
            all.insert(all.end(), f.begin(), f.end());
            one_by_one.push_back(frame_callback(W, H, f, *a.value));
        }
        std::vector<uint8_t> out(all.size());
        auto r = b.value->frame_callback_batch(W, H, all, out);
        bool same_out = r.ok;
        for (uint32_t t = 0; t < n && same_out; ++t)
            same_out = std::memcmp(out.data() + (size_t)t * W * H * 4, one_by_one[t].data(), (size_t)W * H * 4) == 0;
        std::vector<uint8_t> small(10);
        auto refused = b.value->frame_callback_batch(W, H, all, small);
        row("frame_callback_batch", same_out && !refused.ok && refused.err.status == DIPS_ERR_INVALID);
        row("callback_phases_after_call", a.value->callback_phases().has_value());
        auto st = a.value->try_start_texture();
        const size_t fb = (size_t)W * H * 4;
        std::vector<uint8_t> halo(all.begin() + 4 * fb, all.begin() + 7 * fb);
        auto bad = c.value->resume(W, H, st.value.value_or(std::vector<uint8_t>()), std::vector<uint8_t>(10), 7);
        auto rs = c.value->resume(W, H, *st.value, halo, 7);
        bool cont = rs.ok;
        for (uint32_t t = 7; t < n && cont; ++t) {
            std::vector<uint8_t> f(all.begin() + t * fb, all.begin() + (t + 1) * fb);
            cont = frame_callback(W, H, f, *c.value) == one_by_one[t];
        }
        row("resume", st.ok && st.value.has_value() && !bad.ok && cont);
        delete a.value;
        delete b.value;
        delete c.value;
    }

    // DiffSeries: run / run_streamed / run_sharded (loopback) agree; the
    // crate-side refusals never reach the library
    const uint32_t n = 11;
    std::vector<uint8_t> frames;
    for (uint32_t t = 0; t < n; ++t) {
        auto f = frame_rgba(W, H, 100 + t);
        for (size_t i = 0; i < f.size(); i += 4) frames.insert(frames.end(), f.begin() + i, f.begin() + i + 3);
    }
    auto ds = DiffSeries::create_(DIPS_FMT_RGB8, DIPS_MODE_PER_FRAME, 8.0f / 255.0f, 0);
    row("diff_series_new", ds.ok, ds.ok ? "" : ds.err.message);
    if (!ds.ok) return;
    auto one = ds.value->run(W, H, frames, nullptr, nullptr);
    row("diff_series_run", one.ok && one.value.size() == n && one.value[1].sad > 0);
    auto streamed = ds.value->run_streamed(W, H, frames, 4);
    row("diff_series_run_streamed", streamed.ok && same(streamed.value, one.value));
    {
        std::vector<uint8_t> short_ref(10);
        auto r = ds.value->run(W, H, frames, &short_ref, nullptr);
        std::vector<uint8_t> small_map(10);
        auto m = ds.value->run(W, H, frames, nullptr, &small_map);
        std::vector<uint8_t> ragged(frames.begin(), frames.end() - 1);
        auto g = ds.value->run(W, H, ragged, nullptr, nullptr);
        row("diff_series_refusals", !r.ok && r.err.status == DIPS_ERR_INVALID && !m.ok &&
                                        m.err.status == DIPS_ERR_CAPACITY && !g.ok && g.err.status == DIPS_ERR_INVALID);
    }
    {
        auto sr = shard_range(n, 3, 1);
        auto bad = shard_range(n, 3, 3);
        row("shard_range", sr.ok && sr.value.first == 3 && sr.value.second == 4 && !bad.ok);
        auto comms = Comm::loopback(3, 0);
        row("comm_loopback", comms.ok && comms.value.size() == 3 && comms.value[2]->rank == 2 &&
                                 comms.value[0]->nranks == 3);
        if (comms.ok) {
            std::vector<DiffSeries*> ops(3, nullptr);
            bool made_all = true;
            for (auto& o : ops) {
                auto d = DiffSeries::create_(DIPS_FMT_RGB8, DIPS_MODE_PER_FRAME, 8.0f / 255.0f, 0);
                made_all = made_all && d.ok;
                o = d.ok ? d.value : nullptr;
            }
            std::vector<std::vector<dips_series_entry>> all(3);
            std::vector<bool> ok(3, false);
            std::vector<std::thread> th;
            for (int r = 0; r < 3 && made_all; ++r) {
                th.emplace_back([&, r]() {
                    auto range = shard_range(n, 3, r);
                    const size_t fb = (size_t)W * H * 3;
                    auto res = ops[r]->run_sharded(*comms.value[r], W, H, frames.data() + range.value.first * fb,
                                                   (size_t)range.value.second * fb, n);
                    ok[r] = res.ok;
                    if (res.ok) all[r] = res.value.second;
                });
            }
            for (auto& t : th) t.join();
            row("diff_series_run_sharded", made_all && ok[0] && ok[1] && ok[2] && same(all[0], one.value));
            for (auto* o : ops) delete o;
            // a rank whose frame count is not its range: < 0 on that rank alone,
            // before any collective
            auto wrong = ds.value->run_sharded(*comms.value[1], W, H, frames.data(), (size_t)W * H * 3 * 2, n);
            row("diff_series_run_sharded_error", !wrong.ok && wrong.err.status == DIPS_ERR_INVALID &&
                                                     has(wrong.err.message, "owns 4 frames"),
                wrong.ok ? "accepted" : wrong.err.message);
            for (auto* c : comms.value) delete c;
        }
    }
    delete ds.value;

    {
        // ComputeState::frame_callback_batch_sharded over 2 loopback ranks
        // (fresh handles) == one ComputeState's frame_callback_batch; a
        // layout with a rank starting before frame 7 is refused on every rank
        const uint32_t n_total = 16;
        std::vector<uint8_t> all;
        for (uint32_t t = 0; t < n_total; ++t) {
            auto f = frame_rgba(W, H, 200 + t);
            all.insert(all.end(), f.begin(), f.end());
        }
        const size_t fb = (size_t)W * H * 4;
        auto one = ComputeState::on_device(true, 1, 5.0f, DIPS_FILTER_SIGMOID, DIPS_CHROMA_NONE, 0);
        std::vector<uint8_t> want(all.size());
        bool ok = one.ok && one.value->frame_callback_batch(W, H, all, want).ok;
        if (one.ok) delete one.value;
        auto comms = Comm::loopback(2, 0);
        ok = ok && comms.ok;
        std::vector<std::vector<uint8_t>> outs(2);
        std::vector<int> good(2, 0);
        if (ok) {
            std::vector<std::thread> th;
            for (int r = 0; r < 2; ++r)
                th.emplace_back([&, r]() {
                    auto cs = ComputeState::on_device(true, 1, 5.0f, DIPS_FILTER_SIGMOID, DIPS_CHROMA_NONE, 0);
                    if (!cs.ok) return;
                    auto range = shard_range(n_total, 2, r);
                    std::vector<uint8_t> mine(all.begin() + range.value.first * fb,
                                              all.begin() + (range.value.first + range.value.second) * fb);
                    outs[r].resize(mine.size());
                    good[r] = cs.value->frame_callback_batch_sharded(*comms.value[r], W, H, mine, n_total, outs[r]).ok;
                    delete cs.value;
                });
            for (auto& t : th) t.join();
        }
        std::vector<uint8_t> got = outs[0];
        got.insert(got.end(), outs[1].begin(), outs[1].end());
        row("frame_callback_batch_sharded", ok && good[0] && good[1] && got == want);
        if (comms.ok) {
            auto cs = ComputeState::on_device(false, 1, 5.0f, DIPS_FILTER_UNFILTERED, DIPS_CHROMA_NONE, 0);
            std::vector<uint8_t> few(all.begin(), all.begin() + 6 * fb), o(few.size());
            auto bad = cs.ok ? cs.value->frame_callback_batch_sharded(*comms.value[0], W, H, few, 12, o)
                             : Result<int>::Err({0, ""});
            row("frame_callback_batch_sharded_layout", !bad.ok && bad.err.status == DIPS_ERR_INVALID &&
                                                           has(bad.err.message, "< 7"));
            if (cs.ok) delete cs.value;
            for (auto* c : comms.value) delete c;
        }
    }

    // DiPsCompute: (rows, cols) -> dips_alt_create(cols, rows); a wrong frame
    // length is an error, not a panic inside the library
    auto alt = DiPsCompute::create_(2, 16, 24);
    row("dips_compute_new", alt.ok && alt.value->bytes == 16 * 24 * 4, alt.ok ? "" : alt.err.message);
    if (alt.ok) {
        auto good = alt.value->send_frame(frame_rgba(24, 16, 1), false);
        auto bad = alt.value->send_frame(frame_rgba(16, 16, 1), false);
        row("dips_compute_send_frame", good.ok && good.value.size() == alt.value->bytes && !bad.ok &&
                                           bad.err.status == DIPS_ERR_INVALID && has(bad.err.message, "len"));
        std::vector<uint8_t> fr;
        for (uint32_t t = 0; t < 5; ++t) {
            auto f = frame_rgba(24, 16, 60 + t);
            fr.insert(fr.end(), f.begin(), f.end());
        }
        std::vector<uint8_t> out(fr.size()), small(4);
        auto r = alt.value->run(fr, {3}, out);
        auto refused = alt.value->run(fr, {}, small);
        row("dips_compute_run", r.ok && !refused.ok && refused.err.status == DIPS_ERR_INVALID);
        delete alt.value;
    }

    {
        // DiPsCompute::run_sharded over 3 loopback ranks (fresh operators,
        // refresh markers on and across the range edges) == one DiPsCompute's
        // run over every frame; a wrong frame count is refused
        const uint32_t n_total = 15, rows = 16, cols = 24;
        std::vector<uint8_t> all;
        for (uint32_t t = 0; t < n_total; ++t) {
            auto f = frame_rgba(cols, rows, 90 + t);
            all.insert(all.end(), f.begin(), f.end());
        }
        const size_t fb = (size_t)rows * cols * 4;
        const std::vector<uint64_t> markers = {5, 6, 11};
        auto one = DiPsCompute::create_(2, rows, cols);
        std::vector<uint8_t> want(all.size());
        bool ok = one.ok && one.value->run(all, markers, want).ok;
        if (one.ok) delete one.value;
        auto comms = Comm::loopback(3, 0);
        ok = ok && comms.ok;
        std::vector<std::vector<uint8_t>> outs(3);
        std::vector<int> good(3, 0);
        if (ok) {
            std::vector<std::thread> th;
            for (int r = 0; r < 3; ++r)
                th.emplace_back([&, r]() {
                    auto d = DiPsCompute::create_(2, rows, cols);
                    if (!d.ok) return;
                    auto range = shard_range(n_total, 3, r);
                    std::vector<uint8_t> mine(all.begin() + range.value.first * fb,
                                              all.begin() + (range.value.first + range.value.second) * fb);
                    outs[r].resize(mine.size());
                    good[r] = d.value->run_sharded(*comms.value[r], mine, n_total, markers, outs[r]).ok;
                    delete d.value;
                });
            for (auto& t : th) t.join();
        }
        std::vector<uint8_t> got;
        for (auto& o : outs) got.insert(got.end(), o.begin(), o.end());
        row("dips_compute_run_sharded", ok && good[0] && good[1] && good[2] && got == want);
        if (comms.ok) {
            // rank 0 owns 5 of 15 frames: one frame is refused on that rank
            // alone, before any exchange
            auto d = DiPsCompute::create_(2, rows, cols);
            std::vector<uint8_t> few(all.begin(), all.begin() + fb), o(few.size());
            auto bad = d.ok ? d.value->run_sharded(*comms.value[0], few, n_total, {}, o) : Result<int>::Err({0, ""});
            row("dips_compute_run_sharded_error", !bad.ok && bad.err.status == DIPS_ERR_INVALID &&
                                                      has(bad.err.message, "owns 5 frames, n_local is 1"),
                bad.ok ? "accepted" : bad.err.message);
            if (d.ok) delete d.value;
            for (auto* c : comms.value) delete c;
        }
    }

    // Comm::unique_id + Comm::rccl at one rank (ncclCommInitRank)
    auto id = Comm::unique_id();
    auto rc = id.ok ? Comm::rccl(id.value, 1, 0, 0) : Result<Comm*>::Err(id.err);
    row("comm_rccl", rc.ok && rc.value->nranks == 1 && rc.value->rank == 0, rc.ok ? "" : rc.err.message);
    if (rc.ok) delete rc.value;
    auto bad_rank = id.ok ? Comm::rccl(id.value, 1, 1, 0) : Result<Comm*>::Err(id.err);
    row("comm_rccl_error", !bad_rank.ok && bad_rank.err.status == DIPS_ERR_INVALID);
    auto all = Comm::rccl_all({0});
    row("comm_rccl_all", all.ok && all.value.size() == 1 && all.value[0]->nranks == 1, all.ok ? "" : all.err.message);
    if (all.ok)
        for (auto* c : all.value) delete c;

    // abi_version / series_si
    dips_series_entry e{1, 2, 3, 1ull << 32};
    row("series_si", dips_series_si(&e) == 1.0 && dips_abi_version() == DIPS_ABI_VERSION);
}

}  // namespace

int main(int argc, char** argv) {
    auto abi = check_abi();
    row("check_abi", abi.ok, abi.ok ? "" : abi.err.message);
    const bool device = argc > 1 && std::strcmp(argv[1], "--device") == 0;
    if (device) device_rows();
    else no_device_rows();
    std::printf("failures %d\n", failures);
    return failures != 0;
}
