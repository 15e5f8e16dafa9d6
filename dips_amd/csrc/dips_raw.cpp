// dips_raw.cpp -- native host program over the C ABI (include/dips_hip.h),
// the stand-in for the Rust host side (cargo is absent in this image).
//
// It mirrors dips' perform_dips loop (dips/src/frame_extractor.rs:206-276:
// appsink delivers RGBA8 frames, frame_callback (dips/src/lib.rs:233-246)
// turns each into the output frame, the muxer writes it) with the GStreamer
// decode / encode replaced by raw files, and exposes the north-star series:
//
//   dips_raw callback IN.rgba W H OUT.rgba [--colorize] [--window N]
//            [--sensitivity K] [--filter sigmoid|inverse|none]
//            [--chroma none|red|green|blue] [--batch N]
//            [--ranks N [--transport loopback|rccl]]
//                                         -> with --ranks, N ranks (one thread
//            and one fresh handle each) run their frame ranges through
//            dips_frame_callback_batch_sharded
//   dips_raw alt IN.rgba W H OUT.rgba [--markers M1,M2,...] [--window N]
//            [--textures N] [--ranks N [--transport loopback|rccl]]
//                                         -> the dips_alt run_dips_on_file
//            loop (dips_alt/src/lib.rs:588-683) with its refresh markers;
//            with --ranks, dips_alt_run_sharded
//   dips_raw series IN.raw W H rgb8|rgba8|gray8 [--mode overall|per-frame]
//            [--tau T] [--chunk N]        -> CSV frame,sad,sj,count,si
//   dips_raw sharded IN.raw W H rgb8|rgba8|gray8 --ranks N [--mode ...]
//            [--tau T] [--transport loopback|rccl]
//                                         -> the same CSV, computed by N
//            ranks (one thread and one handle each) with
//            dips_diff_series_sharded: each rank hands its frame range of the
//            file to the library, rank 0 prints the gathered series.
//            loopback: every rank on device 0; rccl: rank r on device r, all
//            ranks of this process from dips_comm_create_all -- one process
//            that decodes once and feeds every GPU of a node
//
// Input files are memory-mapped and handed over as host pointers: the
// library stages them through pinned memory and overlaps the PCIe transfers
// with the kernels.  Exit status 0 on success, 1 on a usage error, 2 on a
// library error (message from dips_last_error on stderr).
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/dips_hip.h"

namespace {

struct Mapped {
    const uint8_t* p = nullptr;
    size_t n = 0;
    bool open(const char* path) {
        const int fd = ::open(path, O_RDONLY);
        if (fd < 0) return false;
        struct stat st {};
        if (fstat(fd, &st) != 0 || st.st_size <= 0) {
            ::close(fd);
            return false;
        }
        n = (size_t)st.st_size;
        void* m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
        ::close(fd);
        if (m == MAP_FAILED) return false;
        p = static_cast<const uint8_t*>(m);
        return true;
    }
    ~Mapped() {
        if (p) munmap(const_cast<uint8_t*>(p), n);
    }
};

int usage() {
    std::fprintf(stderr,
                 "usage: dips_raw callback IN.rgba W H OUT.rgba [--colorize] [--window N] [--sensitivity K]\n"
                 "                [--filter sigmoid|inverse|none] [--chroma none|red|green|blue] [--batch N]\n"
                 "                [--ranks N [--transport loopback|rccl]]\n"
                 "       dips_raw alt IN.rgba W H OUT.rgba [--markers M1,M2,...] [--window N] [--textures N]\n"
                 "                [--ranks N [--transport loopback|rccl]]\n"
                 "       dips_raw series IN.raw W H rgb8|rgba8|gray8 [--mode overall|per-frame] [--tau T]\n"
                 "                [--chunk N]\n"
                 "       dips_raw sharded IN.raw W H rgb8|rgba8|gray8 --ranks N [--mode overall|per-frame]\n"
                 "                [--tau T] [--transport loopback|rccl]\n");
    return 1;
}

int lib_error(dips_handle* h, const char* what, int st) {
    std::fprintf(stderr, "dips_raw: %s failed (%d): %s\n", what, st, dips_last_error(h));
    return 2;
}

bool parse_u32(const char* s, uint32_t* v) {
    char* end = nullptr;
    const unsigned long x = std::strtoul(s, &end, 10);
    if (!s[0] || *end || x == 0 || x > 0xFFFFFFFFul) return false;
    *v = (uint32_t)x;
    return true;
}

// `ranks` communicators, loopback on device 0 or RCCL with rank r on device
// r (dips_comm_create_all); 0 or the exit status of the failure
int make_comms(const std::string& transport, uint32_t ranks, std::vector<dips_comm*>& comms) {
    const bool rccl = transport == "rccl";
    comms.assign(ranks, nullptr);
    // RCCL prints its version banner to stdout when a communicator is made:
    // send it to stderr, stdout carries the program's own output only
    std::fflush(stdout);
    const int saved_stdout = dup(1);
    dup2(2, 1);
    const int st = rccl ? dips_comm_create_all((int)ranks, nullptr, comms.data())
                        : dips_comm_create_loopback((int)ranks, 0, comms.data());
    std::fflush(stdout);
    dup2(saved_stdout, 1);
    close(saved_stdout);
    if (st != DIPS_OK) {
        std::fprintf(stderr, "dips_raw: %s failed (%d): %s\n", rccl ? "dips_comm_create_all" : "dips_comm_create_loopback",
                     st, dips_comm_last_error(nullptr));
        return 2;
    }
    return 0;
}

// Run `body(rank, first, count, why)` on one thread per rank; 0, or 2 after
// printing the first failing rank's message
template <typename Body>
int on_ranks(uint32_t ranks, uint64_t n_total, const char* what, Body&& body) {
    std::vector<int> rc(ranks, 0);
    std::vector<std::string> why(ranks);
    std::vector<std::thread> threads;
    for (uint32_t r = 0; r < ranks; ++r)
        threads.emplace_back([&, r]() {
            uint64_t first = 0;
            uint32_t count = 0;
            if (dips_shard_range(n_total, (int)ranks, (int)r, &first, &count) != DIPS_OK) {
                rc[r] = 1;
                why[r] = "bad shard range";
                return;
            }
            rc[r] = body(r, first, count, why[r]);
        });
    for (auto& t : threads) t.join();
    for (uint32_t r = 0; r < ranks; ++r)
        if (rc[r] != 0) {
            std::fprintf(stderr, "dips_raw: rank %u: %s failed (%d): %s\n", r, what, rc[r], why[r].c_str());
            return 2;
        }
    return 0;
}

bool write_all(const char* path, const uint8_t* p, size_t n) {
    FILE* f = std::fopen(path, "wb");
    if (!f) {
        std::fprintf(stderr, "dips_raw: cannot create %s\n", path);
        return false;
    }
    const bool ok = std::fwrite(p, 1, n, f) == n;
    if (std::fclose(f) != 0 || !ok) {
        std::fprintf(stderr, "dips_raw: short write to %s\n", path);
        return false;
    }
    return true;
}

int run_callback(int argc, char** argv) {
    if (argc < 6) return usage();
    uint32_t w = 0, h = 0, batch = 1, ranks = 0;
    std::string transport = "loopback";
    if (!parse_u32(argv[3], &w) || !parse_u32(argv[4], &h)) return usage();
    dips_params p;
    dips_params_default(&p);  // DiPsProperties defaults (dips/src/lib.rs:71-90)
    for (int i = 6; i < argc; ++i) {
        const std::string a = argv[i];
        const bool has = i + 1 < argc;
        if (a == "--colorize") {
            p.colorize = 1;
        } else if (a == "--window" && has) {
            p.spatial_window_size = std::atoi(argv[++i]);
        } else if (a == "--sensitivity" && has) {
            p.sensitivity = std::strtof(argv[++i], nullptr);
        } else if (a == "--filter" && has) {
            const std::string f = argv[++i];
            p.filter_type = f == "sigmoid" ? DIPS_FILTER_SIGMOID
                            : f == "inverse" ? DIPS_FILTER_INVERSE_SIGMOID
                                             : DIPS_FILTER_UNFILTERED;
        } else if (a == "--chroma" && has) {
            const std::string c = argv[++i];
            p.chroma_filter = c == "red" ? DIPS_CHROMA_RED
                              : c == "green" ? DIPS_CHROMA_GREEN
                              : c == "blue" ? DIPS_CHROMA_BLUE
                                            : DIPS_CHROMA_NONE;
        } else if (a == "--batch" && has) {
            if (!parse_u32(argv[++i], &batch)) return usage();
        } else if (a == "--ranks" && has) {
            if (!parse_u32(argv[++i], &ranks) || ranks > 64) return usage();
        } else if (a == "--transport" && has) {
            transport = argv[++i];
            if (transport != "loopback" && transport != "rccl") return usage();
        } else {
            return usage();
        }
    }
    Mapped in;
    if (!in.open(argv[2])) {
        std::fprintf(stderr, "dips_raw: cannot map %s\n", argv[2]);
        return 1;
    }
    const size_t fb = (size_t)w * h * 4u;
    if (in.n % fb != 0) {
        std::fprintf(stderr, "dips_raw: %s is not a whole number of %ux%u RGBA8 frames\n", argv[2], w, h);
        return 1;
    }
    const uint64_t n = in.n / fb;
    if (ranks > 0) {
        // one fresh ComputeState per rank; every output frame is the one
        // ComputeState over the whole file gives
        std::vector<dips_comm*> comms;
        int rc = make_comms(transport, ranks, comms);
        if (rc != 0) return rc;
        std::vector<uint8_t> outbuf(in.n);
        rc = on_ranks(ranks, n, "dips_frame_callback_batch_sharded",
                      [&](uint32_t r, uint64_t first, uint32_t count, std::string& why) {
                          dips_handle* hd = nullptr;
                          int s2 = dips_create(&p, transport == "rccl" ? (int)r : 0, &hd);
                          if (s2 != DIPS_OK) {
                              why = dips_last_error(nullptr);
                              return s2;
                          }
                          s2 = dips_frame_callback_batch_sharded(hd, comms[r], w, h, in.p + first * fb, count, n,
                                                                 outbuf.data() + first * fb);
                          if (s2 != DIPS_OK) why = dips_last_error(hd);
                          dips_destroy(hd);
                          return s2;
                      });
        for (auto* c : comms) dips_comm_destroy(c);
        if (rc != 0) return rc;
        return write_all(argv[5], outbuf.data(), outbuf.size()) ? 0 : 1;
    }
    FILE* out = std::fopen(argv[5], "wb");
    if (!out) {
        std::fprintf(stderr, "dips_raw: cannot create %s\n", argv[5]);
        return 1;
    }
    dips_handle* hd = nullptr;
    int st = dips_create(&p, 0, &hd);
    if (st != DIPS_OK) {
        std::fclose(out);
        return lib_error(nullptr, "dips_create", st);
    }
    std::vector<uint8_t> buf(fb * batch);
    int rc = 0;
    for (uint64_t t = 0; t < n && rc == 0;) {
        const uint32_t m = (uint32_t)std::min<uint64_t>(batch, n - t);
        const uint8_t* src = in.p + t * fb;
        if (batch == 1) {
            // frame_callback: frames 0..2 come back unchanged (lib.rs:241-245)
            st = dips_frame_callback(hd, w, h, src, fb, buf.data(), buf.size());
            if (st < 0) rc = lib_error(hd, "dips_frame_callback", st);
        } else {
            st = dips_frame_callback_batch(hd, w, h, src, m, buf.data());
            if (st != DIPS_OK) rc = lib_error(hd, "dips_frame_callback_batch", st);
        }
        if (rc == 0 && std::fwrite(buf.data(), fb, m, out) != m) {
            std::fprintf(stderr, "dips_raw: short write\n");
            rc = 1;
        }
        t += m;
    }
    dips_destroy(hd);
    if (std::fclose(out) != 0 && rc == 0) rc = 1;
    return rc;
}

void print_series(const dips_series_entry* series, uint64_t n) {
    std::printf("frame,sad,sj,count,si\n");
    for (uint64_t t = 0; t < n; ++t)
        std::printf("%llu,%llu,%llu,%llu,%.17g\n", (unsigned long long)t, (unsigned long long)series[t].sad,
                    (unsigned long long)series[t].sj, (unsigned long long)series[t].count,
                    dips_series_si(&series[t]));
}

int run_sharded(int argc, char** argv) {
    if (argc < 6) return usage();
    uint32_t w = 0, h = 0, ranks = 0;
    std::string transport = "loopback";
    if (!parse_u32(argv[3], &w) || !parse_u32(argv[4], &h)) return usage();
    dips_params p;
    dips_params_default(&p);
    const std::string fmt = argv[5];
    p.format = fmt == "rgb8" ? DIPS_FMT_RGB8 : fmt == "rgba8" ? DIPS_FMT_RGBA8 : fmt == "gray8" ? DIPS_FMT_GRAY8 : 0u;
    if (!p.format) return usage();
    for (int i = 6; i < argc; ++i) {
        const std::string a = argv[i];
        const bool has = i + 1 < argc;
        if (a == "--mode" && has) {
            const std::string m = argv[++i];
            if (m != "overall" && m != "per-frame") return usage();
            p.mode = m == "overall" ? DIPS_MODE_OVERALL : DIPS_MODE_PER_FRAME;
        } else if (a == "--tau" && has) {
            p.tau = std::strtof(argv[++i], nullptr);
        } else if (a == "--ranks" && has) {
            if (!parse_u32(argv[++i], &ranks) || ranks > 64) return usage();
        } else if (a == "--transport" && has) {
            transport = argv[++i];
            if (transport != "loopback" && transport != "rccl") return usage();
        } else {
            return usage();
        }
    }
    if (ranks == 0) return usage();
    Mapped in;
    if (!in.open(argv[2])) {
        std::fprintf(stderr, "dips_raw: cannot map %s\n", argv[2]);
        return 1;
    }
    const size_t fb = (size_t)w * h * p.format;
    if (in.n % fb != 0) {
        std::fprintf(stderr, "dips_raw: %s is not a whole number of %ux%u %s frames\n", argv[2], w, h, fmt.c_str());
        return 1;
    }
    const uint64_t n_total = in.n / fb;
    const bool rccl = transport == "rccl";
    std::vector<dips_comm*> comms;
    int rc = make_comms(transport, ranks, comms);
    if (rc != 0) return rc;
    std::vector<dips_series_entry> all(n_total);
    rc = on_ranks(ranks, n_total, "dips_diff_series_sharded",
                  [&](uint32_t r, uint64_t first, uint32_t count, std::string& why) {
                      dips_handle* hd = nullptr;
                      int s2 = dips_create(&p, rccl ? (int)r : 0, &hd);
                      if (s2 != DIPS_OK) {
                          why = dips_last_error(nullptr);
                          return s2;
                      }
                      std::vector<dips_series_entry> local(count);
                      // host pointers: the rank's frames straight from the mapped file
                      s2 = dips_diff_series_sharded(hd, comms[r], w, h, in.p + first * fb, count, n_total, nullptr, 0,
                                                    local.data(), r == 0 ? all.data() : nullptr);
                      if (s2 != DIPS_OK) why = dips_last_error(hd);
                      dips_destroy(hd);
                      return s2;
                  });
    for (auto* c : comms) dips_comm_destroy(c);
    if (rc != 0) return rc;
    print_series(all.data(), n_total);
    return 0;
}

int run_series(int argc, char** argv) {
    if (argc < 6) return usage();
    uint32_t w = 0, h = 0, chunk = 0;
    if (!parse_u32(argv[3], &w) || !parse_u32(argv[4], &h)) return usage();
    dips_params p;
    dips_params_default(&p);
    const std::string fmt = argv[5];
    p.format = fmt == "rgb8" ? DIPS_FMT_RGB8 : fmt == "rgba8" ? DIPS_FMT_RGBA8 : fmt == "gray8" ? DIPS_FMT_GRAY8 : 0u;
    if (!p.format) return usage();
    for (int i = 6; i < argc; ++i) {
        const std::string a = argv[i];
        const bool has = i + 1 < argc;
        if (a == "--mode" && has) {
            const std::string m = argv[++i];
            if (m != "overall" && m != "per-frame") return usage();
            p.mode = m == "overall" ? DIPS_MODE_OVERALL : DIPS_MODE_PER_FRAME;
        } else if (a == "--tau" && has) {
            p.tau = std::strtof(argv[++i], nullptr);
        } else if (a == "--chunk" && has) {
            if (!parse_u32(argv[++i], &chunk)) return usage();
        } else {
            return usage();
        }
    }
    Mapped in;
    if (!in.open(argv[2])) {
        std::fprintf(stderr, "dips_raw: cannot map %s\n", argv[2]);
        return 1;
    }
    const size_t fb = (size_t)w * h * p.format;
    if (in.n % fb != 0 || in.n / fb > 0xFFFFFFFFull) {
        std::fprintf(stderr, "dips_raw: %s is not a whole number of %ux%u %s frames\n", argv[2], w, h, fmt.c_str());
        return 1;
    }
    const uint32_t n = (uint32_t)(in.n / fb);
    dips_handle* hd = nullptr;
    int st = dips_create(&p, 0, &hd);
    if (st != DIPS_OK) return lib_error(nullptr, "dips_create", st);
    std::vector<dips_series_entry> series(n);
    st = dips_diff_series_streamed(hd, w, h, in.p, n, nullptr, series.data(), chunk);
    if (st != DIPS_OK) {
        const int rc = lib_error(hd, "dips_diff_series_streamed", st);
        dips_destroy(hd);
        return rc;
    }
    print_series(series.data(), n);
    dips_destroy(hd);
    return 0;
}

int alt_error(dips_alt_handle* h, const char* what, int st) {
    std::fprintf(stderr, "dips_raw: %s failed (%d): %s\n", what, st, dips_alt_last_error(h));
    return 2;
}

int run_alt(int argc, char** argv) {
    if (argc < 6) return usage();
    uint32_t w = 0, h = 0, ranks = 0;
    std::string transport = "loopback";
    std::vector<uint64_t> markers;
    if (!parse_u32(argv[3], &w) || !parse_u32(argv[4], &h)) return usage();
    dips_alt_params p;
    dips_alt_params_default(&p);  // DiPsProperties::default() (dips_alt/src/dips_compute/mod.rs:176-186)
    for (int i = 6; i < argc; ++i) {
        const std::string a = argv[i];
        const bool has = i + 1 < argc;
        if (a == "--markers" && has) {
            // comma-separated 1-based frame positions (lib.rs:668-670)
            const std::string list = argv[++i];
            size_t at = 0;
            while (at <= list.size()) {
                const size_t comma = std::min(list.find(',', at), list.size());
                uint32_t m = 0;
                if (!parse_u32(list.substr(at, comma - at).c_str(), &m)) return usage();
                markers.push_back(m);
                at = comma + 1;
            }
        } else if (a == "--window" && has) {
            p.window_size = std::atoi(argv[++i]);
        } else if (a == "--textures" && has) {
            if (!parse_u32(argv[++i], &p.num_textures)) return usage();
        } else if (a == "--ranks" && has) {
            if (!parse_u32(argv[++i], &ranks) || ranks > 64) return usage();
        } else if (a == "--transport" && has) {
            transport = argv[++i];
            if (transport != "loopback" && transport != "rccl") return usage();
        } else {
            return usage();
        }
    }
    Mapped in;
    if (!in.open(argv[2])) {
        std::fprintf(stderr, "dips_raw: cannot map %s\n", argv[2]);
        return 1;
    }
    const size_t fb = (size_t)w * h * 4u;
    if (in.n % fb != 0 || in.n / fb > 0xFFFFFFFFull) {
        std::fprintf(stderr, "dips_raw: %s is not a whole number of %ux%u RGBA8 frames\n", argv[2], w, h);
        return 1;
    }
    const uint64_t n = in.n / fb;
    const uint64_t* mk = markers.empty() ? nullptr : markers.data();
    std::vector<uint8_t> outbuf(in.n);
    if (ranks == 0) {
        dips_alt_handle* hd = nullptr;
        int st = dips_alt_create(&p, w, h, 0, &hd);
        if (st != DIPS_OK) return alt_error(nullptr, "dips_alt_create", st);
        st = dips_alt_run(hd, in.p, (uint32_t)n, mk, (uint32_t)markers.size(), outbuf.data());
        const int rc = st != DIPS_OK ? alt_error(hd, "dips_alt_run", st) : 0;
        dips_alt_destroy(hd);
        if (rc != 0) return rc;
    } else {
        std::vector<dips_comm*> comms;
        int rc = make_comms(transport, ranks, comms);
        if (rc != 0) return rc;
        rc = on_ranks(ranks, n, "dips_alt_run_sharded",
                      [&](uint32_t r, uint64_t first, uint32_t count, std::string& why) {
                          dips_alt_handle* hd = nullptr;
                          int s2 = dips_alt_create(&p, w, h, transport == "rccl" ? (int)r : 0, &hd);
                          if (s2 != DIPS_OK) {
                              why = dips_alt_last_error(nullptr);
                              return s2;
                          }
                          s2 = dips_alt_run_sharded(hd, comms[r], in.p + first * fb, count, n, mk,
                                                    (uint32_t)markers.size(), outbuf.data() + first * fb);
                          if (s2 != DIPS_OK) why = dips_alt_last_error(hd);
                          dips_alt_destroy(hd);
                          return s2;
                      });
        for (auto* c : comms) dips_comm_destroy(c);
        if (rc != 0) return rc;
    }
    return write_all(argv[5], outbuf.data(), outbuf.size()) ? 0 : 1;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) return usage();
    const std::string cmd = argv[1];
    if (cmd == "callback") return run_callback(argc, argv);
    if (cmd == "series") return run_series(argc, argv);
    if (cmd == "sharded") return run_sharded(argc, argv);
    if (cmd == "alt") return run_alt(argc, argv);
    return usage();
}
