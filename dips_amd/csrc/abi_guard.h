// abi_guard.h -- the exception barrier of every extern "C" entry point
// (internal to libdips_hip.so).
//
// no exception or panic crosses the ABI.  A Rust caller
// (rust/dips-hip) aborts on a foreign unwind and a C caller has no handler
// at all, so each exported function's body runs inside dips_abi::guard:
// std::bad_alloc becomes DIPS_ERR_NOMEM, any other C++ exception
// DIPS_ERR_INTERNAL, and the message goes where dips_last_error /
// dips_alt_last_error read it.  tests/test_abi_guard.py parses the sources
// and checks that every function include/dips_hip.h declares is written as
// `{ return dips_abi::guard(h, [&]() -> T { ... }); }`.
//
// The reference swallows or panics instead (dips/src/gpu/mod.rs:189, :206
// ignore add_texture's errors; wgpu panics on device errors); the ABI turns
// both into statuses and leaves the choice to the binding (rust/dips-hip:
// try_* methods return them, the reference-shaped ones panic).
#pragma once

#include <cstddef>
#include <exception>
#include <limits>
#include <new>
#include <type_traits>

#include "../../include/dips_hip.h"

struct dips_handle;
struct dips_alt_handle;
struct dips_comm;

namespace dips_abi {

// Where a caught exception's message goes: the handle's error string, or
// the process-wide creation error of dips_create / dips_alt_create (their
// handle does not exist yet).  Defined next to each handle type; they never
// throw (a failed string assignment leaves the old message).
struct CreateTag {};
struct AltCreateTag {};
struct CommCreateTag {};
void note_error(dips_handle* h, const char* msg) noexcept;
void note_error(dips_alt_handle* h, const char* msg) noexcept;
void note_error(dips_comm* c, const char* msg) noexcept;
void note_error(CreateTag, const char* msg) noexcept;
void note_error(AltCreateTag, const char* msg) noexcept;
void note_error(CommCreateTag, const char* msg) noexcept;
// read-only handles and handle-free functions have nowhere to write
inline void note_error(const dips_handle*, const char*) noexcept {}
inline void note_error(const dips_alt_handle*, const char*) noexcept {}
inline void note_error(const dips_comm*, const char*) noexcept {}
inline void note_error(std::nullptr_t, const char*) noexcept {}

// The value a function of return type R gives for a caught exception.
template <typename R>
R on_exception(dips_status st) noexcept {
    if constexpr (std::is_void_v<R>) {
        return;
    } else if constexpr (std::is_same_v<R, dips_status> || std::is_same_v<R, int>) {
        return static_cast<R>(st);
    } else if constexpr (std::is_floating_point_v<R>) {
        return std::numeric_limits<R>::quiet_NaN();
    } else if constexpr (std::is_same_v<R, const char*>) {
        return "internal error";
    } else {
        static_assert(std::is_void_v<R>, "no error value for this return type");
    }
}

// The calling thread's current HIP device, put back on exit: an entry point
// binds its handle's device (hipSetDevice) and must not leave the caller --
// torch, another library, the rank thread of another GPU -- on it.  Host-only
// functions (guard(nullptr, ...)) skip it and never touch the HIP runtime.
// current_device / set_device are the HIP calls (dips_abi.hip); -1 = none.
int current_device() noexcept;
void set_device(int dev) noexcept;
struct DeviceRestore {
    int dev;
    DeviceRestore() noexcept : dev(current_device()) {}
    ~DeviceRestore() {
        if (dev >= 0 && current_device() != dev) set_device(dev);
    }
    DeviceRestore(const DeviceRestore&) = delete;
    DeviceRestore& operator=(const DeviceRestore&) = delete;
};
struct NoRestore {};

template <typename Where, typename Body>
auto guard(Where where, Body&& body) noexcept -> decltype(body()) {
    using R = decltype(body());
    [[maybe_unused]] std::conditional_t<std::is_same_v<std::decay_t<Where>, std::nullptr_t>, NoRestore, DeviceRestore>
        restore;
    try {
        return body();
    } catch (const std::bad_alloc&) {
        note_error(where, "host allocation failed (std::bad_alloc)");
        return on_exception<R>(DIPS_ERR_NOMEM);
    } catch (const std::exception& ex) {
        note_error(where, ex.what());
        return on_exception<R>(DIPS_ERR_INTERNAL);
    } catch (...) {
        note_error(where, "unknown C++ exception");
        return on_exception<R>(DIPS_ERR_INTERNAL);
    }
}

}  // namespace dips_abi
