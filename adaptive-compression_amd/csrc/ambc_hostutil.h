// ambc_hostutil.h -- error state, timing and tracing of the host code, free of
// HIP types (the CPU sanitizer harness, tests/native/, includes it too).
#pragma once
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>

namespace ambc {

extern thread_local std::string g_err;

inline int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

inline bool trace_on() {
    static int on = -1;
    if (on < 0) on = getenv("AMBC_TRACE") ? 1 : 0;
    return on == 1;
}
#define TRACE(...)                                                   \
    do {                                                             \
        if (::ambc::trace_on()) { fprintf(stderr, "[ambc] " __VA_ARGS__); fputc('\n', stderr); fflush(stderr); } \
    } while (0)

inline uint64_t now_ns() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

}  // namespace ambc
