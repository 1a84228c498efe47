// tuning.hpp -- environment overrides of measured defaults, for A/B builds only.
//
// A product build (the default `make`) reads no environment variable: every
// knob below is its measured default, and the codec handle stays the
// immutable, thread-safe object the reference's `static final` codec is
// (ReedSolomonEncoder.java:17).  `make TUNING=1` defines RSAMD_TUNING_ENV=1
// and lets the RSAMD_* variables named at each use override the default, which
// is how the A/B scripts under tools/ compare choices on one box.
#pragma once

#include <cstddef>
#include <cstdlib>

#ifndef RSAMD_TUNING_ENV
#define RSAMD_TUNING_ENV 0
#endif

namespace rsamd {

// The value of environment variable `name` in a TUNING=1 build, else nullptr.
inline const char *tuning_env(const char *name) {
#if RSAMD_TUNING_ENV
    return std::getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}

// A size knob: the variable's value in a TUNING=1 build (read at each call,
// so a sweep can change it between launches), else `dflt`.
inline size_t tuning_size(const char *name, size_t dflt) {
    const char *e = tuning_env(name);
    return e ? size_t(std::strtoull(e, nullptr, 10)) : dflt;
}

}  // namespace rsamd
