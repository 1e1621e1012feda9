// knobs.hpp -- the library's reads of the process environment.
//
// A release build (the Makefile's default) reads exactly the runtime settings listed in
// kRuntimeSettings below (INTEGRATION.md documents them): every other ADMM_* name in the sources is
// an A/B knob for experiments, compiled to its default unless the library is built with
// -DADMM_AB_BUILD=1 (tools/build_variant.sh).  So a stray environment variable in a user's job cannot
// change kernels, launch shapes or speed.  tests/test_capi_symbols.py scans csrc/ for every
// environment read and checks this split.
#pragma once
#include <cstdlib>

#ifndef ADMM_AB_BUILD
#define ADMM_AB_BUILD 0
#endif

namespace admm_knobs {
inline int env_raw(const char* name, int dflt) {
    const char* s = std::getenv(name);
    return s ? std::atoi(s) : dflt;
}
// the release build's runtime settings (names only; read through env_setting):
//   ADMM_GEN_STREAMS  plane parts (streams) of a generic-size aniso inference solve, 1..4 (default 2)
constexpr const char* kRuntimeSettings[] = {"ADMM_GEN_STREAMS"};
}  // namespace admm_knobs

// an A/B knob: its default in a release build
inline int env_int(const char* name, int dflt) { return ADMM_AB_BUILD ? admm_knobs::env_raw(name, dflt) : dflt; }
// a documented runtime setting (admm_knobs::kRuntimeSettings)
inline int env_setting(const char* name, int dflt) { return admm_knobs::env_raw(name, dflt); }
