// gol_limits.h — bounds shared by the host planner (golhip.hip) and the
// kernels (gol_kernels.hip).  Plain C++: the CPU suite compiles it with g++
// (tests/test_abi_cpu.py::test_resident_turn_bound).
#pragma once
#include <stdint.h>

namespace golk {

// Turns one resident launch (K1p, K1r) may take.  Their super-step arithmetic
// is 32-bit: J = ceil(turns / D), j * D and turns - j * D for depths D <= 64
// (lds_depth, persist depths); a step of more turns runs as several resident
// launches of at most this many (golhip.hip step_locked), so 10^10 turns
// (main.go's default) never wrap an int.
constexpr int64_t kResidentMaxTurns = int64_t(1) << 30;
constexpr int kResidentMaxDepth = 64;
static_assert(kResidentMaxTurns + 2 * kResidentMaxDepth < INT32_MAX, "resident turn arithmetic must fit in int32");

inline int64_t resident_turns(int64_t left, int64_t cap = kResidentMaxTurns) {
    if (cap > kResidentMaxTurns || cap < 1) cap = kResidentMaxTurns;  // (a test hook lowers it, never raises it)
    return left < cap ? left : cap;
}

}  // namespace golk
