// Debug checks inside libmim's kernels.  A shipped build compiles none of them; a debug build
// (MIM_DEBUG=1 at build time: build.py passes -DMIM_DEBUG) prints the failing check from the device.
// Every in-kernel diagnostic goes through this header: no other debug macros in the .hip sources.
#pragma once

// MIM_DEBUG_CHECK prints when the check fails, MIM_DEBUG_PRINT when the condition holds (probes)
#ifdef MIM_DEBUG
#define MIM_DEBUG_CHECK(cond, ...)          \
    do {                                    \
        if (!(cond)) printf(__VA_ARGS__);   \
    } while (0)
#define MIM_DEBUG_PRINT(cond, ...)          \
    do {                                    \
        if (cond) printf(__VA_ARGS__);      \
    } while (0)
#else
#define MIM_DEBUG_CHECK(cond, ...) \
    do {                           \
    } while (0)
#define MIM_DEBUG_PRINT(cond, ...) \
    do {                           \
    } while (0)
#endif
