// Internal helpers shared by the engine and the run driver (not part of the ABI).
#pragma once
#include <stddef.h>

#include "gol_amd.h"

namespace golint {
long long engine_turn(gol_ctx *c);
int engine_device(gol_ctx *c);
}  // namespace golint

// Exported for the CPU tests only (tests/test_abi.py), not declared in include/gol_amd.h: the
// mapping gol_run_start applies to a peer-access call's HIP result (gol_run.cpp).
extern "C" int gol_internal_peer_access_status(const char *call, int hip_error,
                                               const char *hip_name, int dev_a, int dev_b,
                                               char *msg, size_t cap);
