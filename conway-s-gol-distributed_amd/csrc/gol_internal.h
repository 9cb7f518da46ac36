// Internal helpers shared by the engine and the run driver (not part of the ABI).
#pragma once
#include "gol_amd.h"

namespace golint {
long long engine_turn(gol_ctx *c);
int engine_device(gol_ctx *c);
}  // namespace golint
