// mz_mcclendon.h — McClendon difficulty of resident mazes (mz_mcclendon.hip).
// Kept out of mz_kernels.h: that header is part of k_step's source hash (bench.py
// KSTEP_SOURCES), which decides whether the committed PMC traffic record still applies.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "mz_common.h"

// out[i] = {prod, sum} of instance ids[i] (ids null: i); status[i] 0 ok, 1 not a tree, 2 outside
// the kernel's cases (host restatement), 3 invalid. Toroidal handles: the bordered maze.
// limit (device, nullable): only i < min(*limit, n / mult) * mult are scored (the rest untouched).
size_t mz_mcclendon_lds(int P, bool toroidal, int* mm);
hipError_t mz_launch_mcclendon(const MzDev& d, const int32_t* ids, int n, double* out,
                               int32_t* status, hipStream_t s, const int* limit = nullptr,
                               int mult = 1);
// Host restatement (mz_difficulty.hip): *prod = prod_b (C_b + 1) * C_0 of a grid (0 wall, 1 open,
// 2 goal), the quantity k_mcclendon outputs; MZ_OK or an error code.
int mz_mcclendon_host_prod(const uint8_t* g, int32_t H, int32_t W, int32_t sr, int32_t sc,
                           int32_t gr, int32_t gc, double* prod);
