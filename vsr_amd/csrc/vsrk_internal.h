// Internal (non-ABI) helpers shared between the kernel translation units.
#pragma once
#include <algorithm>
#include "vsrk_common.h"

// Per-channel sum (mode 0) or sum + sum of squares (mode 1) over every voxel of
// a view; perm_r maps view channel -> torch channel.  Needs workspace of
// vsrk_channel_reduce_ws_bytes(c) bytes.
size_t vsrk_channel_reduce_ws_bytes(int c);
int vsrk_channel_reduce_internal(const vsrk_tensor5* x, int mode, int perm_r, float scale, float* sum,
                                 float* sumsq, int accumulate, void* ws, size_t ws_bytes, hipStream_t s);
