// The depth-folded rolling forward: conv_roll.hip's kernel with 32-row tiles
// (8 waves x 4 rows) in the (kd, channel)-chunk form SP_FOLD, for a Conv3d
// 3x3x3 with one output depth from three input slices (DUF's last dense
// unit, duf_net.py:214).  A translation unit of its own: the tile height is a
// build constant of the rolling kernel, and the 3-D / 2-D forms keep 16 rows.
#define ROLL_RMS 4
#define ROLL_FOLD_TU 1
#include "conv_roll.hip"
