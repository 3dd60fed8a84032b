/* vsrk data path: the batch assembly before the generator.
 *
 * The reference builds each training sample on CPU workers: temporal window
 * (acdc_vsr_dataset.py:59-76, acdc_misr_dataset.py:53-68), then the
 * augments RandomCropPatch / RandomHorizontalFlip / RandomVerticalFlip
 * (transforms.py:321-450) on numpy arrays.  Here the volumes stay resident
 * in HBM and one launch gathers a whole batch: for every output sample the
 * host resolves the sample's random draws (Python `random`, in the
 * reference's order) into an affine index map and the kernel copies
 *   dst[b, t, y, x] = src[vol, (t0 + t) mod T, y0 + dy*y, x0 + dx*x]
 * (cyclic temporal window, crop offset, flips as dy / dx = -1).  Pure
 * gathers: the result is bit-identical to the CPU pipeline.
 *
 * Same conventions as vsrk.h: int status (0 = ok), vsrk_last_error(),
 * caller-owned buffers, kernels on the caller's stream. */
#ifndef VSRK_DATA_H
#define VSRK_DATA_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* src: nvol volumes of T frames of (h, w) fp32, contiguous.
 * map: nb records of 6 int32 {vol, t0, y0, dy, x0, dx}; frames: frames per
 * output sample; dst: (nb, frames, oh, ow) fp32 contiguous.  Every source
 * index must stay inside its volume (checked on the host by the caller;
 * the kernel clamps nothing). */
int vsrk_gather_windows(const float* src, int32_t nvol, int32_t T, int32_t h, int32_t w, const int32_t* map,
                        int32_t nb, int32_t frames, int32_t oh, int32_t ow, float* dst, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* VSRK_DATA_H */
