// yk_train_amp.h - the mixed-precision train step (yk_train_amp.hip) as the f32 trainer
// (yk_train.hip) drives it: NNetWrapper.train under autocast('cuda') + GradScaler
// (yacht/NNet.py:113-116, 141-155) on hand-written fp16 MFMA kernels with f32 accumulation.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "yacht_hip.h"

namespace yk {

struct AmpTrain;  // device buffers of the mixed-precision step (fp16 weight copies, saved activations)

// P / G: the trainer's flat f32 parameter and gradient buffers in YachtNNet.state_dict() order,
// off[k]: offset of tensor k.  init_scale / growth_interval: GradScaler('cuda') (65536, 2000).
int amp_create(AmpTrain** out, int H, int NB, int Bmax, float* P, float* G, const long* off, float init_scale,
               int growth_interval);
void amp_destroy(AmpTrain* a);
// fp16 copies of every weight matrix (both MFMA operand orientations) from P
int amp_pack(AmpTrain* a, hipStream_t s);
// forward + backward of `B` examples into G (gradients of loss_scale x loss, each fp16-rounded as
// autocast's fp16 GEMMs return them); lrow[i] = (cross-entropy, squared value error) of row i,
// lsum = their column sums.  Dropout masks: rows are numbered row_base + i.  fuse_norm: the
// gradient launches also sum the unscaled sq-norm, and the next amp_apply uses it instead of
// re-reading G (only when nothing changes G in between: yk_trainer_step, not the DDP split).
int amp_backward(AmpTrain* a, const yk_state_t* states, const int32_t* targets, const float* values,
                 const int32_t* idx, int B, float dropout, uint64_t seed, uint64_t step, int64_t row_base,
                 float vloss_weight, float2* lrow, float* lsum, bool fuse_norm, hipStream_t s);
// GradScaler.unscale_ + clip_grad_norm_(max_norm) + AdamW step (skipped, with the scale halved,
// when a gradient is inf / nan) + GradScaler.update + fp16 repack.  sq_out: the unscaled grad
// sq-norm (double).  dropout / seed / next_step: the next backward's dropout draws, which the
// update launch makes ahead (for row offset 0) so that backward needs no mask launch of its own.
int amp_apply(AmpTrain* a, long nparams, float* M, float* V, double* sq_out, float max_norm, float lr, float wd,
              float b1, float b2, float eps, float dropout, uint64_t seed, uint64_t next_step, hipStream_t s);
// HOST out[4]: loss scale, growth tracker, optimiser steps taken, whether the last step found inf
int amp_state(AmpTrain* a, double* out);
int amp_set_steps(AmpTrain* a, int64_t steps);
int64_t amp_steps(AmpTrain* a);

}  // namespace yk
