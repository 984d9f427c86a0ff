// Self-feed state update shared by the device-resident rollouts
// (helper_scripts/infer_self_feed.py:182-194):
//   frame 0: record the initial state; frame f > 0: vel = pred[:, 3:] and
//   pos += pred[:, :3] (target "pos_dt+vel") or pos = pred[:, :3] (any other target, absolute)
// then write frame f of the [B, T, N, 3] trajectories.
#pragma once
#include "nbx_internal.h"

namespace nbx {

static __global__ void rollout_state_kernel(float* __restrict__ pos, float* __restrict__ vel,
                                            const float* __restrict__ out, int64_t V, int N, int64_t frame,
                                            int64_t num_frames, float* __restrict__ tp, float* __restrict__ tv,
                                            int absolute) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= V * 3) return;
    const int64_t node = i / 3;
    const int k = (int)(i - node * 3);
    float p = pos[i], v = vel[i];
    if (frame > 0) {
        p = absolute ? out[6 * node + k] : p + out[6 * node + k];
        v = out[6 * node + 3 + k];
        pos[i] = p;
        vel[i] = v;
    }
    const int64_t b = node / N, d = node - b * N;
    const int64_t o = ((b * num_frames + frame) * N + d) * 3 + k;
    tp[o] = p;
    tv[o] = v;
}

}  // namespace nbx
