// recon.hpp -- the AdaRound reconstruction-loss gradient of one output element, shared by the
// elementwise kernels (adaround.hip) and the fused depthwise step (dwconv.hip).
//
// adaround_loss.py:70-80: loss = mean over (N, spatial) of ||act(q) - act(t)||^2 over dim 1, so
// dloss/dq = scale * (act(q) - act(t)) * act'(q) with scale = 2 / (N * spatial).
// act: 0 none, 1 ReLU (torch threshold_backward: x > 0), 2 ReLU6 (hardtanh(0, 6) backward:
// 0 < x < 6).
#pragma once

namespace aimet_amd
{

__device__ __forceinline__ float recon_g(float q, float t, float scale, int act)
{
    float a = q, b = t, m = 1.0f;
    if (act == 1)
    {
        a = fmaxf(q, 0.0f);
        b = fmaxf(t, 0.0f);
        m = q > 0.0f ? 1.0f : 0.0f;
    }
    else if (act == 2)
    {
        a = fminf(fmaxf(q, 0.0f), 6.0f);
        b = fminf(fmaxf(t, 0.0f), 6.0f);
        m = (q > 0.0f && q < 6.0f) ? 1.0f : 0.0f;
    }
    return scale * (a - b) * m;
}

}   // namespace aimet_amd
