// Probe: torch fused-Adam per-element arithmetic, with and without FMA contraction (tools/studies/adam_probe.py).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>

struct A { double lr, b1, b2, eps; };

__device__ float adam_c(float param, float grad, float& m, float& v, A a, float bc1, float bc2s)
{
    m = a.b1 * m + (1 - a.b1) * grad;
    v = a.b2 * v + (1 - a.b2) * grad * grad;
    const float step_size = a.lr / bc1;
    const float denom = (std::sqrt(v) / bc2s) + a.eps;
    param -= step_size * m / denom;
    return param;
}

__device__ float adam_nc(float param, float grad, float& m, float& v, A a, float bc1, float bc2s)
{
#pragma clang fp contract(off)
    m = a.b1 * m + (1 - a.b1) * grad;
    v = a.b2 * v + (1 - a.b2) * grad * grad;
    const float step_size = a.lr / bc1;
    const float denom = (std::sqrt(v) / bc2s) + a.eps;
    param -= step_size * m / denom;
    return param;
}

__device__ float m_variant(float m, float g, A a, int var)
{
    switch (var)
    {
    case 1: return (float) a.b1 * m + (float) (1 - a.b1) * g;                       // float
    case 2: return m + (float) (1 - a.b1) * (g - m);                                 // float lerp
    case 3: return (float) ((double) m + (1 - a.b1) * ((double) g - (double) m));   // double lerp
    case 4: return fmaf((float) (1 - a.b1), g, (float) a.b1 * m);                   // float fma other order
    case 5: return (float) fma(1 - a.b1, (double) g, a.b1 * (double) m);            // double fma other order
    case 6: { float w = (float) (1 - a.b1); return fabsf(w) < 0.5f ? fmaf(w, g - m, m) : g - (g - m) * (1 - w); }  // at::lerp
    default: return (float) (a.b1 * m + (1 - a.b1) * g);
    }
}

__global__ void k(float* p, const float* g, float* m, float* v, int n, int step, A a, int contract)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float sf = (float) step;
    const float bc1 = (float) (1 - pow(a.b1, (double) sf));
    const float bc2s = (float) sqrt(1 - pow(a.b2, (double) sf));
    float mm = m[i], vv = v[i];
    if (contract >= 10)
    {
        float m2 = m_variant(mm, g[i], a, contract - 10);
        float mm0 = mm;
        p[i] = adam_c(p[i], g[i], mm, vv, a, bc1, bc2s);
        (void) mm0;
        mm = m2;   // moments per variant; param from the default form (moment check only)
    }
    else
        p[i] = contract ? adam_c(p[i], g[i], mm, vv, a, bc1, bc2s) : adam_nc(p[i], g[i], mm, vv, a, bc1, bc2s);
    m[i] = mm; v[i] = vv;
}

extern "C" int adam_probe(float* p, const float* g, float* m, float* v, int n, int step, double lr, double b1,
                          double b2, double eps, int contract)
{
    A a {lr, b1, b2, eps};
    k<<<(n + 255) / 256, 256>>>(p, g, m, v, n, step, a, contract);
    return (int) hipDeviceSynchronize();
}
