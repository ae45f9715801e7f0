// Study: the AdaRound kernels' torch-CPU sigmoid (aimet_amd/csrc/adaround.hip: sigmoidf) in two
// forms, compared bit for bit over ALL 2^32 float inputs on the GPU:
//   old: Sleef expf_u10 with the two-multiply ldexp (vldexp2), then the IEEE division 1 / (e + 1);
//   new: the same polynomial with one v_ldexp_f32, then 1 / y as v_rcp_f32 + one Newton step for
//        y < 2^126 (the IEEE division beyond).
// The two ldexp forms differ only where exp(d) is subnormal (d < -87.3), where e + 1 == 1 in both.
// Also counts, over y in [1, 2^126), where the Newton reciprocal differs from the IEEE division.
// Vector stores and atomics only.
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt \
//         -o tools/studies/sigmoid_fast_check tools/studies/sigmoid_fast_check.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

__device__ __forceinline__ float poly(float d, int& q)
{
    const float qf = __builtin_rintf(d * 1.442695040888963407359924681001892137426645954152985934135449406931f);
    q              = (int) qf;
    float s        = __builtin_fmaf(qf, -0.693145751953125f, d);
    s              = __builtin_fmaf(qf, -1.428606765330187045e-06f, s);
    float u        = 0.000198527617612853646278381f;
    u              = __builtin_fmaf(u, s, 0.00139304355252534151077271f);
    u              = __builtin_fmaf(u, s, 0.00833336077630519866943359f);
    u              = __builtin_fmaf(u, s, 0.0416664853692054748535156f);
    u              = __builtin_fmaf(u, s, 0.166666671633720397949219f);
    u              = __builtin_fmaf(u, s, 0.5f);
    return 1.0f + __builtin_fmaf(s * s, u, s);
}

__device__ __forceinline__ float exp_old(float d)
{
    int q;
    float u      = poly(d, q);
    const int q1 = q >> 1, q2 = q - q1;
    u            = u * __int_as_float((q1 + 127) << 23);
    u            = u * __int_as_float((q2 + 127) << 23);
    u            = d < -104.0f ? 0.0f : u;
    return d > 100.0f ? __builtin_inff() : u;
}

__device__ __forceinline__ float exp_new(float d)
{
    int q;
    float u = __builtin_ldexpf(poly(d, q), q);
    u       = d < -104.0f ? 0.0f : u;
    return d > 100.0f ? __builtin_inff() : u;
}

__device__ __forceinline__ float rcp_nr(float y)
{
    const float r = __builtin_amdgcn_rcpf(y);
    return __builtin_fmaf(__builtin_fmaf(-y, r, 1.0f), r, r);
}

__global__ void check_sigmoid(unsigned long long* bad, uint32_t* first)
{
    for (uint64_t u = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x; u < (1ull << 32);
         u += (uint64_t) gridDim.x * blockDim.x)
    {
        const float a   = __uint_as_float((uint32_t) u);
        const float old = 1.0f / (exp_old(0.0f - a) + 1.0f);
        const float y   = exp_new(0.0f - a) + 1.0f;
        const float nw  = y < 0x1p126f ? rcp_nr(y) : 1.0f / y;
        if (__float_as_uint(old) != __float_as_uint(nw))
        {
            atomicAdd(bad, 1ull);
            atomicMin(first, (uint32_t) u);
        }
    }
}

__global__ void check_rcp(uint32_t lo, uint32_t hi, unsigned long long* bad, uint32_t* first)
{
    for (uint64_t u = lo + (uint64_t) blockIdx.x * blockDim.x + threadIdx.x; u < hi;
         u += (uint64_t) gridDim.x * blockDim.x)
    {
        const float y = __uint_as_float((uint32_t) u);
        if (__float_as_uint(rcp_nr(y)) != __float_as_uint(1.0f / y))
        {
            atomicAdd(bad, 1ull);
            atomicMin(first, (uint32_t) u);
        }
    }
}

int main()
{
    unsigned long long* bad;
    uint32_t* first;
    (void) hipMalloc(&bad, 8);
    (void) hipMalloc(&first, 4);
    unsigned long long h = 0;
    uint32_t f = 0;
    (void) hipMemset(bad, 0, 8);
    (void) hipMemset(first, 0xff, 4);
    check_rcp<<<8192, 256>>>(0x3f800000u, 0x7e800000u, bad, first);
    (void) hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost);
    (void) hipMemcpy(&f, first, 4, hipMemcpyDeviceToHost);
    printf("{\"check\": \"rcp + Newton == 1/y\", \"range\": \"[1, 2^126)\", \"patterns\": %u, \"mismatches\": %llu, "
           "\"first\": \"0x%08x\"}\n", 0x7e800000u - 0x3f800000u, h, f);
    (void) hipMemset(bad, 0, 8);
    (void) hipMemset(first, 0xff, 4);
    check_sigmoid<<<16384, 256>>>(bad, first);
    (void) hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost);
    (void) hipMemcpy(&f, first, 4, hipMemcpyDeviceToHost);
    printf("{\"check\": \"sigmoid new == old\", \"range\": \"all 2^32 inputs\", \"mismatches\": %llu, "
           "\"first\": \"0x%08x\"}\n", h, f);
    (void) hipFree(bad);
    (void) hipFree(first);
    return 0;
}
