// Study: is fma(fma(-b, r, 1), r, r) with r = v_rcp_f32(b) the correctly rounded 1/b (== the IEEE
// division 1.0f / b) for every positive normal b? Exhaustive over the bit patterns on the GPU;
// counts mismatches over all normal b and over [1.5, 3] (the divisor range of Sleef's logkf
// df_div in aimet_amd/csrc/adaround.hip). Vector stores and atomics only.
//   hipcc -O3 --offload-arch=gfx950 -fhip-fp32-correctly-rounded-divide-sqrt -o tools/studies/rcp_newton_check tools/studies/rcp_newton_check.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void check(uint32_t lo, uint32_t hi, unsigned long long* bad, uint32_t* first)
{
    for (uint64_t u = lo + (uint64_t) blockIdx.x * blockDim.x + threadIdx.x; u < hi; u += (uint64_t) gridDim.x * blockDim.x)
    {
        const float b  = __uint_as_float((uint32_t) u);
        const float r  = __builtin_amdgcn_rcpf(b);
        const float r1 = __builtin_fmaf(__builtin_fmaf(-b, r, 1.0f), r, r);
        const float q  = 1.0f / b;
        if (__float_as_uint(r1) != __float_as_uint(q))
        {
            atomicAdd(bad, 1ull);
            atomicMin(first, (uint32_t) u);
        }
    }
}

static void run(uint32_t lo, uint32_t hi, const char* name)
{
    unsigned long long* bad;
    uint32_t* first;
    (void) hipMalloc(&bad, 8);
    (void) hipMalloc(&first, 4);
    (void) hipMemset(bad, 0, 8);
    (void) hipMemset(first, 0xff, 4);
    check<<<8192, 256>>>(lo, hi, bad, first);
    unsigned long long h = 0;
    uint32_t f = 0;
    (void) hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost);
    (void) hipMemcpy(&f, first, 4, hipMemcpyDeviceToHost);
    printf("{\"range\": \"%s\", \"patterns\": %u, \"mismatches\": %llu, \"first\": \"0x%08x\"}\n", name, hi - lo, h, f);
    (void) hipFree(bad);
    (void) hipFree(first);
}

int main()
{
    run(0x3fc00000u, 0x40400001u, "[1.5, 3]");
    run(0x00800000u, 0x7f800000u, "all positive normal");
    return 0;
}
