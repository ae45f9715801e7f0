// Error of f32 natural logarithms over every positive normal f32 x, against log((double) x):
//   hw   -- v_log_f32 (log2) * ln 2 in f32
//   hw2  -- v_log_f32 (log2), the product with ln 2 taken in double
// For each form: max |err| overall, max |err| / |ln x| where |ln x| >= 2^-6, and max |err| where
// |ln x| < 2^-6 (near 1), so that |err| <= A + R |ln x| can be stated with measured A and R.
//   hipcc -O3 --offload-arch=gfx950 tools/studies/log_f32_check.hip -o tools/studies/log_f32_check
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>

#define CK(x)                                                                      \
    do                                                                             \
    {                                                                              \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess)                                                      \
        {                                                                          \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                \
            return 1;                                                              \
        }                                                                          \
    } while (0)

struct Res
{
    double max_abs[2], max_rel[2], max_abs_near1[2];
};

__device__ void atomic_max_d(double* p, double v)
{
    unsigned long long* u = reinterpret_cast<unsigned long long*>(p);
    unsigned long long old = *u;
    while (__longlong_as_double(old) < v)
    {
        const unsigned long long prev = atomicCAS(u, old, __double_as_longlong(v));
        if (prev == old)
            break;
        old = prev;
    }
}

__global__ void check(uint32_t b0, Res* r)
{
    const uint32_t b = b0 + blockIdx.x * 256 + threadIdx.x;
    double ma[2] = {0, 0}, mr[2] = {0, 0}, mn[2] = {0, 0};
    if (b >= 0x00800000u && b < 0x7f800000u)   // positive normal floats
    {
        const float x    = __uint_as_float(b);
        const double ref = log((double) x);
        const float l2   = __builtin_amdgcn_logf(x);
        const double f[2] = {(double) (l2 * 0.693147182f), (double) l2 * 0.69314718055994531};
        for (int k = 0; k < 2; ++k)
        {
            const double e = fabs(f[k] - ref);
            ma[k]          = e;
            if (fabs(ref) >= 0.015625)
                mr[k] = e / fabs(ref);
            else
                mn[k] = e;
        }
    }
    for (int k = 0; k < 2; ++k)
        for (int o = 32; o > 0; o >>= 1)
        {
            ma[k] = fmax(ma[k], __shfl_xor(ma[k], o));
            mr[k] = fmax(mr[k], __shfl_xor(mr[k], o));
            mn[k] = fmax(mn[k], __shfl_xor(mn[k], o));
        }
    if ((threadIdx.x & 63) == 0)
        for (int k = 0; k < 2; ++k)
        {
            atomic_max_d(&r->max_abs[k], ma[k]);
            atomic_max_d(&r->max_rel[k], mr[k]);
            atomic_max_d(&r->max_abs_near1[k], mn[k]);
        }
}

int main()
{
    Res* d;
    CK(hipMalloc(&d, sizeof(Res)));
    CK(hipMemset(d, 0, sizeof(Res)));
    const uint32_t slice = 1u << 26;
    for (uint64_t b0 = 0; b0 < 0x7f800000ull; b0 += slice)
        check<<<slice / 256, 256>>>((uint32_t) b0, d);
    CK(hipDeviceSynchronize());
    Res h;
    CK(hipMemcpy(&h, d, sizeof(Res), hipMemcpyDeviceToHost));
    const char* names[2] = {"v_log_f32 * ln2 (f32)", "v_log_f32, * ln2 in double"};
    for (int k = 0; k < 2; ++k)
        printf("%-28s max |err| %.3e, max |err|/|ln x| (|ln x| >= 2^-6) %.3e = 2^%.2f, max |err| (|ln x| < 2^-6) %.3e = 2^%.2f\n",
               names[k], h.max_abs[k], h.max_rel[k], log2(h.max_rel[k]), h.max_abs_near1[k], log2(h.max_abs_near1[k]));
    return 0;
}
