// Issue rates of the VALU operations the certified pow (sleef_pow.hpp) trades between: f32 FMA,
// packed f32 FMA, f64 FMA, f32<->f64 conversions. Each kernel runs 8 independent chains per lane
// (enough to cover the dependent-issue latency at 8 waves per SIMD) over a full grid; the rate is
// reported in wave-instructions per cycle per SIMD at the measured time and the nominal 2.4 GHz.
//   hipcc -O3 --offload-arch=gfx950 tools/studies/valu_rates.hip -o tools/studies/valu_rates
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kIters = 4096;
typedef float fl2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void k_fma32(float* out, float a)
{
    float v[8];
    for (int j = 0; j < 8; ++j)
        v[j] = threadIdx.x * 1e-3f + j;
    for (int i = 0; i < kIters; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j)
            v[j] = __builtin_fmaf(v[j], a, 0.5f);
    float s = 0;
    for (int j = 0; j < 8; ++j)
        s += v[j];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_pk32(float* out, float a)
{
    fl2 v[8];
    for (int j = 0; j < 8; ++j)
        v[j] = fl2 {threadIdx.x * 1e-3f + j, j * 0.5f};
    const fl2 av {a, a}, c {0.5f, 0.5f};
    for (int i = 0; i < kIters; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j)
            v[j] = __builtin_elementwise_fma(v[j], av, c);
    float s = 0;
    for (int j = 0; j < 8; ++j)
        s += v[j][0] + v[j][1];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_fma64(float* out, float a)
{
    double v[8];
    for (int j = 0; j < 8; ++j)
        v[j] = threadIdx.x * 1e-3 + j;
    const double ad = a;
    for (int i = 0; i < kIters; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j)
            v[j] = fma(v[j], ad, 0.5);
    double s = 0;
    for (int j = 0; j < 8; ++j)
        s += v[j];
    out[blockIdx.x * 256 + threadIdx.x] = (float) s;
}
// f32 -> f64 -> f32 round trips (two conversions per step, each dependent on the last)
__global__ __launch_bounds__(256) void k_cvt(float* out, float a)
{
    float v[8];
    for (int j = 0; j < 8; ++j)
        v[j] = threadIdx.x * 1e-3f + j + a;
    for (int i = 0; i < kIters; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j)
        {
            double d = (double) v[j];
            asm volatile("" : "+v"(d));
            v[j] = (float) d;
            asm volatile("" : "+v"(v[j]));
        }
    float s = 0;
    for (int j = 0; j < 8; ++j)
        s += v[j];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main()
{
    const int blocks = 256 * 8 * 4;   // 8 workgroups per CU, 4 rounds
    float* out;
    hipMalloc(&out, blocks * 256 * sizeof(float));
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    struct K
    {
        const char* name;
        void (*f)(float*, float);
        double insts_per_step;   // wave instructions per chain step
    } ks[] = {{"v_fma_f32", k_fma32, 1}, {"v_pk_fma_f32", k_pk32, 1}, {"v_fma_f64", k_fma64, 1},
              {"v_cvt_f64_f32 + v_cvt_f32_f64", k_cvt, 2}};
    for (auto& k : ks)
    {
        k.f<<<blocks, 256>>>(out, 0.999f);
        hipEventRecord(a);
        for (int r = 0; r < 5; ++r)
            k.f<<<blocks, 256>>>(out, 0.999f);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        ms /= 5;
        const double waves = blocks * 4.0, insts = waves * kIters * 8 * k.insts_per_step;
        const double per_simd_cycle = insts / (1024.0 * ms * 1e-3 * 2.4e9);
        std::printf("%-32s %.3f ms  %.3f wave-instructions / cycle / SIMD (2.4 GHz)  -> %.2f cycles each\n", k.name, ms,
                    per_simd_cycle, 1.0 / per_simd_cycle);
    }
    return 0;
}
