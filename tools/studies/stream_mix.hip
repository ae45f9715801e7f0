// The HBM rate of the AdaRound backward's stream shape without its arithmetic: R 16-B nontemporal
// read streams + one 16-B nontemporal write stream over 2^28 fp32 elements, grid-stride over 8192
// workgroups of 256 (the backward's launch) or one 256-quad tile per workgroup, with `work` dependent FMAs per element added between
// the loads and the store (0 = a pure stream), and the buffers' start addresses optionally skewed
// against each other (skew k x S bytes for buffer k). Prints one JSON line per case.
//   hipcc -O3 --offload-arch=gfx950 tools/studies/stream_mix.hip -o tools/studies/stream_mix
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                       \
    do                                                                                 \
    {                                                                                  \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess)                                                          \
        {                                                                              \
            fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));            \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

template <int R>
__global__ __launch_bounds__(256) void stream_kernel(const f4* __restrict__ a, const f4* __restrict__ b,
                                                     const f4* __restrict__ c, f4* __restrict__ out, uint32_t nq,
                                                     int work, float m)
{
    const uint32_t stride = gridDim.x * 256;
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < nq; i += stride)
    {
        f4 v = __builtin_nontemporal_load(a + i);
        if (R > 1)
            v += __builtin_nontemporal_load(b + i);
        if (R > 2)
            v += __builtin_nontemporal_load(c + i);
#pragma unroll 4
        for (int k = 0; k < work; ++k)
            v = __builtin_elementwise_fma(v, f4 {m, m, m, m}, f4 {0.5f, 0.5f, 0.5f, 0.5f});
        __builtin_nontemporal_store(v, out + i);
    }
}

int main()
{
    const uint64_t n = 1ull << 28, nq = n / 4, bytes = n * 4;
    const uint64_t skews[] = {0, 4096 + 256, (2ull << 20) + 4096 + 256};
    const uint64_t pad    = 3 * ((2ull << 20) + 8192);
    char* raw[4];
    for (int k = 0; k < 4; ++k)
    {
        CHECK(hipMalloc(&raw[k], bytes + pad));
        CHECK(hipMemset(raw[k], 0, bytes + pad));
    }
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const int reps = 10;
    for (int grid : {8192, (int) (nq / 256)})
    for (uint64_t s : skews)
        for (int R : {1, 2, 3})
            for (int work : {0, 8, 16, 32, 58})
            {
                const f4* p[3];
                for (int k = 0; k < 3; ++k)
                    p[k] = reinterpret_cast<const f4*>(raw[k] + k * s);
                f4* o     = reinterpret_cast<f4*>(raw[3] + 3 * s);
                auto go   = [&] {
                    if (R == 1)
                        stream_kernel<1><<<grid, 256>>>(p[0], p[1], p[2], o, (uint32_t) nq, work, 0.999f);
                    else if (R == 2)
                        stream_kernel<2><<<grid, 256>>>(p[0], p[1], p[2], o, (uint32_t) nq, work, 0.999f);
                    else
                        stream_kernel<3><<<grid, 256>>>(p[0], p[1], p[2], o, (uint32_t) nq, work, 0.999f);
                };
                go();
                CHECK(hipDeviceSynchronize());
                CHECK(hipEventRecord(e0));
                for (int r = 0; r < reps; ++r)
                    go();
                CHECK(hipEventRecord(e1));
                CHECK(hipEventSynchronize(e1));
                CHECK(hipGetLastError());
                float ms = 0;
                CHECK(hipEventElapsedTime(&ms, e0, e1));
                ms /= reps;
                const double gbs = (double) (R + 1) * bytes / (ms * 1e-3) / 1e9;
                printf("{\"grid\": %d, \"reads\": %d, \"writes\": 1, \"fma_per_elem\": %d, \"skew_bytes\": %llu, \"avg_ms\": %.4f, "
                       "\"GBps\": %.1f, \"frac_of_8TBps\": %.4f}\n",
                       grid, R, work, (unsigned long long) s, ms, gbs, gbs / 8000.0);
                fflush(stdout);
            }
    for (int k = 0; k < 4; ++k)
        CHECK(hipFree(raw[k]));
    return 0;
}
