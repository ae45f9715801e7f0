// Per-launch time of a 1-read + 1-write fp32 stream (the activation QDQ's shape) by tensor size,
// with Q 16-B quads per lane in one tile per workgroup (quads kBlock apart, all loads issued first)
// for Q = 1, 2, 4: does a longer-lived workgroup cut the fixed cost per launch that the bench's
// small activations pay (tools/runs/r05/gpu_r05_ap.sh: 51 MB at 4.6 TB/s, 1.6 GB at 6.4)?
// 100 back-to-back launches on one stream per case, HIP events around them.
//   hipcc -O3 --offload-arch=gfx950 tools/studies/tile_quads_probe.hip -o tools/studies/tile_quads_probe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                  \
    do                                                                            \
    {                                                                             \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess)                                                     \
        {                                                                         \
            fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));       \
            return 1;                                                             \
        }                                                                         \
    } while (0)

template <int Q>
__global__ __launch_bounds__(256) void tile_kernel(const f4* __restrict__ in, f4* __restrict__ out, uint32_t nq,
                                                   float a, float b)
{
    const uint32_t q0 = blockIdx.x * (256 * Q) + threadIdx.x;
    f4 v[Q];
#pragma unroll
    for (int u = 0; u < Q; ++u)
        if (q0 + u * 256 < nq)
            v[u] = __builtin_nontemporal_load(in + q0 + u * 256);
#pragma unroll
    for (int u = 0; u < Q; ++u)
        if (q0 + u * 256 < nq)
            __builtin_nontemporal_store(v[u] * a + b, out + q0 + u * 256);
}

int main()
{
    const uint64_t sizes[] = {1605632, 3211264, 6422528, 12845056, 25690112, 51380224};   // bench's quads
    const uint64_t maxq    = 51380224;
    f4 *in, *out;
    CHECK(hipMalloc(&in, maxq * 16));
    CHECK(hipMalloc(&out, maxq * 16));
    CHECK(hipMemset(in, 0, maxq * 16));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const int reps = 100;
    for (int pass = 0; pass < 2; ++pass)
        for (uint64_t nq : sizes)
            for (int Q : {1, 2, 4})
            {
                const unsigned grid = (unsigned) ((nq + 256 * Q - 1) / (256 * Q));
                auto go = [&] {
                    if (Q == 1)
                        tile_kernel<1><<<grid, 256>>>(in, out, (uint32_t) nq, 0.5f, 1.0f);
                    else if (Q == 2)
                        tile_kernel<2><<<grid, 256>>>(in, out, (uint32_t) nq, 0.5f, 1.0f);
                    else
                        tile_kernel<4><<<grid, 256>>>(in, out, (uint32_t) nq, 0.5f, 1.0f);
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
                const double us = ms * 1e3 / reps, mb = nq * 32.0 / 1e6;
                printf("{\"pass\": %d, \"quads_per_lane\": %d, \"elems\": %llu, \"MB\": %.1f, \"us_per_launch\": %.2f, "
                       "\"TBps\": %.3f}\n",
                       pass, Q, (unsigned long long) (nq * 4), mb, us, mb / us);
                fflush(stdout);
            }
    CHECK(hipFree(in));
    CHECK(hipFree(out));
    return 0;
}
