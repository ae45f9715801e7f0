// Whether software pipelining lets the AdaRound backward's stream (3 x 16-B nontemporal reads + 1
// x 16-B write per quad, 2^28 fp32 elements) hide its arithmetic: `work` FMAs per element (four
// independent chains per quad, the kernel's ~120 VALU per element is ~2x the FMA count here in
// issue cycles) in
//   tile   -- one 256-quad tile per workgroup (the library's launch),
//   chunk  -- persistent: every workgroup owns a contiguous run of tiles and issues tile k+1's
//             loads before tile k's arithmetic (register double buffer),
//   chunkN -- the same without the prefetch (loads, arithmetic, store per tile).
// Prints one JSON line per case.
//   hipcc -O3 --offload-arch=gfx950 tools/studies/stream_pipe.hip -o tools/studies/stream_pipe
//   tools/studies/stream_pipe [knee]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

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

__device__ __forceinline__ f4 work_on(f4 a, f4 b, f4 c, int work, float m)
{
    f4 v = a + b * c;
#pragma unroll 4
    for (int k = 0; k < work; ++k)
        v = __builtin_elementwise_fma(v, f4 {m, m, m, m}, f4 {0.5f, 0.5f, 0.5f, 0.5f});
    return v;
}

__global__ __launch_bounds__(256) void tile_kernel(const f4* __restrict__ a, const f4* __restrict__ b,
                                                   const f4* __restrict__ c, f4* __restrict__ out, uint32_t nq,
                                                   int work, float m)
{
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= nq)
        return;
    const f4 x = __builtin_nontemporal_load(a + i), y = __builtin_nontemporal_load(b + i),
             z = __builtin_nontemporal_load(c + i);
    __builtin_nontemporal_store(work_on(x, y, z, work, m), out + i);
}

template <bool PREFETCH>
__global__ __launch_bounds__(256) void chunk_kernel(const f4* __restrict__ a, const f4* __restrict__ b,
                                                    const f4* __restrict__ c, f4* __restrict__ out, uint32_t nq,
                                                    uint32_t tiles_per_wg, int work, float m)
{
    const uint32_t t0 = blockIdx.x * tiles_per_wg;
    const uint32_t ntile = (nq + 255) / 256;
    const uint32_t t1 = t0 + tiles_per_wg < ntile ? t0 + tiles_per_wg : ntile;
    if (t0 >= t1)
        return;
    uint32_t i = t0 * 256 + threadIdx.x;
    f4 x, y, z;
    if (i < nq)
    {
        x = __builtin_nontemporal_load(a + i);
        y = __builtin_nontemporal_load(b + i);
        z = __builtin_nontemporal_load(c + i);
    }
    for (uint32_t t = t0; t < t1; ++t)
    {
        const uint32_t cur = i;
        const f4 cx = x, cy = y, cz = z;
        i += 256;
        if (PREFETCH && t + 1 < t1 && i < nq)
        {
            x = __builtin_nontemporal_load(a + i);
            y = __builtin_nontemporal_load(b + i);
            z = __builtin_nontemporal_load(c + i);
        }
        if (cur < nq)
            __builtin_nontemporal_store(work_on(cx, cy, cz, work, m), out + cur);
        if (!PREFETCH && t + 1 < t1 && i < nq)
        {
            x = __builtin_nontemporal_load(a + i);
            y = __builtin_nontemporal_load(b + i);
            z = __builtin_nontemporal_load(c + i);
        }
    }
}

int main(int argc, char** argv)
{
    // "knee": the tile form only, at heavier arithmetic (where the stream stops hiding it)
    const bool knee = argc > 1;
    const uint64_t n = 1ull << 28, nq = n / 4, bytes = n * 4;
    f4* buf[4];
    for (int k = 0; k < 4; ++k)
    {
        CHECK(hipMalloc(&buf[k], bytes));
        CHECK(hipMemset(buf[k], 0, bytes));
    }
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const int reps = 10;
    const uint32_t ntile = (uint32_t) (nq / 256);
    const int works_all[]  = {0, 30, 60, 90};
    const int works_knee[] = {90, 120, 150, 180, 240, 300};
    for (int work : knee ? std::vector<int>(works_knee, works_knee + 6) : std::vector<int>(works_all, works_all + 4))
    {
        for (int form = 0; form < (knee ? 1 : 7); ++form)
        {
            // form 0: tile; 1-3: chunk with prefetch at 2 / 4 / 8 workgroups per CU-resident slot;
            // 4-6: the same without prefetch
            uint32_t tpw = 1, grid = ntile;
            const char* name = "tile";
            if (form > 0)
            {
                const uint32_t wgs = 256u * (form == 1 || form == 4 ? 8u : (form == 2 || form == 5 ? 16u : 32u));
                tpw  = (ntile + wgs - 1) / wgs;
                grid = (ntile + tpw - 1) / tpw;
                name = form <= 3 ? "chunk" : "chunkN";
            }
            auto launch = [&]() {
                if (form == 0)
                    tile_kernel<<<grid, 256>>>(buf[0], buf[1], buf[2], buf[3], (uint32_t) nq, work, 0.999f);
                else if (form <= 3)
                    chunk_kernel<true><<<grid, 256>>>(buf[0], buf[1], buf[2], buf[3], (uint32_t) nq, tpw, work, 0.999f);
                else
                    chunk_kernel<false><<<grid, 256>>>(buf[0], buf[1], buf[2], buf[3], (uint32_t) nq, tpw, work, 0.999f);
            };
            launch();
            CHECK(hipDeviceSynchronize());
            CHECK(hipEventRecord(e0, nullptr));
            for (int r = 0; r < reps; ++r)
                launch();
            CHECK(hipEventRecord(e1, nullptr));
            CHECK(hipEventSynchronize(e1));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            ms /= reps;
            const double gbs = 16.0 * n / (ms * 1e-3) / 1e9;
            printf("{\"form\": \"%s\", \"grid\": %u, \"tiles_per_wg\": %u, \"fma_per_elem\": %d, \"avg_ms\": %.4f, "
                   "\"GBps\": %.1f, \"frac_of_8TBps\": %.4f}\n",
                   name, grid, tpw, work, ms, gbs, gbs / 8000.0);
            fflush(stdout);
        }
    }
    return 0;
}
