// read_ceiling.hip -- the raw streaming-read rate of a list of device buffers (no reduction, no
// LDS): 16-B nontemporal loads, 4 in flight per lane, one 16-KiB tile per workgroup, one launch
// over all buffers (tile -> buffer table). tools/read_ceiling.py compares it with minmax_many.
#include <hip/hip_runtime.h>
#include <cstdint>

typedef float f4 __attribute__((ext_vector_type(4)));
struct Buf { const f4* p; int64_t nq; int64_t tile0; };

__global__ __launch_bounds__(256) void rd_many(const Buf* __restrict__ bufs, const uint16_t* __restrict__ tab,
                                               float* __restrict__ out)
{
    const Buf b = bufs[tab[blockIdx.x]];
    const int64_t base = (int64_t) (blockIdx.x - b.tile0) * 1024 + threadIdx.x;
    float s = 0;
    f4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
    {
        const int64_t i = base + u * 256;
        v[u] = i < b.nq ? __builtin_nontemporal_load(b.p + i) : f4 {0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
        s += v[u].x + v[u].y + v[u].z + v[u].w;
    if (s == 12345.678f)
        out[0] = s;
}

extern "C" int read_many(const Buf* bufs_dev, const uint16_t* tab_dev, int64_t tiles, float* out, void* stream)
{
    rd_many<<<(unsigned) tiles, 256, 0, (hipStream_t) stream>>>(bufs_dev, tab_dev, out);
    return (int) hipGetLastError();
}
