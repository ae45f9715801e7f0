// read_ceiling.hip -- the raw streaming-read rate of a list of device buffers (no reduction, no
// LDS): 16-B nontemporal loads, 4 in flight per lane, one 16-KiB tile per workgroup, one launch
// over all buffers (tile -> buffer table). tools/studies/read_ceiling.py compares it with minmax_many.
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

// variant 1: the raw read + a block min/max (wave shuffles, LDS, one partial per tile)
// variant 2: variant 1 + a per-tile gate read through a second dependent load (like pdf_init)
// variant 3: variant 1 with one partial per WAVE (no LDS, no barrier)
template <int V>
__global__ __launch_bounds__(256) void mm_many(const Buf* __restrict__ bufs, const uint16_t* __restrict__ tab,
                                               const int* __restrict__ gate, float2* __restrict__ part)
{
    const Buf b = bufs[tab[blockIdx.x]];
    if (V == 2 && gate[tab[blockIdx.x]])
        return;
    const int64_t base = (int64_t) (blockIdx.x - b.tile0) * 1024 + threadIdx.x;
    float mn = INFINITY, mx = -INFINITY;
    f4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
    {
        const int64_t i = base + u * 256;
        v[u] = i < b.nq ? __builtin_nontemporal_load(b.p + i) : f4 {NAN, NAN, NAN, NAN};
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
    {
        mn = fminf(fminf(mn, v[u].x), fminf(v[u].y, fminf(v[u].z, v[u].w)));
        mx = fmaxf(fmaxf(mx, v[u].x), fmaxf(v[u].y, fmaxf(v[u].z, v[u].w)));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
    {
        mn = fminf(mn, __shfl_xor(mn, o, 64));
        mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    }
    if (V == 3)
    {
        if ((threadIdx.x & 63) == 0)
            part[blockIdx.x * 4 + (threadIdx.x >> 6)] = make_float2(-mn, mx);
        return;
    }
    __shared__ float smn[4], smx[4];
    if ((threadIdx.x & 63) == 0)
    {
        smn[threadIdx.x >> 6] = mn;
        smx[threadIdx.x >> 6] = mx;
    }
    __syncthreads();
    if (threadIdx.x == 0)
    {
        for (int i = 1; i < 4; ++i)
        {
            mn = fminf(mn, smn[i]);
            mx = fmaxf(mx, smx[i]);
        }
        part[blockIdx.x] = make_float2(-mn, mx);
    }
}

extern "C" int mm_many_v(int variant, const Buf* bufs_dev, const uint16_t* tab_dev, int64_t tiles, const int* gate,
                         float2* part, void* stream)
{
    if (variant == 1)
        mm_many<1><<<(unsigned) tiles, 256, 0, (hipStream_t) stream>>>(bufs_dev, tab_dev, gate, part);
    else if (variant == 2)
        mm_many<2><<<(unsigned) tiles, 256, 0, (hipStream_t) stream>>>(bufs_dev, tab_dev, gate, part);
    else
        mm_many<3><<<(unsigned) tiles, 256, 0, (hipStream_t) stream>>>(bufs_dev, tab_dev, gate, part);
    return (int) hipGetLastError();
}

extern "C" int read_many(const Buf* bufs_dev, const uint16_t* tab_dev, int64_t tiles, float* out, void* stream)
{
    rd_many<<<(unsigned) tiles, 256, 0, (hipStream_t) stream>>>(bufs_dev, tab_dev, out);
    return (int) hipGetLastError();
}
