// hist_variants.hip -- microbenchmark of the 512-bin histogram pass (UpdatePdf's GetHistogram) on
// gfx950 (tuning tool for stats.hip). Build:
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off \
//         -fhip-fp32-correctly-rounded-divide-sqrt -I include -I aimet_amd/csrc tools/studies/hist_variants.hip -o tools/studies/hist_variants
// Two inputs of n floats (default 205,520,896 = 256x64x112x112, ResNet-50's largest activation):
// relu(N(0,1)*1.5+0.2) (about half exact zeros) and N(0,1)*2 (no zeros). Every variant's counts
// are checked against the first variant bit for bit; median GB/s (4 B/elem) over interleaved rounds.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include <hip/hip_runtime.h>

#include "common.hpp"   // round_div_sub (reciprocal fast path)

#define CK(x)                                                                                                  \
    do                                                                                                         \
    {                                                                                                          \
        hipError_t e = (x);                                                                                    \
        if (e != hipSuccess)                                                                                   \
        {                                                                                                      \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);                                   \
            exit(1);                                                                                           \
        }                                                                                                      \
    } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int kBins = 512;

struct Binner
{
    float bucket, offset;
    __device__ __forceinline__ int bin(float x) const
    {
        float r = __builtin_roundf(x / bucket - offset);
        return (r >= 0.0f && r < (float) kBins) ? (int) r : -1;
    }
};

struct BinnerRcp
{
    float bucket, offset, rcp;
    __device__ __forceinline__ int bin(float x) const
    {
        float r = aimet_amd::round_div_sub(x, bucket, rcp, offset);
        return (r >= 0.0f && r < (float) kBins) ? (int) r : -1;
    }
};

// uniform-threshold fast path (stats.hip HistBinner): v = RN(RN(x*rcp) - off) is within
// 6u(|q|+|off|) of the reference's RN(RN(x/bucket) - off); away from half-integers by more than
// thr = (515 + 2|off|) 2^-21 (valid for |v| <= 513; beyond, both roundings are out of range)
// round-half-away(v*) == rint(v). v_fract + one compare instead of floor/abs/abs/add/mul.
struct BinnerFast
{
    float bucket, offset, rcp, thr;
    __device__ __forceinline__ int bin(float x) const
    {
        const float v = x * rcp - offset;
        const float h = __builtin_amdgcn_fractf(v);
        if (__builtin_fabsf(h - 0.5f) > thr)
        {
            const int r = (int) __builtin_rintf(v);
            return (unsigned) r < (unsigned) kBins ? r : -1;
        }
        float r = __builtin_roundf(x / bucket - offset);
        return (r >= 0.0f && r < (float) kBins) ? (int) r : -1;
    }
};

__device__ __forceinline__ uint32_t wave_sum(uint32_t v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
        v += __shfl_xor(v, o, 64);
    return v;
}

// COPIES: LDS histograms per block (1 = shared by the block, BLOCK/64 = one per wave)
template <int BLOCK, int UNROLL, int COPIES, bool NT, bool ZSKIP, bool PART = false, class B = Binner, int LSH = 6>
__global__ __launch_bounds__(BLOCK) void hist_var(const float* __restrict__ x, int64_t n, B bn,
                                                  unsigned long long* __restrict__ counts)
{
    __shared__ uint32_t lds[COPIES][kBins];
    const int copy = (threadIdx.x >> LSH) % COPIES;
    for (int i = threadIdx.x; i < COPIES * kBins; i += BLOCK)
        (&lds[0][0])[i] = 0;
    __syncthreads();
    const int zbin = bn.bin(0.0f);
    uint32_t zc    = 0;
    auto add = [&](float v) {
        if (ZSKIP && v == 0.0f)
        {
            ++zc;
            return;
        }
        int b = bn.bin(v);
        if (b >= 0)
            atomicAdd(&lds[copy][b], 1u);
    };
    const f4* x4         = reinterpret_cast<const f4*>(x);
    const int64_t nv     = n / 4;
    const int64_t stride = (int64_t) gridDim.x * BLOCK * UNROLL;
    for (int64_t base = (int64_t) blockIdx.x * BLOCK * UNROLL + threadIdx.x; base < nv; base += stride)
    {
        f4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
        {
            int64_t i = base + (int64_t) u * BLOCK;
            if (i < nv)
                v[u] = NT ? __builtin_nontemporal_load(x4 + i) : x4[i];
            else
                v[u] = f4 {NAN, NAN, NAN, NAN};
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
        {
            add(v[u].x);
            add(v[u].y);
            add(v[u].z);
            add(v[u].w);
        }
    }
    for (int64_t i = nv * 4 + (int64_t) blockIdx.x * BLOCK + threadIdx.x; i < n; i += (int64_t) gridDim.x * BLOCK)
        add(x[i]);
    if (ZSKIP)
    {
        zc = wave_sum(zc);
        if ((threadIdx.x & 63) == 0 && zbin >= 0 && zc)
            atomicAdd(&lds[copy][zbin], zc);
    }
    __syncthreads();
    for (int b = threadIdx.x; b < kBins; b += BLOCK)
    {
        uint32_t s = 0;
#pragma unroll
        for (int i = 0; i < COPIES; ++i)
            s += lds[i][b];
        if (PART)
            reinterpret_cast<uint32_t*>(counts + 1024)[(int64_t) blockIdx.x * kBins + b] = s;
        else if (s)
            atomicAdd(&counts[b], (unsigned long long) s);
    }
}

// replicated global counts: block b adds into replica (b % R); the last block to finish (atomic
// ticket) folds the R replicas into counts and re-zeroes them -- no second launch, R-fold less
// contention on the 512 global counters
template <int BLOCK, int UNROLL, int COPIES, int R>
__global__ __launch_bounds__(BLOCK) void hist_rep(const float* __restrict__ x, int64_t n, Binner bn,
                                                  unsigned long long* __restrict__ counts)
{
    __shared__ uint32_t lds[COPIES][kBins];
    __shared__ int is_last;
    unsigned long long* rep = counts + 1024;              // [R][512], zero on entry
    unsigned int* ticket    = reinterpret_cast<unsigned int*>(counts + 1024 + R * kBins);
    const int copy = (threadIdx.x >> 6) % COPIES;
    for (int i = threadIdx.x; i < COPIES * kBins; i += BLOCK)
        (&lds[0][0])[i] = 0;
    __syncthreads();
    const int zbin = bn.bin(0.0f);
    uint32_t zc    = 0;
    auto add = [&](float v) {
        if (v == 0.0f)
        {
            ++zc;
            return;
        }
        int b = bn.bin(v);
        if (b >= 0)
            atomicAdd(&lds[copy][b], 1u);
    };
    const f4* x4         = reinterpret_cast<const f4*>(x);
    const int64_t nv     = n / 4;
    const int64_t stride = (int64_t) gridDim.x * BLOCK * UNROLL;
    for (int64_t base = (int64_t) blockIdx.x * BLOCK * UNROLL + threadIdx.x; base < nv; base += stride)
    {
        f4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
        {
            int64_t i = base + (int64_t) u * BLOCK;
            v[u]      = i < nv ? __builtin_nontemporal_load(x4 + i) : f4 {NAN, NAN, NAN, NAN};
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
        {
            add(v[u].x);
            add(v[u].y);
            add(v[u].z);
            add(v[u].w);
        }
    }
    for (int64_t i = nv * 4 + (int64_t) blockIdx.x * BLOCK + threadIdx.x; i < n; i += (int64_t) gridDim.x * BLOCK)
        add(x[i]);
    zc = wave_sum(zc);
    if ((threadIdx.x & 63) == 0 && zbin >= 0 && zc)
        atomicAdd(&lds[copy][zbin], zc);
    __syncthreads();
    unsigned long long* mine = rep + (blockIdx.x % R) * kBins;
    for (int b = threadIdx.x; b < kBins; b += BLOCK)
    {
        uint32_t s = 0;
#pragma unroll
        for (int i = 0; i < COPIES; ++i)
            s += lds[i][b];
        if (s)
            atomicAdd(&mine[b], (unsigned long long) s);
    }
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0)
        is_last = atomicAdd(ticket, 1u) == gridDim.x - 1;
    __syncthreads();
    if (is_last)
    {
        __threadfence();
        for (int b = threadIdx.x; b < kBins; b += BLOCK)
        {
            unsigned long long s = 0;
            for (int r = 0; r < R; ++r)
                s += atomicExch(&rep[r * kBins + b], 0ull);
            if (s)
                counts[b] += s;
        }
        if (threadIdx.x == 0)
            *ticket = 0;
    }
}

template <int BLOCK, int UNROLL, int COPIES, int R, int GRID>
void launch_rep(const float* x, int64_t n, Binner bn, unsigned long long* c, hipStream_t s)
{
    int64_t need = (n / 4 + BLOCK * UNROLL - 1) / (BLOCK * UNROLL);
    int g        = (int) std::max<int64_t>(1, std::min<int64_t>(need, GRID));
    hist_rep<BLOCK, UNROLL, COPIES, R><<<g, BLOCK, 0, s>>>(x, n, bn, c);
}

// sum per-block partial rows [nrows][512] into counts (64-bit): 2-D grid of row slices
__global__ __launch_bounds__(256) void reduce_parts(const uint32_t* __restrict__ part, int nrows,
                                                    unsigned long long* __restrict__ counts)
{
    const int rows_per = (nrows + gridDim.x - 1) / gridDim.x;
    const int r0 = blockIdx.x * rows_per, r1 = min(nrows, r0 + rows_per);
    for (int b = threadIdx.x; b < kBins; b += 256)
    {
        unsigned long long s = 0;
        for (int r = r0; r < r1; ++r)
            s += part[(int64_t) r * kBins + b];
        if (s)
            atomicAdd(&counts[b], s);
    }
}

template <int BLOCK, int UNROLL, int GRID>
void launch_part(const float* x, int64_t n, Binner bn, unsigned long long* c, hipStream_t s)
{
    int64_t need = (n / 4 + BLOCK * UNROLL - 1) / (BLOCK * UNROLL);
    int g        = (int) std::max<int64_t>(1, std::min<int64_t>(need, GRID));
    hist_var<BLOCK, UNROLL, BLOCK / 64, true, true, true><<<g, BLOCK, 0, s>>>(x, n, bn, c);
    reduce_parts<<<std::min(g, 64), 256, 0, s>>>(reinterpret_cast<const uint32_t*>(c + 1024), g, c);
}

// run-length variant: each lane keeps (bin, count) of its current run and only touches LDS when
// the bin changes (hot bins of peaked distributions stop serialising the LDS atomics)
template <int BLOCK, int UNROLL, int COPIES>
__global__ __launch_bounds__(BLOCK) void hist_rl(const float* __restrict__ x, int64_t n, Binner bn,
                                                 unsigned long long* __restrict__ counts)
{
    __shared__ uint32_t lds[COPIES][kBins];
    const int copy = (threadIdx.x >> 6) % COPIES;
    for (int i = threadIdx.x; i < COPIES * kBins; i += BLOCK)
        (&lds[0][0])[i] = 0;
    __syncthreads();
    int cur = -1;
    uint32_t cnt = 0;
    auto add = [&](float v) {
        int b = bn.bin(v);
        if (b == cur)
            ++cnt;
        else
        {
            if (cur >= 0)
                atomicAdd(&lds[copy][cur], cnt);
            cur = b;
            cnt = 1;
        }
    };
    const f4* x4         = reinterpret_cast<const f4*>(x);
    const int64_t nv     = n / 4;
    const int64_t stride = (int64_t) gridDim.x * BLOCK * UNROLL;
    for (int64_t base = (int64_t) blockIdx.x * BLOCK * UNROLL + threadIdx.x; base < nv; base += stride)
    {
        f4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
        {
            int64_t i = base + (int64_t) u * BLOCK;
            v[u]      = i < nv ? __builtin_nontemporal_load(x4 + i) : f4 {NAN, NAN, NAN, NAN};
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
        {
            add(v[u].x);
            add(v[u].y);
            add(v[u].z);
            add(v[u].w);
        }
    }
    for (int64_t i = nv * 4 + (int64_t) blockIdx.x * BLOCK + threadIdx.x; i < n; i += (int64_t) gridDim.x * BLOCK)
        add(x[i]);
    if (cur >= 0)
        atomicAdd(&lds[copy][cur], cnt);
    __syncthreads();
    for (int b = threadIdx.x; b < kBins; b += BLOCK)
    {
        uint32_t s = 0;
#pragma unroll
        for (int i = 0; i < COPIES; ++i)
            s += lds[i][b];
        if (s)
            atomicAdd(&counts[b], (unsigned long long) s);
    }
}

template <int BLOCK, int UNROLL, int COPIES, int GRID>
void launch_rl(const float* x, int64_t n, Binner bn, unsigned long long* c, hipStream_t s)
{
    int64_t need = (n / 4 + BLOCK * UNROLL - 1) / (BLOCK * UNROLL);
    int g        = (int) std::max<int64_t>(1, std::min<int64_t>(need, GRID));
    hist_rl<BLOCK, UNROLL, COPIES><<<g, BLOCK, 0, s>>>(x, n, bn, c);
}

// min/max partials (stats.hip minmax_tensor_kernel shape)
template <int BLOCK, int UNROLL, bool NT>
__global__ __launch_bounds__(BLOCK) void minmax_var(const float* __restrict__ x, int64_t n, float2* __restrict__ part)
{
    const f4* x4         = reinterpret_cast<const f4*>(x);
    const int64_t nv     = n / 4;
    const int64_t stride = (int64_t) gridDim.x * BLOCK * UNROLL;
    float mn = INFINITY, mx = -INFINITY;
    for (int64_t base = (int64_t) blockIdx.x * BLOCK * UNROLL + threadIdx.x; base < nv; base += stride)
    {
        f4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
        {
            int64_t i = base + (int64_t) u * BLOCK;
            v[u]      = i < nv ? (NT ? __builtin_nontemporal_load(x4 + i) : x4[i]) : f4 {NAN, NAN, NAN, NAN};
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
        {
            mn = fminf(fminf(mn, v[u].x), fminf(v[u].y, fminf(v[u].z, v[u].w)));
            mx = fmaxf(fmaxf(mx, v[u].x), fmaxf(v[u].y, fmaxf(v[u].z, v[u].w)));
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
    {
        mn = fminf(mn, __shfl_xor(mn, o, 64));
        mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    }
    __shared__ float smn[BLOCK / 64], smx[BLOCK / 64];
    if ((threadIdx.x & 63) == 0)
    {
        smn[threadIdx.x >> 6] = mn;
        smx[threadIdx.x >> 6] = mx;
    }
    __syncthreads();
    if (threadIdx.x == 0)
    {
        for (int i = 1; i < BLOCK / 64; ++i)
        {
            mn = fminf(mn, smn[i]);
            mx = fmaxf(mx, smx[i]);
        }
        part[blockIdx.x] = make_float2(-mn, mx);
    }
}

template <int BLOCK, int UNROLL, bool NT, int GRID>
void launch_minmax(const float* x, int64_t n, Binner, unsigned long long* c, hipStream_t s)
{
    int64_t need = (n / 4 + BLOCK * UNROLL - 1) / (BLOCK * UNROLL);
    int g        = (int) std::max<int64_t>(1, std::min<int64_t>(need, GRID));
    minmax_var<BLOCK, UNROLL, NT><<<g, BLOCK, 0, s>>>(x, n, (float2*) c);
}

template <int BLOCK, int UNROLL, int COPIES, int GRID>
void launch_hist_rcp(const float* x, int64_t n, Binner bn, unsigned long long* c, hipStream_t s)
{
    int64_t need = (n / 4 + BLOCK * UNROLL - 1) / (BLOCK * UNROLL);
    int g        = (int) std::max<int64_t>(1, std::min<int64_t>(need, GRID));
    BinnerRcp br {bn.bucket, bn.offset, 1.0f / bn.bucket};
    hist_var<BLOCK, UNROLL, COPIES, true, true, false, BinnerRcp><<<g, BLOCK, 0, s>>>(x, n, br, c);
}

// software-pipelined: the next UNROLL float4 are in flight while the current ones are binned
template <int BLOCK, int UNROLL, int COPIES, class B>
__global__ __launch_bounds__(BLOCK) void hist_pipe(const float* __restrict__ x, int64_t n, B bn,
                                                   unsigned long long* __restrict__ counts)
{
    __shared__ uint32_t lds[COPIES][kBins];
    const int copy = (threadIdx.x >> 6) % COPIES;
    for (int i = threadIdx.x; i < COPIES * kBins; i += BLOCK)
        (&lds[0][0])[i] = 0;
    __syncthreads();
    const int zbin = bn.bin(0.0f);
    uint32_t zc    = 0;
    auto add = [&](float v) {
        if (v == 0.0f)
        {
            ++zc;
            return;
        }
        int b = bn.bin(v);
        if (b >= 0)
            atomicAdd(&lds[copy][b], 1u);
    };
    const f4* x4         = reinterpret_cast<const f4*>(x);
    const int64_t nv     = n / 4;
    const int64_t stride = (int64_t) gridDim.x * BLOCK * UNROLL;
    int64_t base         = (int64_t) blockIdx.x * BLOCK * UNROLL + threadIdx.x;
    f4 cur[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
    {
        int64_t i = base + (int64_t) u * BLOCK;
        cur[u]    = i < nv ? __builtin_nontemporal_load(x4 + i) : f4 {NAN, NAN, NAN, NAN};
    }
    for (; base < nv; base += stride)
    {
        f4 nxt[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
        {
            int64_t i = base + stride + (int64_t) u * BLOCK;
            nxt[u]    = i < nv ? __builtin_nontemporal_load(x4 + i) : f4 {NAN, NAN, NAN, NAN};
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
        {
            add(cur[u].x);
            add(cur[u].y);
            add(cur[u].z);
            add(cur[u].w);
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
            cur[u] = nxt[u];
    }
    for (int64_t i = nv * 4 + (int64_t) blockIdx.x * BLOCK + threadIdx.x; i < n; i += (int64_t) gridDim.x * BLOCK)
        add(x[i]);
    zc = wave_sum(zc);
    if ((threadIdx.x & 63) == 0 && zbin >= 0 && zc)
        atomicAdd(&lds[copy][zbin], zc);
    __syncthreads();
    for (int b = threadIdx.x; b < kBins; b += BLOCK)
    {
        uint32_t s = 0;
#pragma unroll
        for (int i = 0; i < COPIES; ++i)
            s += lds[i][b];
        if (s)
            atomicAdd(&counts[b], (unsigned long long) s);
    }
}

template <int BLOCK, int UNROLL, int COPIES, int GRID>
void launch_hist_pipe(const float* x, int64_t n, Binner bn, unsigned long long* c, hipStream_t s)
{
    int64_t need = (n / 4 + BLOCK * UNROLL - 1) / (BLOCK * UNROLL);
    int g        = (int) std::max<int64_t>(1, std::min<int64_t>(need, GRID));
    BinnerRcp br {bn.bucket, bn.offset, 1.0f / bn.bucket};
    hist_pipe<BLOCK, UNROLL, COPIES, BinnerRcp><<<g, BLOCK, 0, s>>>(x, n, br, c);
}

template <int BLOCK, int UNROLL, int COPIES, int GRID, int LSH>
void launch_hist_fast(const float* x, int64_t n, Binner bn, unsigned long long* c, hipStream_t s)
{
    int64_t need = (n / 4 + BLOCK * UNROLL - 1) / (BLOCK * UNROLL);
    int g        = (int) std::max<int64_t>(1, std::min<int64_t>(need, GRID));
    BinnerFast bf {bn.bucket, bn.offset, 1.0f / bn.bucket, (515.0f + 2.0f * fabsf(bn.offset)) * 4.76837158203125e-7f};
    hist_var<BLOCK, UNROLL, COPIES, true, true, false, BinnerFast, LSH><<<g, BLOCK, 0, s>>>(x, n, bf, c);
}

// read-only ceiling: sum of the input (same load pattern)
template <int BLOCK, int UNROLL>
__global__ __launch_bounds__(BLOCK) void read_var(const float* __restrict__ x, int64_t n, float* __restrict__ out)
{
    const f4* x4         = reinterpret_cast<const f4*>(x);
    const int64_t nv     = n / 4;
    const int64_t stride = (int64_t) gridDim.x * BLOCK * UNROLL;
    float s              = 0;
    for (int64_t base = (int64_t) blockIdx.x * BLOCK * UNROLL + threadIdx.x; base < nv; base += stride)
    {
        f4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
        {
            int64_t i = base + (int64_t) u * BLOCK;
            v[u]      = i < nv ? __builtin_nontemporal_load(x4 + i) : f4 {0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
            s += v[u].x + v[u].y + v[u].z + v[u].w;
    }
    if (s == 1234.5f)
        out[0] = s;
}

__global__ void gen_kernel(float* x, int64_t n, int relu, uint32_t seed)
{
    for (int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t) gridDim.x * blockDim.x)
    {
        uint64_t h = (uint64_t) i * 0x9E3779B97F4A7C15ull + seed;
        h ^= h >> 31;
        h *= 0xBF58476D1CE4E5B9ull;
        h ^= h >> 29;
        float u1 = ((h & 0xFFFFFF) + 1) / 16777217.0f, u2 = ((h >> 24) & 0xFFFFFF) / 16777216.0f;
        float z  = sqrtf(-2.0f * logf(u1)) * cosf(6.2831853f * u2);
        x[i]     = relu ? fmaxf(z * 1.5f + 0.2f, 0.0f) : z * 2.0f;
    }
}

struct Variant
{
    const char* name;
    void (*launch)(const float*, int64_t, Binner, unsigned long long*, hipStream_t);
    bool check;
    std::vector<float> ms;
};

template <int BLOCK, int UNROLL, int COPIES, bool NT, bool ZSKIP, int GRID>
void launch_hist(const float* x, int64_t n, Binner bn, unsigned long long* c, hipStream_t s)
{
    int64_t need = (n / 4 + BLOCK * UNROLL - 1) / (BLOCK * UNROLL);
    int g        = (int) std::max<int64_t>(1, std::min<int64_t>(need, GRID));
    hist_var<BLOCK, UNROLL, COPIES, NT, ZSKIP><<<g, BLOCK, 0, s>>>(x, n, bn, c);
}

template <int BLOCK, int UNROLL, int GRID>
void launch_read(const float* x, int64_t n, Binner, unsigned long long* c, hipStream_t s)
{
    read_var<BLOCK, UNROLL><<<GRID, BLOCK, 0, s>>>(x, n, (float*) c);
}

// InitializePdf's range (math_functions.cpp:207-241) for min/max -> UpdatePdf's bucket/offset
Binner binner_for(float mn, float mx)
{
    float center = (mx + mn) / 2.0f;
    float lo = center - 3.0f * (center - mn), hi = center + 3.0f * (mx - center);
    double bs    = ((double) hi - (double) lo) / kBins;
    float bucket = (float) (((double) lo + bs) - (double) lo);
    return Binner {bucket, (float) (double) lo / bucket};
}

int main(int argc, char** argv)
{
    int64_t n  = argc > 1 ? atoll(argv[1]) : 205520896;
    int rounds = argc > 2 ? atoi(argv[2]) : 9;
    float* x;
    unsigned long long *cnt, *ref;
    CK(hipMalloc(&x, n * 4));
    CK(hipMalloc(&cnt, 1024 * 8 + 8192 * 512 * 4));
    CK(hipMalloc(&ref, kBins * 8));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    CK(hipMemset(cnt, 0, 1024 * 8 + 8192 * 512 * 4));
    std::vector<Variant> vs = {
        {"read-only ceiling b256 u4 g4096", launch_read<256, 4, 4096>, false, {}},
        {"hist b256 u4 c4 g2048 nt (division)", launch_hist<256, 4, 4, true, true, 2048>, true, {}},
        {"hist b256 u4 c4 g2048 nt (rcp fast path)", launch_hist_rcp<256, 4, 4, 2048>, true, {}},
        {"hist b1024 u4 c16 g256 nt (division)", launch_hist<1024, 4, 16, true, true, 256>, true, {}},
        {"hist b1024 u4 c16 g256 nt (rcp fast path)", launch_hist_rcp<1024, 4, 16, 256>, true, {}},
        {"hist b256 u4 c4 g2048 nt (uniform thr)", launch_hist_fast<256, 4, 4, 2048, 6>, true, {}},
        {"hist b512 u4 c8 g1024 nt (uniform thr)", launch_hist_fast<512, 4, 8, 1024, 6>, true, {}},
        {"hist b256 u2 c4 g2048 pipelined (rcp)", launch_hist_pipe<256, 2, 4, 2048>, true, {}},
        {"hist b256 u4 c4 g2048 pipelined (rcp)", launch_hist_pipe<256, 4, 4, 2048>, true, {}},
        {"hist b512 u2 c8 g1024 pipelined (rcp)", launch_hist_pipe<512, 2, 8, 1024>, true, {}},
        {"hist b256 u2 c4 g1024 pipelined (rcp)", launch_hist_pipe<256, 2, 4, 1024>, true, {}},
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char* dname[4] = {"relu(N(0,1)*1.5+0.2)", "N(0,1)*2", "N(0,1)*2, range +-30 (outliers)", "relu, range 0..40 (outliers)"};
    for (int dist = 0; dist < 4; ++dist)
    {
        gen_kernel<<<4096, 256, 0, s>>>(x, n, dist == 0 || dist == 3, 1234);
        CK(hipStreamSynchronize(s));
        Binner bn = dist == 0 ? binner_for(0.0f, 9.0f)
                    : dist == 1 ? binner_for(-11.0f, 11.0f)
                    : dist == 2 ? binner_for(-30.0f, 30.0f)
                                : binner_for(0.0f, 40.0f);
        CK(hipMemsetAsync(ref, 0, kBins * 8, s));
        launch_hist<256, 2, 4, false, true, 512>(x, n, bn, ref, s);
        std::vector<unsigned long long> href(kBins), hc(kBins);
        CK(hipMemcpy(href.data(), ref, kBins * 8, hipMemcpyDeviceToHost));
        unsigned long long tot = 0;
        for (auto v: href)
            tot += v;
        for (auto& v: vs)
        {
            v.ms.clear();
            CK(hipMemsetAsync(cnt, 0, 1024 * 8 + 33 * kBins * 8, s));
            v.launch(x, n, bn, cnt, s);
            CK(hipMemcpy(hc.data(), cnt, kBins * 8, hipMemcpyDeviceToHost));
            if (v.check && memcmp(hc.data(), href.data(), kBins * 8) != 0)
                printf("MISMATCH in %s\n", v.name);
        }
        for (int r = 0; r < rounds; ++r)
            for (auto& v: vs)
            {
                CK(hipMemsetAsync(cnt, 0, 1024 * 8 + 33 * kBins * 8, s));
                CK(hipEventRecord(e0, s));
                v.launch(x, n, bn, cnt, s);
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                v.ms.push_back(ms);
            }
        printf("== %s, n=%lld, in-range %llu\n", dname[dist], (long long) n, tot);
        for (auto& v: vs)
        {
            std::sort(v.ms.begin(), v.ms.end());
            float med = v.ms[v.ms.size() / 2];
            printf("%-40s %8.3f ms  %7.1f GB/s\n", v.name, med, n * 4.0 / (med * 1e-3) / 1e9);
        }
    }
    return 0;
}
