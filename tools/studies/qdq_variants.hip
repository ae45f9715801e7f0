// qdq_variants.hip -- microbenchmark of per-tensor QDQ kernel variants on gfx950 (tuning tool).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off
//        -fhip-fp32-correctly-rounded-divide-sqrt -I include -I aimet_amd/csrc tools/studies/qdq_variants.hip -o tools/studies/qdq_variants
// Runs interleaved rounds of every variant on a buffer larger than the 256 MiB Infinity Cache and
// prints median GB/s (8 B/elem for QDQ and copy). Outputs of every variant are checked against
// the baseline kernel bit for bit.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "common.hpp"

using namespace aimet_amd;
typedef float f4 __attribute__((ext_vector_type(4)));

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

template <int BLOCK, int UNROLL, bool NT_LOAD, bool NT_STORE, bool COPY>
__global__ __launch_bounds__(BLOCK) void qdq_var(const float4* __restrict__ in, float4* __restrict__ out, int64_t nvec,
                                                 QdqParams p)
{
    const int64_t stride = (int64_t) gridDim.x * BLOCK * UNROLL;
    for (int64_t base = (int64_t) blockIdx.x * BLOCK * UNROLL + threadIdx.x; base < nvec; base += stride)
    {
        float4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
        {
            int64_t i = base + (int64_t) u * BLOCK;
            if (i < nvec)
            {
                if (NT_LOAD)
                {
                    f4 t = __builtin_nontemporal_load(reinterpret_cast<const f4*>(in) + i);
                    v[u] = make_float4(t.x, t.y, t.z, t.w);
                }
                else
                    v[u] = in[i];
            }
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
        {
            int64_t i = base + (int64_t) u * BLOCK;
            if (i < nvec)
            {
                float4 r = v[u];
                if (!COPY)
                {
                    r.x = dequantize(quantize_nearest(v[u].x, p), p);
                    r.y = dequantize(quantize_nearest(v[u].y, p), p);
                    r.z = dequantize(quantize_nearest(v[u].z, p), p);
                    r.w = dequantize(quantize_nearest(v[u].w, p), p);
                }
                if (NT_STORE)
                {
                    f4 t = {r.x, r.y, r.z, r.w};
                    __builtin_nontemporal_store(t, reinterpret_cast<f4*>(out) + i);
                }
                else
                    out[i] = r;
            }
        }
    }
}

// one tile per block, no grid-stride loop (RCP: reciprocal fast path of common.hpp)
template <int BLOCK, int UNROLL, bool NT = false, bool RCP = false>
__global__ __launch_bounds__(BLOCK) void qdq_tile(const float4* __restrict__ in, float4* __restrict__ out, int64_t nvec,
                                                  QdqParams p)
{
    int64_t base = (int64_t) blockIdx.x * BLOCK * UNROLL + threadIdx.x;
    f4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
        if (base + u * BLOCK < nvec)
        {
            if (NT)
                v[u] = __builtin_nontemporal_load(reinterpret_cast<const f4*>(in) + base + u * BLOCK);
            else
                v[u] = reinterpret_cast<const f4*>(in)[base + u * BLOCK];
        }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
        if (base + u * BLOCK < nvec)
        {
            f4 r;
            if (RCP)
            {
                const float rcp = 1.0f / p.delta;
                r.x = dequantize(quantize_nearest_rcp(v[u].x, p, rcp), p);
                r.y = dequantize(quantize_nearest_rcp(v[u].y, p, rcp), p);
                r.z = dequantize(quantize_nearest_rcp(v[u].z, p, rcp), p);
                r.w = dequantize(quantize_nearest_rcp(v[u].w, p, rcp), p);
            }
            else
            {
                r.x = dequantize(quantize_nearest(v[u].x, p), p);
                r.y = dequantize(quantize_nearest(v[u].y, p), p);
                r.z = dequantize(quantize_nearest(v[u].z, p), p);
                r.w = dequantize(quantize_nearest(v[u].w, p), p);
            }
            if (NT)
                __builtin_nontemporal_store(r, reinterpret_cast<f4*>(out) + base + u * BLOCK);
            else
                reinterpret_cast<f4*>(out)[base + u * BLOCK] = r;
        }
}

struct Variant
{
    const char* name;
    void (*launch)(const float4*, float4*, int64_t, QdqParams, hipStream_t);
    bool copy;
    std::vector<float> ms;
};

template <int BLOCK, int UNROLL, bool NTL, bool NTS, bool COPY, int GRID>
void launch_var(const float4* in, float4* out, int64_t nvec, QdqParams p, hipStream_t s)
{
    int64_t need = (nvec + BLOCK * UNROLL - 1) / (BLOCK * UNROLL);
    int g        = (int) std::min<int64_t>(need, GRID);
    qdq_var<BLOCK, UNROLL, NTL, NTS, COPY><<<g, BLOCK, 0, s>>>(in, out, nvec, p);
}

template <int BLOCK, int UNROLL, bool NT = false, bool RCP = false>
void launch_tile(const float4* in, float4* out, int64_t nvec, QdqParams p, hipStream_t s)
{
    int64_t g = (nvec + BLOCK * UNROLL - 1) / (BLOCK * UNROLL);
    qdq_tile<BLOCK, UNROLL, NT, RCP><<<(int) g, BLOCK, 0, s>>>(in, out, nvec, p);
}

int main(int argc, char** argv)
{
    int64_t n    = argc > 1 ? atoll(argv[1]) : (int64_t(1) << 28);   // 1 GiB per buffer
    int rounds   = argc > 2 ? atoi(argv[2]) : 15;
    int64_t nvec = n / 4;
    float *in, *out, *ref;
    CK(hipMalloc(&in, n * 4));
    CK(hipMalloc(&out, n * 4));
    CK(hipMalloc(&ref, n * 4));
    std::vector<float> h(n);
    srand(1);
    for (int64_t i = 0; i < n; ++i)
        h[i] = ((rand() & 0xFFFF) / 65535.0f - 0.5f) * 12.0f;
    CK(hipMemcpy(in, h.data(), n * 4, hipMemcpyHostToDevice));
    QdqParams p {-3.1f, 5.7f, 0.0345f, -90.0f};
    hipStream_t s;
    CK(hipStreamCreate(&s));

    std::vector<Variant> vs = {
        {"copy b256 u4 g2048 nt-ld+st", launch_var<256, 4, true, true, true, 2048>, true, {}},
        {"qdq  tile b256 u1 nt (division)", launch_tile<256, 1, true>, false, {}},
        {"qdq  tile b256 u1 nt rcp fast path", launch_tile<256, 1, true, true>, false, {}},
        {"qdq  tile b256 u2 nt rcp fast path", launch_tile<256, 2, true, true>, false, {}},
        {"qdq  tile b512 u1 nt rcp fast path", launch_tile<512, 1, true, true>, false, {}},
    };
    // reference output
    launch_var<256, 4, false, false, false, 2048>((const float4*) in, (float4*) ref, nvec, p, s);
    CK(hipStreamSynchronize(s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (auto& v: vs)   // warm + check
    {
        CK(hipMemset(out, 0, n * 4));
        v.launch((const float4*) in, (float4*) out, nvec, p, s);
        CK(hipStreamSynchronize(s));
        if (!v.copy)
        {
            std::vector<float> a(1 << 20), b(1 << 20);
            CK(hipMemcpy(a.data(), out + n - (1 << 20), 4 << 20, hipMemcpyDeviceToHost));
            CK(hipMemcpy(b.data(), ref + n - (1 << 20), 4 << 20, hipMemcpyDeviceToHost));
            if (memcmp(a.data(), b.data(), 4 << 20) != 0)
                printf("MISMATCH in %s\n", v.name);
        }
    }
    for (int r = 0; r < rounds; ++r)
        for (auto& v: vs)
        {
            CK(hipEventRecord(e0, s));
            v.launch((const float4*) in, (float4*) out, nvec, p, s);
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            v.ms.push_back(ms);
        }
    printf("n = %lld elements (%.2f GiB in + out)\n", (long long) n, 2.0 * n * 4 / (1 << 30));
    for (auto& v: vs)
    {
        std::sort(v.ms.begin(), v.ms.end());
        float med = v.ms[v.ms.size() / 2], best = v.ms[0];
        printf("%-34s median %8.4f ms  %7.1f GB/s   best %7.1f GB/s\n", v.name, med, n * 8.0 / med / 1e6,
               n * 8.0 / best / 1e6);
    }
    return 0;
}
