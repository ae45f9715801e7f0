// broadcast.hip -- blockwise (broadcast) quantize-dequantize, the block-layout permutation of the
// blockwise statistics, and the fp16 round trip of float quantizers.
//
// Reference:
//   quantizeDequantizeBroadcast{Cpu,Gpu}  trim_functions.cpp:633-687, trim_functions.cu:96-122
//   permuteTensor{CPU,GPU}                onnx/src/QuantizeDequantizeUtils.cpp:64-95 (+ .cu)
//   quantizeDequantizeFp16{Cpu,Gpu}       onnx/src/AimetOpUtils.cpp:61-67, trim_functions.cu:135-148
//
// The reference walks every dimension of the broadcast view per element with 64-bit divisions
// and int indices (wrapping at 2^31). Here the view is first collapsed on the host: size-1 dims
// are dropped and neighbours that index the encodings the same way (both broadcast, or both
// row-major over the encodings) are merged, so the usual LPBQ / blockwise weight layouts become
// 2-3 dims. The kernel then does one 32-bit multiply-shift division per merged dim per 4
// elements (16-B vectors whenever the innermost run allows), and gathers the per-element
// encoding from the four float arrays (L1/L2-resident: E << N).
#include "common.hpp"

#include <vector>

namespace aimet_amd
{
namespace
{

constexpr int kMaxMerged = 8;
typedef float f4 __attribute__((ext_vector_type(4)));

// A collapsed row-major view: dim d has `size`, tensor stride `tstride` (contiguous) and
// encoding stride `estride` (0 along broadcast dims).
struct View
{
    int nd;
    int64_t size[kMaxMerged];
    int64_t tstride[kMaxMerged];
    int64_t estride[kMaxMerged];
};

// Host: the reference's (input strides, encoding / output strides) description of a contiguous
// tensor of n elements -> collapsed view. Input strides must be those of a row-major tensor.
View collapse(int64_t n, int64_t nd, const int64_t* tstr, const int64_t* estr)
{
    std::vector<int64_t> size(nd), ts(tstr, tstr + nd), es(estr, estr + nd);
    for (int64_t d = 0; d < nd; ++d)
    {
        AIMET_REQUIRE(ts[d] > 0, "input strides must be positive");
        int64_t outer = d == 0 ? n : ts[d - 1];
        AIMET_REQUIRE(outer % ts[d] == 0, "input strides do not describe a contiguous row-major tensor");
        size[d] = outer / ts[d];
    }
    AIMET_REQUIRE(nd == 0 || ts[nd - 1] == 1, "the innermost input stride must be 1");
    // drop size-1 dims, then merge neighbours with estride[d] == estride[d+1] * size[d+1]
    std::vector<int64_t> s2, t2, e2;
    for (int64_t d = 0; d < nd; ++d)
        if (size[d] != 1)
        {
            s2.push_back(size[d]);
            t2.push_back(ts[d]);
            e2.push_back(es[d]);
        }
    std::vector<int64_t> s3, t3, e3;
    for (size_t d = 0; d < s2.size(); ++d)
    {
        if (!s3.empty() && e3.back() == e2[d] * s2[d])
        {
            s3.back() *= s2[d];
            t3.back() = t2[d];
            e3.back() = e2[d];
            continue;
        }
        s3.push_back(s2[d]);
        t3.push_back(t2[d]);
        e3.push_back(e2[d]);
    }
    if (s3.empty())
    {
        s3.push_back(1);
        t3.push_back(1);
        e3.push_back(0);
    }
    AIMET_REQUIRE(s3.size() <= (size_t) kMaxMerged, "broadcast view has too many alternating dimensions");
    View v {};
    v.nd = (int) s3.size();
    for (int d = 0; d < v.nd; ++d)
    {
        v.size[d]    = s3[d];
        v.tstride[d] = t3[d];
        v.estride[d] = e3[d];
    }
    return v;
}

// 32-bit index math (n < 2^31)
struct View32
{
    int nd;
    FastDiv div[kMaxMerged];       // by tstride
    uint32_t tstride[kMaxMerged];
    uint32_t estride[kMaxMerged];
    __device__ __forceinline__ uint32_t index(uint32_t i) const
    {
        uint32_t e = 0, rem = i;
#pragma unroll
        for (int d = 0; d < kMaxMerged; ++d)
        {
            if (d >= nd)
                break;
            uint32_t q = div[d].div(rem);
            rem -= q * tstride[d];
            e += q * estride[d];
        }
        return e;
    }
};

View32 to32(const View& v)
{
    View32 r {};
    r.nd = v.nd;
    for (int d = 0; d < v.nd; ++d)
    {
        r.div[d]     = FastDiv((uint32_t) v.tstride[d]);
        r.tstride[d] = (uint32_t) v.tstride[d];
        r.estride[d] = (uint32_t) v.estride[d];
    }
    return r;
}

__device__ __forceinline__ int64_t index64(const View& v, int64_t i)
{
    int64_t e = 0, rem = i;
    for (int d = 0; d < v.nd; ++d)
    {
        int64_t q = rem / v.tstride[d];
        rem -= q * v.tstride[d];
        e += q * v.estride[d];
    }
    return e;
}

struct EncArrays
{
    const float* __restrict__ mn;
    const float* __restrict__ mx;
    const float* __restrict__ delta;
    const float* __restrict__ offset;
    __device__ __forceinline__ float qdq(float x, uint32_t e) const
    {
        QdqParams p {mn[e], mx[e], delta[e], offset[e]};
        return dequantize(quantize_nearest(x, p), p);
    }
};

// 4 consecutive elements per lane (the innermost merged dim has size % 4 == 0, so they share the
// outer indices and their encodings are e0 + j * inner_estride), kUnroll vectors in flight per
// lane: with LPBQ-sized tables (one encoding per 16-64 elements, tens of MB) the encoding loads
// miss L2 and are as latency-bound as the data.
//   MODE 0: inner_estride == 0 -- one encoding per vector (4 scalar loads)
//   MODE 1: inner_estride == 1, e0 % 4 == 0 and 16-B aligned arrays -- 4 x 16-B vector loads
//   MODE 2: anything else -- 16 scalar gathers
constexpr int kUnroll = 4;

template <int MODE>
__global__ __launch_bounds__(kBlock) void bcast_vec_kernel(const f4* __restrict__ in, f4* __restrict__ out,
                                                           uint32_t nvec, View32 v, uint32_t inner_es, EncArrays enc)
{
    const uint32_t stride = gridDim.x * kBlock * kUnroll;
    for (uint32_t base = blockIdx.x * kBlock * kUnroll + threadIdx.x; base < nvec; base += stride)
    {
        f4 x[kUnroll];
        uint32_t e0[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; ++u)
        {
            const uint32_t i = base + u * kBlock;
            const uint32_t c = i < nvec ? i : nvec - 1;   // clamped (never stored)
            x[u]             = __builtin_nontemporal_load(in + c);
            e0[u]            = v.index(c * 4);
        }
        f4 mn[kUnroll], mx[kUnroll], dl[kUnroll], of[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; ++u)
        {
            const uint32_t e = e0[u];
            if (MODE == 0)
            {
                const float a = enc.mn[e], b = enc.mx[e], d = enc.delta[e], o = enc.offset[e];
                mn[u] = f4 {a, a, a, a};
                mx[u] = f4 {b, b, b, b};
                dl[u] = f4 {d, d, d, d};
                of[u] = f4 {o, o, o, o};
            }
            else if (MODE == 1)
            {
                mn[u] = *reinterpret_cast<const f4*>(enc.mn + e);
                mx[u] = *reinterpret_cast<const f4*>(enc.mx + e);
                dl[u] = *reinterpret_cast<const f4*>(enc.delta + e);
                of[u] = *reinterpret_cast<const f4*>(enc.offset + e);
            }
            else
            {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                {
                    const uint32_t ej = e + j * inner_es;
                    mn[u][j]          = enc.mn[ej];
                    mx[u][j]          = enc.mx[ej];
                    dl[u][j]          = enc.delta[ej];
                    of[u][j]          = enc.offset[ej];
                }
            }
        }
#pragma unroll
        for (int u = 0; u < kUnroll; ++u)
        {
            const uint32_t i = base + u * kBlock;
            if (i >= nvec)
                break;
            f4 r;
            if (MODE == 0)
            {
                // one encoding per vector: its reciprocal and rounding threshold serve 4 elements
                // (qdq_round_fast, common.hpp: bit-identical to the division form)
                const QdqParams p {mn[u][0], mx[u][0], dl[u][0], of[u][0]};
                const float rcp = 1.0f / p.delta, thr = qdq_round_thr(p, rcp);
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    r[j] = dequantize(qdq_round_fast(glibc_fmaxf(glibc_fminf(x[u][j], p.max), p.min), p, rcp, thr), p);
            }
            else
            {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                {
                    QdqParams p {mn[u][j], mx[u][j], dl[u][j], of[u][j]};
                    r[j] = dequantize(quantize_nearest(x[u][j], p), p);
                }
            }
            __builtin_nontemporal_store(r, out + i);
        }
    }
}

// Blocks strided along the outer dim -- the merged view [A][B][C] with encodings [A][C] (ONNX
// MatMul weights [K, N] with blocks along K: channel axis 1, block axis 0). A lane owns 4
// consecutive columns of one block and kRows of its B rows: the 4 x 16-B encoding loads are
// reused kRows times and every row load is coalesced across the wave (lanes = columns).
constexpr int kRows = 16;

template <int RB>
__global__ __launch_bounds__(kBlock) void bcast_colblock_kernel(const f4* __restrict__ in, f4* __restrict__ out,
                                                                uint32_t A, uint32_t B, uint32_t C4, FastDiv divC4,
                                                                FastDiv divRg, uint32_t nrg, EncArrays enc)
{
    const uint32_t items  = A * nrg * C4;
    const uint32_t stride = gridDim.x * kBlock;
    for (uint32_t it = blockIdx.x * kBlock + threadIdx.x; it < items; it += stride)
    {
        const uint32_t t  = divC4.div(it);
        const uint32_t c4 = it - t * C4;
        const uint32_t a  = divRg.div(t);
        const uint32_t rg = t - a * nrg;
        const uint32_t e  = (a * C4 + c4) * 4;
        const f4 mn = *reinterpret_cast<const f4*>(enc.mn + e);
        const f4 mx = *reinterpret_cast<const f4*>(enc.mx + e);
        const f4 dl = *reinterpret_cast<const f4*>(enc.delta + e);
        const f4 of = *reinterpret_cast<const f4*>(enc.offset + e);
        // per-column reciprocal and rounding threshold, reused over the kRows rows (qdq_round_fast)
        f4 rc, th;
#pragma unroll
        for (int j = 0; j < 4; ++j)
        {
            rc[j] = 1.0f / dl[j];
            th[j] = qdq_round_thr(QdqParams {mn[j], mx[j], dl[j], of[j]}, rc[j]);
        }
        const uint32_t b0   = rg * kRows;
        const uint32_t rows = B - b0 < (uint32_t) kRows ? B - b0 : (uint32_t) kRows;
        const uint32_t base = (a * B + b0) * C4 + c4;
        for (uint32_t r0 = 0; r0 < rows; r0 += RB)   // RB row loads in flight per lane
        {
            f4 x[RB];
#pragma unroll
            for (int u = 0; u < RB; ++u)
                if (r0 + u < rows)
                    x[u] = __builtin_nontemporal_load(in + base + (r0 + u) * C4);
#pragma unroll
            for (int u = 0; u < RB; ++u)
            {
                if (r0 + u >= rows)
                    break;
                f4 y;
#pragma unroll
                for (int j = 0; j < 4; ++j)
                {
                    const QdqParams p {mn[j], mx[j], dl[j], of[j]};
                    y[j] = dequantize(qdq_round_fast(glibc_fmaxf(glibc_fminf(x[u][j], p.max), p.min), p, rc[j], th[j]),
                                      p);
                }
                __builtin_nontemporal_store(y, out + base + (r0 + u) * C4);
            }
        }
    }
}

__global__ __launch_bounds__(kBlock) void bcast_scalar_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                              uint32_t n, View32 v, EncArrays enc)
{
    const uint32_t stride = gridDim.x * kBlock;
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
        out[i] = enc.qdq(in[i], v.index(i));
}

__global__ __launch_bounds__(kBlock) void bcast_scalar64_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                                int64_t n, View v, EncArrays enc)
{
    const int64_t stride = (int64_t) gridDim.x * kBlock;
    for (int64_t i = (int64_t) blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
        out[i] = enc.qdq(in[i], (uint32_t) index64(v, i));
}

// permuteTensor: out[sum_d idx_d * ostride_d] = in[i] (the collapsed view's estride holds the
// output strides)
__global__ __launch_bounds__(kBlock) void permute_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                         uint32_t n, View32 v)
{
    const uint32_t stride = gridDim.x * kBlock;
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
        out[v.index(i)] = in[i];
}

__global__ __launch_bounds__(kBlock) void permute64_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                           int64_t n, View v)
{
    const int64_t stride = (int64_t) gridDim.x * kBlock;
    for (int64_t i = (int64_t) blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
        out[index64(v, i)] = in[i];
}

// float -> half (round to nearest even, v_cvt_f16_f32) -> float
__device__ __forceinline__ float fp16_rt(float x)
{
    return (float) (_Float16) x;
}

// one float4 per lane, one 256-lane tile per workgroup (the tensor_vec_kernel form: 6.4 TB/s
// where a 2048-workgroup grid-stride loop reached 5.2)
__global__ __launch_bounds__(kBlock) void fp16_vec_kernel(const f4* __restrict__ in, f4* __restrict__ out,
                                                          int64_t nvec)
{
    const int64_t i = (int64_t) blockIdx.x * kBlock + threadIdx.x;
    if (i >= nvec)
        return;
    f4 x = __builtin_nontemporal_load(in + i);
    f4 r {fp16_rt(x.x), fp16_rt(x.y), fp16_rt(x.z), fp16_rt(x.w)};
    __builtin_nontemporal_store(r, out + i);
}

__global__ __launch_bounds__(kBlock) void fp16_scalar_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                             int64_t begin, int64_t n)
{
    const int64_t stride = (int64_t) gridDim.x * kBlock;
    for (int64_t i = begin + (int64_t) blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
        out[i] = fp16_rt(in[i]);
}

inline bool aligned16(const void* a, const void* b)
{
    return ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b)) & 15) == 0;
}

}   // namespace

void launch_qdq_broadcast(const float* in, float* out, int64_t n, int64_t nd, const int64_t* tstr, const int64_t* estr,
                          const float* mn, const float* mx, const float* delta, const float* offset, hipStream_t s)
{
    if (n == 0)
        return;
    View v = collapse(n, nd, tstr, estr);
    EncArrays enc {mn, mx, delta, offset};
    if (n >= (int64_t(1) << 31))
    {
        bcast_scalar64_kernel<<<kMaxStreamBlocks, kBlock, 0, s>>>(in, out, n, v, enc);
        AIMET_LAUNCH_CHECK();
        return;
    }
    View32 v32 = to32(v);
    if (v.size[v.nd - 1] % 4 == 0 && aligned16(in, out))
    {
        const uint32_t nvec = (uint32_t) (n / 4);
        const uint32_t ies  = (uint32_t) v.estride[v.nd - 1];
        // MODE 1 needs every e0 = sum_d q_d * estride_d to be a multiple of 4: all estrides are
        // (the innermost is 1 and its run is a multiple of 4 elements)
        bool vec_tab = ies == 1 && aligned16(mn, mx) && aligned16(delta, offset);
        for (int d = 0; d + 1 < v.nd; ++d)
            vec_tab = vec_tab && v.estride[d] % 4 == 0;
        // one tile (kBlock x kUnroll vectors) per workgroup: 6.4 TB/s on [4096 x 65536] with
        // 64-blocks, where a 2048-workgroup grid-stride loop reached 5.7 (profiles/r01)
        const int blocks = (int) ceil_div(nvec, (int64_t) kBlock * kUnroll);
        auto in4 = reinterpret_cast<const f4*>(in);
        auto out4 = reinterpret_cast<f4*>(out);
        if (vec_tab && v.nd == 3 && v.estride[1] == 0 && v.estride[0] == v.size[2])
        {
            const uint32_t A = (uint32_t) v.size[0], B = (uint32_t) v.size[1], C4 = (uint32_t) (v.size[2] / 4);
            const uint32_t nrg = (B + kRows - 1) / kRows;
            const int64_t items = (int64_t) A * nrg * C4;
            // 8 row loads in flight per lane (measured: 4 -> 5.2 TB/s, 8 -> 5.4, 16 -> 5.0)
            bcast_colblock_kernel<8><<<(int) ceil_div(items, kBlock), kBlock, 0, s>>>(in4, out4, A, B, C4, FastDiv(C4),
                                                                                     FastDiv(nrg), nrg, enc);
        }
        else if (ies == 0)
            bcast_vec_kernel<0><<<blocks, kBlock, 0, s>>>(in4, out4, nvec, v32, ies, enc);
        else if (vec_tab)
            bcast_vec_kernel<1><<<blocks, kBlock, 0, s>>>(in4, out4, nvec, v32, ies, enc);
        else
            bcast_vec_kernel<2><<<blocks, kBlock, 0, s>>>(in4, out4, nvec, v32, ies, enc);
    }
    else
        bcast_scalar_kernel<<<stream_blocks(n, kBlock), kBlock, 0, s>>>(in, out, (uint32_t) n, v32, enc);
    AIMET_LAUNCH_CHECK();
}

void launch_permute(const float* in, float* out, int64_t n, int64_t nd, const int64_t* istr, const int64_t* ostr,
                    hipStream_t s)
{
    if (n == 0)
        return;
    View v = collapse(n, nd, istr, ostr);
    if (n >= (int64_t(1) << 31))
        permute64_kernel<<<kMaxStreamBlocks, kBlock, 0, s>>>(in, out, n, v);
    else
        permute_kernel<<<stream_blocks(n, kBlock), kBlock, 0, s>>>(in, out, (uint32_t) n, to32(v));
    AIMET_LAUNCH_CHECK();
}

void launch_qdq_fp16(const float* in, float* out, int64_t n, hipStream_t s)
{
    if (n == 0)
        return;
    int64_t done = 0;
    if (aligned16(in, out))
    {
        int64_t nvec = n / 4;
        if (nvec)
        {
            AIMET_REQUIRE(ceil_div(nvec, kBlock) < (int64_t(1) << 31), "tensor too large");
            fp16_vec_kernel<<<(unsigned) ceil_div(nvec, kBlock), kBlock, 0, s>>>(reinterpret_cast<const f4*>(in),
                                                                               reinterpret_cast<f4*>(out), nvec);
            AIMET_LAUNCH_CHECK();
        }
        done = nvec * 4;
    }
    if (done < n)
    {
        fp16_scalar_kernel<<<stream_blocks(n - done, kBlock), kBlock, 0, s>>>(in, out, done, n);
        AIMET_LAUNCH_CHECK();
    }
}

}   // namespace aimet_amd

extern "C" {

int aimet_qdq_broadcast(const float* in, float* out, int64_t n, int64_t num_dims, const int64_t* input_strides,
                        const int64_t* encoding_strides, const float* enc_min, const float* enc_max,
                        const float* enc_delta, const float* enc_offset, void* stream)
{
    using namespace aimet_amd;
    return guarded([&] {
        AIMET_REQUIRE(n >= 0 && num_dims >= 0, "invalid broadcast shape");
        if (n == 0)
            return;
        AIMET_REQUIRE(num_dims > 0 && input_strides && encoding_strides, "null strides");
        require_device_ptr(in, "input");
        require_device_ptr(out, "output");
        require_device_ptr(enc_min, "encoding min");
        require_device_ptr(enc_max, "encoding max");
        require_device_ptr(enc_delta, "encoding delta");
        require_device_ptr(enc_offset, "encoding offset");
        launch_qdq_broadcast(in, out, n, num_dims, input_strides, encoding_strides, enc_min, enc_max, enc_delta,
                             enc_offset, as_stream(stream));
    });
}

int aimet_permute_tensor(const float* in, float* out, int64_t n, int64_t num_dims, const int64_t* input_strides,
                         const int64_t* output_strides, void* stream)
{
    using namespace aimet_amd;
    return guarded([&] {
        AIMET_REQUIRE(n >= 0 && num_dims >= 0, "invalid tensor shape");
        if (n == 0)
            return;
        AIMET_REQUIRE(num_dims > 0 && input_strides && output_strides, "null strides");
        require_device_ptr(in, "input");
        require_device_ptr(out, "output");
        AIMET_REQUIRE(in != out, "permute cannot run in place");
        launch_permute(in, out, n, num_dims, input_strides, output_strides, as_stream(stream));
    });
}

int aimet_qdq_fp16(const float* in, float* out, int64_t n, void* stream)
{
    using namespace aimet_amd;
    return guarded([&] {
        AIMET_REQUIRE(n >= 0, "negative element count");
        if (n == 0)
            return;
        require_device_ptr(in, "input");
        require_device_ptr(out, "output");
        launch_qdq_fp16(in, out, n, as_stream(stream));
    });
}

}   // extern "C"
