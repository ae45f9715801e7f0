// qdq.hip -- quantize-dequantize, quantize-only and STE-backward kernels for gfx950.
//
// Reference: trim_functions.cu:46-92 (one element per thread, 512-thread blocks, fast-math
// division, per-element global loads of the per-channel table, legacy default stream).
// The per-element IEEE division stays (tools/studies/qdq_variants.hip: the reciprocal fast path of
// common.hpp measures 4% slower here -- this kernel is HBM-bound, the fast path's extra VGPRs and
// branch cost more than the division; it pays off in the 16-bit and histogram kernels).
// MI355X design: HBM-bound streaming (8 B/elem fwd, 12 B/elem STE) -> one 16-B vector per lane,
// one tile per 256-thread workgroup (thousands of workgroups fill the 256 CUs), non-temporal
// loads/stores (streamed once, kept out of L2/MALL), scalar encoding parameters in SGPRs,
// per-channel parameters fetched once per 16-B vector (K % 4 == 0) from a device-resident table
// built once per encoding.
#include "common.hpp"

#include <cmath>
#include <vector>

namespace aimet_amd
{

namespace
{

enum class Op
{
    QDQ,        // dequantize(quantize(x))
    QUANTIZE    // quantize(x) - shift
};

template <Op OP, bool STOCHASTIC>
__device__ __forceinline__ float apply(float x, const QdqParams& p, float shift, uint64_t seed, uint64_t idx)
{
    float q = STOCHASTIC ? quantize_stochastic(x, p, seed, idx) : quantize_nearest(x, p);
    if constexpr (OP == Op::QDQ)
        return dequantize(q, p);
    else
        return q - shift;
}

// ---------------------------------------------------------------------------------------
// Per-tensor: parameters are kernel arguments (SGPRs). One 16-B vector per lane, one tile per
// workgroup, non-temporal (streaming) loads and stores: measured on MI355X at 6.6 TB/s for a
// 2 GiB in+out stream vs 5.6 TB/s for a grid-strided 4-vector loop with default cache policy
// (tools/studies/qdq_variants.hip, profiles/r01/qdq_variants.txt).
// ---------------------------------------------------------------------------------------
typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4 load_stream(const f4* p)
{
    return __builtin_nontemporal_load(p);
}
__device__ __forceinline__ void store_stream(f4 v, f4* p)
{
    __builtin_nontemporal_store(v, p);
}

template <Op OP, bool STOCHASTIC>
__global__ __launch_bounds__(kBlock) void tensor_vec_kernel(const f4* __restrict__ in, f4* __restrict__ out,
                                                            int64_t nvec, QdqParams p, float shift, uint64_t seed)
{
    const int64_t i = (int64_t) blockIdx.x * kBlock + threadIdx.x;
    if (i >= nvec)
        return;
    f4 v = load_stream(in + i);
    uint64_t e = (uint64_t) i * 4;
    f4 r;
    r.x = apply<OP, STOCHASTIC>(v.x, p, shift, seed, e + 0);
    r.y = apply<OP, STOCHASTIC>(v.y, p, shift, seed, e + 1);
    r.z = apply<OP, STOCHASTIC>(v.z, p, shift, seed, e + 2);
    r.w = apply<OP, STOCHASTIC>(v.w, p, shift, seed, e + 3);
    store_stream(r, out + i);
}

template <Op OP, bool STOCHASTIC>
__global__ __launch_bounds__(kBlock) void tensor_scalar_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                               int64_t begin, int64_t n, QdqParams p, float shift,
                                                               uint64_t seed)
{
    const int64_t stride = (int64_t) gridDim.x * kBlock;
    for (int64_t i = begin + (int64_t) blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
        out[i] = apply<OP, STOCHASTIC>(in[i], p, shift, seed, (uint64_t) i);
}

template <Op OP, bool STOCHASTIC>
void launch_tensor(const float* in, float* out, int64_t n, const QdqParams& p, float shift, uint64_t seed,
                   hipStream_t s)
{
    if (n <= 0)
        return;
    bool aligned = ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) & 15) == 0;
    int64_t nvec = aligned ? n / 4 : 0;
    if (nvec > 0)
    {
        int64_t blocks = ceil_div(nvec, kBlock);
        tensor_vec_kernel<OP, STOCHASTIC><<<(unsigned) blocks, kBlock, 0, s>>>(reinterpret_cast<const f4*>(in),
                                                                                reinterpret_cast<f4*>(out), nvec, p,
                                                                                shift, seed);
        AIMET_LAUNCH_CHECK();
    }
    int64_t done = nvec * 4;
    if (done < n)
    {
        int blocks = stream_blocks(n - done, kBlock);
        tensor_scalar_kernel<OP, STOCHASTIC><<<blocks, kBlock, 0, s>>>(in, out, done, n, p, shift, seed);
        AIMET_LAUNCH_CHECK();
    }
}

// ---------------------------------------------------------------------------------------
// Per-channel: [outer][C][K], table [4][C] = {min, max, delta, offset}.
// ---------------------------------------------------------------------------------------
struct ChannelMap
{
    FastDiv divK;
    FastDiv divC;
    uint32_t C;
    __device__ __forceinline__ uint32_t channel(uint32_t i) const
    {
        uint32_t row = divK.div(i);
        return row - divC.div(row) * C;
    }
};

__device__ __forceinline__ QdqParams load_params(const float* __restrict__ table, uint32_t C, uint32_t c)
{
    return QdqParams {table[c], table[C + c], table[2 * C + c], table[3 * C + c]};
}

// K % 4 == 0: a 16-B vector never straddles two channels.
template <bool STOCHASTIC>
__global__ __launch_bounds__(kBlock) void channel_vec_kernel(const f4* __restrict__ in, f4* __restrict__ out,
                                                             uint32_t nvec, ChannelMap map,
                                                             const float* __restrict__ table, uint64_t seed)
{
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= nvec)
        return;
    f4 v        = load_stream(in + i);
    QdqParams p = load_params(table, map.C, map.channel(i * 4));
    uint64_t e  = (uint64_t) i * 4;
    f4 r;
    r.x = apply<Op::QDQ, STOCHASTIC>(v.x, p, 0.f, seed, e + 0);
    r.y = apply<Op::QDQ, STOCHASTIC>(v.y, p, 0.f, seed, e + 1);
    r.z = apply<Op::QDQ, STOCHASTIC>(v.z, p, 0.f, seed, e + 2);
    r.w = apply<Op::QDQ, STOCHASTIC>(v.w, p, 0.f, seed, e + 3);
    store_stream(r, out + i);
}

template <bool STOCHASTIC>
__global__ __launch_bounds__(kBlock) void channel_scalar_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                                uint32_t n, ChannelMap map,
                                                                const float* __restrict__ table, uint64_t seed)
{
    const uint32_t stride = gridDim.x * kBlock;
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
    {
        QdqParams p = load_params(table, map.C, map.channel(i));
        out[i]      = apply<Op::QDQ, STOCHASTIC>(in[i], p, 0.f, seed, i);
    }
}

// 64-bit fallback (tensors of >= 2^31 elements).
template <bool STOCHASTIC>
__global__ __launch_bounds__(kBlock) void channel_scalar64_kernel(const float* __restrict__ in,
                                                                  float* __restrict__ out, int64_t n, int64_t C,
                                                                  int64_t K, const float* __restrict__ table,
                                                                  uint64_t seed)
{
    const int64_t stride = (int64_t) gridDim.x * kBlock;
    for (int64_t i = (int64_t) blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
    {
        uint32_t c  = (uint32_t) ((i / K) % C);
        QdqParams p = load_params(table, (uint32_t) C, c);
        out[i]      = apply<Op::QDQ, STOCHASTIC>(in[i], p, 0.f, seed, (uint64_t) i);
    }
}

// ---------------------------------------------------------------------------------------
// STE backward: grad_in = grad * (min <= x <= max)
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ float ste(float x, float g, float mn, float mx)
{
    return g * ((mn <= x && x <= mx) ? 1.0f : 0.0f);
}

__global__ __launch_bounds__(kBlock) void ste_tensor_vec_kernel(const f4* __restrict__ x, const f4* __restrict__ g,
                                                                f4* __restrict__ gi, int64_t nvec, float mn, float mx)
{
    const int64_t i = (int64_t) blockIdx.x * kBlock + threadIdx.x;
    if (i >= nvec)
        return;
    f4 a = load_stream(x + i), b = load_stream(g + i), r;
    r.x = ste(a.x, b.x, mn, mx);
    r.y = ste(a.y, b.y, mn, mx);
    r.z = ste(a.z, b.z, mn, mx);
    r.w = ste(a.w, b.w, mn, mx);
    store_stream(r, gi + i);
}

__global__ __launch_bounds__(kBlock) void ste_scalar_kernel(const float* __restrict__ x, const float* __restrict__ g,
                                                            float* __restrict__ gi, int64_t begin, int64_t n,
                                                            int64_t C, int64_t K, const float* __restrict__ mins,
                                                            const float* __restrict__ maxs, float smin, float smax,
                                                            int use_scalars)
{
    const int64_t stride = (int64_t) gridDim.x * kBlock;
    for (int64_t i = begin + (int64_t) blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
    {
        float mn = smin, mx = smax;
        if (!use_scalars)
        {
            int64_t c = (C == 1) ? 0 : (i / K) % C;
            mn        = mins[c];
            mx        = maxs[c];
        }
        gi[i] = ste(x[i], g[i], mn, mx);
    }
}

__global__ __launch_bounds__(kBlock) void ste_channel_vec_kernel(const f4* __restrict__ x, const f4* __restrict__ g,
                                                                 f4* __restrict__ gi, uint32_t nvec, ChannelMap map,
                                                                 const float* __restrict__ mins,
                                                                 const float* __restrict__ maxs)
{
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= nvec)
        return;
    uint32_t c = map.channel(i * 4);
    float mn = mins[c], mx = maxs[c];
    f4 a = load_stream(x + i), b = load_stream(g + i), r;
    r.x = ste(a.x, b.x, mn, mx);
    r.y = ste(a.y, b.y, mn, mx);
    r.z = ste(a.z, b.z, mn, mx);
    r.w = ste(a.w, b.w, mn, mx);
    store_stream(r, gi + i);
}

// ---------------------------------------------------------------------------------------
// Batched per-channel QDQ (one launch for many tensors)
// ---------------------------------------------------------------------------------------
struct BatchDesc
{
    const float* in;
    float* out;
    const float* table;
    ChannelMap map;
    uint32_t n;           // elements
    uint32_t vec;         // 16-B vector path (K % 4 == 0, aligned)
    uint32_t block0;      // first workgroup of this tensor in the flattened grid
    uint32_t pad;
};

template <bool STOCHASTIC>
__global__ __launch_bounds__(kBlock) void channel_batch_kernel(const BatchDesc* __restrict__ descs, int count,
                                                               uint64_t seed)
{
    // find the tensor of this workgroup (block0 is increasing): scalar binary search
    int lo = 0, hi = count - 1;
    const uint32_t b = blockIdx.x;
    while (lo < hi)
    {
        int mid = (lo + hi + 1) >> 1;
        if (descs[mid].block0 <= b)
            lo = mid;
        else
            hi = mid - 1;
    }
    const BatchDesc& d = descs[lo];
    const uint32_t t   = (b - d.block0) * kBlock + threadIdx.x;
    if (d.vec)
    {
        if (t >= d.n / 4)
            return;
        f4 v        = load_stream(reinterpret_cast<const f4*>(d.in) + t);
        QdqParams p = load_params(d.table, d.map.C, d.map.channel(t * 4));
        uint64_t e  = ((uint64_t) lo << 40) + (uint64_t) t * 4;
        f4 r;
        r.x = apply<Op::QDQ, STOCHASTIC>(v.x, p, 0.f, seed, e + 0);
        r.y = apply<Op::QDQ, STOCHASTIC>(v.y, p, 0.f, seed, e + 1);
        r.z = apply<Op::QDQ, STOCHASTIC>(v.z, p, 0.f, seed, e + 2);
        r.w = apply<Op::QDQ, STOCHASTIC>(v.w, p, 0.f, seed, e + 3);
        store_stream(r, reinterpret_cast<f4*>(d.out) + t);
    }
    else
    {
        if (t >= d.n)
            return;
        QdqParams p = load_params(d.table, d.map.C, d.map.channel(t));
        d.out[t]    = apply<Op::QDQ, STOCHASTIC>(d.in[t], p, 0.f, seed, ((uint64_t) lo << 40) + t);
    }
}

inline bool aligned16(const void* a, const void* b, const void* c = nullptr)
{
    return ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b) | reinterpret_cast<uintptr_t>(c)) & 15) ==
           0;
}

}   // namespace

// -------------------------------------------------------------------------------------------
// Host side of the per-tensor encoding (TensorQuantizationSim.cpp:62-92), exact double math.
// -------------------------------------------------------------------------------------------
aimet_tf_encoding fill_encoding_info(int32_t bw, double mn, double mx);   // encodings.cpp

void per_channel_table_host(const aimet_tf_encoding* encs, int64_t C, float* table);   // encodings.cpp

QdqParams tensor_params(const aimet_tf_encoding& enc)
{
    aimet_tf_encoding e = fill_encoding_info(enc.bw, enc.min, enc.max);
    return QdqParams {(float) e.min, (float) e.max, (float) e.delta, (float) e.offset};
}

}   // namespace aimet_amd

using namespace aimet_amd;

struct aimet_qdq_plan
{
    int device          = 0;
    int count           = 0;
    uint32_t blocks     = 0;
    BatchDesc* descs    = nullptr;   // device
};

extern "C" {

int aimet_qdq_channel_plan_create(const aimet_qdq_channel_desc* descs, int64_t count, int device, aimet_qdq_plan** out)
{
    return guarded([&] {
        AIMET_REQUIRE(out != nullptr && descs != nullptr && count > 0, "empty plan");
        AIMET_REQUIRE(count < (1 << 20), "too many tensors in one plan");
        std::vector<BatchDesc> h((size_t) count);
        uint64_t blocks = 0;
        for (int64_t i = 0; i < count; ++i)
        {
            const auto& d = descs[i];
            AIMET_REQUIRE(d.outer >= 0 && d.C > 0 && d.K >= 0, "invalid per-channel shape");
            int64_t n = d.outer * d.C * d.K;
            AIMET_REQUIRE(n < (int64_t(1) << 31), "batched per-channel QDQ needs < 2^31 elements per tensor");
            if (n > 0)
            {
                require_device_ptr(d.in, "input");
                require_device_ptr(d.out, "output");
                require_device_ptr(d.table, "table");
            }
            BatchDesc& b = h[(size_t) i];
            b.in         = d.in;
            b.out        = d.out;
            b.table      = d.table;
            b.map        = ChannelMap {FastDiv((uint32_t) (d.K > 0 ? d.K : 1)), FastDiv((uint32_t) d.C), (uint32_t) d.C};
            b.n          = (uint32_t) n;
            b.vec        = (d.K % 4 == 0 && aligned16(d.in, d.out)) ? 1u : 0u;
            b.block0     = (uint32_t) blocks;
            b.pad        = 0;
            blocks += (uint64_t) ceil_div(b.vec ? n / 4 : n, kBlock);
        }
        AIMET_REQUIRE(blocks < (uint64_t(1) << 31), "plan too large");
        auto* plan   = new aimet_qdq_plan();
        plan->device = device;
        plan->count  = (int) count;
        plan->blocks = (uint32_t) blocks;
        int prev     = 0;
        AIMET_HIP_CHECK(hipGetDevice(&prev));
        AIMET_HIP_CHECK(hipSetDevice(device));
        hipError_t e = hipMalloc(&plan->descs, sizeof(BatchDesc) * count);
        if (e == hipSuccess)
            e = hipMemcpy(plan->descs, h.data(), sizeof(BatchDesc) * count, hipMemcpyHostToDevice);
        (void) hipSetDevice(prev);
        if (e != hipSuccess)
        {
            if (plan->descs)
                (void) hipFree(plan->descs);
            delete plan;
            throw HipError(std::string("plan upload: ") + hipGetErrorString(e));
        }
        *out = plan;
    });
}

int aimet_qdq_channel_plan_run(aimet_qdq_plan* plan, int round_mode, uint64_t seed, void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(plan != nullptr, "plan is null");
        AIMET_REQUIRE(round_mode == AIMET_ROUND_NEAREST || round_mode == AIMET_ROUND_STOCHASTIC,
                      "Unknown rounding mode.");
        if (plan->blocks == 0)
            return;
        hipStream_t s = as_stream(stream);
        if (round_mode == AIMET_ROUND_STOCHASTIC)
            channel_batch_kernel<true><<<plan->blocks, kBlock, 0, s>>>(plan->descs, plan->count, seed);
        else
            channel_batch_kernel<false><<<plan->blocks, kBlock, 0, s>>>(plan->descs, plan->count, seed);
        AIMET_LAUNCH_CHECK();
    });
}

int aimet_qdq_channel_plan_destroy(aimet_qdq_plan* plan)
{
    return guarded([&] {
        if (!plan)
            return;
        if (plan->descs)
        {
            AIMET_HIP_CHECK(hipDeviceSynchronize());
            AIMET_HIP_CHECK(hipFree(plan->descs));
        }
        delete plan;
    });
}

int aimet_qdq_per_tensor(const float* in, float* out, int64_t n, const aimet_tf_encoding* enc, int round_mode,
                         uint64_t seed, void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(enc != nullptr, "encoding is null");
        AIMET_REQUIRE(n >= 0, "negative element count");
        if (n == 0)
            return;
        require_device_ptr(in, "input");
        require_device_ptr(out, "output");
        QdqParams p = tensor_params(*enc);
        if (round_mode == AIMET_ROUND_NEAREST)
            launch_tensor<Op::QDQ, false>(in, out, n, p, 0.f, seed, as_stream(stream));
        else if (round_mode == AIMET_ROUND_STOCHASTIC)
            launch_tensor<Op::QDQ, true>(in, out, n, p, 0.f, seed, as_stream(stream));
        else
            throw RuntimeError("Unknown rounding mode.");
    });
}

int aimet_quantize_per_tensor(const float* in, float* out, int64_t n, const aimet_tf_encoding* enc, int round_mode,
                              int shift_to_signed, uint64_t seed, void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(enc != nullptr, "encoding is null");
        AIMET_REQUIRE(n >= 0, "negative element count");
        if (n == 0)
            return;
        require_device_ptr(in, "input");
        require_device_ptr(out, "output");
        QdqParams p = tensor_params(*enc);
        // trim_functions.cpp:206-212: unsigned int shift = pow(2, bw-1), subtracted as float
        unsigned int shift = shift_to_signed ? (unsigned int) std::pow(2.0, (double) (enc->bw - 1)) : 0u;
        if (round_mode == AIMET_ROUND_NEAREST)
            launch_tensor<Op::QUANTIZE, false>(in, out, n, p, (float) shift, seed, as_stream(stream));
        else if (round_mode == AIMET_ROUND_STOCHASTIC)
            launch_tensor<Op::QUANTIZE, true>(in, out, n, p, (float) shift, seed, as_stream(stream));
        else
            throw RuntimeError("Unknown rounding mode.");
    });
}

int aimet_per_channel_table(const aimet_tf_encoding* encs, int64_t C, float* table, void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(encs != nullptr && C > 0, "per-channel table needs at least one encoding");
        require_device_ptr(table, "table");
        std::vector<float> t(4 * (size_t) C);
        per_channel_table_host(encs, C, t.data());
        hipStream_t s = as_stream(stream);
        AIMET_HIP_CHECK(hipMemcpyAsync(table, t.data(), sizeof(float) * 4 * C, hipMemcpyHostToDevice, s));
        // pageable source: complete the copy before `t` goes out of scope (once per encoding change)
        AIMET_HIP_CHECK(hipStreamSynchronize(s));
    });
}

int aimet_make_delta_offset(const aimet_tf_encoding* encs, int64_t C, float* table, void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(encs != nullptr && C > 0, "makeDeltaOffsetTensor needs at least one encoding");
        require_device_ptr(table, "table");
        std::vector<float> v(2 * (size_t) C);
        for (int64_t c = 0; c < C; ++c)
        {
            v[c]     = (float) encs[c].delta;
            v[C + c] = (float) encs[c].offset;
        }
        hipStream_t s = as_stream(stream);
        AIMET_HIP_CHECK(hipMemcpyAsync(table, v.data(), sizeof(float) * 2 * C, hipMemcpyHostToDevice, s));
        AIMET_HIP_CHECK(hipStreamSynchronize(s));
    });
}

int aimet_qdq_per_channel(const float* in, float* out, int64_t outer, int64_t C, int64_t K, const float* table,
                          int round_mode, uint64_t seed, void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(outer >= 0 && C > 0 && K >= 0, "invalid per-channel shape");
        int64_t n = outer * C * K;
        if (n == 0)
            return;
        require_device_ptr(in, "input");
        require_device_ptr(out, "output");
        require_device_ptr(table, "table");
        AIMET_REQUIRE(round_mode == AIMET_ROUND_NEAREST || round_mode == AIMET_ROUND_STOCHASTIC,
                      "Unknown rounding mode.");
        bool sto      = round_mode == AIMET_ROUND_STOCHASTIC;
        hipStream_t s = as_stream(stream);
        if (n >= (int64_t(1) << 31))
        {
            int blocks = stream_blocks(n, kBlock);
            if (sto)
                channel_scalar64_kernel<true><<<blocks, kBlock, 0, s>>>(in, out, n, C, K, table, seed);
            else
                channel_scalar64_kernel<false><<<blocks, kBlock, 0, s>>>(in, out, n, C, K, table, seed);
            AIMET_LAUNCH_CHECK();
            return;
        }
        ChannelMap map {FastDiv((uint32_t) K), FastDiv((uint32_t) C), (uint32_t) C};
        if (K % 4 == 0 && aligned16(in, out))
        {
            uint32_t nvec = (uint32_t) (n / 4);
            unsigned blocks = (unsigned) ceil_div(nvec, kBlock);
            if (sto)
                channel_vec_kernel<true><<<blocks, kBlock, 0, s>>>(reinterpret_cast<const f4*>(in),
                                                                    reinterpret_cast<f4*>(out), nvec, map, table,
                                                                    seed);
            else
                channel_vec_kernel<false><<<blocks, kBlock, 0, s>>>(reinterpret_cast<const f4*>(in),
                                                                     reinterpret_cast<f4*>(out), nvec, map, table,
                                                                     seed);
        }
        else
        {
            int blocks = stream_blocks(n, kBlock);
            if (sto)
                channel_scalar_kernel<true><<<blocks, kBlock, 0, s>>>(in, out, (uint32_t) n, map, table, seed);
            else
                channel_scalar_kernel<false><<<blocks, kBlock, 0, s>>>(in, out, (uint32_t) n, map, table, seed);
        }
        AIMET_LAUNCH_CHECK();
    });
}

int aimet_ste_backward_per_tensor(const float* x, const float* g, float* gi, int64_t n, float mn, float mx,
                                  void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(n >= 0, "negative element count");
        if (n == 0)
            return;
        require_device_ptr(x, "x");
        require_device_ptr(g, "grad");
        require_device_ptr(gi, "grad_in");
        hipStream_t s = as_stream(stream);
        int64_t nvec  = aligned16(x, g, gi) ? n / 4 : 0;
        if (nvec > 0)
        {
            ste_tensor_vec_kernel<<<(unsigned) ceil_div(nvec, kBlock), kBlock, 0, s>>>(
                reinterpret_cast<const f4*>(x), reinterpret_cast<const f4*>(g), reinterpret_cast<f4*>(gi), nvec, mn,
                mx);
            AIMET_LAUNCH_CHECK();
        }
        if (nvec * 4 < n)
        {
            int blocks = stream_blocks(n - nvec * 4, kBlock);
            ste_scalar_kernel<<<blocks, kBlock, 0, s>>>(x, g, gi, nvec * 4, n, 1, 1, nullptr, nullptr, mn, mx, 1);
            AIMET_LAUNCH_CHECK();
        }
    });
}

int aimet_ste_backward(const float* x, const float* g, float* gi, int64_t outer, int64_t C, int64_t K,
                       const float* mins, const float* maxs, void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(outer >= 0 && C > 0 && K >= 0, "invalid per-channel shape");
        int64_t n = outer * C * K;
        if (n == 0)
            return;
        require_device_ptr(x, "x");
        require_device_ptr(g, "grad");
        require_device_ptr(gi, "grad_in");
        require_device_ptr(mins, "encoding min");
        require_device_ptr(maxs, "encoding max");
        hipStream_t s = as_stream(stream);
        if (n < (int64_t(1) << 31) && K % 4 == 0 && aligned16(x, g, gi))
        {
            ChannelMap map {FastDiv((uint32_t) K), FastDiv((uint32_t) C), (uint32_t) C};
            uint32_t nvec = (uint32_t) (n / 4);
            ste_channel_vec_kernel<<<(unsigned) ceil_div(nvec, kBlock), kBlock, 0, s>>>(
                reinterpret_cast<const f4*>(x), reinterpret_cast<const f4*>(g), reinterpret_cast<f4*>(gi), nvec, map,
                mins, maxs);
        }
        else
        {
            int blocks = stream_blocks(n, kBlock);
            ste_scalar_kernel<<<blocks, kBlock, 0, s>>>(x, g, gi, 0, n, C, K, mins, maxs, 0.f, 0.f, 0);
        }
        AIMET_LAUNCH_CHECK();
    });
}

}   // extern "C"
