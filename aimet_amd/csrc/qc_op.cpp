// qc_op.cpp -- the ONNX QcQuantizeOp (onnx/src/QcQuantizeOp.cpp:62-113 computeImpl and the
// mode-specific actions of onnx/src/AimetOpUtils.h:101-330) over the library's kernels, plus the
// BroadcastShapeInfo view of blockwise quantization (onnx/src/QuantizeDequantizeUtils.cpp:100-213).
//
// The reference op is an onnxruntime custom op holding one TensorQuantizer per encoding; its CUDA
// flavour synchronises the stream for updateStats / oneShot (the statistics ran on the host),
// slices every channel into a scratch buffer and runs one analyzer update per channel or block.
// Here the op is stream-ordered: statistics of all channels / blocks are ONE per-channel update of
// an aimet_tensor_quantizer with num_channels == num_encodings, read directly in the [outer][C][K]
// layout (blocks that are not contiguous are first permuted into contiguous order, as the
// reference does), and only a oneShot's encoding computation synchronises.
#include <atomic>
#include <cstring>
#include <string>
#include <vector>

#include "common.hpp"

using namespace aimet_amd;

namespace
{

void check(int rc)
{
    if (rc != AIMET_OK)
        throw RuntimeError(aimet_last_error());
}

std::vector<int64_t> row_major_strides(const std::vector<int64_t>& shape)
{
    std::vector<int64_t> st(shape.size());
    int64_t s = 1;
    for (size_t i = shape.size(); i-- > 0;)
    {
        st[i] = s;
        s *= shape[i];
    }
    return st;
}

int64_t product(const std::vector<int64_t>& v)
{
    int64_t p = 1;
    for (int64_t x: v)
        p *= x;
    return p;
}

// QuantizeDequantizeUtils.cpp:100-155
void shape_info(const int64_t* input_shape, int64_t ndims, int channel_axis, int block_axis, int block_size,
                aimet_broadcast_shape_info& out)
{
    AIMET_REQUIRE(ndims >= 0 && (ndims == 0 || input_shape != nullptr), "invalid input shape");
    std::vector<int64_t> tshape, eshape;
    for (int64_t i = 0; i < ndims; ++i)
    {
        AIMET_REQUIRE(input_shape[i] >= 0, "negative dimension");
        if (i == channel_axis)
        {
            tshape.push_back(input_shape[i]);
            eshape.push_back(input_shape[i]);
        }
        else if (i == block_axis)
        {
            AIMET_REQUIRE(block_size > 0, "block size must be positive along the block axis");
            if (input_shape[i] % block_size != 0)
                throw RuntimeError("Block dimension is not evenly divisible by block size.");
            tshape.push_back(input_shape[i] / block_size);
            tshape.push_back(block_size);
            eshape.push_back(input_shape[i] / block_size);
            eshape.push_back(1);
        }
        else
        {
            tshape.push_back(input_shape[i]);
            eshape.push_back(1);
        }
    }
    AIMET_REQUIRE(tshape.size() <= AIMET_BCAST_MAX_DIMS, "too many dimensions");
    std::memset(&out, 0, sizeof(out));
    out.num_dims      = (int64_t) tshape.size();
    out.num_elements  = 1;
    for (int64_t i = 0; i < ndims; ++i)
        out.num_elements *= input_shape[i];
    out.num_encodings = product(eshape);
    auto ts = row_major_strides(tshape), es = row_major_strides(eshape);
    for (size_t i = 0; i < tshape.size(); ++i)
    {
        out.tensor_shape[i]     = tshape[i];
        out.encoding_shape[i]   = eshape[i];
        out.tensor_strides[i]   = ts[i];
        out.encoding_strides[i] = (eshape[i] == 1 && tshape[i] != 1) ? 0 : es[i];
    }
    // hasContiguousBlocks (:157-170): no broadcast dim followed by a non-broadcast one
    bool prev_bcast = false;
    out.contiguous_blocks = 1;
    for (size_t i = 0; i < tshape.size(); ++i)
    {
        if (prev_bcast && tshape[i] == eshape[i])
            out.contiguous_blocks = 0;
        prev_bcast = tshape[i] != eshape[i];
    }
}

// copyToContiguousBlockLayout (:173-213): non-broadcast dims first, broadcast dims last
void block_layout_strides(const aimet_broadcast_shape_info& si, std::vector<int64_t>& ostr)
{
    const int64_t nd = si.num_dims;
    std::vector<int64_t> order;
    for (int64_t i = 0; i < nd; ++i)
        if (si.encoding_strides[i] != 0)
            order.push_back(i);
    for (int64_t i = 0; i < nd; ++i)
        if (si.encoding_strides[i] == 0)
            order.push_back(i);
    ostr.assign(nd, 0);
    ostr[order[nd - 1]] = 1;
    for (int64_t i = nd - 2; i >= 0; --i)
        ostr[order[i]] = ostr[order[i + 1]] * si.tensor_shape[order[i + 1]];
}

// [4][E] float table {min, max, delta, offset} of the host encodings, uploaded stream-ordered
float* encoding_table(const aimet_tf_encoding* encs, int64_t E, hipStream_t s)
{
    std::vector<float> t(4 * (size_t) E);
    for (int64_t i = 0; i < E; ++i)
    {
        t[i]         = (float) encs[i].min;
        t[E + i]     = (float) encs[i].max;
        t[2 * E + i] = (float) encs[i].delta;
        t[3 * E + i] = (float) encs[i].offset;
    }
    return static_cast<float*>(upload_async(t.data(), t.size() * sizeof(float), s));
}

void copy_through(const float* in, float* out, int64_t n, hipStream_t s)
{
    if (in != out && n > 0)
        AIMET_HIP_CHECK(hipMemcpyAsync(out, in, sizeof(float) * n, hipMemcpyDeviceToDevice, s));
}

uint64_t next_seed()
{
    static std::atomic<uint64_t> seed {0x243F6A8885A308D3ull};
    return seed.fetch_add(0x9E3779B97F4A7C15ull);
}

// computeEncoding(enc.bw, useSymmetricEncoding) of every analyzer into the info's encodings
// (min, max, offset, delta; bw kept), one getEncoding per distinct bit-width
void compute_encodings(aimet_qc_quantize_info* info, void* stream)
{
    const int64_t E = info->num_encodings;
    std::vector<aimet_tf_encoding> got((size_t) E);
    std::vector<int32_t> done;
    for (int64_t i = 0; i < E; ++i)
    {
        int32_t bw = info->encodings[i].bw;
        bool seen  = false;
        for (int32_t d: done)
            seen |= d == bw;
        if (seen)
            continue;
        done.push_back(bw);
        int valid = 0;
        check(aimet_tq_get_encoding(info->quantizer, (uint32_t) bw, info->use_symmetric_encoding,
                                    info->use_strict_symmetric, info->use_unsigned_symmetric, got.data(), &valid,
                                    stream));
        for (int64_t j = 0; j < E; ++j)
            if (info->encodings[j].bw == bw)
            {
                info->encodings[j].min    = got[j].min;
                info->encodings[j].max    = got[j].max;
                info->encodings[j].offset = got[j].offset;
                info->encodings[j].delta  = got[j].delta;
            }
    }
}

void require_quantizer(aimet_qc_quantize_info* info, int64_t channels)
{
    AIMET_REQUIRE(info->quantizer != nullptr, "the QcQuantizeInfo has no tensor quantizer");
    int64_t c = 0;
    check(aimet_tq_num_channels(info->quantizer, &c));
    AIMET_REQUIRE(c == channels, "the tensor quantizer has " + std::to_string(c) + " analyzers, the op needs " +
                                     std::to_string(channels));
}

// modeSpecificActionInt (AimetOpUtils.h:101-150)
void per_tensor(aimet_qc_quantize_info* info, int mode, const float* in, float* out, int64_t n, void* stream)
{
    hipStream_t s = as_stream(stream);
    AIMET_REQUIRE(info->num_encodings >= 1, "no encoding");
    aimet_tf_encoding* enc = &info->encodings[0];
    switch (mode)
    {
    case AIMET_OP_ONE_SHOT_QUANTIZE_DEQUANTIZE:
    {
        require_quantizer(info, 1);
        check(aimet_tq_reset_encoding_stats(info->quantizer, stream));
        check(aimet_tq_update_stats(info->quantizer, in, 1, 1, n, stream));
        aimet_tf_encoding e {};
        int valid = 0;
        check(aimet_tq_get_encoding(info->quantizer, (uint32_t) enc->bw, info->use_symmetric_encoding,
                                    info->use_strict_symmetric, info->use_unsigned_symmetric, &e, &valid, stream));
        aimet_tf_encoding q = e;
        q.bw                = enc->bw;
        check(aimet_qdq_per_tensor(in, out, n, &q, info->rounding_mode, next_seed(), stream));
        enc->min    = e.min;
        enc->max    = e.max;
        enc->offset = e.offset;
        enc->delta  = e.delta;
        break;
    }
    case AIMET_OP_UPDATE_STATS:
        require_quantizer(info, 1);
        check(aimet_tq_update_stats(info->quantizer, in, 1, 1, n, stream));
        copy_through(in, out, n, s);
        break;
    case AIMET_OP_QUANTIZE_DEQUANTIZE:
        check(aimet_qdq_per_tensor(in, out, n, enc, info->rounding_mode, next_seed(), stream));
        break;
    case AIMET_OP_PASS_THROUGH:
        copy_through(in, out, n, s);
        break;
    default:
        throw RuntimeError("unknown op mode");
    }
}

// modeSpecificActionPerChannelInt (AimetOpUtils.h:153-216) + quantizeDequantizePerChannel
// (QuantizeDequantizeUtils.hpp:109-163: the raw encodings as the per-channel table)
void per_channel(aimet_qc_quantize_info* info, int mode, const float* in, float* out, const int64_t* shape,
                 int64_t ndims, int64_t n, void* stream)
{
    hipStream_t s = as_stream(stream);
    const int axis = info->channel_axis;
    AIMET_REQUIRE(axis >= 0 && axis < ndims, "channel axis out of range");
    const int64_t C = shape[axis];
    if (C != info->num_encodings)
        throw RuntimeError("Channel dimensions do not match encoding vector size.");
    int64_t outer = 1, K = 1;
    for (int64_t i = 0; i < ndims; ++i)
    {
        if (i < axis)
            outer *= shape[i];
        else if (i > axis)
            K *= shape[i];
    }
    auto qdq = [&] {
        float* t = encoding_table(info->encodings, C, s);
        int rc   = aimet_qdq_per_channel(in, out, outer, C, K, t, info->rounding_mode, next_seed(), stream);
        scratch_free(t, s);
        check(rc);
    };
    switch (mode)
    {
    case AIMET_OP_ONE_SHOT_QUANTIZE_DEQUANTIZE:
        require_quantizer(info, C);
        check(aimet_tq_reset_encoding_stats(info->quantizer, stream));
        check(aimet_tq_update_stats(info->quantizer, in, outer, C, K, stream));
        compute_encodings(info, stream);
        qdq();
        break;
    case AIMET_OP_UPDATE_STATS:
        require_quantizer(info, C);
        check(aimet_tq_update_stats(info->quantizer, in, outer, C, K, stream));
        copy_through(in, out, n, s);
        break;
    case AIMET_OP_QUANTIZE_DEQUANTIZE:
        qdq();
        break;
    case AIMET_OP_PASS_THROUGH:
        copy_through(in, out, n, s);
        break;
    default:
        throw RuntimeError("unknown op mode");
    }
}

// modeSpecificActionBroadcastInt (AimetOpUtils.h:218-297)
void broadcast(aimet_qc_quantize_info* info, int mode, const float* in, float* out, const int64_t* shape,
               int64_t ndims, void* stream)
{
    hipStream_t s = as_stream(stream);
    aimet_broadcast_shape_info si;
    shape_info(shape, ndims, info->channel_axis, info->block_axis, info->block_size, si);
    const int64_t E = si.num_encodings, n = si.num_elements;
    if (E != info->num_encodings)
        throw RuntimeError("Expected number of encodings (" + std::to_string(E) +
                           ") does not match provided encoding list size (" + std::to_string(info->num_encodings) +
                           ").");
    auto stats = [&] {
        require_quantizer(info, E);
        const float* buf = in;
        float* tmp       = nullptr;
        if (!si.contiguous_blocks && n > 0)
        {
            tmp = static_cast<float*>(scratch_alloc(sizeof(float) * n, s));
            check(aimet_copy_to_contiguous_block_layout(in, tmp, &si, stream));
            buf = tmp;
        }
        int rc = aimet_tq_update_stats(info->quantizer, buf, 1, E, E ? n / E : 0, stream);
        if (tmp)
            scratch_free(tmp, s);
        check(rc);
    };
    auto qdq = [&] {
        float* t = encoding_table(info->encodings, E, s);
        int rc   = aimet_qdq_broadcast(in, out, n, si.num_dims, si.tensor_strides, si.encoding_strides, t, t + E,
                                       t + 2 * E, t + 3 * E, stream);
        scratch_free(t, s);
        check(rc);
    };
    switch (mode)
    {
    case AIMET_OP_ONE_SHOT_QUANTIZE_DEQUANTIZE:
        check(aimet_tq_reset_encoding_stats(info->quantizer, stream));
        stats();
        compute_encodings(info, stream);
        qdq();
        break;
    case AIMET_OP_QUANTIZE_DEQUANTIZE:
        qdq();
        break;
    case AIMET_OP_UPDATE_STATS:
        stats();
        copy_through(in, out, n, s);
        break;
    case AIMET_OP_PASS_THROUGH:
        copy_through(in, out, n, s);
        break;
    default:
        throw RuntimeError("unknown op mode");
    }
}

// modeSpecificActionFloat (AimetOpUtils.h:299-330)
void float_path(int mode, const float* in, float* out, int64_t n, void* stream)
{
    switch (mode)
    {
    case AIMET_OP_ONE_SHOT_QUANTIZE_DEQUANTIZE:
    case AIMET_OP_QUANTIZE_DEQUANTIZE:
        check(aimet_qdq_fp16(in, out, n, stream));
        break;
    case AIMET_OP_UPDATE_STATS:
    case AIMET_OP_PASS_THROUGH:
        copy_through(in, out, n, as_stream(stream));
        break;
    default:
        throw RuntimeError("unknown op mode");
    }
}

}   // namespace

extern "C" {

int aimet_broadcast_shape_info_init(const int64_t* input_shape, int64_t ndims, int channel_axis, int block_axis,
                                    int block_size, aimet_broadcast_shape_info* out)
{
    return guarded([&] {
        AIMET_REQUIRE(out != nullptr, "output is null");
        shape_info(input_shape, ndims, channel_axis, block_axis, block_size, *out);
    });
}

int aimet_copy_to_contiguous_block_layout(const float* in, float* out, const aimet_broadcast_shape_info* si,
                                          void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(si != nullptr, "shape info is null");
        AIMET_REQUIRE(si->num_dims > 0 && si->num_dims <= AIMET_BCAST_MAX_DIMS, "invalid shape info");
        std::vector<int64_t> ostr;
        block_layout_strides(*si, ostr);
        check(aimet_permute_tensor(in, out, si->num_elements, si->num_dims, si->tensor_strides, ostr.data(), stream));
    });
}

int aimet_qc_quantize_op_compute(aimet_qc_quantize_info* info, const float* in, float* out, const int64_t* shape,
                                 int64_t ndims, void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(info != nullptr, "quant info is null");
        AIMET_REQUIRE(ndims >= 0 && (ndims == 0 || shape != nullptr), "invalid shape");
        AIMET_REQUIRE(info->num_encodings >= 0 && (info->num_encodings == 0 || info->encodings != nullptr),
                      "encodings are null");
        int64_t n = 1;
        for (int64_t i = 0; i < ndims; ++i)
        {
            AIMET_REQUIRE(shape[i] >= 0, "negative dimension");
            n *= shape[i];
        }
        const int mode = info->enabled ? info->op_mode : AIMET_OP_PASS_THROUGH;   // disabled: pass through
        if (!info->is_int_data_type)
            float_path(mode, in, out, n, stream);
        else if (!info->use_per_channel_mode)
            per_tensor(info, mode, in, out, n, stream);
        else if (info->block_size == 0)
            per_channel(info, mode, in, out, shape, ndims, n, stream);
        else
            broadcast(info, mode, in, out, shape, ndims, stream);
        // oneShot runs once; afterwards the op only quantize-dequantizes (QcQuantizeOp.cpp:108-112)
        if (mode == AIMET_OP_ONE_SHOT_QUANTIZE_DEQUANTIZE)
            info->op_mode = AIMET_OP_QUANTIZE_DEQUANTIZE;
    });
}

}   // extern "C"
