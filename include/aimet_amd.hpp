// aimet_amd.hpp -- the reference's C++-level interfaces for non-Python callers (ONNX / TF custom
// ops), header-only over the C-ABI of aimet_amd.h ("C++-level interfaces").
//
//   IQuantizationEncodingAnalyzer<float>   DlQuantization/IQuantizationEncodingAnalyzer.hpp:48-126
//   getEncodingAnalyzerInstance<float>     DlQuantization/QuantizerFactory.hpp (QuantizerFactory.cpp:74-104)
//   ITensorQuantizationSim<float>          DlQuantization/ITensorQuantizationSim.h:47-123
//   TensorQuantizerOpFacade / TensorQuantizer  DlQuantization/TensorQuantizerOpFacade.h:63-102,
//                                          DlQuantization/TensorQuantizer.h
//
// Same virtual signatures, with `void* stream` = hipStream_t (the overloads without a stream use
// the stream given at construction, default: the legacy default stream). Every tensor pointer is
// MI355X device memory: ComputationMode COMP_MODE_CPU / use_cuda == false, and the host-vector
// entry points of ITensorQuantizationSim (split channel vectors, packed uint8 buffers), throw
// std::runtime_error -- there is no CPU compute path. Errors of the library are rethrown as
// std::invalid_argument / std::runtime_error with aimet_last_error().
#pragma once

#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <tuple>
#include <vector>

#include "aimet_amd.h"

namespace aimet_amd
{

using TfEncoding = aimet_tf_encoding;   // {min, max, delta, offset, bw}: Quantization.hpp:113-120

enum ComputationMode { COMP_MODE_CPU = 0, COMP_MODE_GPU = 1 };   // Quantization.hpp:52-56
enum QuantizationMode {                                          // Quantization.hpp:84-106
    QUANTIZATION_TF = AIMET_QUANTIZATION_TF,
    QUANTIZATION_TF_ENHANCED = AIMET_QUANTIZATION_TF_ENHANCED,
    QUANTIZATION_RANGE_LEARNING = AIMET_QUANTIZATION_RANGE_LEARNING,
    QUANTIZATION_PERCENTILE = AIMET_QUANTIZATION_PERCENTILE,
    QUANTIZATION_MSE = AIMET_QUANTIZATION_MSE,
    QUANTIZATION_ENTROPY = AIMET_QUANTIZATION_ENTROPY
};
enum RoundingMode { ROUND_NEAREST = AIMET_ROUND_NEAREST, ROUND_STOCHASTIC = AIMET_ROUND_STOCHASTIC };
enum class TensorQuantizerOpMode { updateStats, oneShotQuantizeDequantize, quantizeDequantize, passThrough };

// Quantization.hpp:122-129: scratch allocations of the reference. The MI355X kernels keep their
// statistics in a per-quantizer arena, so an allocator passed here is accepted and unused.
class IAllocator
{
public:
    virtual ~IAllocator() = default;
    virtual void* allocateRaw(size_t bytes) = 0;
    virtual void deleteRaw(void* ptr)      = 0;
};

namespace detail
{
inline void check(int rc)
{
    if (rc == AIMET_OK)
        return;
    if (rc == AIMET_ERR_INVALID_ARGUMENT)
        throw std::invalid_argument(aimet_last_error());
    throw std::runtime_error(aimet_last_error());
}

inline void require_device(bool use_cuda)
{
    if (!use_cuda)
        throw std::runtime_error("aimet_amd: device tensors only (MI355X); the core has no CPU path");
}

inline void no_host_path(const char* what)
{
    throw std::runtime_error(std::string("aimet_amd: ") + what +
                             " works on host vectors; the MI355X core has no CPU path");
}

}   // namespace detail

// ---- IQuantizationEncodingAnalyzer<float> -----------------------------------------------------
template <typename DTYPE>
class IQuantizationEncodingAnalyzer
{
public:
    virtual ~IQuantizationEncodingAnalyzer() = default;
    virtual void updateStats(const DTYPE* tensor, const size_t tensorSize, ComputationMode tensorCpuGpuMode) = 0;
    virtual void updateStats(const DTYPE* tensor, const size_t tensorSize, ComputationMode tensorCpuGpuMode,
                             IAllocator* allocator)                                                         = 0;
    virtual TfEncoding computeEncoding(uint8_t bw, bool useSymmetricEncodings, bool useStrictSymmetric,
                                       bool useUnsignedSymmetric) const                                     = 0;
    virtual std::vector<std::tuple<double, double>> getStatsHistogram() const                               = 0;
    virtual void setPercentileValue(float percentile)
    {
        (void) percentile;
        throw std::runtime_error("setPercentileValue: not a percentile analyzer");
    }
    virtual float getPercentileValue()
    {
        throw std::runtime_error("getPercentileValue: not a percentile analyzer");
    }
};

// One analyzer (of any QuantizationMode) whose statistics live in HBM on `device`.
class DeviceEncodingAnalyzer : public IQuantizationEncodingAnalyzer<float>
{
public:
    explicit DeviceEncodingAnalyzer(QuantizationMode mode, int device = 0, void* stream = nullptr)
        : mode_(mode == QUANTIZATION_RANGE_LEARNING ? QUANTIZATION_TF : mode), stream_(stream)
    {
        aimet_tensor_quantizer* q = nullptr;
        detail::check(aimet_tq_create((int) mode_, 1, device, &q));
        q_.reset(q);
    }
    void setStream(void* stream) { stream_ = stream; }
    aimet_tensor_quantizer* handle() const { return q_.get(); }

    void updateStats(const float* tensor, const size_t n, ComputationMode mode) override
    {
        detail::require_device(mode == COMP_MODE_GPU);
        detail::check(aimet_tq_update_stats(q_.get(), tensor, 1, 1, (int64_t) n, stream_));
    }
    void updateStats(const float* tensor, const size_t n, ComputationMode mode, IAllocator*) override
    {
        updateStats(tensor, n, mode);
    }
    TfEncoding computeEncoding(uint8_t bw, bool sym, bool strict, bool unsign) const override
    {
        TfEncoding e {};
        int valid = 0;
        detail::check(aimet_tq_get_encoding(q_.get(), bw, sym, strict, unsign, &e, &valid, stream_));
        return e;   // zeros when no statistics were collected (as the analyzers return)
    }
    std::vector<std::tuple<double, double>> getStatsHistogram() const override
    {
        double xl[512], pdf[512];
        int n = 0;
        detail::check(aimet_tq_get_stats_histogram(q_.get(), 0, xl, pdf, &n, stream_));
        std::vector<std::tuple<double, double>> h;
        for (int i = 0; i < n; ++i)
            h.emplace_back(xl[i], pdf[i]);
        return h;
    }
    void setPercentileValue(float p) override
    {
        if (mode_ != QUANTIZATION_PERCENTILE)
            IQuantizationEncodingAnalyzer<float>::setPercentileValue(p);
        detail::check(aimet_tq_set_percentile_value(q_.get(), p));
    }
    float getPercentileValue() override
    {
        float p = 0;
        detail::check(aimet_tq_get_percentile_value(q_.get(), &p));
        return p;
    }
    void resetStats() { detail::check(aimet_tq_reset_encoding_stats(q_.get(), stream_)); }

private:
    struct Del
    {
        void operator()(aimet_tensor_quantizer* q) const { aimet_tq_destroy(q); }
    };
    QuantizationMode mode_;
    void* stream_;
    std::unique_ptr<aimet_tensor_quantizer, Del> q_;
};

// QuantizerFactory.hpp getEncodingAnalyzerInstance<DTYPE>(QuantizationMode)
template <typename DTYPE>
std::unique_ptr<IQuantizationEncodingAnalyzer<DTYPE>> getEncodingAnalyzerInstance(QuantizationMode mode,
                                                                                  int device = 0)
{
    static_assert(sizeof(DTYPE) == sizeof(float), "the MI355X core analyzes fp32 tensors");
    return std::unique_ptr<IQuantizationEncodingAnalyzer<DTYPE>>(new DeviceEncodingAnalyzer(mode, device));
}

// ---- ITensorQuantizationSim<float> ------------------------------------------------------------
template <typename DTYPE>
class ITensorQuantizationSim
{
public:
    virtual ~ITensorQuantizationSim() = default;
    virtual void quantizeDequantizeTensor(const DTYPE* in, size_t n, DTYPE* out, double encodingMin,
                                          double encodingMax, uint8_t bw, RoundingMode roundMode, bool use_cuda) = 0;
    virtual void quantizeDequantizeTensor(const DTYPE* in, size_t n, DTYPE* out, double encodingMin,
                                          double encodingMax, uint8_t bw, RoundingMode roundMode, bool use_cuda,
                                          void* stream)                                                         = 0;
    virtual void quantizeTensor(const DTYPE* in, size_t n, DTYPE* out, double encodingMin, double encodingMax,
                                uint8_t bw, RoundingMode roundMode, bool use_cuda, bool shiftToSigned)          = 0;
    virtual void quantizeTensorPacked(const DTYPE* in, size_t n, std::vector<uint8_t>& out, double encodingMin,
                                      double encodingMax, uint8_t bw, RoundingMode roundMode, bool useCuda,
                                      bool shiftToSigned)                                                       = 0;
    virtual void dequantizeTensor(const uint8_t* in, size_t n, DTYPE* out, double encodingMin, double encodingMax,
                                  uint8_t bw, bool shiftToSigned)                                               = 0;
    virtual void quantizeDequantizePerChannelTensor(std::vector<std::vector<DTYPE>>& splits,
                                                    std::vector<uint32_t> splitShape, uint32_t axis, DTYPE* out,
                                                    const std::vector<TfEncoding>& encodings, uint8_t bw,
                                                    RoundingMode roundMode, bool useCuda)                       = 0;
    virtual void quantizePerChannelTensorPacked(std::vector<std::vector<DTYPE>>& splits,
                                                std::vector<uint32_t> splitShape, uint32_t axis,
                                                std::vector<uint8_t>& out, const std::vector<TfEncoding>& encodings,
                                                uint8_t bw, RoundingMode roundMode, bool useCuda,
                                                bool shiftToSigned)                                             = 0;
    virtual void dequantizePerChannelTensor(const uint8_t* in, const std::vector<uint32_t>& inputShape, uint32_t axis,
                                            DTYPE* out, uint8_t bw, const std::vector<TfEncoding>& encodings,
                                            bool shiftToSigned)                                                 = 0;
    virtual void fillEncodingInfo(TfEncoding& encoding, uint8_t bw, double encodingMin, double encodingMax)   = 0;
    virtual void generateScaleOffset(double& encodingMin, double& encodingMax, uint8_t bw, double& encodingScale,
                                     double& encodingOffset)                                                    = 0;
    virtual void quantizeDequantizeTensorPerChannel(const DTYPE* in, size_t numChannel, size_t numElement,
                                                    size_t numElementPerChannel, DTYPE* out, DTYPE* encodingMin,
                                                    DTYPE* encodingMax, DTYPE* encodingDelta, DTYPE* encodingOffset,
                                                    RoundingMode roundingMode, bool useCuda)                   = 0;
    virtual void quantizeDequantizeTensorPerChannel(const DTYPE* in, size_t numChannel, size_t numElement,
                                                    size_t numElementPerChannel, DTYPE* out, DTYPE* encodingMin,
                                                    DTYPE* encodingMax, DTYPE* encodingDelta, DTYPE* encodingOffset,
                                                    RoundingMode roundingMode, bool useCuda, void* stream)     = 0;
};

class TensorQuantizationSim : public ITensorQuantizationSim<float>
{
public:
    explicit TensorQuantizationSim(void* stream = nullptr) : stream_(stream) {}

    void quantizeDequantizeTensor(const float* in, size_t n, float* out, double mn, double mx, uint8_t bw,
                                  RoundingMode rm, bool use_cuda) override
    {
        quantizeDequantizeTensor(in, n, out, mn, mx, bw, rm, use_cuda, stream_);
    }
    void quantizeDequantizeTensor(const float* in, size_t n, float* out, double mn, double mx, uint8_t bw,
                                  RoundingMode rm, bool use_cuda, void* stream) override
    {
        detail::require_device(use_cuda);
        TfEncoding e {mn, mx, 0, 0, bw};
        detail::check(aimet_qdq_per_tensor(in, out, (int64_t) n, &e, rm, next_seed(), stream));
    }
    void quantizeTensor(const float* in, size_t n, float* out, double mn, double mx, uint8_t bw, RoundingMode rm,
                        bool use_cuda, bool shiftToSigned) override
    {
        detail::require_device(use_cuda);
        TfEncoding e {mn, mx, 0, 0, bw};
        detail::check(aimet_quantize_per_tensor(in, out, (int64_t) n, &e, rm, shiftToSigned, next_seed(), stream_));
    }
    void quantizeTensorPacked(const float*, size_t, std::vector<uint8_t>&, double, double, uint8_t, RoundingMode,
                              bool, bool) override
    {
        detail::no_host_path("quantizeTensorPacked");
    }
    void dequantizeTensor(const uint8_t*, size_t, float*, double, double, uint8_t, bool) override
    {
        detail::no_host_path("dequantizeTensor (packed host buffer)");
    }
    void quantizeDequantizePerChannelTensor(std::vector<std::vector<float>>&, std::vector<uint32_t>, uint32_t,
                                            float*, const std::vector<TfEncoding>&, uint8_t, RoundingMode,
                                            bool) override
    {
        detail::no_host_path("quantizeDequantizePerChannelTensor (host channel splits)");
    }
    void quantizePerChannelTensorPacked(std::vector<std::vector<float>>&, std::vector<uint32_t>, uint32_t,
                                        std::vector<uint8_t>&, const std::vector<TfEncoding>&, uint8_t, RoundingMode,
                                        bool, bool) override
    {
        detail::no_host_path("quantizePerChannelTensorPacked");
    }
    void dequantizePerChannelTensor(const uint8_t*, const std::vector<uint32_t>&, uint32_t, float*, uint8_t,
                                    const std::vector<TfEncoding>&, bool) override
    {
        detail::no_host_path("dequantizePerChannelTensor (packed host buffer)");
    }
    void fillEncodingInfo(TfEncoding& encoding, uint8_t bw, double mn, double mx) override
    {
        detail::check(aimet_fill_encoding_info(bw, mn, mx, &encoding));
    }
    void generateScaleOffset(double& mn, double& mx, uint8_t bw, double& scale, double& offset) override
    {
        TfEncoding e {};
        detail::check(aimet_fill_encoding_info(bw, mn, mx, &e));
        mn     = e.min;
        mx     = e.max;
        scale  = e.delta;
        offset = e.offset;
    }
    void quantizeDequantizeTensorPerChannel(const float* in, size_t C, size_t n, size_t K, float* out, float* mn,
                                            float* mx, float* delta, float* offset, RoundingMode rm,
                                            bool useCuda) override
    {
        quantizeDequantizeTensorPerChannel(in, C, n, K, out, mn, mx, delta, offset, rm, useCuda, stream_);
    }
    // trim_functions.cpp:697-709: channel = (i / K) % C over n elements, the four encoding arrays
    // (device) used as given. ROUND_NEAREST runs the broadcast kernel over the view [n/(C*K)][C][K].
    void quantizeDequantizeTensorPerChannel(const float* in, size_t C, size_t n, size_t K, float* out, float* mn,
                                            float* mx, float* delta, float* offset, RoundingMode rm, bool useCuda,
                                            void* stream) override
    {
        detail::require_device(useCuda);
        if (rm != ROUND_NEAREST)
            throw std::invalid_argument("quantizeDequantizeTensorPerChannel: ROUND_STOCHASTIC takes the "
                                        "[4][C] table entry point aimet_qdq_per_channel");
        if (n == 0)
            return;
        if (C == 0 || K == 0 || n % (C * K) != 0)
            throw std::invalid_argument("numElement must be a multiple of numChannel * numElementPerChannel");
        int64_t tstr[3] = {(int64_t) (C * K), (int64_t) K, 1};
        int64_t estr[3] = {0, 1, 0};
        detail::check(aimet_qdq_broadcast(in, out, (int64_t) n, 3, tstr, estr, mn, mx, delta, offset, stream));
    }

private:
    static uint64_t next_seed()
    {
        static uint64_t s = 0x853C49E6748FEA9Bull;
        return s += 0x9E3779B97F4A7C15ull;
    }
    void* stream_;
};

// ---- TensorQuantizerOpFacade / TensorQuantizer ------------------------------------------------
class TensorQuantizerOpFacade
{
public:
    virtual ~TensorQuantizerOpFacade()                                                                     = default;
    virtual void resetEncodingStats()                                                                       = 0;
    virtual void updateStats(const float* tensor, std::size_t tensorSize, bool useCuda)                    = 0;
    virtual void updateStats(const float* tensor, std::size_t tensorSize, bool useCuda, IAllocator* alloc) = 0;
    virtual void quantizeDequantize(const float* input, std::size_t tensorSize, float* output, double encodingMin,
                                    double encodingMax, unsigned int bitwidth, bool useCuda)               = 0;
    virtual void quantizeDequantize(const float* input, std::size_t tensorSize, float* output, double encodingMin,
                                    double encodingMax, unsigned int bitwidth, bool useCuda, void* stream) = 0;
    virtual TfEncoding computeEncoding(unsigned int bitwidth, bool useSymmetricEncoding)                   = 0;
    virtual bool getStrictSymmetric()                                                                       = 0;
    virtual bool getUnsignedSymmetric()                                                                     = 0;
};

// TensorQuantizer.cpp:49-343 (the quantizer of the ONNX / TF ops): an analyzer + the sim + flags
class TensorQuantizer : public TensorQuantizerOpFacade
{
public:
    // the analyzer's device state is allocated on first use (host-only calls need no GPU)
    TensorQuantizer(QuantizationMode mode, RoundingMode rm, int device = 0, void* stream = nullptr)
        : roundingMode(rm), sim_(stream), mode_(mode), device_(device), stream_(stream)
    {
    }
    RoundingMode roundingMode;
    bool isEncodingValid = false;

    void resetEncodingStats() override
    {
        analyzer_.reset();   // a fresh analyzer (TensorQuantizer.cpp:91-96), allocated on next use
        validStats_     = false;
        isEncodingValid = false;
    }
    void updateStats(const float* t, std::size_t n, bool useCuda) override
    {
        analyzer().updateStats(t, n, useCuda ? COMP_MODE_GPU : COMP_MODE_CPU);
        validStats_ = true;
    }
    void updateStats(const float* t, std::size_t n, bool useCuda, IAllocator*) override { updateStats(t, n, useCuda); }
    void quantizeDequantize(const float* in, std::size_t n, float* out, double mn, double mx, unsigned int bw,
                            bool useCuda) override
    {
        quantizeDequantize(in, n, out, mn, mx, bw, useCuda, stream_);
    }
    void quantizeDequantize(const float* in, std::size_t n, float* out, double mn, double mx, unsigned int bw,
                            bool useCuda, void* stream) override
    {
        sim_.quantizeDequantizeTensor(in, n, out, mn, mx, (uint8_t) bw, roundingMode, useCuda, stream);
    }
    TfEncoding computeEncoding(unsigned int bw, bool sym) override   // TensorQuantizer.cpp:129-141
    {
        TfEncoding e {};
        if (validStats_)
        {
            e               = analyzer().computeEncoding((uint8_t) bw, sym, strict_, unsigned_);
            isEncodingValid = true;
        }
        return e;
    }
    bool getStrictSymmetric() override { return strict_; }
    bool getUnsignedSymmetric() override { return unsigned_; }
    void setStrictSymmetric(bool v) { strict_ = v; }
    void setUnsignedSymmetric(bool v) { unsigned_ = v; }
    void setQuantScheme(QuantizationMode mode)
    {
        mode_ = mode;
        resetEncodingStats();
    }
    QuantizationMode getQuantScheme() const { return mode_; }
    void setPercentileValue(float p) { analyzer().setPercentileValue(p); }
    float getPercentileValue() { return analyzer().getPercentileValue(); }
    std::vector<std::tuple<double, double>> getStatsHistogram() { return analyzer().getStatsHistogram(); }
    // TensorQuantizer.cpp:327-343 (host math)
    void computePartialEncoding(uint8_t bw, TfEncoding& enc, bool sym, bool unsign, bool strict)
    {
        detail::check(aimet_compute_partial_encoding(bw, &enc, sym, unsign, strict));
    }

private:
    DeviceEncodingAnalyzer& analyzer()
    {
        if (!analyzer_)
            analyzer_.reset(new DeviceEncodingAnalyzer(mode_, device_, stream_));
        return *analyzer_;
    }
    std::unique_ptr<DeviceEncodingAnalyzer> analyzer_;
    TensorQuantizationSim sim_;
    QuantizationMode mode_;
    int device_;
    void* stream_;
    bool validStats_ = false;
    bool strict_     = false;
    bool unsigned_   = false;
};

}   // namespace aimet_amd
