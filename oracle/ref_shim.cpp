// ref_shim.cpp -- TEST INFRASTRUCTURE ONLY.
//
// A thin extern "C" face over the *reference* DlQuantization C++ (compiled from the
// sources where they lie under /root/reference by oracle/build_ref.sh; nothing of the
// reference is copied into this repository). Loaded only by tests/golden/make_golden.py
// to produce golden vectors and by tests/test_oracle_golden.py, tests/test_entropy.py and
// tests/test_blockwise.py to pin oracle/dlq_oracle.c against it.
// The product (aimet_amd/) never loads it.
#include <DlQuantization/IQuantizationEncodingAnalyzer.hpp>
#include <DlQuantization/Quantization.hpp>
#include <DlQuantization/QuantizerFactory.hpp>
#include <TensorQuantizationSim.h>
#include <math_functions.hpp>
#include <quantization_utils.hpp>
#include <trim_functions.hpp>

#include <cstdint>
#include <cstring>
#include <memory>
#include <tuple>

using namespace DlQuantization;

extern "C" {

struct ref_encoding
{
    double min, max, delta, offset;
    int bw;
};

static ref_encoding to_c(const TfEncoding& e)
{
    return ref_encoding {e.min, e.max, e.delta, e.offset, e.bw};
}

// TensorQuantizationSim.cpp:96-114 (CPU)
void ref_qdq_per_tensor(const float* in, float* out, int64_t n, double mn, double mx, int bw)
{
    TensorQuantizationSim<float> sim;
    sim.quantizeDequantizeTensor(in, (size_t) n, out, mn, mx, (uint8_t) bw, ROUND_NEAREST, false);
}

// TensorQuantizationSim.cpp:116-126 (CPU)
void ref_quantize_per_tensor(const float* in, float* out, int64_t n, double mn, double mx, int bw, int shift)
{
    TensorQuantizationSim<float> sim;
    sim.quantizeTensor(in, (size_t) n, out, mn, mx, (uint8_t) bw, ROUND_NEAREST, false, shift != 0);
}

// TensorQuantizationSim.cpp:62-92
void ref_fill_encoding_info(int bw, double mn, double mx, ref_encoding* out)
{
    TensorQuantizationSim<float> sim;
    TfEncoding e {};
    sim.fillEncodingInfo(e, (uint8_t) bw, mn, mx);
    *out = to_c(e);
}

// trim_functions.cpp:607-630 -> :697-709 (CPU)
void ref_qdq_per_channel(const float* in, float* out, int64_t C, int64_t N, int64_t K, float* mins, float* maxs,
                         float* deltas, float* offsets)
{
    quantizeDequantizePerChannel(in, (int) C, (int) N, (int) K, out, mins, maxs, deltas, offsets, COMP_MODE_CPU,
                                 ROUND_NEAREST, nullptr);
}

// quantization_utils.cpp:58-143
void ref_get_computed_encodings(int bw, double mn, double mx, int sym, int strict, int unsign, ref_encoding* out)
{
    *out = to_c(getComputedEncodings((uint8_t) bw, mn, mx, sym != 0, strict != 0, unsign != 0));
}

// quantization_utils.cpp:158-228 (partial encodings); returns -1 when the reference throws
int ref_partial_encoding(int bw, ref_encoding* e, int sym, int unsign, int strict)
{
    TfEncoding t {e->min, e->max, e->delta, e->offset, e->bw};
    try
    {
        if (t.min == 0 && t.max == 0)
            computeMinMaxRangeFromDeltaOffset((uint8_t) bw, t, sym != 0, unsign != 0, strict != 0);
        else if (t.delta == 0)
            computeDeltaAndOffsetFromMinMax((uint8_t) bw, t, sym != 0, unsign != 0, strict != 0);
        else
            return -1;
    }
    catch (...)
    {
        return -1;
    }
    *e = to_c(t);
    return 0;
}

// math_functions.cpp:61-100 (CPU)
float ref_get_min(const float* x, int64_t n)
{
    return GetMin(x, (int) n, COMP_MODE_CPU);
}
float ref_get_max(const float* x, int64_t n)
{
    return GetMax(x, (int) n, COMP_MODE_CPU);
}

// QuantizerFactory.cpp:74-104 + the analyzers
void* ref_analyzer_create(int scheme)
{
    auto p = getEncodingAnalyzerInstance<float>((QuantizationMode) scheme);
    return p.release();
}
void ref_analyzer_destroy(void* a)
{
    delete static_cast<IQuantizationEncodingAnalyzer<float>*>(a);
}
void ref_analyzer_update(void* a, const float* x, int64_t n)
{
    static_cast<IQuantizationEncodingAnalyzer<float>*>(a)->updateStats(x, (size_t) n, COMP_MODE_CPU);
}
void ref_analyzer_compute(void* a, int bw, int sym, int strict, int unsign, ref_encoding* out)
{
    *out = to_c(static_cast<IQuantizationEncodingAnalyzer<float>*>(a)->computeEncoding((uint8_t) bw, sym != 0,
                                                                                        strict != 0, unsign != 0));
}
void ref_analyzer_set_percentile(void* a, float p)
{
    static_cast<IQuantizationEncodingAnalyzer<float>*>(a)->setPercentileValue(p);
}
int ref_analyzer_histogram(void* a, double* xleft, double* pdf)
{
    auto h = static_cast<IQuantizationEncodingAnalyzer<float>*>(a)->getStatsHistogram();
    int i = 0;
    for (auto& t: h)
    {
        xleft[i] = std::get<0>(t);
        pdf[i]   = std::get<1>(t);
        ++i;
    }
    return i;
}

// trim_functions.cpp:633-687 (CPU)
void ref_qdq_broadcast(const float* in, float* out, int64_t n, int64_t nd, const int64_t* istr, const int64_t* estr,
                       const float* mn, const float* mx, const float* delta, const float* offset)
{
    quantizeDequantizeBroadcast(in, out, n, nd, istr, estr, mn, mx, delta, offset, COMP_MODE_CPU, nullptr);
}

// math_functions.cpp:476-560: the entropy analyzer's TensorProfilingParams, driven directly
// (EntropyEncodingAnalyzer keeps its copy private)
void* ref_tpp_create()
{
    auto* t       = new TensorProfilingParams();
    t->min        = 0;
    t->max        = 0;
    t->iterations = 0;
    return t;
}
void ref_tpp_destroy(void* t)
{
    delete static_cast<TensorProfilingParams*>(t);
}
void ref_tpp_update(void* t, const float* x, int64_t n)
{
    updateTensorHistogram_cpu(x, (int) n, *static_cast<TensorProfilingParams*>(t));
}
// returns histogram.size() (0 or 512)
int ref_tpp_get(void* t, double* mn, double* mx, double* hist, int* iterations)
{
    auto* p     = static_cast<TensorProfilingParams*>(t);
    *mn         = p->min;
    *mx         = p->max;
    *iterations = p->iterations;
    for (size_t i = 0; i < p->histogram.size(); ++i)
        hist[i] = p->histogram[i];
    return (int) p->histogram.size();
}

}   // extern "C"
