/*
 * dlq_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference DlQuantization arithmetic (AIMET 1.35.0,
 * /root/reference/ModelOptimizations/DlQuantization). It is the CHECKER for the
 * HIP path and the "port" CPU baseline in bench.py. Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the
 * product (aimet_amd/) never links or calls it.
 *
 * Parity pinning: every function here is checked against
 *   (1) the known-answer tests of the reference's own gtest/pytest suites
 *       (tests/golden/kat.json, see tests/golden/README.md), and
 *   (2) golden vectors produced by the reference C++ itself, compiled from
 *       /root/reference by oracle/build_ref.sh into oracle/_ref/ (not committed),
 *       dumped by tests/golden/make_golden.py into tests/golden/ (npz files).
 *
 * Every C++ expression of the reference is restated with its exact evaluation
 * types: the reference is instantiated with DTYPE=float, mixes float and double,
 * uses std::min/std::max ((b<a)?b:a / (a<b)?b:a), std::round (half away from
 * zero) and is compiled for x86-64 without FMA.  Build with -ffp-contract=off.
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define PDF_SIZE 512                 /* math_functions.hpp:80 */
#define EPSILON_GATE 1e-5            /* quantization_utils.hpp:51 */
#define MIN_RANGE 0.01               /* TfEncodingAnalyzer.h:81, TfEnhancedEncodingAnalyzer.h:105 */
#define TFE_GAMMA 3.0f               /* TfEnhancedEncodingAnalyzer.h:102 (static constexpr DTYPE) */

enum { QUANTIZATION_TF = 0, QUANTIZATION_TF_ENHANCED = 1, QUANTIZATION_RANGE_LEARNING = 2,
       QUANTIZATION_PERCENTILE = 3, QUANTIZATION_MSE = 4, QUANTIZATION_ENTROPY = 5 }; /* Quantization.hpp:84-106 */

typedef struct {
    double min, max, delta, offset;
    int bw;
} orc_encoding; /* Quantization.hpp:113-120 */

/* std::min / std::max as libstdc++ defines them. */
static inline double dmin_(double a, double b) { return (b < a) ? b : a; }
static inline double dmax_(double a, double b) { return (a < b) ? b : a; }
static inline float fmin_(float a, float b) { return (b < a) ? b : a; }
static inline float fmax_(float a, float b) { return (a < b) ? b : a; }
static inline int imin_(int a, int b) { return (b < a) ? b : a; }
static inline int imax_(int a, int b) { return (a < b) ? b : a; }

/* ------------------------------------------------------------------------- */
/* quantization_utils.cpp                                                     */
/* ------------------------------------------------------------------------- */

/* quantization_utils.cpp:145-156 gateMinMax */
void orc_gate_min_max(double* mn, double* mx)
{
    *mn = dmin_(*mn, 0.0);
    *mx = dmax_(*mx, 0.0);
    *mx = dmax_(*mx, *mn + EPSILON_GATE);
}

/* quantization_utils.cpp:58-143 getComputedEncodings */
orc_encoding orc_get_computed_encodings(int bw, double mn, double mx, int sym, int strict, int unsign)
{
    orc_encoding e;
    double numSteps = pow(2.0, (double) bw) - 1;
    if (sym && strict)
        numSteps -= 1;
    e.bw = bw;
    if (isinf(mn))
        mn = -FLT_MAX;
    if (isinf(mx))
        mx = FLT_MAX;
    if (sym && ((mn < 0.0) || (!unsign))) {
        mx = dmax_(fabs(mx), fabs(mn));
        unsigned int numPositiveSteps = (unsigned int) floor(numSteps / 2);
        e.delta = mx / numPositiveSteps;
        e.offset = -ceil(numSteps / 2);
        e.min = dmax_(e.offset * e.delta, (double) -FLT_MAX);
        e.max = dmin_(e.delta * numPositiveSteps, (double) FLT_MAX);
    } else {
        e.delta = (mx - mn) / numSteps;
        if (mn < 0 && mx > 0) {
            double bZero = round(-mn / e.delta);
            bZero = dmin_(numSteps, dmax_(0.0, bZero));
            e.offset = -bZero;
        } else {
            e.offset = round(mn / e.delta);
            e.min = mn;
            e.max = mx;
            return e;
        }
        if (e.delta * e.offset >= (double) -FLT_MAX && e.delta * e.offset <= (double) FLT_MAX)
            e.min = e.delta * e.offset;
        else
            e.min = (double) -FLT_MAX;
        e.max = mx - mn + e.min;
        if (e.max > (double) FLT_MAX)
            e.max = FLT_MAX;
    }
    return e;
}

/* TensorQuantizationSim.cpp:62-92 generateScaleOffset + fillEncodingInfo */
orc_encoding orc_fill_encoding_info(int bw, double mn, double mx)
{
    orc_encoding e;
    e.bw = bw;
    orc_gate_min_max(&mn, &mx);
    double numSteps = pow(2.0, (double) bw) - 1;
    if (mn == -mx)
        numSteps -= 1;
    e.delta = (mx - mn) / numSteps;                /* trim_functions.cpp:61-65 */
    e.offset = round(mn / e.delta);                /* trim_functions.cpp:68-73 */
    e.min = e.offset * e.delta;
    e.max = e.delta * numSteps + e.min;
    return e;
}

/* quantization_utils.cpp:158-200 computeMinMaxRangeFromDeltaOffset (partial encodings).
 * Returns 0 on success, -1 if the reference would throw. */
int orc_min_max_from_delta_offset(int bw, orc_encoding* e, int sym, int unsign, int strict)
{
    if (e->bw == 0) return -1;
    if (e->min != 0 && e->max != 0) return -1;
    if (e->delta == 0 && e->offset > 0) return -1;
    double numSteps = pow(2.0, (double) bw) - 1;
    if (sym && strict) numSteps -= 1;
    e->min = e->offset * e->delta;
    if (sym && ((e->min < 0.0) || (!unsign))) {
        double numPositiveSteps = floor(numSteps / 2);
        e->max = e->delta * numPositiveSteps;
    } else {
        e->max = e->delta * numSteps + e->min;
    }
    if (e->max - e->min < EPSILON_GATE)
        orc_gate_min_max(&e->min, &e->max);
    return 0;
}

/* quantization_utils.cpp:202-228 computeDeltaAndOffsetFromMinMax */
int orc_delta_offset_from_min_max(int bw, orc_encoding* e, int sym, int unsign, int strict)
{
    orc_encoding orig = *e;
    if (e->bw == 0) return -1;
    if (orig.delta != 0 && orig.offset != 0) return -1;
    *e = orc_get_computed_encodings(bw, e->min, e->max, sym, strict, unsign);
    e->min = orig.min;
    e->max = orig.max;
    return 0;
}

/* ------------------------------------------------------------------------- */
/* trim_functions.cpp -- QDQ element arithmetic (DTYPE = float)               */
/* ------------------------------------------------------------------------- */

/* trim_functions.cpp:140-165 quantizeValueCpu, ROUND_NEAREST */
static inline float quantize_value(float x, float emin, float emax, float edelta, float eoff)
{
    float o = fmaxf(fminf(x, emax), emin);
    o = o / edelta - eoff;
    return roundf(o);
}

/* trim_functions.cpp:167-171 dequantizeValueCpu */
static inline float dequantize_value(float q, float edelta, float eoff)
{
    return edelta * (q + eoff);
}

/* TensorQuantizationSim.cpp:96-114 quantizeDequantizeTensor -> trim_functions.cpp:173-182.
 * enc_min/enc_max are the raw encoding.min/.max the caller passes (AimetTensorQuantizer.cpp:150-152). */
void orc_qdq_per_tensor(const float* in, float* out, int64_t n, double enc_min, double enc_max, int bw)
{
    orc_encoding e = orc_fill_encoding_info(bw, enc_min, enc_max);
    float mn = (float) e.min, mx = (float) e.max, d = (float) e.delta, off = (float) e.offset;
    for (int64_t i = 0; i < n; ++i)
        out[i] = dequantize_value(quantize_value(in[i], mn, mx, d, off), d, off);
}

/* TensorQuantizationSim.cpp:116-126 quantizeTensor -> trim_functions.cpp:202-218 quantizeToFxpCpu */
void orc_quantize_per_tensor(const float* in, float* out, int64_t n, double enc_min, double enc_max, int bw,
                             int shift_to_signed)
{
    orc_encoding e = orc_fill_encoding_info(bw, enc_min, enc_max);
    unsigned int shift = 0;
    if (shift_to_signed)
        shift = (unsigned int) pow(2.0, (double) (e.bw - 1));
    float mn = (float) e.min, mx = (float) e.max, d = (float) e.delta, off = (float) e.offset;
    for (int64_t i = 0; i < n; ++i)
        out[i] = quantize_value(in[i], mn, mx, d, off) - (float) shift;
}

/* AimetTensorQuantizer.cpp:233-307: per-channel encoding tensors built with torch float32
 * ops on the host (CPU path): min/max cast to float, torch.minimum/maximum (NaN-propagating),
 * `+ 1e-5` and `/ numSteps` as float32 ops with the scalar cast to float32, at::round
 * (half-to-even).  table layout: [4][C] = min, max, delta, offset. */
static inline float torch_minimum(float a, float b) { return (isnan(a) || isnan(b)) ? NAN : (a < b ? a : b); }
static inline float torch_maximum(float a, float b) { return (isnan(a) || isnan(b)) ? NAN : (a > b ? a : b); }

void orc_per_channel_table(const orc_encoding* encs, int64_t C, float* table)
{
    double numSteps = pow(2.0, (double) encs[0].bw) - 1;
    if (encs[0].min == -encs[0].max)
        numSteps -= 1;
    float fsteps = (float) numSteps;
    for (int64_t c = 0; c < C; ++c) {
        float mn = (float) encs[c].min, mx = (float) encs[c].max;
        mn = torch_minimum(mn, 0.0f);
        mx = torch_maximum(mx, 0.0f);
        mx = torch_maximum(mx, mn + (float) 1e-5);
        float d = (mx - mn) / fsteps;
        float off = nearbyintf(mn / d); /* default FE_TONEAREST: half-to-even */
        table[c] = mn;
        table[C + c] = mx;
        table[2 * C + c] = d;
        table[3 * C + c] = off;
    }
}

/* trim_functions.cpp:697-709 quantizeDequantizePerChannelCpu; channel = (i / K) % C */
void orc_qdq_per_channel(const float* in, float* out, int64_t C, int64_t N, int64_t K, const float* table)
{
    for (int64_t i = 0; i < N; ++i) {
        int64_t c = (i / K) % C;
        float mn = table[c], mx = table[C + c], d = table[2 * C + c], off = table[3 * C + c];
        out[i] = dequantize_value(quantize_value(in[i], mn, mx, d, off), d, off);
    }
}

/* OpenMP variants of the two QDQ loops (the cpu_baseline's multi-core figure):
 * the same element arithmetic, iterations split statically over `threads` threads. */
void orc_qdq_per_tensor_omp(const float* in, float* out, int64_t n, double enc_min, double enc_max, int bw,
                            int threads)
{
    orc_encoding e = orc_fill_encoding_info(bw, enc_min, enc_max);
    float mn = (float) e.min, mx = (float) e.max, d = (float) e.delta, off = (float) e.offset;
#pragma omp parallel for num_threads(threads) schedule(static)
    for (int64_t i = 0; i < n; ++i)
        out[i] = dequantize_value(quantize_value(in[i], mn, mx, d, off), d, off);
}

void orc_qdq_per_channel_omp(const float* in, float* out, int64_t C, int64_t N, int64_t K, const float* table,
                             int threads)
{
#pragma omp parallel for num_threads(threads) schedule(static)
    for (int64_t i = 0; i < N; ++i) {
        int64_t c = (i / K) % C;
        float mn = table[c], mx = table[C + c], d = table[2 * C + c], off = table[3 * C + c];
        out[i] = dequantize_value(quantize_value(in[i], mn, mx, d, off), d, off);
    }
}

int orc_openmp_enabled(void)
{
#ifdef _OPENMP
    return 1;
#else
    return 0;
#endif
}

/* quantsim_straight_through_grad.py:91-118 compute_dloss_by_dx: grad * (min <= x <= max),
 * min/max are float32 tensors broadcast along ch_axis (C==1: per-tensor). Layout [outer][C][K]. */
void orc_ste_backward(const float* x, const float* g, float* gin, int64_t N, int64_t C, int64_t K,
                      const float* mins, const float* maxs)
{
    for (int64_t i = 0; i < N; ++i) {
        int64_t c = (C == 1) ? 0 : (i / K) % C;
        float m = (mins[c] <= x[i] && x[i] <= maxs[c]) ? 1.0f : 0.0f;
        gin[i] = g[i] * m;
    }
}

/* ------------------------------------------------------------------------- */
/* math_functions.cpp -- reductions, histogram, PDF (DTYPE = float)           */
/* ------------------------------------------------------------------------- */

/* math_functions.cpp:327-336 GetMax_cpu: starts at (float)-DBL_MAX = -inf, std::max (NaN ignored) */
float orc_get_max(const float* x, int64_t n)
{
    float v = (float) -DBL_MAX;
    for (int64_t i = 0; i < n; ++i)
        v = fmax_(v, x[i]);
    return v;
}

/* math_functions.cpp:338-347 GetMin_cpu */
float orc_get_min(const float* x, int64_t n)
{
    float v = (float) DBL_MAX;
    for (int64_t i = 0; i < n; ++i)
        v = fmin_(v, x[i]);
    return v;
}

typedef struct {
    int initialized;   /* pdf.xLeft.size() != 0 */
    int iterations;
    double xLeft[PDF_SIZE];
    double pdf[PDF_SIZE];
    float hist_min;       /* InitializePdf's min_val after widening: xLeft[i] = hist_min + i*bucket_size */
    double bucket_size;
} orc_pdf; /* math_functions.hpp:70-77 */

/* math_functions.cpp:207-241 InitializePdf<float> */
void orc_initialize_pdf(orc_pdf* p, float min_val, float max_val, int signed_vals)
{
    if (min_val == max_val)
        max_val = fmax_(max_val, min_val + (float) 0.01);
    float center = (max_val + min_val) / 2;
    min_val = fmax_(-FLT_MAX, center - 3 * (center - min_val));
    max_val = fmin_(FLT_MAX, center + 3 * (max_val - center));
    double bucket_size;
    if (signed_vals) {
        bucket_size = ((double) max_val - (double) min_val) / PDF_SIZE;
    } else {
        float max_abs_val = fmax_(fabsf(max_val), fabsf(min_val));
        bucket_size = (double) (max_abs_val / PDF_SIZE);
    }
    for (int i = 0; i < PDF_SIZE; ++i) {
        if (signed_vals)
            p->xLeft[i] = (double) min_val + (double) i * bucket_size;
        else
            p->xLeft[i] = (double) i * bucket_size;
    }
    memset(p->pdf, 0, sizeof(p->pdf));
    p->iterations = 0;
    p->initialized = 1;
    p->hist_min = min_val;
    p->bucket_size = bucket_size;
}

/* math_functions.cpp:367-384 GetHistogram_cpu. Out-of-range/NaN indices (x86 cvttss2si
 * yields INT_MIN for them) are dropped. */
void orc_get_histogram(const float* x, int64_t n, uint32_t* hist, float bucket_size, float pdf_offset, int is_signed)
{
    for (int64_t i = 0; i < n; ++i) {
        float v = is_signed ? (x[i] / bucket_size - pdf_offset) : (fabsf(x[i]) / bucket_size - pdf_offset);
        float r = roundf(v);
        if (r >= 0.0f && r < (float) PDF_SIZE)
            hist[(int) r] += 1;
    }
}

/* math_functions.cpp:243-288 UpdatePdf<float>; cnt is the int element count */
void orc_update_pdf(orc_pdf* p, const float* x, int64_t n, int signed_vals)
{
    if (!p->initialized) {
        float mn = orc_get_min(x, n);
        float mx = orc_get_max(x, n);
        if (mn == 0 && mx == 0)
            return;
        orc_initialize_pdf(p, mn, mx, signed_vals);
    }
    float bucket_size = (float) (p->xLeft[1] - p->xLeft[0]);
    float min_val = signed_vals ? (float) p->xLeft[0] : 0.0f;
    float pdf_offset = min_val / bucket_size;
    uint32_t hist[PDF_SIZE];
    memset(hist, 0, sizeof(hist));
    orc_get_histogram(x, n, hist, bucket_size, pdf_offset, signed_vals);
    for (int i = 0; i < PDF_SIZE; ++i) {
        double prob = (double) hist[i] / (double) n;
        p->pdf[i] = (p->pdf[i] * p->iterations + prob) / (p->iterations + 1);
    }
    p->iterations++;
}

/* Same update from externally summed counts (sharded calibration: counts summed over ranks,
 * n = global element count). */
void orc_update_pdf_from_counts(orc_pdf* p, const uint64_t* counts, int64_t n)
{
    for (int i = 0; i < PDF_SIZE; ++i) {
        double prob = (double) counts[i] / (double) n;
        p->pdf[i] = (p->pdf[i] * p->iterations + prob) / (p->iterations + 1);
    }
    p->iterations++;
}

/* math_functions.cpp:404-439 findOriginalRange<float> (also TfEnhanced _findRangeOfAggregateStats,
 * TfEnhancedEncodingAnalyzer.cpp:255-291, identical arithmetic) */
static void find_original_range(const orc_pdf* p, float* outMin, float* outMax)
{
    float minVal = (float) p->xLeft[0];
    float maxVal = (float) p->xLeft[PDF_SIZE - 1];
    for (int i = 0; i < PDF_SIZE; ++i)
        if (p->pdf[i] > 0) { minVal = (float) p->xLeft[i]; break; }
    for (int i = PDF_SIZE - 1; i > 0; --i)
        if (p->pdf[i] > 0) { maxVal = (float) p->xLeft[i]; break; }
    minVal = fmin_(minVal, 0.0f);
    maxVal = fmax_(maxVal, 0.0f);
    maxVal = fmax_(maxVal, minVal + (float) MIN_RANGE);
    *outMin = minVal;
    *outMax = maxVal;
}

/* ------------------------------------------------------------------------- */
/* TfEnhancedEncodingAnalyzer.cpp (DTYPE = float)                             */
/* ------------------------------------------------------------------------- */

/* TfEnhancedEncodingAnalyzer.cpp:293-355 _quantAndSatCost */
static double tfe_cost(const orc_pdf* pdf, int bw, float delta, int offset)
{
    float minVal = delta * (float) offset;
    float stepSize = (float) (pow(2.0, (double) bw) - 1);
    float maxVal = delta * ((float) offset + stepSize);
    float pdfStart = (float) pdf->xLeft[0];
    double pdfStep = pdf->xLeft[1] - pdf->xLeft[0];
    int minInd = (int) floor((double) (minVal - pdfStart) / pdfStep);
    minInd = imin_(imax_(0, minInd), PDF_SIZE - 1);
    int maxInd = (int) floor((double) (maxVal - pdfStart) / pdfStep);
    maxInd = imin_(imax_(0, maxInd), PDF_SIZE - 1);

    double satCostBottom = 0;
    float minValMiddle = (float) ((double) pdfStart + (minInd * pdfStep) + pdfStep / 2);
    for (int i = 0; i < minInd; ++i) {
        double midVal = (double) pdfStart + i * pdfStep + pdfStep / 2;
        double d = midVal - (double) minValMiddle;
        satCostBottom += pdf->pdf[i] * (d * d);
    }
    double satCostTop = 0;
    float maxValMiddle = (float) ((double) pdfStart + (maxInd * pdfStep) + pdfStep / 2);
    for (int i = maxInd; i < PDF_SIZE; ++i) {
        double midVal = (double) pdfStart + i * pdfStep + pdfStep / 2;
        double d = midVal - (double) maxValMiddle;
        satCostTop += pdf->pdf[i] * (d * d);
    }
    double quantCost = 0;
    for (int i = minInd; i < maxInd; ++i) {
        float floatVal = (float) ((double) pdfStart + i * pdfStep + pdfStep / 2);
        int quantized = (int) roundf(floatVal / delta - (float) offset);
        float dequantized = delta * (float) (quantized + offset);
        double d = (double) (floatVal - dequantized);
        quantCost += pdf->pdf[i] * (d * d);
    }
    double sqnr = (double) TFE_GAMMA * (satCostBottom + satCostTop) + quantCost;
    return dmin_(sqnr, DBL_MAX);
}

/* TfEnhancedEncodingAnalyzer.cpp:144-170 _clampToObservedMinMax */
static int tfe_clamp(float observedMin, float observedMax, float numSteps, float* testDelta, int* testOffset)
{
    float testMin = fmax_(*testDelta * (float) *testOffset, -FLT_MAX);
    float testMax = fmin_(*testDelta * ((float) *testOffset + numSteps), FLT_MAX);
    if ((testMin < observedMin) && (testMax > observedMax))
        return 0;
    testMin = fmax_(observedMin, testMin);
    testMax = fmin_(observedMax, testMax);
    if (testMin == testMax)
        return 0;
    *testDelta = (float) (((double) testMax - (double) testMin) / (double) numSteps);
    *testOffset = (int) roundf(testMin / *testDelta);
    return 1;
}

#define TFE_MAX_CAND 512
typedef struct { float delta; int offset; } tfe_cand;

/* TfEnhancedEncodingAnalyzer.cpp:172-205 _pickTestCandidatesAsymmetric */
static int tfe_cands_asym(float observedMin, float observedMax, float numSteps, tfe_cand* c)
{
    int n = 0;
    float observedDelta = (float) (((double) observedMax - (double) observedMin) / (double) numSteps);
    int observedOffset = (int) roundf(observedMin / observedDelta);
    observedMin = fmax_(observedDelta * (float) observedOffset, -FLT_MAX);
    observedMax = fmin_(observedDelta * ((float) observedOffset + numSteps), FLT_MAX);
    float deltaMax = observedDelta;
    for (float f = (float) (1.0 / 16); (double) f <= 1 + 1.0 / 16; f = (float) ((double) f + 1.0 / 16)) {
        for (int i = 0; i <= 20; ++i) {
            float testDelta = f * deltaMax;
            int testOffset = (int) ((double) (-numSteps) + (double) numSteps / 20.0 * i);
            if (!tfe_clamp(observedMin, observedMax, numSteps, &testDelta, &testOffset))
                continue;
            c[n].delta = testDelta;
            c[n].offset = testOffset;
            n++;
        }
    }
    c[n].delta = observedDelta;
    c[n].offset = observedOffset;
    n++;
    return n;
}

/* TfEnhancedEncodingAnalyzer.cpp:207-241 _pickTestCandidatesSymmetric */
static int tfe_cands_sym(float minVal, float maxVal, float numSteps, tfe_cand* c, int unsign)
{
    int n = 0;
    float deltaMax = 0.0f;
    int testOffset = 0;
    if ((minVal == 0.0f) && unsign) {
        deltaMax = maxVal / numSteps;
        testOffset = 0;
    } else {
        float absoluteMax = fmax_(fabsf(maxVal), fabsf(minVal));
        deltaMax = (float) ((double) absoluteMax / ((double) numSteps / 2.0));
        testOffset = (int) floorf(-numSteps / 2);
    }
    for (float f = (float) (1.0 / 100); (double) f <= 1 + 1.0 / 100; f = (float) ((double) f + 1.0 / 100)) {
        c[n].delta = f * deltaMax;
        c[n].offset = testOffset;
        n++;
    }
    return n;
}

/* TfEnhancedEncodingAnalyzer.cpp:78-113 computeEncoding + :357-392 getComputedEncodings */
static orc_encoding tfe_compute(const orc_pdf* p, int stats_updated, int bw, int sym, int strict, int unsign)
{
    orc_encoding e = {0, 0, 0, 0, 0};
    float numSteps = (float) (pow(2.0, (double) bw) - 1);
    if (!p->initialized) {
        if (stats_updated) {
            e.min = -1;
            e.max = 1;
            e.delta = (e.max - e.min) / (int) numSteps;
            e.offset = floor(e.min / e.delta);
            e.min = e.offset * e.delta;
            e.max = e.min + (int) numSteps * e.delta;
            e.bw = bw;
        }
        return e;
    }
    float minVal, maxVal;
    find_original_range(p, &minVal, &maxVal);
    tfe_cand cands[TFE_MAX_CAND];
    int n;
    if (sym) {
        if (strict)
            numSteps -= 1;
        n = tfe_cands_sym(minVal, maxVal, numSteps, cands, unsign);
    } else {
        n = tfe_cands_asym(minVal, maxVal, numSteps, cands);
    }
    /* :115-142 _findBestCandidate */
    float bestDelta = -1;
    int bestOffset = -1;
    double bestCost = DBL_MAX;
    for (int i = 0; i < n; ++i) {
        double cost = tfe_cost(p, bw, cands[i].delta, cands[i].offset);
        if (cost < bestCost) {
            bestCost = cost;
            bestDelta = cands[i].delta;
            bestOffset = cands[i].offset;
        }
    }
    float bestMin = fmax_(bestDelta * (float) bestOffset, -FLT_MAX);
    float bestMax = fmin_(bestDelta * ((float) bestOffset + numSteps), FLT_MAX);
    e.delta = bestDelta;
    e.offset = bestOffset;
    e.bw = bw;
    e.min = bestMin;
    e.max = bestMax;
    return e;
}

/* ------------------------------------------------------------------------- */
/* PercentileEncodingAnalyzer.cpp (DTYPE = float)                             */
/* ------------------------------------------------------------------------- */

static orc_encoding zero_data_encoding(int bw, float numSteps)
{
    orc_encoding e;
    e.min = -1;
    e.max = 1;
    e.delta = (e.max - e.min) / (int) numSteps;
    e.offset = floor(e.min / e.delta);
    e.min = e.offset * e.delta;
    e.max = e.min + (int) numSteps * e.delta;
    e.bw = bw;
    return e;
}

/* PercentileEncodingAnalyzer.cpp:127-190 _computePercentileRange */
static void percentile_range(const orc_pdf* p, float percentile, float* outMin, float* outMax)
{
    float minVal, maxVal;
    find_original_range(p, &minVal, &maxVal);
    if (percentile == 100.0f) {
        *outMin = minVal;
        *outMax = maxVal;
        return;
    }
    const float histBinWidth = (float) (p->xLeft[1] - p->xLeft[0]);
    float histMin = (float) p->xLeft[0];
    float histMax = (float) p->xLeft[PDF_SIZE - 1] + histBinWidth;
    float percentileMin = histMin, percentileMax = histMax;
    double cdf[PDF_SIZE];
    memcpy(cdf, p->pdf, sizeof(cdf));
    for (int i = 1; i < PDF_SIZE; i++)
        cdf[i] += cdf[i - 1];
    float leftPercentile = 1 - percentile / 100;
    for (int i = 0; i < PDF_SIZE; i++)
        if (cdf[i] >= (double) leftPercentile) { percentileMin = (float) p->xLeft[i]; break; }
    float rightPercentile = percentile / 100;
    for (int i = PDF_SIZE - 1; i >= 0; i--) {
        if (cdf[i] < (double) rightPercentile && p->xLeft[i] < (double) maxVal) {
            percentileMax = (float) (p->xLeft[i] + (double) histBinWidth);
            break;
        }
    }
    if (percentileMin == percentileMax)
        percentileMax += histBinWidth;
    *outMin = percentileMin;
    *outMax = percentileMax;
}

/* PercentileEncodingAnalyzer.cpp:78-125 computeEncoding */
static orc_encoding percentile_compute(const orc_pdf* p, int stats_updated, float percentile, int bw, int sym,
                                       int strict, int unsign)
{
    orc_encoding e = {0, 0, 0, 0, 0};
    float numSteps = (float) (pow(2.0, (double) bw) - 1);
    if (sym && strict)
        numSteps -= 1;
    if (!p->initialized)
        return stats_updated ? zero_data_encoding(bw, numSteps) : e;
    float aMin, aMax;
    percentile_range(p, percentile, &aMin, &aMax);
    aMin = fmin_(aMin, 0.0f);
    aMax = fmax_(aMax, 0.0f);
    return orc_get_computed_encodings(bw, aMin, aMax, sym, strict, unsign);
}

/* ------------------------------------------------------------------------- */
/* MseEncodingAnalyzer.cpp (DTYPE = float)                                    */
/* ------------------------------------------------------------------------- */

/* MseEncodingAnalyzer.cpp:240-264 _computeMSECost */
static float mse_cost(int bw, const float* centers, const float* cpdf, int nc, float cMin, float cMax, int sym,
                      int strict, int unsign)
{
    orc_encoding e = orc_get_computed_encodings(bw, cMin, cMax, sym, strict, unsign);
    float w = 0;
    for (int i = 0; i < nc; i++) {
        float floatVal = centers[i];
        float clamped = fmax_(cMin, fmin_(floatVal, cMax));
        int quantized = (int) round((double) clamped / e.delta - e.offset);
        float dequantized = (float) (e.delta * (quantized + e.offset));
        double d = (double) (floatVal - dequantized);
        w = (float) ((double) w + (double) cpdf[i] * (d * d));
    }
    return w;
}

/* MseEncodingAnalyzer.cpp:130-204 _minimizeMSE + :206-238 _pickMinMaxCandidatesMSECalib */
static void mse_minimize(const orc_pdf* p, int bw, int sym, int strict, int unsign, float* outMin, float* outMax)
{
    const float histBinWidth = (float) (p->xLeft[1] - p->xLeft[0]);
    float histMin = (float) p->xLeft[0];
    float histMax = (float) p->xLeft[PDF_SIZE - 1] + histBinWidth;
    float minVal, maxVal;
    find_original_range(p, &minVal, &maxVal);
    maxVal = maxVal + histBinWidth;

    /* bin edges: at most PDF_SIZE + 2 entries plus float accumulation slack */
    int cap = 4 * PDF_SIZE + 8, ne = 0;
    float* edges = (float*) malloc(sizeof(float) * cap);
    edges[ne++] = minVal;
    for (float i = histMin; i <= histMax; i += histBinWidth) {
        if (i >= minVal && i <= maxVal) {
            if (ne == cap) { cap *= 2; edges = (float*) realloc(edges, sizeof(float) * cap); }
            edges[ne++] = i;
        }
    }
    /* candidates */
    float* minC = (float*) malloc(sizeof(float) * (ne + 1));
    float* maxC = (float*) malloc(sizeof(float) * (ne + 1));
    int nmin = 0, nmax = 0;
    for (int k = 0; k < ne; ++k) {
        if (edges[k] < 0) minC[nmin++] = edges[k];
        else if (edges[k] > 0) maxC[nmax++] = edges[k];
    }
    minC[nmin++] = 0;
    maxC[nmax++] = 0;

    float pdfStart = (float) p->xLeft[0];
    float pdfStep = (float) (p->xLeft[1] - p->xLeft[0]);
    int nc = ne - 1;
    float* centers = (float*) malloc(sizeof(float) * (nc > 0 ? nc : 1));
    float* cpdf = (float*) malloc(sizeof(float) * (nc > 0 ? nc : 1));
    for (int i = 0; i < nc; i++) {
        centers[i] = (i == 0) ? (minVal + histBinWidth / 2) : (centers[i - 1] + histBinWidth);
        int ind = (int) floorf((centers[i] - pdfStart) / pdfStep);
        ind = imin_(imax_(0, ind), PDF_SIZE - 1);
        cpdf[i] = (float) p->pdf[ind];
    }
    float mseMin = FLT_MAX;
    float bestMin = minVal, bestMax = maxVal;
    int total = nmin * nmax - 1; /* last pair {0,0} popped */
    for (int t = 0; t < total; ++t) {
        float cmin = minC[t / nmax], cmax = maxC[t % nmax];
        float mse = mse_cost(bw, centers, cpdf, nc, cmin, cmax, sym, strict, unsign);
        if (mse < mseMin) {
            mseMin = mse;
            bestMin = cmin;
            bestMax = cmax;
        }
    }
    free(edges); free(minC); free(maxC); free(centers); free(cpdf);
    *outMin = bestMin;
    *outMax = bestMax;
}

/* MseEncodingAnalyzer.cpp:79-128 computeEncoding */
static orc_encoding mse_compute(const orc_pdf* p, int stats_updated, int bw, int sym, int strict, int unsign)
{
    orc_encoding e = {0, 0, 0, 0, 0};
    float numSteps = (float) (pow(2.0, (double) bw) - 1);
    if (sym && strict)
        numSteps -= 1;
    if (!p->initialized)
        return stats_updated ? zero_data_encoding(bw, numSteps) : e;
    float aMin, aMax;
    mse_minimize(p, bw, sym, strict, unsign, &aMin, &aMax);
    aMin = fmin_(aMin, 0.0f);
    aMax = fmax_(aMax, 0.0f);
    return orc_get_computed_encodings(bw, aMin, aMax, sym, strict, unsign);
}

/* ------------------------------------------------------------------------- */
/* Entropy analyzer: TensorProfilingParams histogram + KL-divergence range search              */
/* (math_functions.cpp:470-641, EntropyEncodingAnalyzer.cpp:97-435)                            */
/* ------------------------------------------------------------------------- */

typedef struct {
    double min, max;           /* TensorProfilingParams (math_functions.hpp:71-77) */
    double hist[PDF_SIZE];
    int has_hist;              /* histogram.size() != 0 */
    int iterations;
} orc_tpp;

/* math_functions.cpp:470-474 getBin. The (size_t) conversion of a float is the x86-64 one gcc
 * emits (NaN and values <= -1 land in the last bin, values >= 2^64 in bin 0), as in the
 * reference build. */
static size_t ent_get_bin(size_t nBins, float binWidth, float minValue, float value)
{
    if (binWidth == 0)
        return 0;
    size_t b = (size_t) ((value - minValue) / binWidth);
    return (nBins - 1 < b) ? nBins - 1 : b;
}

/* math_functions.cpp:476-560 updateTensorHistogram_cpu */
void orc_entropy_update(orc_tpp* t, const float* x, int64_t n)
{
    double minInput = (double) orc_get_min(x, n);
    double maxInput = (double) orc_get_max(x, n);
    if (minInput == 0 && maxInput == 0)
        return;
    if (minInput == maxInput)
        maxInput = dmax_(maxInput, minInput + (double) 0.01f);
    if (!t->has_hist) {
        memset(t->hist, 0, sizeof(t->hist));
        t->has_hist = 1;
        t->min = minInput;
        t->max = maxInput;
    }
    if (minInput < t->min || maxInput > t->max) {
        double newMin = dmin_(minInput, t->min);
        double newMax = dmax_(maxInput, t->max);
        double destBinWidth = (newMax - newMin) / PDF_SIZE;
        double srcBinWidth = (t->max - t->min) / PDF_SIZE;
        double scaled[PDF_SIZE];
        memset(scaled, 0, sizeof(scaled));
        for (size_t i = 0; i < PDF_SIZE; ++i) {
            if (t->hist[i] == 0)
                continue;
            double srcBinBegin = t->min + srcBinWidth * (double) i;
            size_t destBin = (size_t) ((srcBinBegin - newMin) / destBinWidth);
            double destBinEnd = newMin + destBinWidth * (double) (destBin + 1);
            double dstBinCnt = dmin_(round((destBinEnd - srcBinBegin) / srcBinWidth * t->hist[i]), t->hist[i]);
            scaled[ent_get_bin(PDF_SIZE, (float) destBinWidth, (float) newMin, (float) srcBinBegin)] += dstBinCnt;
            if (dstBinCnt < t->hist[i])
                scaled[ent_get_bin(PDF_SIZE, (float) destBinWidth, (float) newMin,
                                   (float) (srcBinBegin + destBinWidth))] += t->hist[i] - dstBinCnt;
        }
        memcpy(t->hist, scaled, sizeof(scaled));
        t->min = newMin;
        t->max = newMax;
    }
    float binWidth = (float) ((t->max - t->min) / PDF_SIZE);
    float fmin = (float) t->min;
    for (int64_t i = 0; i < n; ++i)
        t->hist[ent_get_bin(PDF_SIZE, binWidth, fmin, x[i])] += 1;
    t->iterations++;
}

/* math_functions.cpp:562-641 rescaleHistogram (non-empty source) */
static void ent_rescale(const double* src, double srcMin, double srcMax, double dstMin, double dstMax, double* dst)
{
    if (srcMin == dstMin && srcMax == dstMax) {
        memcpy(dst, src, PDF_SIZE * sizeof(double));
        return;
    }
    const size_t numBins = PDF_SIZE;
    const double srcBinWidth = (srcMax - srcMin) / (double) numBins;
    const double destBinWidth = (dstMax - dstMin) / (double) numBins;
    memset(dst, 0, PDF_SIZE * sizeof(double));
    for (size_t s = 0; s < numBins; s++) {
        double v = src[s];
        if (v == 0)
            continue;
        double sStart = srcMin + (double) s * srcBinWidth;
        double sStop = srcMin + (double) (s + 1) * srcBinWidth;
        double startF = floor((sStart - dstMin) / destBinWidth);
        double stopF = ceil((sStop - dstMin) / destBinWidth);
        size_t i0 = (size_t) dmax_(startF, 0.0);
        size_t i1 = (size_t) dmax_(stopF, 0.0);
        if (i0 >= numBins) i0 = numBins - 1;
        if (i1 >= numBins) i1 = numBins - 1;
        double rem = v;
        for (size_t d = i0; d <= i1; d++) {
            double dStart = dstMin + (double) d * destBinWidth;
            double dStop = dstMin + (double) (d + 1) * destBinWidth;
            double oStart = dmax_(sStart, dStart);
            double oStop = dmin_(sStop, dStop);
            double ratio = (oStop - oStart) / srcBinWidth;
            ratio = ratio >= 0.0f ? ratio : 0.0f;
            ratio = ratio <= 1.0f ? ratio : 1.0f;
            double dist = round(ratio * v);
            dist = dist <= rem ? dist : rem;
            dst[d] += dist;
            rem -= dist;
        }
    }
}

/* std::accumulate(first, last, 0.f): the running sum is a float */
static double ent_accumulate_f(const double* p, size_t n)
{
    float acc = 0.f;
    for (size_t i = 0; i < n; i++)
        acc = (float) ((double) acc + p[i]);
    return (double) acc;
}

/* EntropyEncodingAnalyzer.cpp:156-198 _conditionHistogram */
static void ent_condition(double* h, size_t n)
{
    const double epsZero = 0.0001;
    size_t numZeros = 0;
    for (size_t i = 0; i < n; i++)
        numZeros += (h[i] == 0.f);
    if (numZeros == n)
        return;
    double epsNonZero = epsZero * (double) numZeros / (double) (n - numZeros);
    if (epsNonZero >= 1.0)
        return;
    for (size_t i = 0; i < n; i++) {
        int z = (h[i] == 0.f);
        h[i] += epsZero * z;
        h[i] -= epsNonZero * (1 - z);
    }
}

/* EntropyEncodingAnalyzer.cpp:200-224 _computeKL */
static double ent_kl(double* P, double* Q, size_t n)
{
    double sumP = ent_accumulate_f(P, n);
    double sumQ = ent_accumulate_f(Q, n);
    double divergence = 0;
    for (size_t i = 0; i < n; i++) {
        P[i] /= sumP;
        Q[i] /= sumQ;
        if (P[i] > 0 && Q[i] > 0)
            divergence += P[i] * log(P[i] / Q[i]);
    }
    return divergence;
}

/* EntropyEncodingAnalyzer.cpp:226-435 _optimizeKL (the DTYPE=float tuple it returns) */
static void ent_optimize_kl(const orc_tpp* t, int bw, int sym, int strict, int unsign, float* outMin, float* outMax)
{
    double histMin = t->min, histMax = t->max;
    double hist[PDF_SIZE];
    if (sym && ((histMin < 0.0) || (!unsign))) {
        float absoluteMax = (float) dmax_(fabs(histMax), fabs(histMin));
        float absoluteMin = -absoluteMax;
        ent_rescale(t->hist, histMin, histMax, absoluteMin, absoluteMax, hist);
        histMin = absoluteMin;
        histMax = absoluteMax;
    } else {
        memcpy(hist, t->hist, sizeof(hist));
    }
    const size_t numBins = PDF_SIZE, numQ = 255;
    if (bw != 8) {
        *outMin = (float) histMin;
        *outMax = (float) histMax;
        return;
    }
    const double binWidth = (histMax - histMin) / (double) numBins;
    double divOpt = INFINITY;
    double thrMin = histMin, thrMax = histMax;
    size_t start = 0, stop = numBins - 1;
    double P[PDF_SIZE], Q[PDF_SIZE];
    while ((stop - start + 1) >= numQ) {
        const size_t win = stop - start + 1;
        const double* hw = hist + start;
        memset(P, 0, win * sizeof(double));
        double leftSum = 0;
        for (size_t i = 0; i <= start; i++)
            leftSum += hist[i];
        P[0] += leftSum;
        for (size_t i = start + 1; i < stop; i++)
            P[i - start] = hist[i];
        double rightSum = 0;
        for (size_t i = stop; i < numBins; i++)
            rightSum += hist[i];
        P[win - 1] += rightSum;
        const double merged = (double) win / (double) numQ;
        memset(Q, 0, win * sizeof(double));
        for (size_t q = 0; q < numQ; q++) {
            const size_t i0 = (size_t) ceil((double) q * merged);
            const size_t i1 = (q < numQ - 1) ? (size_t) ceil((double) (q + 1) * merged) : win;
            double sum = 0, norm = 0;
            for (size_t i = i0; i < i1; i++) {
                sum += hw[i];
                norm += (hw[i] != 0);
            }
            if (norm != 0)
                for (size_t i = i0; i < i1; i++)
                    if (hw[i] != 0)
                        Q[i] = sum / norm;
        }
        if (ent_accumulate_f(P, win) == 0 || ent_accumulate_f(Q, win) == 0)
            break;
        ent_condition(P, win);
        ent_condition(Q, win);
        double dv = ent_kl(P, Q, win);
        if (dv < divOpt) {
            divOpt = dv;
            thrMin = histMin + (double) start * binWidth;
            thrMax = histMin + (double) (stop + 1) * binWidth;
        }
        if (sym || strict) {
            start++;
            stop--;
        } else {
            double loss[3] = {hist[start] + hist[stop], hist[start] + hist[start + 1], hist[stop] + hist[stop - 1]};
            int k = 0;
            if (loss[1] < loss[k]) k = 1;
            if (loss[2] < loss[k]) k = 2;
            if ((k == 0 && (histMin + (double) (start + 1) * binWidth) > 0) ||
                (k == 1 && (histMin + (double) (start + 2) * binWidth) > 0))
                k = 2;
            else if ((k == 0 && (histMin + (double) stop * binWidth) < 0) ||
                     (k == 2 && (histMin + (double) (stop - 1) * binWidth) < 0))
                k = 1;
            if (k == 0) {
                start++;
                stop--;
            } else if (k == 1) {
                start += 2;
            } else {
                stop -= 2;
            }
        }
    }
    *outMin = (float) thrMin;
    *outMax = (float) thrMax;
}

/* EntropyEncodingAnalyzer.cpp:97-148 computeEncoding */
orc_encoding orc_entropy_compute(const orc_tpp* t, int stats_updated, int bw, int sym, int strict, int unsign)
{
    orc_encoding e = {0, 0, 0, 0, 0};
    float numSteps = (float) (pow(2.0, (double) bw) - 1);
    if (sym && strict)
        numSteps -= 1;
    if (!t->has_hist)
        return stats_updated ? zero_data_encoding(bw, numSteps) : e;
    float aMin, aMax;
    ent_optimize_kl(t, bw, sym, strict, unsign, &aMin, &aMax);
    aMin = fmin_(aMin, 0.0f);
    aMax = fmax_(aMax, 0.0f);
    return orc_get_computed_encodings(bw, aMin, aMax, sym, strict, unsign);
}

/* ------------------------------------------------------------------------- */
/* Analyzer facade (IQuantizationEncodingAnalyzer<float>, QuantizerFactory.cpp:74-104)          */
/* ------------------------------------------------------------------------- */

typedef struct {
    int scheme;
    int stats_updated;
    double acc_min, acc_max;   /* TfEncodingAnalyzer.h:86-91 */
    float percentile;          /* PercentileEncodingAnalyzer.h:100 */
    orc_pdf pdf;
    orc_tpp tpp;               /* EntropyEncodingAnalyzer.h: _tensorProfilingParams */
} orc_analyzer;

size_t orc_analyzer_size(void) { return sizeof(orc_analyzer); }

int orc_analyzer_init(orc_analyzer* a, int scheme)
{
    memset(a, 0, sizeof(*a));
    if (scheme == QUANTIZATION_RANGE_LEARNING)   /* QuantizerFactory.cpp:93-96 */
        scheme = QUANTIZATION_TF;
    a->scheme = scheme;
    a->acc_min = DBL_MAX;
    a->acc_max = -DBL_MAX;
    a->percentile = 100.0f;
    return 0;
}

void orc_analyzer_set_percentile(orc_analyzer* a, float p) { a->percentile = p; }

/* TfEncodingAnalyzer.cpp:59-72; TfEnhanced/Percentile/Mse updateStats -> UpdatePdf(signed=true) */
void orc_analyzer_update(orc_analyzer* a, const float* x, int64_t n)
{
    a->stats_updated = 1;
    if (a->scheme == QUANTIZATION_TF) {
        double cmin = (double) orc_get_min(x, n);
        double cmax = (double) orc_get_max(x, n);
        a->acc_min = dmin_(a->acc_min, cmin);
        a->acc_max = dmax_(a->acc_max, cmax);
    } else if (a->scheme == QUANTIZATION_ENTROPY) {
        orc_entropy_update(&a->tpp, x, n);
    } else {
        orc_update_pdf(&a->pdf, x, n, 1);
    }
}

/* TfEncodingAnalyzer.cpp:80-101 */
static orc_encoding tf_compute(const orc_analyzer* a, int bw, int sym, int strict, int unsign)
{
    double newMin = dmin_(0.0, a->acc_min);
    double newMax = dmax_(0.0, a->acc_max);
    newMax = dmax_(newMax, newMin + MIN_RANGE);
    return orc_get_computed_encodings(bw, newMin, newMax, sym, strict, unsign);
}

orc_encoding orc_analyzer_compute(const orc_analyzer* a, int bw, int sym, int strict, int unsign)
{
    switch (a->scheme) {
    case QUANTIZATION_TF: return tf_compute(a, bw, sym, strict, unsign);
    case QUANTIZATION_TF_ENHANCED: return tfe_compute(&a->pdf, a->stats_updated, bw, sym, strict, unsign);
    case QUANTIZATION_PERCENTILE:
        return percentile_compute(&a->pdf, a->stats_updated, a->percentile, bw, sym, strict, unsign);
    case QUANTIZATION_MSE: return mse_compute(&a->pdf, a->stats_updated, bw, sym, strict, unsign);
    case QUANTIZATION_ENTROPY: return orc_entropy_compute(&a->tpp, a->stats_updated, bw, sym, strict, unsign);
    default: { orc_encoding z = {0, 0, 0, 0, 0}; return z; }
    }
}

/* getStatsHistogram (math_functions.cpp:386-402): copies xLeft/pdf; returns element count */
int orc_analyzer_histogram(const orc_analyzer* a, double* xleft, double* pdf)
{
    if (!a->pdf.initialized) return 0;
    memcpy(xleft, a->pdf.xLeft, sizeof(a->pdf.xLeft));
    memcpy(pdf, a->pdf.pdf, sizeof(a->pdf.pdf));
    return PDF_SIZE;
}

/* Reduced statistics, as the HIP path keeps them (tests of the host-side encoding math) */
void orc_analyzer_stats(const orc_analyzer* a, int* stats_updated, double* acc_min, double* acc_max,
                        int* initialized, float* hist_min, double* bucket_size, int* iterations)
{
    *stats_updated = a->stats_updated;
    *acc_min = a->acc_min;
    *acc_max = a->acc_max;
    *initialized = a->pdf.initialized;
    *hist_min = a->pdf.hist_min;
    *bucket_size = a->pdf.bucket_size;
    *iterations = a->pdf.iterations;
}

/* Fold a batch's (already exchanged) min/max into the analyzer: TF running min/max, or the PDF
 * range on the first non-zero batch -- the same step UpdatePdf / TfEncodingAnalyzer::updateStats
 * take after GetMin/GetMax (math_functions.cpp:249-260, TfEncodingAnalyzer.cpp:63-71).
 * Returns 1 when a histogram update must follow (PDF initialised). */
int orc_analyzer_fold_minmax(orc_analyzer* a, float mn, float mx)
{
    a->stats_updated = 1;
    if (a->scheme == QUANTIZATION_TF) {
        a->acc_min = dmin_(a->acc_min, (double) mn);
        a->acc_max = dmax_(a->acc_max, (double) mx);
        return 0;
    }
    if (!a->pdf.initialized) {
        if (mn == 0 && mx == 0)
            return 0;
        orc_initialize_pdf(&a->pdf, mn, mx, 1);
    }
    return 1;
}

/* Entropy statistics (TensorProfilingParams) for tests of the device path */
orc_tpp* orc_analyzer_tpp(orc_analyzer* a) { return &a->tpp; }

/* Direct PDF access for tests of the sharded path */
orc_pdf* orc_analyzer_pdf(orc_analyzer* a) { return &a->pdf; }

/* ------------------------------------------------------------------------- */
/* Blockwise (broadcast) QDQ and the block-layout permutation                  */
/* ------------------------------------------------------------------------- */

/* trim_functions.cpp:633-660 quantizeDequantizeBroadcastCpu (int index arithmetic as written) */
void orc_qdq_broadcast(const float* in, float* out, int64_t n, int64_t nd, const int64_t* istr, const int64_t* estr,
                       const float* emin, const float* emax, const float* edelta, const float* eoff)
{
    for (size_t i = 0; i < (size_t) n; i++) {
        int e = 0;
        int rem = (int) i;
        for (int d = 0; d < nd; d++) {
            int q = (int) (rem / istr[d]);
            rem = (int) (rem - q * istr[d]);
            e += (int) (estr[d] * q);
        }
        float v = quantize_value(in[i], emin[e], emax[e], edelta[e], eoff[e]);
        out[i] = dequantize_value(v, edelta[e], eoff[e]);
    }
}

/* onnx/src/QuantizeDequantizeUtils.cpp:64-95 permuteTensorCPU */
void orc_permute(const float* in, float* out, int64_t n, int64_t nd, const int64_t* istr, const int64_t* ostr)
{
    int64_t chunk = n;
    for (int64_t i = nd - 1; i >= 0; i--)
        if (istr[i] != ostr[i]) {
            chunk = istr[i];
            break;
        }
    for (size_t i = 0; i < (size_t) n; i += (size_t) chunk) {
        size_t o = 0, rem = i;
        for (int d = 0; d < nd; d++) {
            size_t q = rem / (size_t) istr[d];
            rem = rem - q * (size_t) istr[d];
            o += (size_t) ostr[d] * q;
        }
        memcpy(out + o, in + i, (size_t) chunk * sizeof(float));
    }
}
