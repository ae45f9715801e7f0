// tfe_core.hpp -- TF-Enhanced encoding search, one source for the host (encodings.cpp) and the
// device (tfe_search.hip): TfEnhancedEncodingAnalyzer.cpp:115-392 with DTYPE = float.
//
// Every expression keeps the reference's evaluation types (float vs double), std::min/std::max
// tie rules and std::round (half away from zero); pow(v, 2) is v*v as the reference build
// (-O3) folds it. Compiled with -ffp-contract=off on both sides, IEEE fp32/fp64 division.
#pragma once

#include <cfloat>
#include <cmath>

#if defined(__HIPCC__)
#define AIMET_HD __host__ __device__
#else
#define AIMET_HD
#endif

namespace aimet_amd
{
namespace tfe
{

constexpr int kBins        = 512;
constexpr float kGamma     = 3.0f;     // TfEnhancedEncodingAnalyzer.h:102 (DTYPE)
constexpr float kMinRangeF = (float) 0.01;
constexpr int kAsymF       = 17;       // deltas f = 1/16 .. 17/16
constexpr int kAsymO       = 21;       // offsets i = 0 .. 20
constexpr int kSymF        = 101;      // deltas f = 1/100 .. 101/100
constexpr int kMaxCand     = kAsymF * kAsymO + 1;

template <class T>
AIMET_HD inline T smin(T a, T b)
{
    return (b < a) ? b : a;   // std::min
}
template <class T>
AIMET_HD inline T smax(T a, T b)
{
    return (a < b) ? b : a;   // std::max
}

// PDF of one channel: xLeft[i] = (double)hist_min + (double)i * bucket (InitializePdf)
struct Hist
{
    float hist_min;
    double bucket;
    const double* pdf;
    AIMET_HD double xl(int i) const
    {
        return (double) hist_min + (double) i * bucket;
    }
};

// _findRangeOfAggregateStats (:255-291) given the first / last non-empty bins (-1: none;
// `last` only scans i > 0 like the reference loop).
AIMET_HD inline void observed_range(const Hist& h, int first, int last, float& lo, float& hi)
{
    lo = (float) h.xl(0);
    hi = (float) h.xl(kBins - 1);
    if (first >= 0)
        lo = (float) h.xl(first);
    if (last >= 0)
        hi = (float) h.xl(last);
    lo = smin(lo, 0.0f);
    hi = smax(hi, 0.0f);
    hi = smax(hi, lo + kMinRangeF);
}

// first non-empty bin and last non-empty bin with i > 0 (-1: none), serial form
AIMET_HD inline void first_last(const double* pdf, int& first, int& last)
{
    first = last = -1;
    for (int i = 0; i < kBins; ++i)
        if (pdf[i] > 0)
        {
            first = i;
            break;
        }
    for (int i = kBins - 1; i > 0; --i)
        if (pdf[i] > 0)
        {
            last = i;
            break;
        }
}

// f sequences of the candidate loops: float accumulator, double comparison (data independent)
AIMET_HD inline int fseq_asym(float* f)
{
    int n = 0;
    for (float v = 1.0 / 16; v <= 1 + 1.0 / 16; v += 1.0 / 16)
        f[n++] = v;
    return n;
}
AIMET_HD inline int fseq_sym(float* f)
{
    int n = 0;
    for (float v = 1.0 / 100; v <= 1 + 1.0 / 100; v += 1.0 / 100)
        f[n++] = v;
    return n;
}

// _clampToObservedMinMax (:144-170)
AIMET_HD inline bool clamp_candidate(float obsLo, float obsHi, float steps, float& delta, int& offset)
{
    float lo = smax(delta * offset, -FLT_MAX);
    float hi = smin(delta * (offset + steps), FLT_MAX);
    if (lo < obsLo && hi > obsHi)
        return false;
    lo = smax(obsLo, lo);
    hi = smin(obsHi, hi);
    if (lo == hi)
        return false;
    delta  = (float) (((double) hi - lo) / steps);
    offset = (int) roundf(lo / delta);
    return true;
}

// Search parameters of one channel, derived from the observed range.
struct Setup
{
    bool sym;
    float steps;        // numSteps (strict-reduced for symmetric strict)
    // asymmetric
    float obsLo, obsHi, d0;
    int o0;
    // symmetric
    float dmax;
    int symOffset;
    int ncand;
};

AIMET_HD inline Setup setup(float lo, float hi, int bw, bool sym, bool strict, bool unsign)
{
    Setup s {};
    s.sym   = sym;
    s.steps = (float) (ldexp(1.0, bw) - 1);   // pow(2, bw) - 1, exact
    if (sym)
    {
        if (strict)
            s.steps -= 1;
        if ((lo == 0.0) && unsign)
        {
            s.dmax      = hi / s.steps;
            s.symOffset = 0;
        }
        else
        {
            float absmax = smax(fabsf(hi), fabsf(lo));
            s.dmax       = (float) (absmax / (s.steps / 2.0));
            s.symOffset  = (int) floorf(-s.steps / 2);
        }
        s.ncand = kSymF;
    }
    else
    {
        s.d0    = (float) (((double) hi - (double) lo) / s.steps);
        s.o0    = (int) roundf(lo / s.d0);
        s.obsLo = smax(s.d0 * s.o0, -FLT_MAX);
        s.obsHi = smin(s.d0 * (s.o0 + s.steps), FLT_MAX);
        s.ncand = kAsymF * kAsymO + 1;
    }
    return s;
}

// Candidate t in the reference's order; false when _clampToObservedMinMax drops it.
AIMET_HD inline bool candidate(const Setup& s, const float* fseq, int t, float& delta, int& offset)
{
    if (s.sym)
    {
        delta  = fseq[t] * s.dmax;
        offset = s.symOffset;
        return true;
    }
    if (t == kAsymF * kAsymO)
    {
        delta  = s.d0;
        offset = s.o0;
        return true;
    }
    int k  = t / kAsymO, i = t % kAsymO;
    delta  = fseq[k] * s.d0;
    offset = (int) (-s.steps + s.steps / 20.0 * i);
    return clamp_candidate(s.obsLo, s.obsHi, s.steps, delta, offset);
}

// Per-channel precomputation shared by every candidate of _quantAndSatCost (:293-355):
//   cd[i] = start + i*step + step/2 (double, the bin centre as the reference evaluates it)
//   cf[i] = (float) cd[i]            (loMid / hiMid / the quantised value v)
// and, over the bins the cost loops must visit (ascending bin index, k = 0..nnz):
//   pdf_c[k], cd_c[k], cf_c[k]       (the visited bins' pdf and centres, compacted)
//   pos[i] = number of visited bins with index < i   (i = 0..kBins-1)
// A bin whose pdf is 0 adds exactly +0.0 to its sum as long as its squared distance is finite,
// so such bins are skipped when the histogram range is bounded (|x| <= 1e30 keeps every
// distance finite); otherwise every bin is visited, as in the reference.
struct Bins
{
    float start;
    double step;
    const float* cf;
    const double* pdf_c;
    const double* cd_c;
    const float* cf_c;
    const short* pos;
    int nnz;
};

AIMET_HD inline float bins_start(const Hist& h)
{
    return (float) h.xl(0);
}
AIMET_HD inline double bins_step(const Hist& h)
{
    return h.xl(1) - h.xl(0);
}
AIMET_HD inline double bin_centre(float start, double step, int i)
{
    return start + i * step + step / 2;
}
AIMET_HD inline bool bins_skip_empty(const Hist& h)
{
    double a = h.xl(0), b = h.xl(kBins - 1) + (h.xl(1) - h.xl(0));
    return a >= -1e30 && a <= 1e30 && b >= -1e30 && b <= 1e30;
}

// (int) std::round(v / delta - offset) exactly as the reference evaluates it (float division,
// half away from zero). On the device the IEEE division is taken only near half-integers: with
// rcp = RN(1/delta) and thr >= 2^-21 (|v*rcp| + |offset| + 1) for every v of the loop, rint of
// RN(RN(v*rcp) - offset) equals the reference's rounding whenever the fractional part is more
// than thr away from 1/2 (the round_div_sub / qdq_round_fast argument, common.hpp); the int
// conversion drops the sign of a zero code, so no sign test is needed.
AIMET_HD inline int quant_code(float v, float delta, int offset, float rcp, float thr)
{
#if defined(__HIP_DEVICE_COMPILE__)
    const float x = v * rcp - (float) offset;
    if (fabsf(__builtin_amdgcn_fractf(x) - 0.5f) > thr)   // false for NaN
        return (int) __builtin_rintf(x);
#else
    (void) rcp;
    (void) thr;
#endif
    return (int) roundf(v / delta - offset);
}

// The three sums of _quantAndSatCost over visited bins [k0, k1), ascending. Four bins' terms are
// formed at once (independent LDS loads and products: a lane's loop is latency-bound otherwise)
// and added in the serial order, so every sum is the reference's, bit for bit.
AIMET_HD inline double sat_sum(const Bins& B, int k0, int k1, double mid)
{
    double s = 0;
    int k    = k0;
    for (; k + 4 <= k1; k += 4)
    {
        double t[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
        {
            double d = B.cd_c[k + u] - mid;
            t[u]     = B.pdf_c[k + u] * (d * d);
        }
        s += t[0];
        s += t[1];
        s += t[2];
        s += t[3];
    }
    for (; k < k1; ++k)
    {
        double d = B.cd_c[k] - mid;
        s += B.pdf_c[k] * (d * d);
    }
    return s;
}

AIMET_HD inline double quant_term(const Bins& B, int k, float delta, int offset, float rcp, float thr)
{
    float v   = B.cf_c[k];
    int q     = quant_code(v, delta, offset, rcp, thr);
    float deq = delta * (q + offset);
    double d  = (double) (v - deq);
    return B.pdf_c[k] * (d * d);
}

AIMET_HD inline double quant_sum(const Bins& B, int k0, int k1, float delta, int offset, float rcp, float thr)
{
    double s = 0;
    int k    = k0;
#if defined(__HIP_DEVICE_COMPILE__)
    // Four bins at once with ONE exactness test for the four codes (a branch per bin serialised
    // the wave). quantized + offset is formed in float, rint(x) + offset, where that sum is exact:
    // thr = 2^-21 (vmax * rcp + |offset| + 1) < 4 bounds |rint(x) + offset| ~ |v * rcp| below
    // 2^23 and both integer operands below 2^24, so it is the reference's int sum converted for
    // the multiply, without the two conversions.
    const float of   = (float) offset;
    const bool fsum  = thr < 4.0f;   // false for a NaN thr
    for (; k + 4 <= k1; k += 4)
    {
        float v[4], x[4], qf[4];
        bool fast = fsum;
#pragma unroll
        for (int u = 0; u < 4; ++u)
        {
            v[u] = B.cf_c[k + u];
            x[u] = v[u] * rcp - of;
            fast &= __builtin_fabsf(__builtin_amdgcn_fractf(x[u]) - 0.5f) > thr;
        }
        if (fast)
        {
#pragma unroll
            for (int u = 0; u < 4; ++u)
                qf[u] = __builtin_rintf(x[u]) + of;
        }
        else
        {
#pragma unroll
            for (int u = 0; u < 4; ++u)
                qf[u] = (float) (quant_code(v[u], delta, offset, rcp, thr) + offset);
        }
        double t[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
        {
            const double d = (double) (v[u] - delta * qf[u]);
            t[u]           = B.pdf_c[k + u] * (d * d);
        }
        s += t[0];
        s += t[1];
        s += t[2];
        s += t[3];
    }
#else
    for (; k + 4 <= k1; k += 4)
    {
        double t[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            t[u] = quant_term(B, k + u, delta, offset, rcp, thr);
        s += t[0];
        s += t[1];
        s += t[2];
        s += t[3];
    }
#endif
    for (; k < k1; ++k)
        s += quant_term(B, k, delta, offset, rcp, thr);
    return s;
}

// _quantAndSatCost (:293-355) over the prepared bins. The reference's three loops are kept as
// three loops, each over its own contiguous range of visited bins (i < iLo, i >= iHi,
// iLo <= i < iHi) in ascending order, so every sum adds the same terms in the same order; a bin
// can belong to both saturation ranges exactly as in the reference. `split` picks between running
// them as three loops (the lanes of a wave, one candidate each, run branch-free bodies: the
// symmetric grid, whose candidates' ranges nest) or as one guarded loop; both give identical sums.
template <bool split>
AIMET_HD inline double cost(const Bins& B, int bw, float delta, int offset)
{
    const float lo    = delta * offset;
    const float steps = (float) (ldexp(1.0, bw) - 1);
    const float hi    = delta * (offset + steps);
    int iLo           = (int) floor((lo - B.start) / B.step);
    iLo               = smin(smax(0, iLo), kBins - 1);
    int iHi           = (int) floor((hi - B.start) / B.step);
    iHi               = smin(smax(0, iHi), kBins - 1);
    const float loMid = B.cf[iLo];
    const float hiMid = B.cf[iHi];
    // every v of the quantisation loop lies in [cf[iLo], cf[iHi]] (bin centres ascend)
    const float rcp = 1.0f / delta;
    const float vmax = (loMid != loMid || hiMid != hiMid) ? NAN : smax(fabsf(loMid), fabsf(hiMid));   // NaN: exact path
    const float thr  = (vmax * rcp + fabsf((float) offset) + 1.0f) * 4.76837158203125e-7f;
    const int kLo = B.pos[iLo];   // visited bins below iLo: k in [0, kLo)
    const int kHi = B.pos[iHi];   // visited bins at or above iHi: k in [kHi, nnz)
    double satLo = 0, satHi = 0, quant = 0;
    if constexpr (!split)
    {
        // one pass with the three bodies guarded: the lanes of a wave share each bin's loads,
        // which wins when their candidates' ranges differ widely (the asymmetric grid)
        for (int k = 0; k < B.nnz; ++k)
        {
            if (k < kLo)
            {
                double d = B.cd_c[k] - loMid;
                satLo += B.pdf_c[k] * (d * d);
            }
            if (k >= kHi)
            {
                double d = B.cd_c[k] - hiMid;
                satHi += B.pdf_c[k] * (d * d);
            }
            if (k >= kLo && k < kHi)
            {
                float v   = B.cf_c[k];
                int q     = quant_code(v, delta, offset, rcp, thr);
                float deq = delta * (q + offset);
                double d  = (double) (v - deq);
                quant += B.pdf_c[k] * (d * d);
            }
        }
        double c = kGamma * (satLo + satHi) + quant;
        return smin(c, DBL_MAX);
    }
    satLo = sat_sum(B, 0, kLo, loMid);
    satHi = sat_sum(B, kHi, B.nnz, hiMid);
    quant = quant_sum(B, kLo, kHi, delta, offset, rcp, thr);   // empty unless iLo < iHi
    double c = kGamma * (satLo + satHi) + quant;
    return smin(c, DBL_MAX);
}

struct Result
{
    double min, max, delta, offset;
};

// getComputedEncodings (:357-392) tail from the best candidate
AIMET_HD inline Result finish(const Setup& s, float bestDelta, int bestOffset)
{
    float lo = smax(bestDelta * bestOffset, -FLT_MAX);
    float hi = smin(bestDelta * (bestOffset + s.steps), FLT_MAX);
    return Result {lo, hi, bestDelta, (double) bestOffset};
}

}   // namespace tfe
}   // namespace aimet_amd
