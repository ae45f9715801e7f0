// entropy_kl.hpp -- the entropy analyzer's KL-divergence range search, one source for the host
// (encodings.cpp: kl_range) and the device (entropy_search.hip): EntropyEncodingAnalyzer.cpp:
// 156-435 (_conditionHistogram, _computeKL, _optimizeKL) over rescaleHistogram
// (math_functions.cpp:562-641).
//
// The reference loop shrinks a window [a, b] over the 512 bins and keeps the window whose
// 255-level requantisation Q is closest (KL) to the saturated P. Which window comes next depends
// only on the histogram, never on a KL value, so the windows are enumerated first (`windows`) and
// each one's KL is an independent computation (`window_kl`): P and Q are streamed bin by bin in
// the reference's order instead of being materialised, with the same float / double operations
// (std::accumulate(..., 0.f) sums in float, the conditioning, the normalisation and the
// p * log(p / q) sum in ascending order). The only operation that differs between the host and
// the device is the natural logarithm (glibc vs the device library: both within an ulp or two of
// the true value), which `window_kl` takes as a parameter; the device search re-checks near-ties
// on the host (entropy_search.hip).
//
// Compiled with -ffp-contract=off on both sides.
#pragma once

#include "entropy_core.hpp"

#include <cmath>

namespace aimet_amd
{
namespace entropy
{

constexpr int kLevels  = 255;                          // requantisation levels of _optimizeKL (8 bit)
constexpr int kWindows = (kBins - kLevels) / 2 + 1;    // every step shrinks the window by 2 bins: 129

template <class T>
AIMET_ENT_HD T kmin(T a, T b)
{
    return (b < a) ? b : a;   // std::min
}
template <class T>
AIMET_ENT_HD T kmax(T a, T b)
{
    return (a < b) ? b : a;   // std::max
}

// rescaleHistogram (math_functions.cpp:562-641) of a non-empty source: redistribute the bins of
// [srcMin, srcMax] over [dstMin, dstMax]; every part is a rounded share of the source bin, capped
// by what is left of it, added to the destination bins in ascending source order.
AIMET_ENT_HD void rescale_histogram(const double* src, double srcMin, double srcMax, double dstMin, double dstMax,
                                    double* dst)
{
    if (srcMin == dstMin && srcMax == dstMax)
    {
        for (int i = 0; i < kBins; ++i)
            dst[i] = src[i];
        return;
    }
    const uint64_t n  = kBins;
    const double srcW = (srcMax - srcMin) / (double) n;
    const double dstW = (dstMax - dstMin) / (double) n;
    for (int i = 0; i < kBins; ++i)
        dst[i] = 0.0;
    for (uint64_t b = 0; b < n; ++b)
    {
        const double v = src[b];
        if (v == 0)
            continue;
        const double s0 = srcMin + (double) b * srcW;
        const double s1 = srcMin + (double) (b + 1) * srcW;
        uint64_t d0     = x86_d2u64(kmax(floor((s0 - dstMin) / dstW), 0.0));
        uint64_t d1     = x86_d2u64(kmax(ceil((s1 - dstMin) / dstW), 0.0));
        d0              = kmin(d0, n - 1);
        d1              = kmin(d1, n - 1);
        double rem      = v;
        for (uint64_t k = d0; k <= d1; ++k)
        {
            const double o0 = kmax(s0, dstMin + (double) k * dstW);
            const double o1 = kmin(s1, dstMin + (double) (k + 1) * dstW);
            double ratio    = (o1 - o0) / srcW;
            ratio           = ratio >= 0.0f ? ratio : 0.0f;
            ratio           = ratio <= 1.0f ? ratio : 1.0f;
            double part     = round(ratio * v);
            part            = part <= rem ? part : rem;
            dst[k] += part;
            rem -= part;
        }
    }
}

// _optimizeKL (:226-270): the histogram the windows run over and its range. Symmetric encodings
// (unless unsigned over a non-negative range) first rescale to [-absmax, absmax].
AIMET_ENT_HD void kl_histogram(double tmin, double tmax, const double* tpp_hist, bool sym, bool unsign, double* hist,
                               double& lo, double& hi)
{
    lo = tmin;
    hi = tmax;
    if (sym && (lo < 0.0 || !unsign))
    {
        const float amax = (float) kmax(fabs(hi), fabs(lo));
        const float amin = -amax;
        rescale_histogram(tpp_hist, lo, hi, amin, amax, hist);
        lo = amin;
        hi = amax;
    }
    else
        for (int i = 0; i < kBins; ++i)
            hist[i] = tpp_hist[i];
}

// The windows the reference visits, in order (:272-435): both ends shrink at once for symmetric
// or strict encodings; otherwise the end(s) losing the least mass, keeping 0 inside the range.
// Returns the count (kWindows); wa/wb[k] = the inclusive bounds of window k.
AIMET_ENT_HD int windows(const double* hist, double lo, double w, bool both_ends, short* wa, short* wb)
{
    int a = 0, b = kBins - 1;   // the reference's size_t indices: the same values, converted to double exactly
    int n = 0;
    while (b - a + 1 >= kLevels)
    {
        wa[n] = (short) a;
        wb[n] = (short) b;
        ++n;
        if (both_ends)
        {
            ++a;
            --b;
            continue;
        }
        const double loss[3] = {hist[a] + hist[b], hist[a] + hist[a + 1], hist[b] + hist[b - 1]};
        int k                = 0;   // std::min_element: the first minimum
        if (loss[1] < loss[k])
            k = 1;
        if (loss[2] < loss[k])
            k = 2;
        if ((k == 0 && lo + (double) (a + 1) * w > 0) || (k == 1 && lo + (double) (a + 2) * w > 0))
            k = 2;   // keep 0 representable: only shrink from the right
        else if ((k == 0 && lo + (double) b * w < 0) || (k == 2 && lo + (double) (b - 1) * w < 0))
            k = 1;   // ... or only from the left
        if (k == 0)
        {
            ++a;
            --b;
        }
        else if (k == 1)
            a += 2;
        else
            b -= 2;
    }
    return n;
}

// One window's P (saturated) and Q (255-level requantisation) streamed in bin order. For each
// bin i of the window, emit(i, P[i], Q[i]) is called in ascending i.
template <class Emit>
AIMET_ENT_HD void stream_pq(const double* hist, int a, int b, double left, double right, Emit&& emit)
{
    const int win        = b - a + 1;
    const double* hw     = hist + a;
    const double merged  = (double) win / (double) kLevels;
    for (int q = 0; q < kLevels; ++q)
    {
        const int i0 = (int) (uint64_t) ceil((double) q * merged);
        const int i1 = q < kLevels - 1 ? (int) (uint64_t) ceil((double) (q + 1) * merged) : win;
        double sum = 0, norm = 0;
        for (int i = i0; i < i1; ++i)
        {
            sum += hw[i];
            norm += (hw[i] != 0);
        }
        for (int i = i0; i < i1; ++i)
        {
            const double Qi = (norm != 0 && hw[i] != 0) ? sum / norm : 0.0;
            const double Pi = i == 0 ? 0.0 + left : (i == win - 1 ? 0.0 + right : hw[i]);
            emit(i, Pi, Qi);
        }
    }
}

// _conditionHistogram (:156-198) of one value: `h += epsZero * z; h -= epsNonZero * (1 - z)`
struct Cond
{
    bool skip;     // every bin zero, or epsNonZero >= 1: the histogram is left as it is
    double eps;    // epsNonZero
};
AIMET_ENT_HD Cond cond_of(uint64_t zeros, uint64_t n)
{
    const double epsZero = 0.0001;
    if (zeros == n)
        return Cond {true, 0.0};
    const double e = epsZero * (double) zeros / (double) (n - zeros);
    return Cond {e >= 1.0, e};
}
AIMET_ENT_HD double cond_apply(const Cond& c, double h)
{
    if (c.skip)
        return h;
    const int z = (h == 0.f);
    h += 0.0001 * z;
    h -= c.eps * (1 - z);
    return h;
}

struct WindowKl
{
    bool brk;      // the reference loop stops at this window (P or Q sums to 0)
    double dv;     // KL(P || Q)
    double mag;    // sum of |p * log(p / q)| (the device's near-tie tolerance scales with it)
};

// Per-histogram tables shared by every window (built once, in the reference's summation order):
//   left[a]  = hist[0] + ... + hist[a]          (sequential double sum, as the window loop adds it)
//   zeros[k] = number of zero bins in hist[0, k)
//   q_zero_rule: every bin is 0 or in [1e-300, DBL_MAX] (bin counts always are). Then Q[i] == 0
//   exactly when hw[i] == 0 (a non-empty level's sum / norm cannot underflow), so both zero
//   counts of the conditioning are known before the window is streamed.
struct Prefix
{
    const double* left;   // [kBins]
    const int* zeros;     // [kBins + 1]
    bool q_zero_rule;
};

AIMET_ENT_HD void build_prefix(const double* hist, double* left, int* zeros, bool& q_zero_rule)
{
    double l = 0;
    int z    = 0;
    bool ok  = true;
    zeros[0] = 0;
    for (int i = 0; i < kBins; ++i)
    {
        l += hist[i];
        left[i] = l;
        z += hist[i] == 0;
        zeros[i + 1] = z;
        ok = ok && (hist[i] == 0 || (hist[i] >= 1e-300 && hist[i] <= 1.7976931348623157e308));
    }
    q_zero_rule = ok;
}

// _computeKL (:200-224) of window [a, b] over `hist`, with `lg` the natural logarithm. With a
// Prefix whose q_zero_rule holds, the accumulate() sums and the conditioned normalisers come
// from one streamed pass instead of two (same operations, same order).
template <class Log>
AIMET_ENT_HD WindowKl window_kl(const double* hist, int a, int b, Log&& lg, const Prefix* pre = nullptr)
{
    const int win = b - a + 1;
    double left = 0, right = 0;
    if (pre)
        left = pre->left[a];
    else
        for (int i = 0; i <= a; ++i)
            left += hist[i];
    for (int i = b; i < kBins; ++i)
        right += hist[i];
    float aP = 0.f, aQ = 0.f, sP = 0.f, sQ = 0.f;
    Cond cP, cQ;
    if (pre && pre->q_zero_rule)
    {
        // P = {left, hist[a+1 .. b-1], right}, Q is zero exactly where hist[a .. b] is
        const uint64_t zP = (uint64_t) (pre->zeros[b] - pre->zeros[a + 1]) + (left == 0.f) + (right == 0.f);
        const uint64_t zQ = (uint64_t) (pre->zeros[b + 1] - pre->zeros[a]);
        cP = cond_of(zP, (uint64_t) win);
        cQ = cond_of(zQ, (uint64_t) win);
        stream_pq(hist, a, b, left, right, [&](int, double p, double q) {
            aP = (float) ((double) aP + p);
            aQ = (float) ((double) aQ + q);
            sP = (float) ((double) sP + cond_apply(cP, p));
            sQ = (float) ((double) sQ + cond_apply(cQ, q));
        });
        if (aP == 0 || aQ == 0)
            return WindowKl {true, 0.0, 0.0};
    }
    else
    {
        // pass 1: accumulate(P), accumulate(Q) (float) and the zero counts of the conditioning
        uint64_t zP = 0, zQ = 0;
        stream_pq(hist, a, b, left, right, [&](int, double p, double q) {
            aP = (float) ((double) aP + p);
            aQ = (float) ((double) aQ + q);
            zP += (p == 0.f);
            zQ += (q == 0.f);
        });
        if (aP == 0 || aQ == 0)
            return WindowKl {true, 0.0, 0.0};
        cP = cond_of(zP, (uint64_t) win);
        cQ = cond_of(zQ, (uint64_t) win);
        // pass 2: the normalisers of the conditioned histograms (float accumulate)
        stream_pq(hist, a, b, left, right, [&](int, double p, double q) {
            sP = (float) ((double) sP + cond_apply(cP, p));
            sQ = (float) ((double) sQ + cond_apply(cQ, q));
        });
    }
    // the divergence, ascending
    double dv = 0, mag = 0;
    const double dP = sP, dQ = sQ;
    stream_pq(hist, a, b, left, right, [&](int, double p, double q) {
        const double pn = cond_apply(cP, p) / dP;
        const double qn = cond_apply(cQ, q) / dQ;
        if (pn > 0 && qn > 0)
        {
            const double t = pn * lg(pn / qn);
            dv += t;
            mag += fabs(t);
        }
    });
    return WindowKl {false, dv, mag};
}

}   // namespace entropy
}   // namespace aimet_amd
