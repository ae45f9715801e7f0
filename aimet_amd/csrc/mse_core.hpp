// mse_core.hpp -- MSE encoding search, one source for the host (encodings.cpp) and the device
// (mse_search.hip): MseEncodingAnalyzer.cpp:79-264 with DTYPE = float, plus getComputedEncodings
// (quantization_utils.cpp:58-143) which every MSE candidate evaluates.
//
// Same evaluation types (float accumulator of the cost, double encoding math), std::min/std::max
// tie rules and std::round; compiled with -ffp-contract=off on both sides.
#pragma once

#include "tfe_core.hpp"

#include "../../include/aimet_amd.h"

namespace aimet_amd
{
namespace mse
{

constexpr int kMaxEdges = tfe::kBins + 4;   // lo + every bucket edge in [lo, hi]

// getComputedEncodings (quantization_utils.cpp:58-143)
AIMET_HD inline aimet_tf_encoding computed_encoding(int bw, double mn, double mx, bool sym, bool strict, bool unsign)
{
    double steps = ldexp(1.0, bw) - 1;   // pow(2, bw) - 1, exact
    if (sym && strict)
        steps -= 1;
    if (fabs(mn) == (double) INFINITY)
        mn = -FLT_MAX;
    if (fabs(mx) == (double) INFINITY)
        mx = FLT_MAX;
    aimet_tf_encoding e {0, 0, 0, 0, bw};
    if (sym && (mn < 0.0 || !unsign))
    {
        double absmax         = tfe::smax(fabs(mx), fabs(mn));
        unsigned int posSteps = (unsigned int) floor(steps / 2);
        e.delta               = absmax / posSteps;
        e.offset              = -ceil(steps / 2);
        e.min                 = tfe::smax(e.offset * e.delta, (double) -FLT_MAX);
        e.max                 = tfe::smin(e.delta * posSteps, (double) FLT_MAX);
        return e;
    }
    e.delta = (mx - mn) / steps;
    if (!(mn < 0 && mx > 0))
    {
        // one end is zero: 0 is already on the grid
        e.offset = round(mn / e.delta);
        e.min    = mn;
        e.max    = mx;
        return e;
    }
    double zeroCode = round(-mn / e.delta);
    zeroCode        = tfe::smin(steps, tfe::smax(0.0, zeroCode));
    e.offset        = -zeroCode;
    double lo       = e.delta * e.offset;
    e.min           = (lo >= (double) -FLT_MAX && lo <= (double) FLT_MAX) ? lo : (double) -FLT_MAX;
    e.max           = mx - mn + e.min;
    if (e.max > (double) FLT_MAX)
        e.max = FLT_MAX;
    return e;
}

// Candidate grid of _minimizeMSE (:137-200): every bucket edge inside the observed range splits
// into the negative mins and positive maxs (+ 0 each); bin centres carry the PDF mass.
struct Setup
{
    float lo, hi;   // observed range; hi includes one more bucket
    int nmins, nmaxs, nc;
    long long total;   // nmins * nmaxs - 1 (the trailing {0, 0} pair is not a candidate)
};

// the mass of the bin that holds centre c (setup's second loop, one centre)
AIMET_HD inline float centre_mass(const tfe::Hist& h, float c)
{
    const float start = (float) h.xl(0);
    const float step  = (float) (h.xl(1) - h.xl(0));
    int idx           = (int) floor((c - start) / step);
    idx               = tfe::smin(tfe::smax(0, idx), tfe::kBins - 1);
    return (float) h.pdf[idx];
}

// setup without the centres' masses: the edges and the centres, whose float sums are sequential
// (the device fills the masses in parallel after it, mse_search.hip)
AIMET_HD inline Setup setup_centres(const tfe::Hist& h, int first, int last, float* mins, float* maxs, float* cv);

// mins/maxs: >= kMaxEdges + 1 floats; cv/cw (centre value / mass): >= kMaxEdges floats.
// first/last: first and last (i > 0) non-empty bins, -1 for none (as tfe::observed_range).
AIMET_HD inline Setup setup(const tfe::Hist& h, int first, int last, float* mins, float* maxs, float* cv, float* cw)
{
    const Setup s = setup_centres(h, first, last, mins, maxs, cv);
    for (int i = 0; i < s.nc; ++i)
        cw[i] = centre_mass(h, cv[i]);
    return s;
}

AIMET_HD inline Setup setup_centres(const tfe::Hist& h, int first, int last, float* mins, float* maxs, float* cv)
{
    Setup s {};
    const float width = (float) (h.xl(1) - h.xl(0));
    const float hMin  = (float) h.xl(0);
    const float hMax  = (float) h.xl(tfe::kBins - 1) + width;
    float olo, ohi;
    tfe::observed_range(h, first, last, olo, ohi);
    s.lo = olo;
    s.hi = ohi + width;
    // edges = {lo} + {e in [lo, hi]} (float accumulator, as the reference loop)
    int nm = 0, nx = 0, ne = 0;
    float prev_edge = 0;
    auto take_edge = [&](float e) {
        if (e < 0)
            mins[nm++] = e;
        else if (e > 0)
            maxs[nx++] = e;
        ++ne;
        prev_edge = e;
    };
    take_edge(s.lo);
    // The reference loop never ends when `e += width` stops advancing (|hMin| / width > 2^24);
    // capping the iterations only changes that case (kBins + 1 edges otherwise).
    int iters = 0;
    for (float e = hMin; e <= hMax && iters < 4 * tfe::kBins; e += width, ++iters)
        if (e >= s.lo && e <= s.hi && ne < kMaxEdges)
            take_edge(e);
    (void) prev_edge;
    mins[nm++] = 0;
    maxs[nx++] = 0;
    s.nmins = nm;
    s.nmaxs = nx;
    s.nc    = ne - 1 > 0 ? ne - 1 : 0;
    s.total = (long long) nm * nx - 1;
    for (int i = 0; i < s.nc; ++i)
        cv[i] = (i == 0) ? s.lo + width / 2 : cv[i - 1] + width;
    return s;
}

AIMET_HD inline void candidate(const Setup& s, const float* mins, const float* maxs, long long t, float& cLo,
                               float& cHi)
{
    cLo = mins[t / s.nmaxs];
    cHi = maxs[t % s.nmaxs];
}

// _computeMSECost (:202-264)
AIMET_HD inline float cost(int bw, const float* cv, const float* cw, int nc, float cLo, float cHi, bool sym,
                           bool strict, bool unsign)
{
    aimet_tf_encoding e = computed_encoding(bw, cLo, cHi, sym, strict, unsign);
    float err           = 0;
    for (int i = 0; i < nc; ++i)
    {
        float v       = cv[i];
        float clamped = tfe::smax(cLo, tfe::smin(v, cHi));
        int q         = (int) round(clamped / e.delta - e.offset);
        float deq     = e.delta * (q + e.offset);
        double d      = (double) (v - deq);
        err += cw[i] * (d * d);
    }
    return err;
}

// the encoding of the chosen range (histogram_encoding's tail, MseEncodingAnalyzer.cpp:100-113)
AIMET_HD inline aimet_tf_encoding finish(int bw, float rlo, float rhi, bool sym, bool strict, bool unsign)
{
    float lo = tfe::smin(rlo, 0.0f);
    float hi = tfe::smax(rhi, 0.0f);
    return computed_encoding(bw, lo, hi, sym, strict, unsign);
}

}   // namespace mse
}   // namespace aimet_amd
