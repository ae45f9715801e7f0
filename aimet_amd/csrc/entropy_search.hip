// entropy_search.hip -- the entropy analyzer's KL range search on the device, every channel of
// every quantizer in one launch.
//
// Reference: EntropyEncodingAnalyzer::computeEncoding -> _optimizeKL (EntropyEncodingAnalyzer.cpp:
// 226-435) runs on the host, one channel at a time: 129 windows x ~5 passes over up to 512 bins,
// with a log per bin (~3 ms per channel). Here: one workgroup per channel:
//  1. the histogram the windows run over (the symmetric rescale) and its prefix tables: in
//     parallel over the bins when every bin count is an integer below 2^43 (bin counts always
//     are: sums of integers are then exact in any order), else by lane 0 as the reference loops;
//     the windows (entropy_kl.hpp: the window sequence never depends on a KL value): listed in
//     parallel when both ends shrink together (symmetric / strict), else by lane 0;
//  2. one window per lane: the reference's float normalisers of P and Q, streamed level by level
//     in bin order with its float / double operations (exact); with integral bins the level sums,
//     the zero counts and the saturated ends come from the prefix tables, and the same pass
//     accumulates an f32 estimate of the window's divergence with a rigorous error bound
//     (window_norms_integral: the filter);
//  3. the windows the estimates cannot rule out (candidates: possibly the minimum or within the
//     near-tie tolerance of it; usually a handful of the 129) get the divergence
//     sum_i p_i log(p_i / q_i) in double, split into kSegs segments of their 255 levels over all
//     lanes, the segments' sums added per window; a window's empty bins all have the same term,
//     evaluated once and counted; without the filter (non-integral bins) every window is one;
//  4. the first strict minimum among the candidates and the near-tie test by wave reductions
//     (a window ruled out by the filter exceeds the minimum by more than the tolerance);
//  5. for a batched request, the channel's finished encoding (entropy_out: the host's
//     entropy_encoding_from_range on the chosen range), so the host only re-runs flagged channels.
// The asymmetric (not strict) window lists are walked before the search by entropy_walk_kernel,
// one lane per channel (the walk is 129 dependent steps; inside the search one lane had taken
// them while its workgroup waited).
//
// Bit parity: every operation of 1, 2 and the window choice equals the host's. The divergence
// differs from the host's (log_kl, relative error < 2^-49, for glibc's log; p and q as multiplies
// by reciprocals -- the levels' by v_rcp_f64 and two Newton steps -- instead of divisions; the
// empty bins' equal terms counted; the segments' sums re-associated): per term by at most 2^-48
// |t| plus 2^-51 p, and the sums' order by 2^-44 sum|t|, so the two sums differ by
// < 2^-42 sum|t| + 1e-15. A window is accepted as
// the winner only when every other window's divergence exceeds it by more than
// 1e-11 * (sum |t| of both) + 1e-14; otherwise (and for non-finite ranges) the channel is flagged
// and the host re-runs the glibc search for it (quantizer.cpp). The accepted winner is then the
// host's winner too.
#include "entropy_kl.hpp"
#include "mse_core.hpp"
#include "tq_state.hpp"

namespace aimet_amd
{
namespace
{

constexpr int kEntBlock = 192;   // >= kWindows (129): one window per lane in step 2
static_assert(kEntBlock >= entropy::kWindows, "one window per lane");
constexpr int kSegs   = 4;                              // step 3: segments of 64 levels per window
constexpr int kSegLev = (entropy::kLevels + kSegs - 1) / kSegs;

struct EntJob
{
    const double* acc;          // [C][2] TensorProfilingParams {min, max}
    const int32_t* pdf_init;    // [C] histogram allocated
    const double* hist;         // [C][512] bin counts
    EntropyRange* out;          // [C]
    int64_t start;              // first global channel of this job
    EntropyOut* flat;           // optional: every job's finished encodings concatenated (+ start)
};

// a window's step-2 results, read by step 3
struct WinState
{
    double left, right;       // the saturated end bins of P
    double rdP, rdQ;          // 1 / the normalisers of the conditioned P and Q
    double rqz;               // 1 / (the conditioned Q of an empty bin / dQ)
    entropy::Cond cP, cQ;
    int brk;                  // the reference loop stops at this window (P or Q sums to 0)
};

// ln x for a positive finite double (the divergence terms' logarithm): x = 2^k m, m in [sqrt(1/2),
// sqrt(2)), ln m = 2 atanh(s) = 2 s (1 + s^2/3 + ... + s^16/17), s = (m - 1) / (m + 1) (|s| <=
// 0.1716; m - 1 exact; the quotient from v_rcp_f64 and two Newton steps). Relative error of ln m
// below 2^-49 (series truncation 2^-50, roundings a few ulp; ln m is small only where s is, so
// the error stays relative near x = 1), k ln2 in two parts: ~30 instructions where the device
// library's correctly rounded log takes ~95 (double-double arithmetic) -- the divergence only
// needs the accuracy its near-tie tolerance assumes (file header)
__device__ __forceinline__ double log_kl(double x)
{
    int k    = __builtin_amdgcn_frexp_exp(x);
    double m = __builtin_amdgcn_frexp_mant(x);   // [0.5, 1)
    if (m < 0.70710678118654752440)
    {
        m += m;
        --k;
    }
    const double f = m - 1.0;
    const double d = m + 1.0;
    double r       = __builtin_amdgcn_rcp(d);
    r              = __builtin_fma(__builtin_fma(-d, r, 1.0), r, r);
    r              = __builtin_fma(__builtin_fma(-d, r, 1.0), r, r);
    const double s = f * r, z = s * s;
    double p = 1.0 / 17.0;
    p        = __builtin_fma(p, z, 1.0 / 15.0);
    p        = __builtin_fma(p, z, 1.0 / 13.0);
    p        = __builtin_fma(p, z, 1.0 / 11.0);
    p        = __builtin_fma(p, z, 1.0 / 9.0);
    p        = __builtin_fma(p, z, 1.0 / 7.0);
    p        = __builtin_fma(p, z, 1.0 / 5.0);
    p        = __builtin_fma(p, z, 1.0 / 3.0);
    const double lm = 2.0 * __builtin_fma(s * z, p, s);
    const double kd = (double) k;
    return __builtin_fma(kd, 6.93147180369123816490e-01, __builtin_fma(kd, 1.90821492927058770002e-10, lm));
}

// a level's Q where its bins are non-empty: the reference's sum / norm, exactly (norm 1 and 2 --
// nearly every level of a window of 256-512 bins over 255 levels -- without the division)
__device__ __forceinline__ double level_q(double sum, double norm)
{
    return norm == 1.0 ? sum : (norm == 2.0 ? sum * 0.5 : sum / norm);
}

// [i0, i1) of level q of a window of `win` bins (stream_pq's bounds: ceil of the double products)
__device__ __forceinline__ int level_end(int q, double merged, int win)
{
    return q < entropy::kLevels - 1 ? (int) __builtin_ceil((double) (q + 1) * merged) : win;
}

// step 2 for window [a, b] of an integral histogram (every bin an integer below 2^43, so every
// sum of bins is exact in any order): the float normalisers of the conditioned P and Q in the
// reference's bin order (exact: the same float / double operations), with the level sums, the
// zero counts and the right-hand saturation from the prefix tables, and whether the reference
// loop stops here (the float sums of P or Q are 0 exactly when every bin of P or Q is 0)
// The filter (round 6): while the exact normalisers are streamed, the same pass accumulates an
// estimate of the window's divergence in f32 arithmetic, KL = (S1 + ln(dQ / dP) S0) / dP with
// S1 = sum cP ln(cP / cQ) and S0 = sum cP over the terms the reference adds (cP, cQ the
// conditioned P and Q; p = cP / dP, q = cQ / dQ), and a bound on its error: per term the f32
// ratio (reciprocal of the level's cQ, one product) is within 2^-22 relative, v_log_f32 * ln2
// within kLogAbs + kLogRel |ln| (tools/studies/log_f32_check.hip, profiles/r06/log_f32_check.txt),
// the f32 product within 2^-23; summed in double. Only windows whose estimate could be the
// minimum or a near-tie of it are then evaluated exactly (step 3).
constexpr double kLogAbs = 0x1p-20, kLogRel = 0x1p-20;   // >= 4x the measured bounds plus the ratio's
struct WinEstimate
{
    double kl, err, mag;   // estimate, bound on |estimate - divergence|, bound on sum |p ln(p / q)|
};

__device__ void window_norms_integral(const double* hist, int a, int b, const entropy::Prefix& pre, WinState& st,
                                      WinEstimate& est)
{
    using namespace entropy;
    const int win       = b - a + 1;
    const double total  = pre.left[kBins - 1];
    const double left   = pre.left[a];
    const double right  = total - (b > 0 ? pre.left[b - 1] : 0.0);
    const uint64_t zP   = (uint64_t) (pre.zeros[b] - pre.zeros[a + 1]) + (left == 0.0) + (right == 0.0);
    const uint64_t zQ   = (uint64_t) (pre.zeros[b + 1] - pre.zeros[a]);
    const Cond cP = cond_of(zP, (uint64_t) win), cQ = cond_of(zQ, (uint64_t) win);
    const double merged = (double) win / (double) kLevels;
    // cond_apply in select form (the same value: h + 0.0001 * 1 - eps * 0 = 0.0001 for an empty
    // bin, h + 0.0001 * 0 - eps * 1 = h - eps otherwise)
    auto cfast = [](const Cond& c, double h) { return c.skip ? h : (h == 0 ? 0.0001 : h - c.eps); };
    const double cQz = cfast(cQ, 0.0);
    const float rqz32 = __builtin_amdgcn_rcpf((float) cQz);
    float sP = 0.f, sQ = 0.f;
    double S1 = 0.0, M1 = 0.0, S0 = 0.0;   // the filter's sums
    // level by level (255 iterations for every lane), each level's 1-3 bins in order; the level's
    // sum and non-empty count from the prefix tables at its two bounds, the lower one carried over
    double Lprev = a > 0 ? pre.left[a - 1] : 0.0;   // hist[0, a + i0)
    int Zprev    = pre.zeros[a];
    int i0       = 0;
    for (int q = 0; q < kLevels; ++q)
    {
        const int i1      = level_end(q, merged, win);
        const double Lcur = pre.left[a + i1 - 1];
        const int Zcur    = pre.zeros[a + i1];
        const int norm    = (i1 - i0) - (Zcur - Zprev);
        const double sum  = Lcur - Lprev;
        double qv         = norm == 2 ? sum * 0.5 : sum;
        if (norm > 2)   // three bins per level: only the widest windows, rarely
            qv = sum / (double) norm;
        const double cQn = norm != 0 ? cfast(cQ, qv) : cQz;   // the level's non-empty bins
        const float rqn32 = __builtin_amdgcn_rcpf((float) cQn);
        for (int i = i0; i < i1; ++i)
        {
            const double h  = hist[a + i];
            const double Pi = i == 0 ? 0.0 + left : (i == win - 1 ? 0.0 + right : h);
            const double cp = cfast(cP, Pi), cq = h != 0 ? cQn : cQz;
            sP              = (float) ((double) sP + cp);
            sQ              = (float) ((double) sQ + cq);
            // the filter's term (p > 0 and q > 0 exactly when cP > 0 and cQ > 0)
            const bool inc  = cp > 0 && cq > 0;
            const float c32 = (float) cp;
            const float l   = __builtin_amdgcn_logf(c32 * (h != 0 ? rqn32 : rqz32)) * 0.693147182f;
            const float tt  = inc ? c32 * l : 0.0f;
            S1 += (double) tt;
            M1 += (double) __builtin_fabsf(tt);
            S0 += inc ? cp : 0.0;
        }
        i0    = i1;
        Lprev = Lcur;
        Zprev = Zcur;
    }
    st.left  = left;
    st.right = right;
    st.cP    = cP;
    st.cQ    = cQ;
    st.brk   = (zP == (uint64_t) win || zQ == (uint64_t) win) ? 1 : 0;
    const double dP = sP, dQ = sQ;
    st.rdP = 1.0 / dP;
    st.rdQ = 1.0 / dQ;
    st.rqz = 1.0 / (cond_apply(cQ, 0.0) * st.rdQ);
    // KL = sum p ln(p / q) = (S1 + ln(dQ / dP) S0) / dP; |sum p ln(p / q)| terms <= (M1 + |L| S0) / dP
    const double L   = log_kl(dQ * st.rdP);
    const double mag = (M1 + __builtin_fabs(L) * S0) * st.rdP;
    est.kl  = (S1 + L * S0) * st.rdP;
    est.err = ((kLogAbs * S0 + kLogRel * M1) * st.rdP + 0x1p-40 * mag) * 1.0009765625 + 1e-300;
    est.mag = mag * (1.0 + 0x1p-20) + est.err;
}

// step 2 for window [a, b] without the integral tables' shortcuts (lane per window, two streamed
// passes, as entropy::window_kl)
__device__ void window_norms(const double* hist, int a, int b, const entropy::Prefix* pre, WinState& st)
{
    using namespace entropy;
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
    }
    else
    {
        uint64_t zP = 0, zQ = 0;
        stream_pq(hist, a, b, left, right, [&](int, double p, double q) {
            aP = (float) ((double) aP + p);
            aQ = (float) ((double) aQ + q);
            zP += (p == 0.f);
            zQ += (q == 0.f);
        });
        cP = cond_of(zP, (uint64_t) win);
        cQ = cond_of(zQ, (uint64_t) win);
        if (!(aP == 0 || aQ == 0))
            stream_pq(hist, a, b, left, right, [&](int, double p, double q) {
                sP = (float) ((double) sP + cond_apply(cP, p));
                sQ = (float) ((double) sQ + cond_apply(cQ, q));
            });
    }
    st.left  = left;
    st.right = right;
    st.cP    = cP;
    st.cQ    = cQ;
    st.brk   = (aP == 0 || aQ == 0) ? 1 : 0;
    const double dP = sP, dQ = sQ;
    st.rdP = 1.0 / dP;
    st.rdQ = 1.0 / dQ;
    st.rqz = 1.0 / (cond_apply(cQ, 0.0) * st.rdQ);
}

// step 3: the divergence terms of levels [q0, q1) of window [a, b] (entropy::stream_pq's levels),
// p = cond(P) / dP, q = cond(Q) / dQ, sum of p log(p / q) over p, q > 0, and of its magnitudes
__device__ void window_segment(const double* hist, int a, int b, int q0, int q1, const WinState& st,
                               const entropy::Prefix& pre, bool integral, double& dv, double& mag)
{
    using namespace entropy;
    const int win       = b - a + 1;
    const double* hw    = hist + a;
    const double merged = (double) win / (double) kLevels;
    const double qz     = cond_apply(st.cQ, 0.0) * st.rdQ;
    dv = 0;
    mag = 0;
    int zeros_inside = 0;
    int i1 = (int) (uint64_t) ceil((double) q0 * merged);
    // integral bins: the levels' sums and non-empty counts from the prefix tables (exact), the
    // lower bound's entries carried over from the previous level
    double Lprev = 0.0;
    int Zprev    = 0;
    if (integral)
    {
        Lprev = a + i1 > 0 ? pre.left[a + i1 - 1] : 0.0;
        Zprev = pre.zeros[a + i1];
    }
    for (int q = q0; q < q1; ++q)
    {
        const int i0 = i1;
        i1           = level_end(q, merged, win);
        double sum = 0, norm = 0;
        if (integral)
        {
            const double Lcur = pre.left[a + i1 - 1];
            const int Zcur    = pre.zeros[a + i1];
            sum               = Lcur - Lprev;
            norm              = (double) ((i1 - i0) - (Zcur - Zprev));
            Lprev             = Lcur;
            Zprev             = Zcur;
        }
        else
            for (int i = i0; i < i1; ++i)
            {
                sum += hw[i];
                norm += (hw[i] != 0);
            }
        // the level's Q where its bin is non-empty (the reference's sum / norm, per bin), and its
        // reciprocal (v_rcp_f64 + two Newton steps: within an ulp, inside the terms' error bound)
        double qnz = 0.0, rqnz = 0.0;
        if (norm != 0)
        {
            double qv = norm == 2 ? sum * 0.5 : sum;
            if (norm > 2)   // three bins per level: only the widest windows, rarely
                qv = sum / norm;
            qnz  = cond_apply(st.cQ, qv) * st.rdQ;
            rqnz = __builtin_amdgcn_rcp(qnz);
            rqnz = __builtin_fma(__builtin_fma(-qnz, rqnz, 1.0), rqnz, rqnz);
            rqnz = __builtin_fma(__builtin_fma(-qnz, rqnz, 1.0), rqnz, rqnz);
        }
        for (int i = i0; i < i1; ++i)
        {
            const double h = hw[i];
            if (h == 0 && i != 0 && i != win - 1)
            {
                ++zeros_inside;   // the window's constant empty-bin term, added once below
                continue;
            }
            const bool nz   = norm != 0 && h != 0;
            const double Pi = i == 0 ? 0.0 + st.left : (i == win - 1 ? 0.0 + st.right : h);
            const double pn = cond_apply(st.cP, Pi) * st.rdP;
            const double qn = nz ? qnz : qz;
            if (pn > 0 && qn > 0)
            {
                const double t = pn * log_kl(pn * (nz ? rqnz : st.rqz));
                dv += t;
                mag += fabs(t);
            }
        }
    }
    // every empty bin inside the window has P = cond(0) / dP and Q = cond(0) / dQ: one term,
    // counted (the sum re-associated: within the terms' error bound)
    const double pz = cond_apply(st.cP, 0.0) * st.rdP;
    if (zeros_inside && pz > 0 && qz > 0)
    {
        const double t = pz * log_kl(pz * st.rqz);
        dv += (double) zeros_inside * t;
        mag += (double) zeros_inside * fabs(t);
    }
}

// the job holding global channel g (the last one with start <= g)
__device__ __forceinline__ int find_job(const EntJob* __restrict__ jobs, int njobs, int64_t g)
{
    int lo_j = 0, hi_j = njobs - 1;
    while (lo_j < hi_j)
    {
        const int mid = (lo_j + hi_j + 1) >> 1;
        if (jobs[mid].start <= g)
            lo_j = mid;
        else
            hi_j = mid - 1;
    }
    return lo_j;
}

// The asymmetric (not strict) window list of every channel, one lane per channel: entropy::windows
// on the channel's histogram where it lies (an asymmetric search runs on the histogram as
// accumulated, unrescaled). The walk is 129 dependent steps; inside the search kernel one lane
// took them while its workgroup's other 191 lanes waited (~0.8 ms for ResNet-50's 27,560
// channels, profiles/r06/entropy_step_shares.txt); here 64 channels walk side by side per wave.
// walks[g][0][n] / walks[g][1][n]: window n's first / last bin (every walk has kWindows windows:
// each step narrows the window by two bins, from 512 to 256).
__global__ __launch_bounds__(64) void entropy_walk_kernel(const EntJob* __restrict__ jobs, int njobs, int64_t total,
                                                          short* __restrict__ walks)
{
    const int64_t g = (int64_t) blockIdx.x * 64 + threadIdx.x;
    if (g >= total)
        return;
    const EntJob& j = jobs[find_job(jobs, njobs, g)];
    const int64_t c    = g - j.start;
    const double tmin = j.acc[2 * c], tmax = j.acc[2 * c + 1];
    if (!j.pdf_init[c] || !__builtin_isfinite(tmin) || !__builtin_isfinite(tmax))
        return;   // the search decides these channels without a window list
    short* w = walks + g * 2 * entropy::kWindows;
    entropy::windows(j.hist + c * entropy::kBins, tmin, (tmax - tmin) / (double) entropy::kBins, false, w,
                     w + entropy::kWindows);
}

// A channel's finished encoding: entropy_encoding_from_range of the KL range (kEntFinal) or
// unseen_or_zero's all-zero encoding (kEntNoHist; encodings.cpp), the same double operations
// (mse::computed_encoding is the host's own getComputedEncodings); kEntHost: left to the host
__device__ __noinline__ EntropyOut entropy_out(float kl_lo, float kl_hi, int status, int bw, bool sym, bool strict, bool unsign)
{
    EntropyOut o {0, 0, 0, 0, 0, status};
    if (status == kEntFinal)
    {
        const float lo          = 0.0f < kl_lo ? 0.0f : kl_lo;   // std::min(kl_lo, 0.0f)
        const float hi          = kl_hi < 0.0f ? 0.0f : kl_hi;   // std::max(kl_hi, 0.0f)
        const aimet_tf_encoding e = mse::computed_encoding(bw, (double) lo, (double) hi, sym, strict, unsign);
        o = EntropyOut {e.min, e.max, e.delta, e.offset, e.bw, status};
    }
    else if (status == kEntNoHist)
    {
        float steps = (float) (ldexp(1.0, bw) - 1);   // (float) (std::pow(2.0, bw) - 1)
        if (sym && strict)
            steps -= 1;
        const int isteps   = (int) steps;
        const double delta = (1.0 - (-1.0)) / isteps;
        const double off   = floor(-1.0 / delta);
        const double lo    = off * delta;
        o = EntropyOut {lo, lo + isteps * delta, delta, off, bw, status};
    }
    return o;
}

// 5 waves per SIMD (<= 96 VGPRs, a few spills): with the kernel's 23.6 KB of LDS (step 1's scratch
// in `left` / `ws`, step 3's segments added by shuffles), 6 workgroups of 3 waves per CU, where
// 29.8 KB had allowed 5. At 137 VGPRs (entropy_out inlined) 4 had fit, and the kernel took 6.0 ms
// instead of 5.15 on ResNet-50's weights (profiles/r06/entropy_waves_ab.txt): entropy_out stays a
// call (one lane per channel)
__global__ __launch_bounds__(kEntBlock) __attribute__((amdgpu_waves_per_eu(5))) void entropy_search_kernel(const EntJob* __restrict__ jobs, int njobs,
                                                                   int64_t total, int sym, int strict, int unsign,
                                                                   int bw, const short* __restrict__ walks)
{
    // step 1's source histogram and integer accumulators share their LDS with step 3's sums
    __shared__ double hist[entropy::kBins];
    __shared__ short wa[entropy::kWindows], wb[entropy::kWindows];
    __shared__ WinState ws[entropy::kWindows];
    __shared__ double left[entropy::kBins];
    // step 1's source histogram and integer accumulators in the LDS of `left` and `ws`, which
    // step 1 writes only after it is done with them (the prefix tables) or not at all (ws: step 2)
    double* tpp               = left;
    unsigned long long* acc_u = reinterpret_cast<unsigned long long*>(ws);
    static_assert(sizeof(WinState) * entropy::kWindows >= sizeof(unsigned long long) * entropy::kBins,
                  "step 1's accumulators fit the window states");
    __shared__ double s_vt[entropy::kWindows], s_mt[entropy::kWindows];   // step 3's sums per candidate
    __shared__ int zeros[entropy::kBins + 1];
    __shared__ double s_lo, s_hi;
    __shared__ int s_n, s_rule, s_integral;
    __shared__ int s_first_brk[kEntBlock / 64], s_best_k[kEntBlock / 64], s_tie, s_ncand[kEntBlock / 64];
    __shared__ double s_best_v[kEntBlock / 64], s_best_m, s_mag[kEntBlock / 64];
    __shared__ short s_cand[entropy::kWindows];
    const int t = threadIdx.x;
    const int lane = t & 63;
    for (int64_t g = blockIdx.x; g < total; g += gridDim.x)
    {
        const EntJob& j = jobs[find_job(jobs, njobs, g)];
        const int64_t c = g - j.start;
        const double tmin = j.acc[2 * c], tmax = j.acc[2 * c + 1];
        if (!j.pdf_init[c] || !__builtin_isfinite(tmin) || !__builtin_isfinite(tmax))
        {
            // no histogram (the host returns the unseen / all-zero encoding), or a non-finite
            // range: the host search decides
            if (t == 0)
            {
                const EntropyRange r {0.f, 0.f, j.pdf_init[c] ? kEntHost : kEntNoHist, 0};
                j.out[c] = r;
                if (j.flat)
                    j.flat[j.start + c] = entropy_out(r.lo, r.hi, r.status, bw, sym, strict, unsign);
            }
            continue;
        }
        // ---- 1. the histogram, its prefix tables, the windows ----------------------------------
        if (t == 0)
            s_integral = 1;
        __syncthreads();
        for (int i = t; i < entropy::kBins; i += kEntBlock)
        {
            const double v = j.hist[c * entropy::kBins + i];
            tpp[i]         = v;
            acc_u[i]       = 0;
            // an integer in [0, 2^43): every sum of the 512 bins below is exact in any order
            if (!(v >= 0.0 && v < 8796093022208.0 && __builtin_floor(v) == v))
                s_integral = 0;
        }
        __syncthreads();
        const bool integral = s_integral != 0;
        // the symmetric rescale (kl_histogram) and whether it applies
        const bool rescale = sym && (tmin < 0.0 || !unsign);
        const float amax   = (float) entropy::kmax(fabs(tmax), fabs(tmin));
        const double dlo = rescale ? (double) -amax : tmin, dhi = rescale ? (double) amax : tmax;
        const bool same = !rescale || (tmin == dlo && tmax == dhi);
        if (integral)
        {
            if (same)
            {
                for (int i = t; i < entropy::kBins; i += kEntBlock)
                    hist[i] = tpp[i];
            }
            else
            {
                // rescale_histogram with every source bin's parts added as integers (any order)
                const uint64_t n  = entropy::kBins;
                const double srcW = (tmax - tmin) / (double) n;
                const double dstW = (dhi - dlo) / (double) n;
                for (int bb = t; bb < entropy::kBins; bb += kEntBlock)
                {
                    const double v = tpp[bb];
                    if (v == 0)
                        continue;
                    const double s0 = tmin + (double) bb * srcW;
                    const double s1 = tmin + (double) (bb + 1) * srcW;
                    uint64_t d0     = entropy::x86_d2u64(entropy::kmax(floor((s0 - dlo) / dstW), 0.0));
                    uint64_t d1     = entropy::x86_d2u64(entropy::kmax(ceil((s1 - dlo) / dstW), 0.0));
                    d0              = entropy::kmin(d0, n - 1);
                    d1              = entropy::kmin(d1, n - 1);
                    double rem      = v;
                    for (uint64_t k = d0; k <= d1; ++k)
                    {
                        const double o0 = entropy::kmax(s0, dlo + (double) k * dstW);
                        const double o1 = entropy::kmin(s1, dlo + (double) (k + 1) * dstW);
                        double ratio    = (o1 - o0) / srcW;
                        ratio           = ratio >= 0.0f ? ratio : 0.0f;
                        ratio           = ratio <= 1.0f ? ratio : 1.0f;
                        double part     = round(ratio * v);
                        part            = part <= rem ? part : rem;
                        atomicAdd(&acc_u[k], (unsigned long long) part);
                        rem -= part;
                    }
                }
                __syncthreads();
                for (int i = t; i < entropy::kBins; i += kEntBlock)
                    hist[i] = (double) acc_u[i];
            }
            __syncthreads();
            // prefix tables: wave 0, 8 bins per lane, then the lanes' running totals
            if (t < 64)
            {
                double l = 0;
                int z    = 0;
                for (int k = 0; k < 8; ++k)
                {
                    const double h = hist[8 * lane + k];
                    l += h;
                    z += h == 0;
                }
                double lx = l;
                int zx    = z;
                for (int o = 1; o < 64; o <<= 1)   // inclusive scan
                {
                    const double lo = __shfl_up(lx, o, 64);
                    const int zo    = __shfl_up(zx, o, 64);
                    if (lane >= o)
                    {
                        lx += lo;
                        zx += zo;
                    }
                }
                double run = lx - l;
                int zr     = zx - z;
                for (int k = 0; k < 8; ++k)
                {
                    const double h = hist[8 * lane + k];
                    run += h;
                    zr += h == 0;
                    left[8 * lane + k]      = run;
                    zeros[8 * lane + k + 1] = zr;
                }
                if (lane == 0)
                    zeros[0] = 0;
            }
            __syncthreads();
            if (sym || strict)   // both ends shrink by one bin per window: window n is [n, 511 - n]
            {
                for (int n = t; n < entropy::kWindows; n += kEntBlock)
                {
                    wa[n] = (short) n;
                    wb[n] = (short) (entropy::kBins - 1 - n);
                }
            }
            else if (walks)   // the walk of this histogram (no rescale here: hist is the source)
            {
                const short* w = walks + g * 2 * entropy::kWindows;
                for (int n = t; n < entropy::kWindows; n += kEntBlock)
                {
                    wa[n] = w[n];
                    wb[n] = w[entropy::kWindows + n];
                }
            }
            if (t == 0)
            {
                s_lo   = dlo;
                s_hi   = dhi;
                s_n    = (sym || strict || walks) ? entropy::kWindows
                                         : entropy::windows(hist, dlo, (dhi - dlo) / (double) entropy::kBins, false, wa, wb);
                s_rule = 1;   // integral bins: 0 or >= 1
            }
        }
        else if (t == 0)
        {
            double lo, hi;
            entropy::kl_histogram(tmin, tmax, tpp, sym != 0, unsign != 0, hist, lo, hi);
            s_lo = lo;
            s_hi = hi;
            s_n  = entropy::windows(hist, lo, (hi - lo) / (double) entropy::kBins, sym || strict, wa, wb);
            bool rule;
            entropy::build_prefix(hist, left, zeros, rule);
            s_rule = rule ? 1 : 0;
        }
        __syncthreads();
        // ---- 2. the normalisers of every window (exact) and the filter's estimate ---------------
        const entropy::Prefix pre {left, zeros, s_rule != 0};
        WinEstimate est {0.0, __builtin_inf(), __builtin_inf()};   // (no filter: every window exact)
        if (t < s_n)
        {
            if (integral)
                window_norms_integral(hist, wa[t], wb[t], pre, ws[t], est);
            else
                window_norms(hist, wa[t], wb[t], &pre, ws[t]);
        }
        const int wave = t >> 6;
        const bool brk = t >= s_n || ws[t].brk != 0;
        const uint64_t brk_mask = __ballot(brk);
        if (lane == 0)
            s_first_brk[wave] = brk_mask ? wave * 64 + __ffsll((long long) brk_mask) - 1 : kEntBlock;
        __syncthreads();
        // the reference loop stops at the first breaking window (nv)
        int nv = kEntBlock;
        for (int k = 0; k < kEntBlock / 64; ++k)
            nv = s_first_brk[k] < nv ? s_first_brk[k] : nv;
        nv = nv < s_n ? nv : s_n;
        // ---- 3a. the windows the estimate cannot rule out --------------------------------------
        // U = min (kl + err) >= the smallest divergence; a window with kl - err > U + T, T above
        // the near-tie tolerance 1e-11 (mag_k + mag_best) + 1e-14, is larger than the minimum by
        // more than that tolerance: it is neither the winner nor a near-tie, and is not evaluated
        double up = t < nv ? est.kl + est.err : __builtin_inf();
        double mg = t < nv ? est.mag : 0.0;
        for (int o = 32; o > 0; o >>= 1)
        {
            up = __builtin_fmin(up, __shfl_xor(up, o, 64));
            mg = __builtin_fmax(mg, __shfl_xor(mg, o, 64));
        }
        if (lane == 0)
        {
            s_best_v[wave] = up;
            s_mag[wave]    = mg;
        }
        __syncthreads();
        double U = __builtin_inf(), maxmag = 0.0;
        for (int k = 0; k < kEntBlock / 64; ++k)
        {
            U      = __builtin_fmin(U, s_best_v[k]);
            maxmag = __builtin_fmax(maxmag, s_mag[k]);
        }
        // (a NaN estimate, an infinite bound or no filter: a candidate)
        const double T  = 1e-11 * (est.mag + maxmag) * 1.0009765625 + 1e-14;
        const bool cand = t < nv && !(est.kl - est.err > U + T);
        const uint64_t cand_mask = __ballot(cand);
        if (lane == 0)
            s_ncand[wave] = __popcll(cand_mask);
        __syncthreads();
        int cbase = 0, ncand = 0;
        for (int k = 0; k < kEntBlock / 64; ++k)
        {
            cbase += k < wave ? s_ncand[k] : 0;
            ncand += s_ncand[k];
        }
        if (cand)
            s_cand[cbase + (int) __builtin_amdgcn_mbcnt_hi((uint32_t) (cand_mask >> 32),
                                                           __builtin_amdgcn_mbcnt_lo((uint32_t) cand_mask, 0u))] = (short) t;
        __syncthreads();
        // ---- 3b. the candidates' divergences, (window, segment) items over every lane ------------
        // a candidate's kSegs segments sit on 4 adjacent lanes of one wave (kEntBlock and 64 are
        // multiples of kSegs, and every lane of such a group runs the same iterations): the first
        // adds them, in segment order
        static_assert(kSegs == 4 && kEntBlock % kSegs == 0, "a candidate's segments on 4 adjacent lanes");
        for (int it = t; it < ncand * kSegs; it += kEntBlock)
        {
            const int w = s_cand[it / kSegs], sgm = it % kSegs;
            const int q0 = sgm * kSegLev, q1 = q0 + kSegLev < entropy::kLevels ? q0 + kSegLev : entropy::kLevels;
            double dv = 0, mag = 0;
            window_segment(hist, wa[w], wb[w], q0, q1, ws[w], pre, integral, dv, mag);
            const double d1 = __shfl(dv, lane + 1, 64), d2 = __shfl(dv, lane + 2, 64), d3 = __shfl(dv, lane + 3, 64);
            const double m1 = __shfl(mag, lane + 1, 64), m2 = __shfl(mag, lane + 2, 64),
                         m3 = __shfl(mag, lane + 3, 64);
            if (sgm == 0)
            {
                s_vt[w] = (((0.0 + dv) + d1) + d2) + d3;
                s_mt[w] = (((0.0 + mag) + m1) + m2) + m3;
            }
        }
        __syncthreads();
        // ---- 4. the first strict minimum among the candidates (wave reductions), near-tie test ---
        // the window is accepted only if every other one before nv exceeds it by more than the
        // tolerance (a near-tie or a NaN: the host's glibc search decides)
        double v = __builtin_inf(), m = 0.0;
        if (cand)
        {
            v = s_vt[t];
            m = s_mt[t];
        }
        // (value, index) argmin: the smallest value below +inf, the first index among equals
        double bv = (t < nv && v < __builtin_inf()) ? v : __builtin_inf();
        int bk    = bv < __builtin_inf() ? t : kEntBlock;
        for (int o = 32; o > 0; o >>= 1)
        {
            const double ov = __shfl_xor(bv, o, 64);
            const int ok    = __shfl_xor(bk, o, 64);
            if (ov < bv || (ov == bv && ok < bk))
            {
                bv = ov;
                bk = ok;
            }
        }
        if (lane == 0)
        {
            s_best_v[wave] = bv;
            s_best_k[wave] = bk;
        }
        if (t == 0)
            s_tie = 0;
        __syncthreads();
        int best      = kEntBlock;
        double best_v = __builtin_inf();
        for (int k = 0; k < kEntBlock / 64; ++k)
            if (s_best_v[k] < best_v || (s_best_v[k] == best_v && s_best_k[k] < best))
            {
                best_v = s_best_v[k];
                best   = s_best_k[k];
            }
        if (best < kEntBlock && t == best)
            s_best_m = m;
        __syncthreads();
        if (best < kEntBlock && t < nv && t != best)
        {
            const double tol = 1e-11 * (m + s_best_m) + 1e-14;
            if (!(v - best_v > tol))
                s_tie = 1;
        }
        __syncthreads();
        if (t == 0)
        {
            const int status = s_tie ? kEntHost : kEntFinal;
            const double w   = (s_hi - s_lo) / (double) entropy::kBins;
            float lo         = (float) s_lo, hi = (float) s_hi;
            if (best < kEntBlock)
            {
                lo = (float) (s_lo + (double) wa[best] * w);
                hi = (float) (s_lo + (double) (wb[best] + 1) * w);
            }
            j.out[c] = EntropyRange {lo, hi, status, 0};
            if (j.flat)
                j.flat[j.start + c] = entropy_out(lo, hi, status, bw, sym, strict, unsign);
        }
        __syncthreads();
    }
}

}   // namespace

void launch_entropy_search_many(const TqDevice* const* ds, const int64_t* Cs, int n, bool sym, bool strict, bool unsign,
                                hipStream_t s, EntropyOut* pinned_dst, int bw)
{
    if (n == 0)
        return;
    std::vector<EntJob> jobs((size_t) n);
    int64_t total = 0;
    for (int i = 0; i < n; ++i)
        total += Cs[i];
    // every quantizer's encodings side by side, for one copy into the caller's pinned block
    auto* flat = pinned_dst ? static_cast<EntropyOut*>(scratch_alloc(sizeof(EntropyOut) * total, s)) : nullptr;
    total = 0;
    for (int i = 0; i < n; ++i)
    {
        jobs[(size_t) i] = EntJob {ds[i]->acc, ds[i]->pdf_init, ds[i]->pdf, entropy_ranges(*ds[i]), total, flat};
        total += Cs[i];
    }
    auto* dj       = static_cast<EntJob*>(upload_async(jobs.data(), sizeof(EntJob) * (size_t) n, s));
    const int grid = (int) (total < 65536 ? total : 65536);
    // asymmetric, not strict: every channel's window list first, 64 channels per wave
    short* walks = nullptr;
    if (!sym && !strict)
    {
        walks = static_cast<short*>(scratch_alloc(sizeof(short) * 2 * entropy::kWindows * (size_t) total, s));
        entropy_walk_kernel<<<(int) ((total + 63) / 64), 64, 0, s>>>(dj, n, total, walks);
        AIMET_LAUNCH_CHECK();
    }
    entropy_search_kernel<<<grid, kEntBlock, 0, s>>>(dj, n, total, sym ? 1 : 0, strict ? 1 : 0, unsign ? 1 : 0,
                                                               bw, walks);
    AIMET_LAUNCH_CHECK();
    if (walks)
        scratch_free(walks, s);
    scratch_free(dj, s);
    if (flat)
    {
        AIMET_HIP_CHECK(hipMemcpyAsync(pinned_dst, flat, sizeof(EntropyOut) * total, hipMemcpyDeviceToHost, s));
        scratch_free(flat, s);
    }
}

}   // namespace aimet_amd
