// entropy_search.hip -- the entropy analyzer's KL range search on the device, every channel of
// every quantizer in one launch.
//
// Reference: EntropyEncodingAnalyzer::computeEncoding -> _optimizeKL (EntropyEncodingAnalyzer.cpp:
// 226-435) runs on the host, one channel at a time: 129 windows x ~5 passes over up to 512 bins,
// with a log per bin (~3 ms per channel). Here: one workgroup per channel; lane 0 prepares the
// histogram (symmetric rescale) and enumerates the windows (entropy_kl.hpp: the window sequence
// never depends on a KL value), then one window per lane computes its KL divergence with the
// reference's float/double arithmetic streamed in bin order, and lane 0 picks the first strict
// minimum.
//
// Bit parity: every operation equals the host's except the natural logarithm (device library vs
// glibc, each within a couple of ulp of the true value). With t_i = p_i log(p_i/q_i), the two
// sums differ by at most ~2^-43 * sum |t_i| for <= 512 terms; a window is accepted as the winner
// only when every other window's divergence exceeds it by more than 1e-11 * (sum |t| of both),
// otherwise (and for non-finite ranges) the channel is flagged and the host re-runs the glibc
// search for it (quantizer.cpp). The accepted winner is then the host's winner too.
#include "entropy_kl.hpp"
#include "tq_state.hpp"

namespace aimet_amd
{
namespace
{

constexpr int kEntBlock = 192;   // >= kWindows (129): one window per lane
static_assert(kEntBlock >= entropy::kWindows, "one window per lane");

struct EntJob
{
    const double* acc;          // [C][2] TensorProfilingParams {min, max}
    const int32_t* pdf_init;    // [C] histogram allocated
    const double* hist;         // [C][512] bin counts
    EntropyRange* out;          // [C]
    int64_t start;              // first global channel of this job
};

__global__ __launch_bounds__(kEntBlock) void entropy_search_kernel(const EntJob* __restrict__ jobs, int njobs,
                                                                   int64_t total, int sym, int strict, int unsign)
{
    __shared__ double tpp[entropy::kBins];
    __shared__ double hist[entropy::kBins];
    __shared__ short wa[entropy::kWindows], wb[entropy::kWindows];
    __shared__ double dv[entropy::kWindows], mag[entropy::kWindows];
    __shared__ int brk[entropy::kWindows];
    __shared__ double left[entropy::kBins];
    __shared__ int zeros[entropy::kBins + 1];
    __shared__ double s_lo, s_hi;
    __shared__ int s_n, s_rule;
    const int t = threadIdx.x;
    for (int64_t g = blockIdx.x; g < total; g += gridDim.x)
    {
        int lo_j = 0, hi_j = njobs - 1;   // last job with start <= g
        while (lo_j < hi_j)
        {
            int mid = (lo_j + hi_j + 1) >> 1;
            if (jobs[mid].start <= g)
                lo_j = mid;
            else
                hi_j = mid - 1;
        }
        const EntJob& j = jobs[lo_j];
        const int64_t c = g - j.start;
        const double tmin = j.acc[2 * c], tmax = j.acc[2 * c + 1];
        if (!j.pdf_init[c] || !__builtin_isfinite(tmin) || !__builtin_isfinite(tmax))
        {
            // no histogram (the host returns the unseen / all-zero encoding), or a non-finite
            // range: the host search decides
            if (t == 0)
                j.out[c] = EntropyRange {0.f, 0.f, j.pdf_init[c] ? kEntHost : kEntNoHist, 0};
            continue;
        }
        for (int i = t; i < entropy::kBins; i += kEntBlock)
            tpp[i] = j.hist[c * entropy::kBins + i];
        __syncthreads();
        if (t == 0)
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
        if (t < s_n)
        {
            const entropy::Prefix pre {left, zeros, s_rule != 0};
            const entropy::WindowKl r =
                entropy::window_kl(hist, wa[t], wb[t], [](double v) { return log(v); }, &pre);
            dv[t]  = r.dv;
            mag[t] = r.mag;
            brk[t] = r.brk ? 1 : 0;
        }
        __syncthreads();
        if (t == 0)
        {
            // the reference loop: stop at the first breaking window, keep the first strict minimum
            int nv = 0;
            while (nv < s_n && !brk[nv])
                ++nv;
            int best = -1;
            for (int k = 0; k < nv; ++k)
                if (best < 0 ? dv[k] < __builtin_inf() : dv[k] < dv[best])
                    best = k;
            int status = kEntFinal;
            for (int k = 0; k < nv && best >= 0; ++k)
            {
                if (k == best)
                    continue;
                const double tol = 1e-11 * (mag[k] + mag[best]) + 1e-300;
                if (!(dv[k] - dv[best] > tol))   // a near-tie (or NaN): glibc decides
                {
                    status = kEntHost;
                    break;
                }
            }
            const double w = (s_hi - s_lo) / (double) entropy::kBins;
            float lo       = (float) s_lo, hi = (float) s_hi;
            if (best >= 0)
            {
                lo = (float) (s_lo + (double) wa[best] * w);
                hi = (float) (s_lo + (double) (wb[best] + 1) * w);
            }
            j.out[c] = EntropyRange {lo, hi, status, 0};
        }
        __syncthreads();
    }
}

}   // namespace

void launch_entropy_search_many(const TqDevice* const* ds, const int64_t* Cs, int n, bool sym, bool strict, bool unsign,
                                hipStream_t s)
{
    if (n == 0)
        return;
    std::vector<EntJob> jobs((size_t) n);
    int64_t total = 0;
    for (int i = 0; i < n; ++i)
    {
        jobs[(size_t) i] = EntJob {ds[i]->acc, ds[i]->pdf_init, ds[i]->pdf, entropy_ranges(*ds[i]), total};
        total += Cs[i];
    }
    auto* dj       = static_cast<EntJob*>(upload_async(jobs.data(), sizeof(EntJob) * (size_t) n, s));
    const int grid = (int) (total < 65536 ? total : 65536);
    entropy_search_kernel<<<grid, kEntBlock, 0, s>>>(dj, n, total, sym ? 1 : 0, strict ? 1 : 0, unsign ? 1 : 0);
    AIMET_LAUNCH_CHECK();
    scratch_free(dj, s);
}

}   // namespace aimet_amd
