// mse_search.hip -- MSE encoding search on the device.
//
// Reference: MseEncodingAnalyzer::computeEncoding (MseEncodingAnalyzer.cpp:79-264) evaluates
// every (min edge, max edge) pair of the observed range -- up to ~257^2 candidates x 512 bin
// centres -- on the host, one channel at a time (10.5 ms per tensor). Here: a 2-D grid
// (channel, candidate slice); each workgroup rebuilds the channel's candidate grid in LDS (one
// lane, ~1k serial float ops exactly as the reference loops), evaluates its slice with one
// candidate per lane, and keeps the first minimum; a second launch folds the slices in candidate
// order. Arithmetic: mse_core.hpp, shared with the host path (bit-exact).
#include "mse_core.hpp"
#include "tq_state.hpp"

namespace aimet_amd
{
namespace
{

struct MsePart
{
    float err;
    int idx;   // candidate index, -1: none selected in this slice
    float lo, hi;
    float obs_lo, obs_hi;   // the search range: result when no candidate is ever selected
};

// round(c / delta - offset) of the reference (mse::cost) for a clamped value c, exactly
__device__ __forceinline__ int code_exact(float c, const aimet_tf_encoding& e)
{
    return (int) round(c / e.delta - e.offset);
}

// mse::cost (_computeMSECost, MseEncodingAnalyzer.cpp:202-264) over the bins (zv[i], zw[i]),
// i < n, in the same order and float / double arithmetic, for a channel whose observed range is
// finite (every bin centre, candidate end and term finite; compact_bins), with two exact shortcuts:
//  * the double division c / delta is a multiply by RN(1 / delta): y' = fma(c, RN(1/delta), -offset)
//    lies within 2^-50 (|c / delta| + |offset| + 1) of the reference's RN(RN(c / delta) - offset),
//    so round() picks the same integer wherever y' is farther than `thr` >= that from a
//    half-integer (no tie: rint == round); otherwise, and for any non-finite y', the division
//    decides. |c / delta| <= steps + 1 and |offset| <= steps for every MSE candidate (0 lies in
//    [cLo, cHi]), so thr = 2^(bw + 2 - 48) bounds it;
//  * monotone early exit: every term cw * d^2 is >= 0, so the float sum never decreases; once it
//    exceeds `prune` (an error some candidate of this slice reached) the candidate cannot be the
//    first minimum, and it is dropped (`pruned`).
// The bin values come as double (zvd, zwd: exact copies of the float centres and masses) and as
// float (zv, for the float subtraction v - deq).
__device__ __forceinline__ float cost_fast(int bw, const float* zv, const double* zvd, const double* zwd, int n,
                                           float cLo, float cHi, bool sym, bool strict, bool unsign, float prune,
                                           bool& pruned)
{
    const aimet_tf_encoding e = mse::computed_encoding(bw, cLo, cHi, sym, strict, unsign);
    const double rcp          = 1.0 / e.delta;
    const double lo = cLo, hi = cHi, off = e.offset;
    const double thr = __builtin_ldexp(1.0, bw - 46);
    float err        = 0;
    pruned           = false;
    for (int i = 0; i < n; ++i)
    {
        // std::max(cLo, std::min(v, cHi)) for finite values (the sign of a zero does not matter:
        // it only meets 0 / delta)
        const double c = __builtin_fmax(lo, __builtin_fmin(zvd[i], hi));
        const double y = __builtin_fma(c, rcp, -off);
        double k;
        if (__builtin_fabs((y - __builtin_floor(y)) - 0.5) > thr)   // false for NaN
            k = __builtin_rint(y) + off;
        else
            k = (double) code_exact((float) c, e) + off;
        const float deq = (float) (e.delta * k);
        const double d  = (double) (zv[i] - deq);
        err += zwd[i] * (d * d);
        if ((i & 7) == 7 && err > prune)
        {
            pruned = true;
            break;
        }
    }
    return err;
}

// The bins of non-zero mass (cv, cw) -> (zv, zw) in order (and as double in zvd, zwd), by wave 0;
// returns how many; `finite`: the observed range is finite (cost_fast applies). Skipping a
// zero-mass bin is exact when its term cw * d^2 is +0, i.e. d finite: |d| <= |v| + |deq| with v a
// bin centre and deq inside the candidate range, both within the observed range, so every term
// is finite when the range stays below 2^100 in magnitude. Otherwise (and with a NaN mass, which
// is kept) the full list is used.
__device__ int compact_bins(const mse::Setup& st, const float* cv, const float* cw, float* zv, float* zw, double* zvd,
                             double* zwd, bool& finite)
{
    __shared__ int count;
    const bool finite_range = __builtin_fabsf(st.lo) < 1.2676506e30f && __builtin_fabsf(st.hi) < 1.2676506e30f;
    if (threadIdx.x < 64)
    {
        const int lane = threadIdx.x;
        int base       = 0;
        for (int i0 = 0; i0 < st.nc; i0 += 64)
        {
            const int i     = i0 + lane;
            const bool keep = i < st.nc && (!finite_range || !(cw[i] == 0.0f));
            const unsigned long long m = __ballot(keep);
            if (keep)
            {
                const int pos = base + __popcll(m & ((1ull << lane) - 1ull));
                zv[pos]       = cv[i];
                zw[pos]       = cw[i];
                zvd[pos]      = (double) cv[i];
                zwd[pos]      = (double) cw[i];
            }
            base += __popcll(m);
        }
        if (lane == 0)
            count = base;
    }
    __syncthreads();
    finite = finite_range;
    return count;
}

// exclusive prefix sum over the workgroup's kBlock threads (and the total), in thread order
__device__ __forceinline__ int block_exscan(int v, int& total)
{
    __shared__ int wsum[kBlock / 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int x = v;
    for (int o = 1; o < 64; o <<= 1)
    {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o)
            x += y;
    }
    if (lane == 63)
        wsum[wave] = x;
    __syncthreads();
    int before = 0;
    total      = 0;
    for (int w = 0; w < kBlock / 64; ++w)
    {
        before += w < wave ? wsum[w] : 0;
        total += wsum[w];
    }
    __syncthreads();   // wsum is reused by the next call
    return before + x - v;
}

// mse::setup_centres on the device, the same values: the edge walk e += width and the centres'
// chain cv[i] = cv[i - 1] + width are sequential float sums, each a tight loop on one lane (two
// lanes of different waves, side by side); which edges are taken (in [lo, hi], the first
// kMaxEdges - 1 of them) and where they go (mins / maxs, in order) is decided over the workgroup
// by prefix sums. E: >= 4 kBins floats of scratch. Every thread calls it; the result in `st`.
__device__ void setup_centres_device(const tfe::Hist& h, int first, int last, float* mins, float* maxs, float* cv,
                                     float* E, mse::Setup& st)
{
    __shared__ int s_nE;
    constexpr int kIters = 4 * tfe::kBins;
    constexpr int kPer   = kIters / kBlock;   // consecutive edges per thread in the classification
    static_assert(kIters % kBlock == 0, "edges split evenly");
    const float width = (float) (h.xl(1) - h.xl(0));
    float olo, ohi;
    tfe::observed_range(h, first, last, olo, ohi);
    const float lo = olo, hi = ohi + width;
    if (threadIdx.x == 0)
    {
        const float hMin = (float) h.xl(0);
        const float hMax = (float) h.xl(tfe::kBins - 1) + width;
        int k   = 0;
        float e = hMin;
        for (; e <= hMax && k < kIters; e += width, ++k)
            E[k] = e;
        s_nE = k;
    }
    else if (threadIdx.x == 64)
    {
        // the centres for the longest possible list (kMaxEdges - 1); the caller uses st.nc of them
        float c = lo + width / 2;
        for (int i = 0; i < mse::kMaxEdges - 1; ++i)
        {
            cv[i] = c;
            c     = c + width;
        }
    }
    __syncthreads();
    const int nE = s_nE;
    // lo itself is taken first (ne = 1); then an edge in [lo, hi] while ne < kMaxEdges
    const int nm0 = lo < 0 ? 1 : 0, nx0 = lo > 0 ? 1 : 0;
    int q = 0;
    bool inr[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u)
    {
        const int k = threadIdx.x * kPer + u;
        inr[u]      = k < nE && E[k] >= lo && E[k] <= hi;
        q += inr[u] ? 1 : 0;
    }
    int nq;
    int rank = block_exscan(q, nq);
    int neg = 0, pos = 0;
    bool take[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u)
    {
        const int k = threadIdx.x * kPer + u;
        take[u]     = inr[u] && rank < mse::kMaxEdges - 1;
        rank += inr[u] ? 1 : 0;
        neg += take[u] && E[k] < 0 ? 1 : 0;
        pos += take[u] && E[k] > 0 ? 1 : 0;
    }
    int nneg, npos;
    int in = block_exscan(neg, nneg) + nm0;
    int ix = block_exscan(pos, npos) + nx0;
#pragma unroll
    for (int u = 0; u < kPer; ++u)
    {
        const int k = threadIdx.x * kPer + u;
        if (take[u] && E[k] < 0)
            mins[in++] = E[k];
        else if (take[u] && E[k] > 0)
            maxs[ix++] = E[k];
    }
    if (threadIdx.x == 0)
    {
        if (lo < 0)
            mins[0] = lo;
        else if (lo > 0)
            maxs[0] = lo;
        const int nm = nm0 + nneg, nx = nx0 + npos;
        const int ne = 1 + (nq < mse::kMaxEdges - 1 ? nq : mse::kMaxEdges - 1);
        mins[nm] = 0;
        maxs[nx] = 0;
        mse::Setup r {};
        r.lo    = lo;
        r.hi    = hi;
        r.nmins = nm + 1;
        r.nmaxs = nx + 1;
        r.nc    = ne - 1 > 0 ? ne - 1 : 0;
        r.total = (long long) r.nmins * r.nmaxs - 1;
        st      = r;
    }
    __syncthreads();
}

__device__ __forceinline__ bool better(float e, long long t, float be, long long bt)
{
    if (t < 0)
        return false;
    if (bt < 0)
        return true;
    return (e < be) || (e == be && t < bt);
}

// slice y (of `splits`) of channel c's candidate grid -> parts[c * splits + y]. Every lane of the
// workgroup calls it with the same (c, y).
__device__ void search_slice(const TqDevice& d, int64_t c, int y, int splits, int bw, int sym, int strict, int unsign)
{
    __shared__ double pdf[tfe::kBins];
    __shared__ float mins[mse::kMaxEdges + 1], maxs[mse::kMaxEdges + 1], cv[mse::kMaxEdges], cw[mse::kMaxEdges];
    __shared__ float zv[mse::kMaxEdges], zw[mse::kMaxEdges];
    // zvd / zwd (after the setup) share their 8 KiB with the setup's edge scratch (before it)
    __shared__ double zbuf[2 * mse::kMaxEdges];
    static_assert(2 * mse::kMaxEdges * sizeof(double) >= 4 * tfe::kBins * sizeof(float), "edge scratch fits");
    double* zvd = zbuf;
    double* zwd = zbuf + mse::kMaxEdges;
    __shared__ float wg_best, wmin[kBlock / 64];
    __shared__ mse::Setup st;
    __shared__ int first, last;
    __shared__ float werr[kBlock / 64];
    __shared__ long long widx[kBlock / 64];
    __shared__ float wlo[kBlock / 64], whi[kBlock / 64];
    const int lane = threadIdx.x & 63;
    MsePart* parts = reinterpret_cast<MsePart*>(d.search_part);
    {
        if (!d.pdf_init[c])
            return;   // the finish step writes the all-zero-data encoding
        for (int i = threadIdx.x; i < tfe::kBins; i += kBlock)
            pdf[i] = d.pdf[c * tfe::kBins + i];
        __syncthreads();
        if (threadIdx.x < 64)
        {
            int fst = -1, lst = -1;
            for (int i0 = 0; i0 < tfe::kBins; i0 += 64)
            {
                unsigned long long o = __ballot(pdf[i0 + lane] > 0);
                if (o)
                {
                    if (fst < 0)
                        fst = i0 + __ffsll((long long) o) - 1;
                    lst = i0 + 63 - __clzll(o);
                }
            }
            if (lane == 0)
            {
                first = fst;
                last  = lst > 0 ? lst : -1;
            }
        }
        __syncthreads();
        // mse::setup over the workgroup: the edges and the bin centres (sequential float sums) as
        // tight one-lane loops, their classification and the centres' masses (a division each) in
        // parallel -- the one-lane setup had been ~1.1 ms of the 5-ms ResNet-50 search
        // (profiles/r06/mse_preamble.txt)
        const tfe::Hist h {d.hist_min[c], d.bucket_size[c], pdf};
        setup_centres_device(h, first, last, mins, maxs, cv, reinterpret_cast<float*>(zbuf), st);
        for (int i = threadIdx.x; i < st.nc; i += kBlock)
            cw[i] = mse::centre_mass(h, cv[i]);
        __syncthreads();
        bool finite;
        const int nz = compact_bins(st, cv, cw, zv, zw, zvd, zwd, finite);
        // candidates in the order j: iMin ascending (widest low end first), iMax from the widest
        // positive end down (maxs[nx - 2] ... maxs[0], then the 0 end): the first round holds the
        // near-full ranges, whose errors are small, and later rounds are pruned against the best
        // error the workgroup has reached (cost_fast). The selection still compares the reference's
        // candidate index t = iMin * nx + iMax (the first minimum in its order).
        const int nx          = st.nmaxs;
        const long long full  = (long long) st.nmins * nx;   // t = full - 1 is not a candidate
        const long long chunk = (full + splits - 1) / splits;
        const long long j0    = (long long) y * chunk;
        const long long j1    = j0 + chunk < full ? j0 + chunk : full;
        if (threadIdx.x == 0)
            wg_best = FLT_MAX;
        __syncthreads();
        float be = 0, blo = 0, bhi = 0;
        long long bt = -1;
        for (long long jb = j0; jb < j1; jb += kBlock)
        {
            const long long j = jb + threadIdx.x;
            const float prune = bt >= 0 && be < wg_best ? be : wg_best;
            if (j < j1)
            {
                const int iMin = (int) (j / nx);
                const int jm   = (int) (j - (long long) iMin * nx);
                const int iMax = jm < nx - 1 ? nx - 2 - jm : nx - 1;
                const long long t = (long long) iMin * nx + iMax;
                if (t != full - 1)
                {
                    const float cLo = mins[iMin], cHi = maxs[iMax];
                    bool pruned     = false;
                    const float err = finite ? cost_fast(bw, zv, zvd, zwd, nz, cLo, cHi, sym != 0, strict != 0,
                                                         unsign != 0, prune, pruned)
                                             : mse::cost(bw, zv, zw, nz, cLo, cHi, sym != 0, strict != 0, unsign != 0);
                    // `err < bestErr` with bestErr = FLT_MAX never selects err >= FLT_MAX
                    if (!pruned && err < FLT_MAX && better(err, t, be, bt))
                    {
                        be  = err;
                        bt  = t;
                        blo = cLo;
                        bhi = cHi;
                    }
                }
            }
            // the workgroup's best error so far (every lane's selected error is a complete one)
            float m = bt >= 0 ? be : FLT_MAX;
            for (int k = 32; k > 0; k >>= 1)
                m = fminf(m, __shfl_xor(m, k, 64));
            if (lane == 0)
                wmin[threadIdx.x >> 6] = m;
            __syncthreads();
            if (threadIdx.x == 0)
                for (int w = 0; w < kBlock / 64; ++w)
                    wg_best = fminf(wg_best, wmin[w]);
            __syncthreads();
        }
        for (int k = 32; k > 0; k >>= 1)
        {
            float oe       = __shfl_xor(be, k, 64);
            long long ot   = __shfl_xor(bt, k, 64);
            float olo      = __shfl_xor(blo, k, 64);
            float ohi      = __shfl_xor(bhi, k, 64);
            if (better(oe, ot, be, bt))
            {
                be  = oe;
                bt  = ot;
                blo = olo;
                bhi = ohi;
            }
        }
        if (lane == 0)
        {
            werr[threadIdx.x >> 6] = be;
            widx[threadIdx.x >> 6] = bt;
            wlo[threadIdx.x >> 6]  = blo;
            whi[threadIdx.x >> 6]  = bhi;
        }
        __syncthreads();
        if (threadIdx.x == 0)
        {
            for (int w = 1; w < kBlock / 64; ++w)
                if (better(werr[w], widx[w], be, bt))
                {
                    be  = werr[w];
                    bt  = widx[w];
                    blo = wlo[w];
                    bhi = whi[w];
                }
            parts[c * splits + y] = MsePart {be, bt >= 0 ? (int) bt : -1, blo, bhi, st.lo, st.hi};
        }
        __syncthreads();
    }
}

// 6 waves per SIMD, the most the kernel's 24.9 KB of LDS allows (80 VGPRs, a few spills): 3.80 ms
// against 4.08 at 5 waves (96 VGPRs, no spills) and 4.69 at 4 (106 VGPRs) on ResNet-50's weights
// (profiles/r06/mse_preamble.txt)
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(6))) void mse_search_kernel(TqDevice d, int64_t C, int splits, int bw, int sym,
                                                            int strict, int unsign)
{
    for (int64_t c = blockIdx.x; c < C; c += gridDim.x)
        search_slice(d, c, (int) blockIdx.y, splits, bw, sym, strict, unsign);
}

// many quantizers in one launch: work item g = (job, channel, slice), flattened in job order
struct MseJob
{
    TqDevice d;
    int64_t C;
    int splits;
    int64_t wstart;            // first work item (channel x slice) of this job
    int64_t cstart;            // first channel of this job
    aimet_tf_encoding* flat;   // optional: the encodings of every job concatenated (+ cstart)
};

__device__ __forceinline__ int job_of(const MseJob* jobs, int njobs, int64_t g, bool by_channel)
{
    int lo = 0, hi = njobs - 1;   // last job whose start <= g
    while (lo < hi)
    {
        int mid = (lo + hi + 1) >> 1;
        if ((by_channel ? jobs[mid].cstart : jobs[mid].wstart) <= g)
            lo = mid;
        else
            hi = mid - 1;
    }
    return lo;
}

__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(6))) void mse_search_many_kernel(const MseJob* __restrict__ jobs, int njobs,
                                                                 int64_t total, int bw, int sym, int strict, int unsign)
{
    for (int64_t g = blockIdx.x; g < total; g += gridDim.x)
    {
        const MseJob& j      = jobs[job_of(jobs, njobs, g, false)];
        const int64_t local  = g - j.wstart;
        search_slice(j.d, local / j.splits, (int) (local % j.splits), j.splits, bw, sym, strict, unsign);
    }
}

// fold the slices of every channel (in candidate order) and write the encodings
__device__ void finish_channel(const TqDevice& d, int64_t c, int splits, int bw, int sym, int strict, int unsign,
                               aimet_tf_encoding* flat = nullptr)
{
    if (!d.pdf_init[c])
    {
        // statistics updated but no histogram (all data zero): MseEncodingAnalyzer.cpp:86-99,
        // numSteps reduced first for strict symmetric
        float steps = (float) (ldexp(1.0, bw) - 1);
        if (sym && strict)
            steps -= 1;
        int isteps = (int) steps;
        aimet_tf_encoding e;
        e.delta  = (1.0 - (-1.0)) / isteps;
        e.offset = floor(-1.0 / e.delta);
        e.min    = e.offset * e.delta;
        e.max    = e.min + isteps * e.delta;
        e.bw     = bw;
        d.enc[c] = e;
        if (flat)
            flat[c] = e;
        return;
    }
    const MsePart* parts = reinterpret_cast<const MsePart*>(d.search_part) + c * splits;
    float be = 0, blo = parts[0].obs_lo, bhi = parts[0].obs_hi;
    long long bt = -1;
    for (int y = 0; y < splits; ++y)
        if (better(parts[y].err, parts[y].idx, be, bt))
        {
            be  = parts[y].err;
            bt  = parts[y].idx;
            blo = parts[y].lo;
            bhi = parts[y].hi;
        }
    const aimet_tf_encoding e = mse::finish(bw, blo, bhi, sym != 0, strict != 0, unsign != 0);
    d.enc[c] = e;
    if (flat)
        flat[c] = e;
}

__global__ __launch_bounds__(kBlock) void mse_finish_kernel(TqDevice d, int64_t C, int splits, int bw, int sym,
                                                            int strict, int unsign)
{
    const int64_t c = (int64_t) blockIdx.x * kBlock + threadIdx.x;
    if (c < C)
        finish_channel(d, c, splits, bw, sym, strict, unsign);
}

__global__ __launch_bounds__(kBlock) void mse_finish_many_kernel(const MseJob* __restrict__ jobs, int njobs,
                                                                 int64_t total, int bw, int sym, int strict, int unsign)
{
    const int64_t g = (int64_t) blockIdx.x * kBlock + threadIdx.x;
    if (g >= total)
        return;
    const MseJob& j = jobs[job_of(jobs, njobs, g, true)];
    finish_channel(j.d, g - j.cstart, j.splits, bw, sym, strict, unsign, j.flat ? j.flat + j.cstart : nullptr);
}

}   // namespace

size_t mse_part_bytes(int64_t C)
{
    return sizeof(MsePart) * (size_t) (C > kMseMaxSplits ? C : kMseMaxSplits);
}

namespace
{
// slices per channel: fill the chip when there are few channels (per-tensor: 128 workgroups);
// the result does not depend on it (slices are folded in candidate order)
int mse_splits(int64_t C)
{
    return C >= kMseMaxSplits ? 1 : (int) (kMseMaxSplits / C);
}
}   // namespace

void launch_mse_search_many(const TqDevice* const* ds, const int64_t* Cs, int n, int bw, bool sym, bool strict,
                            bool unsign, hipStream_t s, aimet_tf_encoding* pinned_dst)
{
    if (n == 0)
        return;
    std::vector<MseJob> jobs((size_t) n);
    int64_t work = 0, chans = 0;
    for (int i = 0; i < n; ++i)
        chans += Cs[i];
    // the encodings of every quantizer side by side, for one copy into the caller's pinned block
    auto* flat = pinned_dst ? static_cast<aimet_tf_encoding*>(scratch_alloc(sizeof(aimet_tf_encoding) * chans, s))
                            : nullptr;
    chans = 0;
    for (int i = 0; i < n; ++i)
    {
        const int splits = mse_splits(Cs[i]);
        jobs[(size_t) i] = MseJob {*ds[i], Cs[i], splits, work, chans, flat};
        work += Cs[i] * splits;
        chans += Cs[i];
    }
    auto* dj = static_cast<MseJob*>(upload_async(jobs.data(), sizeof(MseJob) * (size_t) n, s));
    mse_search_many_kernel<<<(unsigned) (work < 65536 ? work : 65536), kBlock, 0, s>>>(
        dj, n, work, bw, sym ? 1 : 0, strict ? 1 : 0, unsign ? 1 : 0);
    AIMET_LAUNCH_CHECK();
    mse_finish_many_kernel<<<(unsigned) ceil_div(chans, kBlock), kBlock, 0, s>>>(dj, n, chans, bw, sym ? 1 : 0,
                                                                                 strict ? 1 : 0, unsign ? 1 : 0);
    AIMET_LAUNCH_CHECK();
    scratch_free(dj, s);
    if (flat)
    {
        AIMET_HIP_CHECK(hipMemcpyAsync(pinned_dst, flat, sizeof(aimet_tf_encoding) * chans, hipMemcpyDeviceToHost, s));
        scratch_free(flat, s);
    }
}

void launch_mse_search(const TqDevice& d, int64_t C, int bw, bool sym, bool strict, bool unsign, hipStream_t s)
{
    const int splits = mse_splits(C);
    dim3 grid((unsigned) (C < 65536 ? C : 65536), (unsigned) splits);
    mse_search_kernel<<<grid, kBlock, 0, s>>>(d, C, splits, bw, sym, strict, unsign);
    AIMET_LAUNCH_CHECK();
    mse_finish_kernel<<<(unsigned) ceil_div(C, kBlock), kBlock, 0, s>>>(d, C, splits, bw, sym, strict, unsign);
    AIMET_LAUNCH_CHECK();
}

}   // namespace aimet_amd
