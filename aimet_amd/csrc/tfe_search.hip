// tfe_search.hip -- TF-Enhanced encoding search on the device, all channels in one launch.
//
// Reference: TfEnhancedEncodingAnalyzer::computeEncoding (TfEnhancedEncodingAnalyzer.cpp:78-392)
// runs on the host, one channel at a time: 101 (symmetric) or 358 (asymmetric) candidates x 512
// bins of mixed float/double arithmetic per channel -- 3.3 s (sym) / 10.7 s (asym) for ResNet-50's
// 27,560 weight channels. Here: one workgroup per channel, one candidate per lane
// (each lane evaluates its candidate's cost over the 512 bins in the reference's order, the PDF
// broadcast from LDS), then a first-minimum argmin across the workgroup. The arithmetic is the
// shared header tfe_core.hpp, compiled for the host and the device from one source (bit-exact).
#include "tfe_core.hpp"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include "tq_state.hpp"

#include <mutex>
#include <vector>

namespace aimet_amd
{
namespace
{

// (cost, index) of the first strict minimum below DBL_MAX: exactly `if (cost < bestCost)` over
// candidates in index order with bestCost starting at DBL_MAX (NaN / DBL_MAX never selected).
struct Best
{
    double cost;
    int idx;
    float delta;
    int offset;
};

__device__ __forceinline__ bool better(const Best& a, const Best& b)
{
    if (a.idx < 0)
        return false;
    if (b.idx < 0)
        return true;
    return (a.cost < b.cost) || (a.cost == b.cost && a.idx < b.idx);
}

// Channel g's candidates over `splits` workgroups (few channels: the activations' quantizers of a
// batch): workgroup (g, s) takes candidates s * BLOCK + lane, s * BLOCK + lane + BLOCK * splits, ...,
// publishes its first minimum (cost, index) write-through, and the last of the g's workgroups to
// arrive (tickets[g]) takes the first minimum of those -- `better` orders by (cost, index), so the
// choice is the one-workgroup argmin's -- and finishes the encoding. splits == 1: one workgroup
// per channel, no hand-off. SYMFORM: tfe::cost's branch-free symmetric loops (same sums).
template <int BLOCK, bool SYMFORM>
__global__ __launch_bounds__(BLOCK, BLOCK == 128 ? 5 : (BLOCK == 64 ? 2 : 7)) void tfe_search_kernel(
    TfeJob one, const TfeJob* __restrict__ jobs, int njobs, int64_t total, int bw, int sym, int strict, int unsign,
    int splits, uint64_t* __restrict__ part, unsigned* __restrict__ tickets)
{
    constexpr int kW = BLOCK / 64;
    __shared__ double pdf_c[tfe::kBins];
    __shared__ double cd_c[tfe::kBins];
    __shared__ float cf_c[tfe::kBins];
    __shared__ float cf[tfe::kBins];
    __shared__ short pos[tfe::kBins];
    __shared__ float fseq[tfe::kSymF + 8];
    __shared__ int first, last, nnz;
    __shared__ Best wbest[kW];
    if (threadIdx.x == 0)
    {
        if (sym)
            tfe::fseq_sym(fseq);
        else
            tfe::fseq_asym(fseq);
    }
    const int lane = threadIdx.x & 63;
    for (int64_t gs = blockIdx.x; gs < total * splits; gs += gridDim.x)
    {
        const int64_t g = gs / splits;
        const int sp    = (int) (gs - g * splits);
        TfeJob j = one;
        if (jobs)
        {
            int lo = 0, hi = njobs - 1;   // last job with start <= g
            while (lo < hi)
            {
                int mid = (lo + hi + 1) >> 1;
                if (jobs[mid].start <= g)
                    lo = mid;
                else
                    hi = mid - 1;
            }
            j = jobs[lo];
        }
        const int64_t c = g - j.start;
        if (!j.pdf_init[c])
        {
            if (threadIdx.x == 0 && sp == 0)
            {
                // statistics updated but all data zero (TfEnhancedEncodingAnalyzer.cpp:86-99)
                int isteps = (int) (float) (ldexp(1.0, bw) - 1);
                aimet_tf_encoding e;
                e.delta    = (1.0 - (-1.0)) / isteps;
                e.offset   = floor(-1.0 / e.delta);
                e.min      = e.offset * e.delta;
                e.max      = e.min + isteps * e.delta;
                e.bw       = bw;
                j.out[c]   = e;
            }
            continue;
        }
        tfe::Hist h {j.hist_min[c], j.bucket_size[c], nullptr};
        const float start = tfe::bins_start(h);
        const double step = tfe::bins_step(h);
        for (int i = threadIdx.x; i < tfe::kBins; i += BLOCK)   // staged by every wave
            pdf_c[i] = j.pdf[c * tfe::kBins + i];
        __syncthreads();
        if (threadIdx.x < 64)
        {
            // ascending compaction of the bins the cost must visit (pdf and centres gathered
            // into k order, pos[i] = visited bins below i) + first/last non-empty bins. In place:
            // chunk r is read before any of its lanes writes, and every write goes to k <= i.
            const bool skip = tfe::bins_skip_empty(h);
            const unsigned long long below = (1ull << lane) - 1;
            int base = 0, fst = -1, lst = -1;
            for (int i0 = 0; i0 < tfe::kBins; i0 += 64)
            {
                const int i          = i0 + lane;
                const double pi      = pdf_c[i];
                const double m_c     = tfe::bin_centre(start, step, i);
                const bool occupied  = pi > 0;
                const bool visit     = occupied || !skip;
                unsigned long long m = __ballot(visit);
                unsigned long long o = __ballot(occupied);
                const int k          = base + __popcll(m & below);
                cf[i]                = (float) m_c;
                pos[i]               = (short) k;
                if (visit)
                {
                    pdf_c[k] = pi;
                    cd_c[k]  = m_c;
                    cf_c[k]  = (float) m_c;
                }
                base += __popcll(m);
                if (o)
                {
                    if (fst < 0)
                        fst = i0 + __ffsll((long long) o) - 1;
                    lst = i0 + 63 - __clzll(o);
                }
            }
            if (lane == 0)
            {
                nnz   = base;
                first = fst;
                last  = lst > 0 ? lst : -1;   // the reference's backward scan stops before bin 0
            }
        }
        __syncthreads();
        float lo, hi;
        tfe::observed_range(h, first, last, lo, hi);
        tfe::Setup st = tfe::setup(lo, hi, bw, sym != 0, strict != 0, unsign != 0);
        const tfe::Bins B {start, step, cf, pdf_c, cd_c, cf_c, pos, nnz};

        Best b {0.0, -1, -1.0f, -1};
        for (int t = threadIdx.x + sp * BLOCK; t < st.ncand; t += BLOCK * splits)
        {
            float dl;
            int o;
            if (!tfe::candidate(st, fseq, t, dl, o))
                continue;
            double cst = tfe::cost<SYMFORM>(B, bw, dl, o);
            if (!(cst < DBL_MAX))
                continue;
            Best me {cst, t, dl, o};
            if (better(me, b))
                b = me;
        }
        // wave argmin, then across waves
        for (int k = 32; k > 0; k >>= 1)
        {
            Best o;
            o.cost   = __shfl_xor(b.cost, k, 64);
            o.idx    = __shfl_xor(b.idx, k, 64);
            o.delta  = __shfl_xor(b.delta, k, 64);
            o.offset = __shfl_xor(b.offset, k, 64);
            if (better(o, b))
                b = o;
        }
        if (lane == 0)
            wbest[threadIdx.x >> 6] = b;
        __syncthreads();
        if (threadIdx.x == 0)
            for (int w = 1; w < kW; ++w)
                if (better(wbest[w], b))
                    b = wbest[w];
        bool finish = splits == 1;
        if (!finish)
        {
            // publish (cost, index) write-through; the last of channel g's workgroups takes the
            // first minimum over them: lane q loads split q's pair, lane 0 scans them in order
            __shared__ int lastw;
            if (threadIdx.x == 0)
            {
                uint64_t* my = part + 2 * gs;
                publish_u64(my, (uint64_t) __double_as_longlong(b.cost));
                publish_u64(my + 1, (uint64_t) (uint32_t) b.idx);
                lastw = arrive_is_last(tickets + g, (unsigned) splits);
            }
            __syncthreads();
            if (lastw)
            {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                double qc = 0.0;
                int qi    = -1;
                if (threadIdx.x < (unsigned) splits)
                {
                    const uint64_t* pq = part + 2 * (g * splits + threadIdx.x);
                    qc                 = __longlong_as_double((long long) consume_u64(pq));
                    qi                 = (int) (uint32_t) consume_u64(pq + 1);
                }
                Best m {0.0, -1, -1.0f, -1};
                for (int q = 0; q < splits; ++q)   // uniform over the wave (splits <= 64)
                {
                    Best o {__shfl(qc, q, 64), __shfl(qi, q, 64), -1.0f, -1};
                    if (better(o, m))
                        m = o;
                }
                if (threadIdx.x == 0)
                {
                    finish = true;
                    b      = m;
                    if (b.idx >= 0)   // the winner's delta / offset, as its lane formed them
                        tfe::candidate(st, fseq, b.idx, b.delta, b.offset);
                    ticket_reset(tickets + g);
                }
            }
        }
        if (threadIdx.x == 0 && finish)
        {
            float bd = b.idx >= 0 ? b.delta : -1.0f;
            int bo   = b.idx >= 0 ? b.offset : -1;
            tfe::Result r = tfe::finish(st, bd, bo);
            j.out[c]      = aimet_tf_encoding {r.min, r.max, r.delta, r.offset, bw};
        }
        __syncthreads();
    }
}

// one candidate per lane: 101 symmetric candidates -> 2 waves, 358 asymmetric -> 6 waves; one
// workgroup per channel (capped grids measured no faster beside the activation passes,
// profiles/r04/enc_split_tfe_grid.jsonl)
constexpr int kSearchGridCap = 65536;

// channels below which each one's candidates are split over one-wave workgroups (the activations'
// quantizers of a batch: ResNet-50's 55 asymmetric searches took 58 us as 55 workgroups)
constexpr int64_t kTfeSplitBelow = 512;

// the split search's launch (part: 2 * total * splits, tickets: total zeroed counters)
void launch_split(const TfeJob& one, const TfeJob* jobs, int njobs, int64_t total, int bw, bool sym, bool strict,
                  bool unsign, int splits, uint64_t* part, unsigned* tickets, hipStream_t s)
{
    const int grid = (int) std::min<int64_t>(total * splits, kSearchGridCap);
    if (sym)
        tfe_search_kernel<64, true><<<grid, 64, 0, s>>>(one, jobs, njobs, total, bw, 1, strict, unsign, splits, part,
                                                      tickets);
    else
        tfe_search_kernel<64, false><<<grid, 64, 0, s>>>(one, jobs, njobs, total, bw, 0, strict, unsign, splits, part,
                                                       tickets);
    AIMET_LAUNCH_CHECK();
}

void launch_kernel(const TfeJob& one, const TfeJob* jobs, int njobs, int64_t total, int bw, bool sym, bool strict,
                   bool unsign, hipStream_t s, size_t lds_pad = 0)
{
    const int cap    = kSearchGridCap;
    const int splits = tfe_splits(total, sym);
    if (splits > 1)
    {
        unsigned* tickets = ticket_alloc(s, (unsigned) total);
        if (tickets)
        {
            auto* part = static_cast<uint64_t*>(scratch_alloc(sizeof(uint64_t) * 2 * total * splits, s));
            launch_split(one, jobs, njobs, total, bw, sym, strict, unsign, splits, part, tickets, s);
            scratch_free(part, s);
            return;
        }
    }
    const int grid = (int) (total < cap ? total : cap);
    if (sym)
        tfe_search_kernel<128, true><<<grid, 128, lds_pad, s>>>(one, jobs, njobs, total, bw, 1, strict, unsign, 1, nullptr,
                                                        nullptr);
    else
        tfe_search_kernel<384, false><<<grid, 384, lds_pad, s>>>(one, jobs, njobs, total, bw, 0, strict, unsign, 1, nullptr,
                                                         nullptr);
    AIMET_LAUNCH_CHECK();
}

}   // namespace

int tfe_splits(int64_t total, bool sym)
{
    if (total >= kTfeSplitBelow)
        return 1;
    return (int) ceil_div(sym ? tfe::kSymF : tfe::kMaxCand, 64);
}

void launch_tfe_table(const TfeTable& t, int bw, bool sym, bool strict, bool unsign, hipStream_t s)
{
    const int per_cu = t.per_cu;
    if (t.total == 0)
        return;
    const int splits = tfe_splits(t.total, sym);
    if (splits > 1)
    {
        AIMET_REQUIRE(t.part != nullptr && t.tickets != nullptr, "split TF-Enhanced search without its buffers");
        launch_split(t.first, t.dev, t.n, t.total, bw, sym, strict, unsign, splits, t.part, t.tickets, s);
        return;
    }
    // at most `per_cu` workgroups per CU: dynamic LDS beyond the kernel's own keeps more from being
    // resident (the wave slots left to an HBM-bound pass running beside the search)
    size_t pad = 0;
    if (per_cu > 0)
    {
        constexpr size_t kLdsPerCu = 160 * 1024, kStatic = 14 * 1024;   // the kernel's own ~13.3 KB
        const size_t want          = kLdsPerCu / (size_t) (per_cu + 1) + 1;
        pad                        = want > kStatic ? want - kStatic : 0;
    }
    launch_kernel(t.first, t.dev, t.n, t.total, bw, sym, strict, unsign, s, pad);
}

namespace
{

TfeJob job_of(const TqDevice& d, int64_t start)
{
    return TfeJob {d.pdf_init, d.hist_min, d.bucket_size, d.pdf, d.enc, start};
}

// Grow-only pinned host buffer per device for the batched searches' results (a D2H copy into
// pageable memory is staged through the driver's bounce buffer: 0.56 ms for ResNet-50's 27,560
// encodings, against ~0.01 ms pinned); held under the lock until the call has synchronised.
struct PinnedOut
{
    std::mutex m;
    void* p[64]    = {};
    size_t cap[64] = {};
};
PinnedOut& pinned_out()
{
    static PinnedOut s;
    return s;
}
}   // namespace

void launch_tfe_search(const TqDevice& d, int64_t C, int bw, bool sym, bool strict, bool unsign, hipStream_t s)
{
    launch_kernel(job_of(d, 0), nullptr, 0, C, bw, sym, strict, unsign, s);
}

void launch_tfe_search_many_to(const TqDevice* const* ds, const int64_t* Cs, int n, int bw, bool sym, bool strict,
                               bool unsign, aimet_tf_encoding* pinned_dst, hipStream_t s, hipStream_t prep)
{
    if (n == 0)
        return;
    std::vector<TfeJob> jobs(n);
    int64_t total = 0;
    for (int i = 0; i < n; ++i)
    {
        jobs[i] = job_of(*ds[i], total);
        total += Cs[i];
    }
    auto* dout = static_cast<aimet_tf_encoding*>(scratch_alloc(sizeof(aimet_tf_encoding) * total, s));
    for (int i = 0; i < n; ++i)
        jobs[i].out = dout + jobs[i].start;
    const hipStream_t us = (prep != nullptr && prep != s) ? prep : s;
    auto* djobs = static_cast<TfeJob*>(upload_async(jobs.data(), sizeof(TfeJob) * n, us));
    if (us != s)
        stream_join(s, us);   // the copy ran long before s gets here (the statistics passes)
    launch_kernel(jobs[0], djobs, n, total, bw, sym, strict, unsign, s);
    AIMET_HIP_CHECK(hipMemcpyAsync(pinned_dst, dout, sizeof(aimet_tf_encoding) * total, hipMemcpyDeviceToHost, s));
    scratch_free(djobs, s);
    scratch_free(dout, s);
}

void launch_tfe_search_many(const TqDevice* const* ds, const int64_t* Cs, int n, int bw, bool sym, bool strict,
                            bool unsign, aimet_tf_encoding* host_out, hipStream_t s)
{
    if (n == 0)
        return;
    std::vector<TfeJob> jobs(n);
    int64_t total = 0;
    for (int i = 0; i < n; ++i)
    {
        jobs[i] = job_of(*ds[i], total);
        total += Cs[i];
    }
    int dev = 0;
    AIMET_HIP_CHECK(hipGetDevice(&dev));
    AIMET_REQUIRE(dev >= 0 && dev < 64, "device id out of range");
    auto* dout = static_cast<aimet_tf_encoding*>(scratch_alloc(sizeof(aimet_tf_encoding) * total, s));
    for (int i = 0; i < n; ++i)
        jobs[i].out = dout + jobs[i].start;
    auto* djobs = static_cast<TfeJob*>(upload_async(jobs.data(), sizeof(TfeJob) * n, s));
    launch_kernel(jobs[0], djobs, n, total, bw, sym, strict, unsign, s);
    const size_t out_bytes = sizeof(aimet_tf_encoding) * total;
    PinnedOut& po = pinned_out();
    std::lock_guard<std::mutex> lock(po.m);
    if (po.cap[dev] < out_bytes)
    {
        if (po.p[dev])
            AIMET_HIP_CHECK(hipHostFree(po.p[dev]));
        po.p[dev]   = nullptr;
        po.cap[dev] = 0;
        AIMET_HIP_CHECK(hipHostMalloc(&po.p[dev], out_bytes, hipHostMallocDefault));
        po.cap[dev] = out_bytes;
    }
    AIMET_HIP_CHECK(hipMemcpyAsync(po.p[dev], dout, out_bytes, hipMemcpyDeviceToHost, s));
    scratch_free(djobs, s);
    scratch_free(dout, s);
    AIMET_HIP_CHECK(hipStreamSynchronize(s));
    std::memcpy(host_out, po.p[dev], out_bytes);
}

}   // namespace aimet_amd
