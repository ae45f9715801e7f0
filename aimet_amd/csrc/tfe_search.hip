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
#include "tq_state.hpp"

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

__global__ __launch_bounds__(kBlock) void tfe_search_kernel(TqDevice d, int64_t C, int bw, int sym, int strict,
                                                            int unsign, int stats_updated,
                                                            aimet_tf_encoding* __restrict__ out)
{
    __shared__ double pdf[tfe::kBins];
    __shared__ float fseq[tfe::kSymF + 8];
    __shared__ int first, last;
    __shared__ Best wbest[kBlock / 64];
    if (threadIdx.x == 0)
    {
        if (sym)
            tfe::fseq_sym(fseq);
        else
            tfe::fseq_asym(fseq);
    }
    for (int64_t c = blockIdx.x; c < C; c += gridDim.x)
    {
        if (!d.pdf_init[c])
        {
            if (threadIdx.x == 0)
            {
                aimet_tf_encoding e {0, 0, 0, 0, 0};
                if (stats_updated)   // all-zero data seen (TfEnhancedEncodingAnalyzer.cpp:86-99)
                {
                    int isteps = (int) (float) (ldexp(1.0, bw) - 1);
                    e.delta    = (1.0 - (-1.0)) / isteps;
                    e.offset   = floor(-1.0 / e.delta);
                    e.min      = e.offset * e.delta;
                    e.max      = e.min + isteps * e.delta;
                    e.bw       = bw;
                }
                out[c] = e;
            }
            continue;
        }
        for (int i = threadIdx.x; i < tfe::kBins; i += kBlock)
            pdf[i] = d.pdf[c * tfe::kBins + i];
        if (threadIdx.x == 0)
        {
            first = tfe::kBins;
            last  = -1;
        }
        __syncthreads();
        for (int i = threadIdx.x; i < tfe::kBins; i += kBlock)
            if (pdf[i] > 0)
            {
                atomicMin(&first, i);
                if (i > 0)
                    atomicMax(&last, i);
            }
        __syncthreads();
        tfe::Hist h {d.hist_min[c], d.bucket_size[c], pdf};
        float lo, hi;
        tfe::observed_range(h, first < tfe::kBins ? first : -1, last, lo, hi);
        tfe::Setup st = tfe::setup(lo, hi, bw, sym != 0, strict != 0, unsign != 0);

        Best b {0.0, -1, -1.0f, -1};
        for (int t = threadIdx.x; t < st.ncand; t += kBlock)
        {
            float dl;
            int o;
            if (!tfe::candidate(st, fseq, t, dl, o))
                continue;
            double cst = tfe::cost(h, bw, dl, o);
            if (!(cst < DBL_MAX))
                continue;
            Best me {cst, t, dl, o};
            if (better(me, b))
                b = me;
        }
        // wave argmin
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
        if ((threadIdx.x & 63) == 0)
            wbest[threadIdx.x >> 6] = b;
        __syncthreads();
        if (threadIdx.x == 0)
        {
            for (int w = 1; w < kBlock / 64; ++w)
                if (better(wbest[w], b))
                    b = wbest[w];
            float bd = b.idx >= 0 ? b.delta : -1.0f;
            int bo   = b.idx >= 0 ? b.offset : -1;
            tfe::Result r = tfe::finish(st, bd, bo);
            out[c]        = aimet_tf_encoding {r.min, r.max, r.delta, r.offset, bw};
        }
        __syncthreads();
    }
}

}   // namespace

void launch_tfe_search(const TqDevice& d, int64_t C, int bw, bool sym, bool strict, bool unsign, bool stats_updated,
                       aimet_tf_encoding* out, hipStream_t s)
{
    int grid = (int) (C < 65536 ? C : 65536);
    tfe_search_kernel<<<grid, kBlock, 0, s>>>(d, C, bw, sym, strict, unsign, stats_updated, out);
    AIMET_LAUNCH_CHECK();
}

}   // namespace aimet_amd
