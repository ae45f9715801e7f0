// tq_state.hpp -- device-resident statistics of one aimet_tensor_quantizer (C channels).
//
// The reference keeps statistics on the host (TfEncodingAnalyzer::_accumulatedStats, PDF in a
// std::vector) and synchronises the device 1-3x per updateStats (thrust D2H + histogram memcpy,
// math_functions.cu:52-64,174-211). Here every field lives in HBM and updateStats is a chain
// of stream-ordered kernels with no host round trip; only getEncoding reads them back.
#pragma once

#include <cstddef>
#include <functional>

#include "common.hpp"

#include <vector>

namespace aimet_amd
{

struct TqDevice
{
    // phase-1 output, exchanged between ranks with all_reduce(MAX): {-min, max} per channel
    float* minmax;          // [C][2]
    float* partials;        // [kMinmaxParts][2]   (C == 1: per-block partial {-min, max})
    // TF analyzer (TfEncodingAnalyzer.h:86-91), double
    double* acc;            // [C][2] {min, max}
    // PDF (math_functions.hpp:70-77) of histogram analyzers
    int32_t* pdf_init;      // [C] xLeft.size() != 0
    int32_t* iterations;    // [C]
    float* hist_min;        // [C] min_val of InitializePdf (xLeft[i] = min_val + i*bucket_size)
    double* bucket_size;    // [C]
    float* bin_bucket;      // [C] (float)(xLeft[1]-xLeft[0])      UpdatePdf:264
    float* bin_offset;      // [C] (float)xLeft[0] / bin_bucket    UpdatePdf:265-268
    double* pdf;            // [C][512]
    unsigned long long* counts;   // [C][512] histogram of the current batch
    // Entropy analyzer (TensorProfilingParams, math_functions.hpp:71-77) reuses: acc = {min, max},
    // pdf_init = histogram allocated, pdf = the 512 bin counts (integers in double), iterations,
    // bin_bucket / bin_offset = the float (binWidth, min) of the current batch, and
    int32_t* active;        // [C] the current batch is binned (not all-zero, :482-487)
    aimet_tf_encoding* enc; // [C] device-computed encodings (TF-Enhanced / MSE search)
    void* search_part;      // MSE search slices (mse_part_bytes(C))
};

// statistics family of a quantizer's analyzer
enum StatsKind
{
    kKindTf      = 0,   // running min/max (TF)
    kKindPdf     = 1,   // PDF histogram, range fixed on the first batch (TF-E, percentile, MSE)
    kKindEntropy = 2    // TensorProfilingParams histogram, range widened every batch (entropy)
};

constexpr int kMinmaxParts  = 1024;   // grid of the per-tensor min/max pass
constexpr int kMseMaxSplits = 128;    // candidate slices of a per-tensor MSE search

// stats.hip
void launch_batch_minmax(const TqDevice& d, const float* x, int64_t outer, int64_t C, int64_t K, int skip_if_init,
                         hipStream_t s);
void launch_fold_minmax(const TqDevice& d, int64_t C, StatsKind kind, hipStream_t s);
void launch_batch_histogram(const TqDevice& d, const float* x, int64_t outer, int64_t C, int64_t K, StatsKind kind,
                            hipStream_t s);
void launch_fold_histogram(const TqDevice& d, int64_t C, int64_t count, StatsKind kind, hipStream_t s);
void launch_reset_state(const TqDevice& d, int64_t C, bool hist, hipStream_t s);
// the TF accumulators of many quantizers (aimet_tq_create_many) in one launch
struct ResetJob
{
    double* acc;
    int64_t C;
};
void launch_reset_state_many(const std::vector<ResetJob>& jobs, hipStream_t s);
// zero many device ranges in one launch (16-B aligned starts; any length)
struct ZeroJob
{
    void* p;
    int64_t bytes;
};
void launch_zero_many(const std::vector<ZeroJob>& jobs, hipStream_t s);
// the same two resets over device tables (`most`: the largest range in bytes)
void launch_zero_table(const ZeroJob* dj, int n, int64_t most, hipStream_t s);
void launch_reset_table(const ResetJob* dj, int n, hipStream_t s);
// Many per-tensor quantizers (C == 1) in one launch per phase (stats.hip: launch_stats_many)
struct StatsJob
{
    const float* x;
    int64_t n;       // elements of this quantizer's tensor
    int64_t count;   // element count of the PDF fold (the global count when sharded)
    const int64_t* count_dev;   // when set: the count is read on the device (summed over ranks in HBM)
    int64_t* count_out;         // when set: the combine writes this rank's element count n there (the
                                // sharded calibration's SUM then forms count_dev in place)
    TqDevice d;
    uint32_t mm_block0, mm_blocks, h_block0, h_blocks;   // filled by launch_stats_many
    float* mm_part;  // [mm_blocks][2] per-tile {-min, max} (launch_stats_many's scratch)
    int32_t hist, vec;
    int32_t ent;     // entropy analyzer (hist == 1 too): min/max every batch, TensorProfilingParams
    int32_t seen;    // the quantizer has seen a batch since its reset (host flag; a schedule hint only)
    int32_t fresh;   // reset in this call after the min/max pass (launch_stats_many's `between`): its
                     // PDF range counts as unset whatever the device state still says
};
enum StatsPhase
{
    kPhaseMinmax        = 1,   // min/max pass + combine into minmax[0]
    kPhaseFoldMinmax    = 2,   // TF running min/max / PDF range initialisation
    kPhaseHistogram     = 4,
    kPhaseFoldHistogram = 8
};
// `between` (optional) runs on the host right after the min/max pass is enqueued and before its
// combine / fold: the calibration enqueues the quantizers' reset and the parameters' work there
void launch_stats_many(std::vector<StatsJob>& jobs, int phases, hipStream_t s,
                       const std::function<void()>& between = {});
// launch_stats_many in two halves, for job tables kept on the device (calibration plans): the
// workgroup layout (mm_block0 / h_block0 of every job; *mm, *hb the two passes' grids), then the
// phases over a device copy `dj` of those jobs (whose mm_part point into 2 * mm floats of scratch).
// walk: the min/max pass walks the tiles (launch_stats_many decides it from the jobs' seen flags)
void stats_layout(std::vector<StatsJob>& jobs, uint64_t* mm, uint64_t* hb);
bool stats_walk(const StatsJob* jobs, int n);
void launch_stats_table(const StatsJob* dj, int n, uint64_t mm, uint64_t hb, bool walk, int phases, hipStream_t s,
                        const std::function<void()>& between = {});
// Many per-channel quantizers ([outer][C][K] tensors) with the whole updateStats (min/max, fold,
// histogram, fold) in TWO launches: every channel of every quantizer is one workgroup, and the
// fold of a channel needs only that channel's statistics, so it runs in the workgroup that
// produced them (stats.hip: launch_channel_stats_many).
struct ChannelJob
{
    const float* x;
    int64_t outer, C, K;
    TqDevice d;
    uint32_t block0;   // first workgroup (filled by launch_channel_stats_many)
    int32_t kind;      // StatsKind
    int32_t vec;       // 16-B aligned rows
};
void launch_channel_stats_many(std::vector<ChannelJob>& jobs, hipStream_t s);
// the same over a device job table (block0 filled: channel_layout), `blocks` channels in all
uint64_t channel_layout(std::vector<ChannelJob>& jobs, bool* any_hist);
void launch_channel_table(const ChannelJob* dj, int n, uint64_t blocks, bool any_hist, hipStream_t s);
// tfe_search.hip
// One quantizer's statistics and output; a batched search passes one job per quantizer.
struct TfeJob
{
    const int32_t* pdf_init;
    const float* hist_min;
    const double* bucket_size;
    const double* pdf;
    aimet_tf_encoding* out;
    int64_t start;   // first global channel of this job
};
// A TF-Enhanced search whose job table is already on the device (calibration plans, calib_plan.cpp):
// one launch, the results straight into each job's `out` (device-accessible memory: a plan points
// them into pinned host memory, so no copy follows the search)
struct TfeTable
{
    TfeJob first {};                 // jobs[0] (the kernel's by-value job)
    const TfeJob* dev = nullptr;     // every job, on the device
    int n = 0;
    int64_t total = 0;               // channels
    uint64_t* part = nullptr;        // split search: 2 * total * splits (tfe_splits)
    unsigned* tickets = nullptr;     // split search: `total` zeroed counters
    int per_cu = 0;                  // > 0: at most that many workgroups resident per CU (its work
                                     // beside an HBM-bound pass on another stream)
};
// workgroups per channel of a batched search of `total` channels (1: one workgroup per channel)
int tfe_splits(int64_t total, bool sym);
void launch_tfe_table(const TfeTable& t, int bw, bool sym, bool strict, bool unsign, hipStream_t s);
// d.enc[c] <- TF-Enhanced encoding of channel c (statistics updated; see aimet_tq_get_encoding)
void launch_tfe_search(const TqDevice& d, int64_t C, int bw, bool sym, bool strict, bool unsign, hipStream_t s);
// the same for n quantizers in one launch; host_out <- their encodings concatenated
// (sum of Cs). Synchronises s.
void launch_tfe_search_many(const TqDevice* const* ds, const int64_t* Cs, int n, int bw, bool sym, bool strict,
                            bool unsign, aimet_tf_encoding* host_out, hipStream_t s);
// the same, asynchronous: the encodings are copied into pinned_dst (host-pinned, sum of Cs entries)
// on s; the caller synchronises before reading it. `prep` (optional, another stream): the job
// table's upload runs there, so it is done before s reaches the search (s waits for prep's work
// enqueued so far) instead of adding a copy's latency between the statistics and the search
void launch_tfe_search_many_to(const TqDevice* const* ds, const int64_t* Cs, int n, int bw, bool sym, bool strict,
                               bool unsign, aimet_tf_encoding* pinned_dst, hipStream_t s, hipStream_t prep = nullptr);
// quantizer.cpp: `waiter` continues after everything enqueued on `from` so far (no host wait)
void stream_join(hipStream_t waiter, hipStream_t from);
// mse_search.hip: d.enc[c] <- MSE encoding of channel c (statistics updated)
size_t mse_part_bytes(int64_t C);
void launch_mse_search(const TqDevice& d, int64_t C, int bw, bool sym, bool strict, bool unsign, hipStream_t s);
// the same for n quantizers in one launch (+ one fold launch); pinned_dst (optional, host-pinned,
// sum of Cs entries): the encodings concatenated, copied there on s (the caller synchronises)
void launch_mse_search_many(const TqDevice* const* ds, const int64_t* Cs, int n, int bw, bool sym, bool strict,
                            bool unsign, hipStream_t s, aimet_tf_encoding* pinned_dst = nullptr);

// entropy_search.hip: the KL range of every channel of an 8-bit entropy getEncoding, written over
// the first 16 B per channel of d.enc (the quantizer's encoding scratch, 40 B per channel)
enum EntropyStatus
{
    kEntFinal  = 0,   // [lo, hi] is the reference's _optimizeKL range
    kEntHost   = 1,   // near-tie or non-finite range: the host search decides (glibc log)
    kEntNoHist = 2    // histogram never allocated: the unseen / all-zero encoding
};
struct EntropyRange
{
    float lo, hi;
    int32_t status;
    int32_t pad;
};
static_assert(sizeof(EntropyRange) <= sizeof(aimet_tf_encoding), "fits the encoding scratch");
inline EntropyRange* entropy_ranges(const TqDevice& d)
{
    return reinterpret_cast<EntropyRange*>(d.enc);
}
// A batched request's result per channel: the finished encoding (computed on the device from the
// KL range as entropy_encoding_from_range / unseen_or_zero do on the host) with the status in the
// encoding's tail padding, so that a block of them is copied into the caller's encodings as is
// (status kEntHost: the host search overwrites that channel)
struct EntropyOut
{
    double min, max, delta, offset;
    int32_t bw;
    int32_t status;
};
static_assert(sizeof(EntropyOut) == sizeof(aimet_tf_encoding) && offsetof(EntropyOut, bw) == offsetof(aimet_tf_encoding, bw),
              "an encoding with its status in the padding");
// pinned_dst (optional, host-pinned, sum of Cs entries): the finished encodings concatenated,
// copied there on s (bw: the request's bitwidth, 8)
void launch_entropy_search_many(const TqDevice* const* ds, const int64_t* Cs, int n, bool sym, bool strict, bool unsign,
                                hipStream_t s, EntropyOut* pinned_dst = nullptr, int bw = 8);

}   // namespace aimet_amd
