// tq_internal.hpp -- the aimet_tensor_quantizer object and the batched-encoding request, shared by
// quantizer.cpp (the per-call C-ABI) and calib_plan.cpp (calibration plans: the same launches with
// every job table built once). Not part of the public interface (include/aimet_amd.h).
#pragma once

#include <vector>

#include "tq_state.hpp"

struct Slab;

struct aimet_tensor_quantizer
{
    int scheme       = AIMET_QUANTIZATION_TF;
    int64_t C        = 1;
    int device       = 0;
    float percentile = 100.0f;   // PercentileEncodingAnalyzer.h:100
    bool stats_updated = false;  // AimetTensorQuantizer::_isEncodingValid / analyzer _statsUpdated
    bool hist        = false;    // histogram-based analyzer (TF-E, percentile, MSE, entropy)
    aimet_amd::StatsKind kind = aimet_amd::kKindTf;
    void* arena      = nullptr;
    size_t arena_bytes = 0;
    // quantizers made by aimet_tq_create_many share one allocation; the last one destroyed frees it
    Slab* slab = nullptr;
    aimet_amd::TqDevice d {};
};

// A batched getEncoding in flight: every device search enqueued on `stream`, the TF-Enhanced
// results on their way into a pinned block, `done` recorded after them.
struct aimet_encoding_request
{
    std::vector<aimet_tensor_quantizer*> qs;
    int32_t b  = 0;
    int sym    = 0, strict = 0, unsign = 0;
    int device = 0;
    hipStream_t stream = nullptr;   // where the search and its result copy were enqueued
    hipEvent_t done = nullptr;
    void* pinned    = nullptr;   // TF-Enhanced encodings, concatenated
    size_t pinned_bytes = 0;
    bool pinned_borrowed = false;   // a calibration plan's block: not returned to the pool
    int* busy = nullptr;            // a calibration plan's in-flight count, decremented on release
    std::vector<int64_t> tfe_offs, tfe_Cs;   // per TF-E quantizer: offset in `out`, channels
    // the MSE encodings and the entropy KL ranges of the device searches, copied into one pinned
    // block of their own (MSE encodings first, then the ranges); per quantizer its index in qs
    void* pinned_dev        = nullptr;
    size_t pinned_dev_bytes = 0;
    std::vector<int64_t> mse_q, ent_q;
    int64_t mse_total = 0;
};

namespace aimet_amd
{

struct DeviceGuard
{
    int prev = -1;
    explicit DeviceGuard(int dev)
    {
        AIMET_HIP_CHECK(hipGetDevice(&prev));
        if (prev != dev)
            AIMET_HIP_CHECK(hipSetDevice(dev));
    }
    ~DeviceGuard()
    {
        int cur = -1;
        if (hipGetDevice(&cur) == hipSuccess && cur != prev && prev >= 0)
            (void) hipSetDevice(prev);
    }
};

// jobs of a many-quantizer statistics call (per-tensor quantizers of one device)
std::vector<StatsJob> make_jobs(aimet_tensor_quantizer* const* qs, const float* const* xs, const int64_t* ns,
                                const int64_t* counts, int64_t count, const int64_t* counts_dev = nullptr);
// the job of one per-channel statistics update ([outer][C][K] tensor)
ChannelJob make_channel_job(aimet_tensor_quantizer* q, const float* x, int64_t outer, int64_t C, int64_t K);
// the device ranges resetEncodingStats clears and the running min/max it re-initialises. `light`:
// the PDF (and a per-channel quantizer's bin counts) are left as they are -- only for a reset that
// the same call follows with a full statistics update of the quantizer, which rewrites both
// wherever the PDF range gets set (the first batch's fold does not read the old PDF) and leaves
// them unread where it does not (pdf_init stays 0)
void reset_ranges(const aimet_tensor_quantizer* q, bool light, std::vector<ZeroJob>& zero,
                  std::vector<ResetJob>& resets);
// the host half of a reset (a fresh analyzer, AimetTensorQuantizer.cpp:89-96)
void mark_reset(aimet_tensor_quantizer* q);

bool device_search(const aimet_tensor_quantizer* q);
bool entropy_device(const aimet_tensor_quantizer* q, int32_t b);

// pinned result blocks and events of encoding requests (pooled)
void* take_pinned(size_t bytes, size_t* real);
hipEvent_t take_event();
void give_event(hipEvent_t e);
void release_request(aimet_encoding_request* r);
// the host's wait for an event it is about to read results behind: polls, then blocks (quantizer.cpp)
void await_event(hipEvent_t e);
void release_request_after_error(aimet_encoding_request* r);

// The device half of a batched getEncoding (throws; the caller releases `req` on failure): every
// device search enqueued on `st`, the TF-Enhanced ones from `tfe` when given (its quantizers must be
// exactly the stats-updated TF-Enhanced ones of qs, in order).
aimet_encoding_request* encodings_launch(aimet_tensor_quantizer* const* qs, int64_t nq, uint32_t bw, int sym,
                                         int strict, int unsign, hipStream_t st, aimet_encoding_request*& req,
                                         hipStream_t prep = nullptr, const TfeTable* tfe = nullptr);

}   // namespace aimet_amd
