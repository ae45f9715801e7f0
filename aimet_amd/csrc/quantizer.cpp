// quantizer.cpp -- aimet_tensor_quantizer: the AimetTensorQuantizer / TensorQuantizer object of the
// reference (AimetTensorQuantizer.cpp:79-315, TensorQuantizer.cpp:49-343) with its analyzer state
// held in HBM. One object carries the analyzers of all channels of a tensor (the reference
// allocates one C++ analyzer per channel and loops over channels in Python).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "encodings.hpp"
#include "tq_internal.hpp"

using namespace aimet_amd;

struct Slab
{
    void* base   = nullptr;
    size_t bytes = 0;
    std::atomic<int64_t> refs {0};
};

namespace
{

size_t align256(size_t b)
{
    return (b + 255) & ~size_t(255);
}

void layout(aimet_tensor_quantizer* q, bool assign)
{
    const int64_t C = q->C;
    size_t off      = 0;
    char* base      = static_cast<char*>(q->arena);
    auto take       = [&](size_t bytes) -> void* {
        void* p = assign ? base + off : nullptr;
        off += align256(bytes);
        return p;
    };
    q->d.minmax      = (float*) take(sizeof(float) * 2 * C);
    q->d.partials    = (float*) take(sizeof(float) * 2 * kMinmaxParts);
    q->d.acc         = (double*) take(sizeof(double) * 2 * C);
    q->d.pdf_init    = (int32_t*) take(sizeof(int32_t) * C);
    q->d.iterations  = (int32_t*) take(sizeof(int32_t) * C);
    q->d.hist_min    = (float*) take(sizeof(float) * C);
    q->d.bucket_size = (double*) take(sizeof(double) * C);
    q->d.bin_bucket  = (float*) take(sizeof(float) * C);
    q->d.bin_offset  = (float*) take(sizeof(float) * C);
    q->d.active      = (int32_t*) take(sizeof(int32_t) * C);
    if (q->hist)
    {
        q->d.pdf    = (double*) take(sizeof(double) * kPdfSize * C);
        q->d.counts = (unsigned long long*) take(sizeof(unsigned long long) * kPdfSize * C);
        q->d.enc    = (aimet_tf_encoding*) take(sizeof(aimet_tf_encoding) * C);
        q->d.search_part = q->scheme == AIMET_QUANTIZATION_MSE ? take(mse_part_bytes(C)) : nullptr;
    }
    else
    {
        q->d.pdf         = nullptr;
        q->d.counts      = nullptr;
        q->d.enc         = nullptr;
        q->d.search_part = nullptr;
    }
    q->arena_bytes = off;
}

bool in_arena(const aimet_tensor_quantizer* q, const void* p)
{
    auto b = static_cast<const char*>(q->arena), c = static_cast<const char*>(p);
    return c >= b && c < b + q->arena_bytes;
}

void reset_device_state(aimet_tensor_quantizer* q, hipStream_t s)
{
    AIMET_HIP_CHECK(hipMemsetAsync(q->arena, 0, q->arena_bytes, s));
    // exchange buffers bound outside the arena (aimet_tq_bind_exchange)
    if (q->d.minmax && !in_arena(q, q->d.minmax))
        AIMET_HIP_CHECK(hipMemsetAsync(q->d.minmax, 0, sizeof(float) * 2 * q->C, s));
    if (q->d.counts && !in_arena(q, q->d.counts))
        AIMET_HIP_CHECK(hipMemsetAsync(q->d.counts, 0, sizeof(unsigned long long) * kPdfSize * q->C, s));
    launch_reset_state(q->d, q->C, q->hist, s);
}

void check_shape(aimet_tensor_quantizer* q, int64_t outer, int64_t C, int64_t K)
{
    AIMET_REQUIRE(q != nullptr, "tensor quantizer is null");
    AIMET_REQUIRE(outer >= 0 && K >= 0, "invalid tensor shape");
    AIMET_REQUIRE(C == q->C, "channel count of the tensor (" + std::to_string(C) +
                                 ") does not match the quantizer (" + std::to_string(q->C) + ")");
}

template <class T>
std::vector<T> d2h(const T* dev, size_t n)
{
    std::vector<T> h(n);
    if (n)
        AIMET_HIP_CHECK(hipMemcpy(h.data(), dev, sizeof(T) * n, hipMemcpyDeviceToHost));
    return h;
}

template <class F>
void parallel_channels(int64_t C, F&& f, int64_t grain = 64)   // grain: fewest tasks worth a thread
{
    unsigned hw   = std::max(1u, std::thread::hardware_concurrency());
    int64_t nthr  = std::min<int64_t>({(int64_t) hw, 16, (C + grain - 1) / grain});
    if (nthr <= 1)
    {
        for (int64_t c = 0; c < C; ++c)
            f(c);
        return;
    }
    std::vector<std::thread> th;
    for (int64_t t = 0; t < nthr; ++t)
        th.emplace_back([&, t] {
            for (int64_t c = t; c < C; c += nthr)
                f(c);
        });
    for (auto& x: th)
        x.join();
}

// Released quantizer state is cached for reuse (as torch's caching allocator does) instead of
// hipDeviceSynchronize + hipFree at destruction: destroying a quantizer then never blocks the host
// nor breaks a HIP graph being captured on another stream, and a calibration that creates a
// model's quantizers again reuses the allocation. Work queued on any stream may still use a
// released block, so it is handed out again only after a device synchronisation (by the creating
// call, outside any capture). Blocks that do not fit are freed when an allocation misses.
struct StateCache
{
    struct Block
    {
        int device;
        void* p;
        size_t bytes;
    };
    std::mutex m;
    std::vector<Block> blocks;
};
StateCache& state_cache()
{
    static StateCache* c = new StateCache();   // never destroyed: blocks live until process exit
    return *c;
}

// device memory for quantizer state on the current device (the caller holds a DeviceGuard)
void* state_alloc(int device, size_t bytes)
{
    StateCache& c = state_cache();
    void* p       = nullptr;
    std::vector<void*> misfits;
    {
        std::lock_guard<std::mutex> lock(c.m);
        size_t best = (size_t) -1;
        for (size_t i = 0; i < c.blocks.size(); ++i)
        {
            const StateCache::Block& b = c.blocks[i];
            if (b.device == device && b.bytes >= bytes && b.bytes <= 2 * bytes &&
                (best == (size_t) -1 || b.bytes < c.blocks[best].bytes))
                best = i;
        }
        if (best != (size_t) -1)
        {
            p = c.blocks[best].p;
            c.blocks.erase(c.blocks.begin() + (std::ptrdiff_t) best);
        }
        else
            for (size_t i = 0; i < c.blocks.size();)
                if (c.blocks[i].device == device)
                {
                    misfits.push_back(c.blocks[i].p);
                    c.blocks.erase(c.blocks.begin() + (std::ptrdiff_t) i);
                }
                else
                    ++i;
    }
    if (p)
    {
        AIMET_HIP_CHECK(hipDeviceSynchronize());   // the previous owner's queued work is done
        return p;
    }
    for (void* m: misfits)
        AIMET_HIP_CHECK(hipFree(m));
    hipError_t e = hipMalloc(&p, bytes);
    if (e != hipSuccess)
        throw HipError(std::string("hipMalloc(tensor quantizer state): ") + hipGetErrorString(e));
    return p;
}

void state_release(int device, void* p, size_t bytes)
{
    StateCache& c = state_cache();
    std::lock_guard<std::mutex> lock(c.m);
    c.blocks.push_back(StateCache::Block {device, p, bytes});
}

aimet_tensor_quantizer* new_quantizer(int scheme, int64_t num_channels, int device)
{
    AIMET_REQUIRE(num_channels >= 1, "num_channels must be >= 1");
    if (scheme == AIMET_QUANTIZATION_RANGE_LEARNING)   // QuantizerFactory.cpp:93-96
        scheme = AIMET_QUANTIZATION_TF;
    AIMET_REQUIRE(scheme >= AIMET_QUANTIZATION_TF && scheme <= AIMET_QUANTIZATION_ENTROPY, "Unknown quant scheme");
    auto* q   = new aimet_tensor_quantizer();
    q->scheme = scheme;
    q->C      = num_channels;
    q->device = device;
    q->hist   = scheme != AIMET_QUANTIZATION_TF;
    q->kind   = scheme == AIMET_QUANTIZATION_TF ? kKindTf : scheme == AIMET_QUANTIZATION_ENTROPY ? kKindEntropy : kKindPdf;
    layout(q, false);
    return q;
}

// resetEncodingStats of many quantizers of one device in two launches (the zeroing of every state
// range, the running min/max re-initialised), no host synchronisation
void reset_many(aimet_tensor_quantizer* const* qs, int64_t nq, hipStream_t st)
{
    AIMET_REQUIRE(nq >= 0 && (qs != nullptr || nq == 0), "null argument");
    if (nq == 0)
        return;
    std::vector<ZeroJob> zero;
    std::vector<ResetJob> resets;
    for (int64_t i = 0; i < nq; ++i)
    {
        AIMET_REQUIRE(qs[i] != nullptr, "null quantizer");
        AIMET_REQUIRE(qs[i]->device == qs[0]->device, "quantizers of one batched reset share a device");
        reset_ranges(qs[i], false, zero, resets);
    }
    DeviceGuard g(qs[0]->device);
    launch_zero_many(zero, st);
    launch_reset_state_many(resets, st);
    for (int64_t i = 0; i < nq; ++i)
        mark_reset(qs[i]);
}

}   // namespace

void aimet_amd::reset_ranges(const aimet_tensor_quantizer* q, bool light, std::vector<ZeroJob>& zero,
                             std::vector<ResetJob>& resets)
{
    char* a = static_cast<char*>(q->arena);
    // layout(): the PDF, then the bin counts, then the encodings scratch, at the arena's end
    if (light && q->kind == kKindPdf && q->d.pdf && in_arena(q, q->d.pdf))
    {
        char* pdf = reinterpret_cast<char*>(q->d.pdf);
        zero.push_back(ZeroJob {a, (int64_t) (pdf - a)});
        // a per-channel quantizer's histogram writes every bin of a binned channel (no
        // accumulation); a per-tensor one adds into its counts, which must start at zero
        char* keep_end = (q->C > 1 && q->d.counts && in_arena(q, q->d.counts))
                             ? reinterpret_cast<char*>(q->d.counts) + align256(sizeof(unsigned long long) * kPdfSize * q->C)
                             : pdf + align256(sizeof(double) * kPdfSize * q->C);
        zero.push_back(ZeroJob {keep_end, (int64_t) (a + q->arena_bytes - keep_end)});
    }
    else
        zero.push_back(ZeroJob {a, (int64_t) q->arena_bytes});
    if (q->d.minmax && !in_arena(q, q->d.minmax))
        zero.push_back(ZeroJob {q->d.minmax, (int64_t) (sizeof(float) * 2 * q->C)});
    if (q->d.counts && !in_arena(q, q->d.counts))
        zero.push_back(ZeroJob {q->d.counts, (int64_t) (sizeof(unsigned long long) * kPdfSize * q->C)});
    resets.push_back(ResetJob {q->d.acc, q->C});
}

void aimet_amd::mark_reset(aimet_tensor_quantizer* q)
{
    q->stats_updated = false;
    q->percentile    = 100.0f;
}

extern "C" {

int aimet_tq_create_many(const int* schemes, const int64_t* num_channels, int64_t count, int device,
                         aimet_tensor_quantizer** out)
{
    return guarded([&] {
        AIMET_REQUIRE(count >= 0, "negative quantizer count");
        if (count == 0)
            return;
        AIMET_REQUIRE(schemes && num_channels && out, "null argument");
        std::vector<aimet_tensor_quantizer*> qs;
        std::vector<size_t> offs;
        size_t total = 0;
        try
        {
            for (int64_t i = 0; i < count; ++i)
            {
                qs.push_back(new_quantizer(schemes[i], num_channels[i], device));
                offs.push_back(total);
                total += align256(qs.back()->arena_bytes);
            }
        }
        catch (...)
        {
            for (auto* q: qs)
                delete q;
            throw;
        }
        DeviceGuard g(device);
        auto* sl = new Slab();
        try
        {
            sl->base = state_alloc(device, total);
        }
        catch (...)
        {
            delete sl;
            for (auto* q: qs)
                delete q;
            throw;
        }
        sl->bytes = total;
        sl->refs  = count;
        AIMET_HIP_CHECK(hipMemsetAsync(sl->base, 0, total, nullptr));
        std::vector<ResetJob> resets;
        for (int64_t i = 0; i < count; ++i)
        {
            aimet_tensor_quantizer* q = qs[(size_t) i];
            q->arena = static_cast<char*>(sl->base) + offs[(size_t) i];
            q->slab  = sl;
            layout(q, true);
            resets.push_back(ResetJob {q->d.acc, q->C});
            out[i] = q;
        }
        launch_reset_state_many(resets, nullptr);
        AIMET_HIP_CHECK(hipStreamSynchronize(nullptr));
    });
}

int aimet_tq_create(int scheme, int64_t num_channels, int device, aimet_tensor_quantizer** out)
{
    return guarded([&] {
        AIMET_REQUIRE(out != nullptr, "output handle is null");
        auto* q = new_quantizer(scheme, num_channels, device);
        DeviceGuard g(device);
        try
        {
            q->arena = static_cast<char*>(state_alloc(device, q->arena_bytes));
        }
        catch (...)
        {
            delete q;
            throw;
        }
        layout(q, true);
        reset_device_state(q, nullptr);
        AIMET_HIP_CHECK(hipStreamSynchronize(nullptr));
        *out = q;
    });
}

int aimet_tq_destroy(aimet_tensor_quantizer* q)
{
    return guarded([&] {
        if (!q)
            return;
        // the memory goes back to the state cache (no synchronisation here: see state_alloc)
        if (q->slab)
        {
            Slab* sl = q->slab;
            if (--sl->refs == 0)
            {
                state_release(q->device, sl->base, sl->bytes);
                delete sl;
            }
        }
        else if (q->arena)
            state_release(q->device, q->arena, q->arena_bytes);
        delete q;
    });
}

int aimet_tq_reset_encoding_stats(aimet_tensor_quantizer* q, void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(q != nullptr, "tensor quantizer is null");
        DeviceGuard g(q->device);
        reset_device_state(q, as_stream(stream));
        q->stats_updated = false;
        q->percentile    = 100.0f;   // a fresh analyzer (AimetTensorQuantizer.cpp:89-96)
    });
}

int aimet_tq_reset_encoding_stats_many(aimet_tensor_quantizer* const* qs, int64_t nq, void* stream)
{
    return guarded([&] { reset_many(qs, nq, as_stream(stream)); });
}

int aimet_tq_set_percentile_value(aimet_tensor_quantizer* q, float p)
{
    return guarded([&] {
        AIMET_REQUIRE(q != nullptr, "tensor quantizer is null");
        if (q->scheme == AIMET_QUANTIZATION_PERCENTILE)   // only for the percentile scheme
        {
            // PercentileEncodingAnalyzer.cpp setPercentileValue: valid range (0, 100]? The reference
            // asserts 50 <= p <= 100 in Python (v1/quantsim.py:1009) and not in C++.
            q->percentile = p;
        }
    });
}

int aimet_tq_get_percentile_value(aimet_tensor_quantizer* q, float* p)
{
    return guarded([&] {
        AIMET_REQUIRE(q != nullptr && p != nullptr, "null argument");
        if (q->scheme != AIMET_QUANTIZATION_PERCENTILE)
            throw RuntimeError("Percentile Value only exists in case of percentile quant scheme.");
        *p = q->percentile;
    });
}

int aimet_tq_batch_minmax(aimet_tensor_quantizer* q, const float* x, int64_t outer, int64_t C, int64_t K,
                          void* stream)
{
    return guarded([&] {
        check_shape(q, outer, C, K);
        if (outer * K > 0)
            require_device_ptr(x, "input");
        DeviceGuard g(q->device);
        launch_batch_minmax(q->d, x, outer, C, K, q->kind == kKindPdf ? 1 : 0, as_stream(stream));
        q->stats_updated = true;
    });
}

int aimet_tq_fold_minmax(aimet_tensor_quantizer* q, void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(q != nullptr, "tensor quantizer is null");
        DeviceGuard g(q->device);
        launch_fold_minmax(q->d, q->C, q->kind, as_stream(stream));
    });
}

int aimet_tq_batch_histogram(aimet_tensor_quantizer* q, const float* x, int64_t outer, int64_t C, int64_t K,
                             void* stream)
{
    return guarded([&] {
        check_shape(q, outer, C, K);
        if (!q->hist)
            return;
        if (outer * K > 0)
            require_device_ptr(x, "input");
        DeviceGuard g(q->device);
        launch_batch_histogram(q->d, x, outer, C, K, q->kind, as_stream(stream));
    });
}

int aimet_tq_fold_histogram(aimet_tensor_quantizer* q, int64_t count, void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(q != nullptr, "tensor quantizer is null");
        AIMET_REQUIRE(count >= 0, "negative element count");
        if (!q->hist)
            return;
        DeviceGuard g(q->device);
        launch_fold_histogram(q->d, q->C, count, q->kind, as_stream(stream));
    });
}

int aimet_tq_update_stats(aimet_tensor_quantizer* q, const float* x, int64_t outer, int64_t C, int64_t K,
                          void* stream)
{
    return guarded([&] {
        check_shape(q, outer, C, K);
        if (outer * K > 0)
            require_device_ptr(x, "input");
        DeviceGuard g(q->device);
        hipStream_t s = as_stream(stream);
        launch_batch_minmax(q->d, x, outer, C, K, q->kind == kKindPdf ? 1 : 0, s);
        launch_fold_minmax(q->d, q->C, q->kind, s);
        if (q->hist)
        {
            launch_batch_histogram(q->d, x, outer, C, K, q->kind, s);
            launch_fold_histogram(q->d, q->C, outer * K, q->kind, s);
        }
        q->stats_updated = true;
    });
}

}   // extern "C"

// jobs of a many-quantizer call: per-tensor quantizers of one device
std::vector<StatsJob> aimet_amd::make_jobs(aimet_tensor_quantizer* const* qs, const float* const* xs,
                                           const int64_t* ns, const int64_t* counts, int64_t count,
                                           const int64_t* counts_dev)
{
    AIMET_REQUIRE(qs != nullptr && count >= 0, "null argument");
    std::vector<StatsJob> jobs((size_t) count);
    for (int64_t i = 0; i < count; ++i)
    {
        aimet_tensor_quantizer* q = qs[i];
        AIMET_REQUIRE(q != nullptr, "tensor quantizer is null");
        AIMET_REQUIRE(q->C == 1, "the *_many entry points take per-tensor quantizers (num_channels == 1)");
        AIMET_REQUIRE(q->device == qs[0]->device, "quantizers of one *_many call share a device");
        StatsJob& j = jobs[(size_t) i];
        j.x         = xs ? xs[i] : nullptr;
        j.n         = ns ? ns[i] : 0;
        AIMET_REQUIRE(j.n >= 0, "negative element count");
        if (xs && j.n > 0)
            require_device_ptr(j.x, "input");
        j.count = counts ? counts[i] : j.n;
        AIMET_REQUIRE(j.count >= 0, "negative element count");
        j.count_dev = counts_dev ? counts_dev + i : nullptr;
        j.count_out = nullptr;
        j.d     = q->d;
        j.hist  = q->hist ? 1 : 0;
        j.ent   = q->kind == kKindEntropy ? 1 : 0;
        j.vec   = (reinterpret_cast<uintptr_t>(j.x) & 15) == 0 ? 1 : 0;
        j.seen  = q->stats_updated ? 1 : 0;
        j.fresh = 0;
    }
    return jobs;
}

ChannelJob aimet_amd::make_channel_job(aimet_tensor_quantizer* q, const float* x, int64_t outer, int64_t C, int64_t K)
{
    check_shape(q, outer, C, K);
    if (outer * K > 0)
        require_device_ptr(x, "input");
    ChannelJob j {};
    j.x     = x;
    j.outer = outer;
    j.C     = C;
    j.K     = K;
    j.d     = q->d;
    j.kind  = (int32_t) q->kind;
    j.vec   = ((reinterpret_cast<uintptr_t>(x) & 15) == 0 && K % 4 == 0) ? 1 : 0;
    return j;
}

namespace
{

// per-channel statistics of many quantizers (two launches): the jobs of updateStatsPerChannelMany
void channel_stats_many(aimet_tensor_quantizer* const* qs, const float* const* xs, const int64_t* outers,
                        const int64_t* Cs, const int64_t* Ks, int64_t count, hipStream_t st)
{
    AIMET_REQUIRE(count >= 0, "negative quantizer count");
    if (count == 0)
        return;
    AIMET_REQUIRE(qs && xs && outers && Cs && Ks, "null argument");
    std::vector<ChannelJob> jobs;
    jobs.reserve((size_t) count);
    for (int64_t i = 0; i < count; ++i)
    {
        aimet_tensor_quantizer* q = qs[i];
        AIMET_REQUIRE(q != nullptr, "tensor quantizer is null");
        AIMET_REQUIRE(q->device == qs[0]->device, "quantizers of one *_many call share a device");
        jobs.push_back(make_channel_job(q, xs[i], outers[i], Cs[i], Ks[i]));
    }
    DeviceGuard g(qs[0]->device);
    launch_channel_stats_many(jobs, st);
    for (int64_t i = 0; i < count; ++i)
        qs[i]->stats_updated = true;
}

int run_many(aimet_tensor_quantizer* const* qs, const float* const* xs, const int64_t* ns, const int64_t* counts,
             int64_t count, int phases, bool marks_updated, void* stream, const int64_t* counts_dev = nullptr)
{
    return guarded([&] {
        if (counts_dev)
            require_device_ptr(counts_dev, "element counts");
        auto jobs = make_jobs(qs, xs, ns, counts, count, counts_dev);
        if (jobs.empty())
            return;
        DeviceGuard g(qs[0]->device);
        launch_stats_many(jobs, phases, as_stream(stream));
        if (marks_updated)
            for (int64_t i = 0; i < count; ++i)
                qs[i]->stats_updated = true;
    });
}

}   // namespace

extern "C" {

int aimet_tq_update_stats_many(aimet_tensor_quantizer* const* qs, const float* const* xs, const int64_t* ns,
                               int64_t count, void* stream)
{
    return run_many(qs, xs, ns, nullptr, count,
                    kPhaseMinmax | kPhaseFoldMinmax | kPhaseHistogram | kPhaseFoldHistogram, true, stream);
}

int aimet_tq_batch_minmax_many(aimet_tensor_quantizer* const* qs, const float* const* xs, const int64_t* ns,
                               int64_t count, void* stream)
{
    return run_many(qs, xs, ns, nullptr, count, kPhaseMinmax, true, stream);
}

int aimet_tq_fold_minmax_many(aimet_tensor_quantizer* const* qs, int64_t count, void* stream)
{
    return run_many(qs, nullptr, nullptr, nullptr, count, kPhaseFoldMinmax, false, stream);
}

int aimet_tq_batch_histogram_many(aimet_tensor_quantizer* const* qs, const float* const* xs, const int64_t* ns,
                                  int64_t count, void* stream)
{
    return run_many(qs, xs, ns, nullptr, count, kPhaseHistogram, false, stream);
}

int aimet_tq_fold_histogram_many(aimet_tensor_quantizer* const* qs, const int64_t* counts, int64_t count,
                                 void* stream)
{
    if (counts == nullptr && count > 0)
        return guarded([] { AIMET_REQUIRE(false, "null element counts"); });
    return run_many(qs, nullptr, nullptr, counts, count, kPhaseFoldHistogram, false, stream);
}

int aimet_tq_fold_histogram_many_dev(aimet_tensor_quantizer* const* qs, const int64_t* counts_dev, int64_t count,
                                     void* stream)
{
    if (counts_dev == nullptr && count > 0)
        return guarded([] { AIMET_REQUIRE(false, "null element counts"); });
    return run_many(qs, nullptr, nullptr, nullptr, count, kPhaseFoldHistogram, false, stream, counts_dev);
}

int aimet_tq_update_stats_channels_many(aimet_tensor_quantizer* const* qs, const float* const* xs,
                                        const int64_t* outers, const int64_t* Cs, const int64_t* Ks, int64_t count,
                                        void* stream)
{
    return guarded([&] { channel_stats_many(qs, xs, outers, Cs, Ks, count, as_stream(stream)); });
}

int aimet_tq_minmax_buffer(aimet_tensor_quantizer* q, float** dev, int64_t* n)
{
    return guarded([&] {
        AIMET_REQUIRE(q && dev && n, "null argument");
        *dev = q->d.minmax;
        *n   = 2 * q->C;
    });
}

int aimet_tq_counts_buffer(aimet_tensor_quantizer* q, uint64_t** dev, int64_t* n)
{
    return guarded([&] {
        AIMET_REQUIRE(q && dev && n, "null argument");
        *dev = reinterpret_cast<uint64_t*>(q->d.counts);
        *n   = q->hist ? (int64_t) kPdfSize * q->C : 0;
    });
}

int aimet_tq_bind_exchange(aimet_tensor_quantizer* q, float* minmax, uint64_t* counts)
{
    return guarded([&] {
        AIMET_REQUIRE(q != nullptr, "tensor quantizer is null");
        require_device_ptr(minmax, "minmax exchange buffer");
        if (q->hist)
        {
            require_device_ptr(counts, "counts exchange buffer");
            q->d.counts = reinterpret_cast<unsigned long long*>(counts);
        }
        q->d.minmax = minmax;
    });
}

int aimet_tq_mark_stats_updated(aimet_tensor_quantizer* q)
{
    return guarded([&] {
        AIMET_REQUIRE(q != nullptr, "tensor quantizer is null");
        q->stats_updated = true;
    });
}

}   // extern "C"

bool aimet_amd::device_search(const aimet_tensor_quantizer* q)
{
    return q->hist && (q->scheme == AIMET_QUANTIZATION_TF_ENHANCED || q->scheme == AIMET_QUANTIZATION_MSE);
}

// the entropy KL search runs on the device for 8-bit encodings (the only width _optimizeKL
// searches; other widths take the histogram range as it is)
bool aimet_amd::entropy_device(const aimet_tensor_quantizer* q, int32_t b)
{
    return q->kind == kKindEntropy && b == 8;
}

extern "C" {

namespace
{

// getEncoding, part 1: enqueue the device-side search (TF-Enhanced, MSE, entropy) on the stream.
void launch_encoding(aimet_tensor_quantizer* q, int32_t b, int sym, int strict, int unsign, hipStream_t s)
{
    if (entropy_device(q, b))
    {
        const TqDevice* d = &q->d;
        launch_entropy_search_many(&d, &q->C, 1, sym != 0, strict != 0, unsign != 0, s);
        return;
    }
    if (!device_search(q))
        return;
    if (q->scheme == AIMET_QUANTIZATION_TF_ENHANCED)
        launch_tfe_search(q->d, q->C, b, sym, strict, unsign, s);
    else
        launch_mse_search(q->d, q->C, b, sym, strict, unsign, s);
}

// getEncoding, part 2 (stream already synchronised): read back the statistics of a quantizer whose
// encoding is finished on the host (TF, percentile, entropy); the device-searched ones (MSE) copy
// their encodings straight into `out`.
struct HostStats
{
    aimet_tensor_quantizer* q = nullptr;
    aimet_tf_encoding* out    = nullptr;
    std::vector<double> acc, bsz, pdf;
    std::vector<int32_t> init;
    std::vector<float> hmin;
    std::vector<EntropyRange> ent;   // device KL ranges (entropy, 8 bit)
    const EntropyOut* dev = nullptr; // or a batched request's finished encodings (already in out)
    bool host_search = false;        // some channel still needs the host KL search
    std::vector<int32_t> pdf_row;    // when only some rows were read back: channel -> row of pdf
    bool only_host(int64_t c) const  // the channels of `dev` the host finishes
    {
        return dev == nullptr || dev[c].status == kEntHost;
    }
    const double* pdf_of(int64_t c) const
    {
        return pdf.data() + kPdfSize * (pdf_row.empty() ? c : (int64_t) pdf_row[(size_t) c]);
    }
};

bool fetch_stats(aimet_tensor_quantizer* q, int32_t b, aimet_tf_encoding* out, HostStats& h,
                 const EntropyOut* dev = nullptr)
{
    const int64_t C = q->C;
    h.q   = q;
    h.out = out;
    if (entropy_device(q, b))
    {
        // a batched request's encodings arrive finished in its pinned block (only its kEntHost
        // channels are left); else the ranges are read back here
        h.dev = dev;
        if (dev == nullptr)
            h.ent = d2h(entropy_ranges(q->d), C);
        std::vector<int64_t> flagged;
        for (int64_t c = 0; c < C; ++c)
            if (dev ? dev[c].status == kEntHost : h.ent[(size_t) c].status == kEntHost)
                flagged.push_back(c);
        h.host_search = !flagged.empty();
        if (h.host_search)
        {
            // near-ties (or non-finite ranges) on some channel: its statistics for the glibc search
            // (a few flagged channels: their histogram rows only)
            h.init = d2h(q->d.pdf_init, C);
            h.acc  = d2h(q->d.acc, 2 * C);
            if ((int64_t) flagged.size() * 8 >= C)
                h.pdf = d2h(q->d.pdf, (size_t) kPdfSize * C);
            else
            {
                h.pdf.resize((size_t) kPdfSize * flagged.size());
                h.pdf_row.assign((size_t) C, 0);
                for (size_t k = 0; k < flagged.size(); ++k)
                {
                    h.pdf_row[(size_t) flagged[k]] = (int32_t) k;
                    AIMET_HIP_CHECK(hipMemcpy(h.pdf.data() + kPdfSize * k, q->d.pdf + kPdfSize * flagged[k],
                                              sizeof(double) * kPdfSize, hipMemcpyDeviceToHost));
                }
            }
        }
        return dev == nullptr || h.host_search;
    }
    if (!q->hist)
    {
        h.acc = d2h(q->d.acc, 2 * C);
        return true;
    }
    if (device_search(q))
    {
        // candidate search ran on the device (tfe_search.hip / mse_search.hip): only the
        // encodings come back
        AIMET_HIP_CHECK(hipMemcpy(out, q->d.enc, sizeof(aimet_tf_encoding) * C, hipMemcpyDeviceToHost));
        return false;
    }
    h.init = d2h(q->d.pdf_init, C);
    h.pdf  = d2h(q->d.pdf, (size_t) kPdfSize * C);
    if (q->kind == kKindEntropy)
        h.acc = d2h(q->d.acc, 2 * C);   // TensorProfilingParams {min, max}; the KL search runs here
    else
    {
        h.hmin = d2h(q->d.hist_min, C);
        h.bsz  = d2h(q->d.bucket_size, C);
    }
    return true;
}

void host_encoding(const HostStats& h, int64_t c, int32_t b, int sym, int strict, int unsign)
{
    const aimet_tensor_quantizer* q = h.q;
    if (!h.only_host(c))
        return;   // finished on the device, already in out
    if (!q->hist)
        h.out[c] = tf_encoding(h.acc[2 * c], h.acc[2 * c + 1], b, sym, strict, unsign);
    else if (!h.ent.empty() && h.ent[(size_t) c].status != kEntHost)
        h.out[c] = h.ent[(size_t) c].status == kEntFinal
                       ? entropy_encoding_from_range(h.ent[(size_t) c].lo, h.ent[(size_t) c].hi, b, sym, strict, unsign)
                       : entropy_encoding(false, true, 0.0, 0.0, nullptr, b, sym, strict, unsign);
    else if (q->kind == kKindEntropy)
        h.out[c] = entropy_encoding(h.init[c] != 0, true, h.acc[2 * c], h.acc[2 * c + 1], h.pdf_of(c), b, sym, strict,
                                    unsign);
    else
        h.out[c] = histogram_encoding(q->scheme, h.init[c] != 0, true, h.hmin[c], h.bsz[c], h.pdf.data() + kPdfSize * c,
                                      q->percentile, b, sym, strict, unsign);
}

// the host-finished encodings of every (quantizer, channel) in one thread pool: the entropy KL
// search is ~3 ms per channel, so a model's per-tensor entropy quantizers run in parallel too
void collect_encodings(aimet_tensor_quantizer* const* qs, aimet_tf_encoding* const* outs, int64_t n, int32_t b,
                       int sym, int strict, int unsign, const EntropyOut* const* dev = nullptr)
{
    std::vector<HostStats> hs;
    hs.reserve((size_t) n);
    for (int64_t i = 0; i < n; ++i)
    {
        HostStats h;
        if (fetch_stats(qs[i], b, outs[i], h, dev ? dev[i] : nullptr))
            hs.push_back(std::move(h));
    }
    std::vector<std::pair<int32_t, int64_t>> tasks;
    bool costly = false;   // the host entropy KL search: ~3 ms per channel, worth a thread each
    for (size_t k = 0; k < hs.size(); ++k)
    {
        costly = costly || (hs[k].q->kind == kKindEntropy && (hs[k].ent.empty() || hs[k].host_search));
        for (int64_t c = 0; c < hs[k].q->C; ++c)
            if (hs[k].only_host(c))
                tasks.emplace_back((int32_t) k, c);
    }
    parallel_channels(
        (int64_t) tasks.size(),
        [&](int64_t t) {
            host_encoding(hs[(size_t) tasks[(size_t) t].first], tasks[(size_t) t].second, b, sym, strict, unsign);
        },
        costly ? 1 : 64);
}

void collect_encoding(aimet_tensor_quantizer* q, int32_t b, int sym, int strict, int unsign, aimet_tf_encoding* out)
{
    collect_encodings(&q, &out, 1, b, sym, strict, unsign);
}

}   // namespace

int aimet_tq_get_encoding(aimet_tensor_quantizer* q, uint32_t bw, int sym, int strict, int unsign,
                          aimet_tf_encoding* out, int* valid, void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(q != nullptr && out != nullptr, "null argument");
        std::memset(out, 0, sizeof(aimet_tf_encoding) * q->C);
        if (valid)
            *valid = q->stats_updated ? 1 : 0;
        if (!q->stats_updated)
            return;   // AimetTensorQuantizer.cpp:185-189: encoding left default, valid = false
        DeviceGuard g(q->device);
        const int32_t b = (int32_t) (uint8_t) bw;   // computeEncoding(uint8_t bw, ...)
        launch_encoding(q, b, sym, strict, unsign, as_stream(stream));
        AIMET_HIP_CHECK(hipStreamSynchronize(as_stream(stream)));
        collect_encoding(q, b, sym, strict, unsign, out);
    });
}

}   // extern "C"

namespace
{

// pinned result blocks and events, reused across requests (two may be in flight at once: the
// parameters' on a side stream and the activations' on the main stream)
struct RequestPool
{
    std::mutex m;
    std::vector<std::pair<void*, size_t>> blocks;
    std::vector<hipEvent_t> events;
};
RequestPool& request_pool()
{
    static RequestPool* p = new RequestPool;   // outlives static destruction (no HIP calls at exit)
    return *p;
}

}   // namespace

void* aimet_amd::take_pinned(size_t bytes, size_t* real)
{
    RequestPool& p = request_pool();
    {
        std::lock_guard<std::mutex> lock(p.m);
        size_t best = p.blocks.size();
        for (size_t i = 0; i < p.blocks.size(); ++i)
            if (p.blocks[i].second >= bytes && (best == p.blocks.size() || p.blocks[i].second < p.blocks[best].second))
                best = i;
        if (best != p.blocks.size())
        {
            auto blk = p.blocks[best];
            p.blocks.erase(p.blocks.begin() + (std::ptrdiff_t) best);
            *real = blk.second;
            return blk.first;
        }
    }
    void* ptr = nullptr;
    AIMET_HIP_CHECK(hipHostMalloc(&ptr, bytes, hipHostMallocDefault));
    *real = bytes;
    return ptr;
}

hipEvent_t aimet_amd::take_event()
{
    RequestPool& p = request_pool();
    {
        std::lock_guard<std::mutex> lock(p.m);
        if (!p.events.empty())
        {
            hipEvent_t e = p.events.back();
            p.events.pop_back();
            return e;
        }
    }
    hipEvent_t e = nullptr;
    AIMET_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    return e;
}

void aimet_amd::give_event(hipEvent_t e)
{
    if (e == nullptr)
        return;
    RequestPool& p = request_pool();
    std::lock_guard<std::mutex> lock(p.m);
    p.events.push_back(e);
}

void aimet_amd::release_request(aimet_encoding_request* r)
{
    if (r == nullptr)
        return;
    RequestPool& p = request_pool();
    {
        std::lock_guard<std::mutex> lock(p.m);
        if (r->pinned && !r->pinned_borrowed)
            p.blocks.emplace_back(r->pinned, r->pinned_bytes);
        if (r->pinned_dev)
            p.blocks.emplace_back(r->pinned_dev, r->pinned_dev_bytes);
        if (r->done)
            p.events.push_back(r->done);
    }
    if (r->busy)
        --*r->busy;   // the plan may launch again (its pinned block is idle: the request was waited for)
    delete r;
}

// release on an error path: the request's result copy may already be queued into its pinned block,
// so the block goes back to the pool only after the stream has drained (else the next take_pinned
// could hand it out while the copy still writes into it)
void aimet_amd::release_request_after_error(aimet_encoding_request* r)
{
    if (r == nullptr)
        return;
    if (r->pinned || r->pinned_dev)
    {
        DeviceGuard g(r->device);
        if (hipStreamSynchronize(r->stream) != hipSuccess)
        {
            // the stream is broken: leak the block rather than risk a live copy into a reused one
            // (a plan's block: the plan keeps counting the request as in flight, so it never
            // launches into that block again)
            r->pinned     = nullptr;
            r->pinned_dev = nullptr;
            r->busy       = nullptr;
            (void) hipGetLastError();
        }
    }
    release_request(r);
}

// The device half of a batched getEncoding (throws; the caller releases `req` on failure): every
// TF-Enhanced search in ONE launch (one workgroup per channel of every quantizer), results back in
// one copy (a plan's table: written by the search into its pinned block); the MSE / entropy
// searches enqueued beside it; the other schemes read back their statistics when the request is
// finished.
aimet_encoding_request* aimet_amd::encodings_launch(aimet_tensor_quantizer* const* qs, int64_t nq, uint32_t bw,
                                                    int sym, int strict, int unsign, hipStream_t st,
                                                    aimet_encoding_request*& req, hipStream_t prep,
                                                    const TfeTable* table)
{
    AIMET_REQUIRE(nq >= 0 && (qs != nullptr || nq == 0), "null argument");
    for (int64_t i = 0; i < nq; ++i)
    {
        AIMET_REQUIRE(qs[i] != nullptr, "null quantizer");
        AIMET_REQUIRE(qs[i]->device == qs[0]->device, "quantizers of one batched getEncoding share a device");
    }
    req         = new aimet_encoding_request;
    req->qs.assign(qs, qs + nq);
    req->b      = (int32_t) (uint8_t) bw;   // computeEncoding(uint8_t bw, ...)
    req->sym    = sym;
    req->strict = strict;
    req->unsign = unsign;
    if (nq == 0)
        return req;
    req->device = qs[0]->device;
    req->stream = st;
    DeviceGuard g(req->device);
    const int32_t b = req->b;
    std::vector<const TqDevice*> tfe, ent, mse;
    std::vector<int64_t> entC, mseC;
    int64_t off = 0, tfe_total = 0;
    for (int64_t i = 0; i < nq; ++i)
    {
        aimet_tensor_quantizer* q = qs[i];
        if (q->stats_updated && q->hist && q->scheme == AIMET_QUANTIZATION_TF_ENHANCED)
        {
            tfe.push_back(&q->d);
            req->tfe_Cs.push_back(q->C);
            req->tfe_offs.push_back(off);
            tfe_total += q->C;
        }
        else if (q->stats_updated && entropy_device(q, b))
        {
            ent.push_back(&q->d);
            entC.push_back(q->C);
            req->ent_q.push_back(i);
        }
        else if (q->stats_updated && q->hist && q->scheme == AIMET_QUANTIZATION_MSE)
        {
            mse.push_back(&q->d);
            mseC.push_back(q->C);
            req->mse_q.push_back(i);
            req->mse_total += q->C;
        }
        off += q->C;
    }
    // the MSE encodings and the entropy ranges come back in one pinned block (two copies enqueued
    // behind the searches), not in a synchronous copy per quantizer when the request is finished
    int64_t ent_total = 0;
    for (int64_t c: entC)
        ent_total += c;
    aimet_tf_encoding* mse_dst = nullptr;
    EntropyOut* ent_dst        = nullptr;
    if (req->mse_total + ent_total > 0)
    {
        const size_t mse_bytes = sizeof(aimet_tf_encoding) * (size_t) req->mse_total;
        req->pinned_dev = take_pinned(mse_bytes + sizeof(EntropyOut) * (size_t) ent_total, &req->pinned_dev_bytes);
        mse_dst         = req->mse_total ? static_cast<aimet_tf_encoding*>(req->pinned_dev) : nullptr;
        ent_dst = ent_total ? reinterpret_cast<EntropyOut*>(static_cast<char*>(req->pinned_dev) + mse_bytes) : nullptr;
    }
    launch_mse_search_many(mse.data(), mseC.data(), (int) mse.size(), b, sym != 0, strict != 0, unsign != 0, st,
                           mse_dst);
    launch_entropy_search_many(ent.data(), entC.data(), (int) ent.size(), sym != 0, strict != 0, unsign != 0, st,
                               ent_dst, b);
    if (tfe_total > 0 && table != nullptr)
    {
        AIMET_REQUIRE(table->total == tfe_total && table->n == (int) tfe.size(),
                      "calibration plan: the TF-Enhanced search table does not match the quantizers");
        launch_tfe_table(*table, b, sym != 0, strict != 0, unsign != 0, st);
    }
    else if (tfe_total > 0)
    {
        req->pinned = take_pinned(sizeof(aimet_tf_encoding) * (size_t) tfe_total, &req->pinned_bytes);
        launch_tfe_search_many_to(tfe.data(), req->tfe_Cs.data(), (int) tfe.size(), b, sym, strict, unsign,
                                  static_cast<aimet_tf_encoding*>(req->pinned), st, prep);
    }
    req->done = take_event();
    AIMET_HIP_CHECK(hipEventRecord(req->done, st));
    return req;
}

// The host waits for a request's device work by polling its event: the caller is about to read the
// results (a calibration's last step), and hipEventSynchronize's wake-up after the kernel has ended
// was measured at up to ~0.25 ms in some processes (profiles/r05/README.md), 6 % of a ResNet-50
// compute_encodings. After 20 ms of polling the blocking wait takes over (a long device queue).
// The first 200 us poll back to back; after that each poll is followed by a 20 us sleep, so a wait
// that several ranks (or loader threads) share a host with does not hold a core at 100 %.
void aimet_amd::await_event(hipEvent_t e)
{
    const auto t0 = std::chrono::steady_clock::now();
    for (;;)
    {
        const hipError_t q = hipEventQuery(e);
        if (q == hipSuccess)
            return;
        if (q != hipErrorNotReady)
            AIMET_HIP_CHECK(q);
        const auto waited = std::chrono::steady_clock::now() - t0;
        if (waited > std::chrono::milliseconds(20))
            break;
        if (waited > std::chrono::microseconds(200))
            std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    AIMET_HIP_CHECK(hipEventSynchronize(e));
}

// `waiter` continues after everything enqueued on `from` so far (a pooled event, no host wait)
void aimet_amd::stream_join(hipStream_t waiter, hipStream_t from)
{
    hipEvent_t e = take_event();
    RequestPool& p = request_pool();
    try
    {
        AIMET_HIP_CHECK(hipEventRecord(e, from));
        AIMET_HIP_CHECK(hipStreamWaitEvent(waiter, e, 0));
    }
    catch (...)
    {
        std::lock_guard<std::mutex> lock(p.m);
        p.events.push_back(e);
        throw;
    }
    std::lock_guard<std::mutex> lock(p.m);
    p.events.push_back(e);   // a later record does not affect the wait already enqueued
}

extern "C" {

int aimet_tq_get_encodings_launch(aimet_tensor_quantizer* const* qs, int64_t nq, uint32_t bw, int sym, int strict,
                                  int unsign, void* stream, aimet_encoding_request** req_out)
{
    aimet_encoding_request* req = nullptr;
    const int rc = guarded([&] {
        AIMET_REQUIRE(req_out != nullptr, "null argument");
        *req_out = nullptr;
        encodings_launch(qs, nq, bw, sym, strict, unsign, as_stream(stream), req);
    });
    if (rc != AIMET_OK)
    {
        release_request_after_error(req);
        return rc;
    }
    *req_out = req;
    return rc;
}

int aimet_calibrate_launch(aimet_tensor_quantizer* const* act_qs, const float* const* act_x, const int64_t* act_n,
                           int64_t n_act, aimet_tensor_quantizer* const* par_qs, const float* const* par_x,
                           const int64_t* par_outer, const int64_t* par_C, const int64_t* par_K, int64_t n_par,
                           const int32_t* act_settings, const int32_t* par_settings, int reset, void* main_stream,
                           void* side_stream, aimet_encoding_request** act_req, aimet_encoding_request** par_req)
{
    aimet_encoding_request *ra = nullptr, *rp = nullptr;
    const int rc = guarded([&] {
        AIMET_REQUIRE(act_req != nullptr && par_req != nullptr && act_settings != nullptr && par_settings != nullptr,
                      "null argument");
        AIMET_REQUIRE(n_act >= 0 && n_par >= 0, "negative quantizer count");
        *act_req = *par_req = nullptr;
        const int dev = n_act ? act_qs[0]->device : (n_par ? par_qs[0]->device : -1);
        for (int64_t i = 0; i < n_par; ++i)
            AIMET_REQUIRE(par_qs[i] != nullptr && par_qs[i]->device == dev, "quantizers of one calibration share a device");
        hipStream_t ms = as_stream(main_stream), ss = as_stream(side_stream);
        if (dev < 0)
            return;
        DeviceGuard g(dev);
        // the parameters' stream starts after everything already queued on the main stream (the
        // inputs are ordered there), before the activation passes are added to it
        if (n_par && ss != ms)
            stream_join(ss, ms);
        // enqueued right after the activations' min/max pass (launch_stats_many's `between`), so that
        // pass starts at once: the resets (the activations' ones joined back into the main stream
        // before the pass's combine / fold; the pass itself treats the quantizers as reset,
        // StatsJob::fresh), then the parameters' statistics and search, run on the high-priority
        // parameters' stream beside the activation passes (aimet_amd/calibration.py)
        auto rest = [&] {
            if (reset && n_act)
            {
                // on the parameters' stream, beside the min/max pass (it treats the quantizers as
                // reset already): the main stream waits for it before the pass's combine / fold
                reset_many(act_qs, n_act, ss);
                if (ss != ms)
                    stream_join(ms, ss);
            }
            if (n_par)
            {
                if (reset)
                    reset_many(par_qs, n_par, ss);
                channel_stats_many(par_qs, par_x, par_outer, par_C, par_K, n_par, ss);
                encodings_launch(par_qs, n_par, (uint32_t) par_settings[0], par_settings[1], par_settings[2],
                                 par_settings[3], ss, rp);
            }
        };
        if (n_act)
        {
            auto jobs = make_jobs(act_qs, act_x, act_n, nullptr, n_act);
            if (reset)
                for (auto& j: jobs)
                {
                    j.fresh = 1;
                    j.seen  = 0;
                }
            launch_stats_many(jobs, kPhaseMinmax | kPhaseFoldMinmax | kPhaseHistogram | kPhaseFoldHistogram, ms,
                              rest);
            for (int64_t i = 0; i < n_act; ++i)
                act_qs[i]->stats_updated = true;
        }
        else
            rest();
        // the search's job table goes up on the main stream itself: on the parameters' stream it
        // would sit behind all of their work, and the join would make the search wait for that
        // work (a calibration plan, calib_plan.cpp, has no upload at all)
        encodings_launch(act_qs, n_act, (uint32_t) act_settings[0], act_settings[1], act_settings[2],
                         act_settings[3], ms, ra);
        if (n_par && ss != ms)
            stream_join(ms, ss);   // later work on the main stream sees the parameters' state too
    });
    if (rc != AIMET_OK)
    {
        release_request_after_error(ra);
        release_request_after_error(rp);
        return rc;
    }
    *act_req = ra;
    *par_req = rp;
    return rc;
}

int aimet_tq_get_encodings_finish(aimet_encoding_request* req, aimet_tf_encoding* out, int* valid)
{
    const int rc = guarded([&] {
        AIMET_REQUIRE(req != nullptr, "request is null");
        const int64_t nq = (int64_t) req->qs.size();
        if (out == nullptr && valid == nullptr)
        {
            // discard: the request's result copy may still be writing into its pinned block, which
            // goes back to the pool below -- wait for the request's device work first
            if (nq && req->done)
            {
                DeviceGuard g(req->device);
                AIMET_HIP_CHECK(hipEventSynchronize(req->done));
            }
            return;
        }
        int64_t total = 0;
        for (aimet_tensor_quantizer* q: req->qs)
            total += q->C;
        AIMET_REQUIRE(out != nullptr || total == 0, "out is null");
        if (total)
            std::memset(out, 0, sizeof(aimet_tf_encoding) * total);
        for (int64_t i = 0; i < nq; ++i)
            if (valid)
                valid[i] = req->qs[i]->stats_updated ? 1 : 0;
        if (nq == 0)
            return;
        DeviceGuard g(req->device);
        await_event(req->done);
        auto* tfe = static_cast<const aimet_tf_encoding*>(req->pinned);
        for (size_t k = 0, src = 0; k < req->tfe_Cs.size(); src += req->tfe_Cs[k], ++k)
            std::memcpy(out + req->tfe_offs[k], tfe + src, sizeof(aimet_tf_encoding) * req->tfe_Cs[k]);
        // the device-searched MSE and entropy encodings, from the request's pinned block
        std::vector<int64_t> offs((size_t) nq);
        for (int64_t i = 0, o = 0; i < nq; o += req->qs[(size_t) i]->C, ++i)
            offs[(size_t) i] = o;
        std::vector<char> from_pinned((size_t) nq, 0);
        std::vector<const EntropyOut*> dev((size_t) nq, nullptr);
        {
            auto* m = static_cast<const aimet_tf_encoding*>(req->pinned_dev);
            for (int64_t i: req->mse_q)
            {
                const int64_t C = req->qs[(size_t) i]->C;
                std::memcpy(out + offs[(size_t) i], m, sizeof(aimet_tf_encoding) * C);
                m += C;
                from_pinned[(size_t) i] = 1;
            }
            auto* r = reinterpret_cast<const EntropyOut*>(static_cast<const char*>(req->pinned_dev) +
                                                          sizeof(aimet_tf_encoding) * (size_t) req->mse_total);
            for (int64_t i: req->ent_q)
            {
                // every channel's encoding as the device finished it; the host search then
                // overwrites the flagged (kEntHost) ones
                const int64_t C = req->qs[(size_t) i]->C;
                aimet_tf_encoding* o = out + offs[(size_t) i];
                bool flagged = false;
                for (int64_t c = 0; c < C; ++c)
                {
                    o[c]    = aimet_tf_encoding {r[c].min, r[c].max, r[c].delta, r[c].offset, r[c].bw};
                    flagged = flagged || r[c].status == kEntHost;
                }
                dev[(size_t) i]         = r;
                from_pinned[(size_t) i] = flagged ? 0 : 1;
                r += C;
            }
        }
        std::vector<aimet_tensor_quantizer*> host_q;
        std::vector<aimet_tf_encoding*> host_out;
        std::vector<const EntropyOut*> host_dev;
        for (int64_t i = 0; i < nq; ++i)
        {
            aimet_tensor_quantizer* q = req->qs[(size_t) i];
            if (q->stats_updated && !(q->hist && q->scheme == AIMET_QUANTIZATION_TF_ENHANCED) && !from_pinned[(size_t) i])
            {
                host_q.push_back(q);
                host_out.push_back(out + offs[(size_t) i]);
                host_dev.push_back(dev[(size_t) i]);
            }
        }
        collect_encodings(host_q.data(), host_out.data(), (int64_t) host_q.size(), req->b, req->sym, req->strict,
                          req->unsign, host_dev.data());
    });
    if (rc != AIMET_OK)
        release_request_after_error(req);   // the copy may not have been waited for
    else
        release_request(req);
    return rc;
}

int aimet_tq_get_encodings(aimet_tensor_quantizer* const* qs, int64_t nq, uint32_t bw, int sym, int strict,
                           int unsign, aimet_tf_encoding* out, int* valid, void* stream)
{
    if (out == nullptr && valid == nullptr && nq > 0)
        return guarded([] { AIMET_REQUIRE(false, "out is null"); });   // not a discard here
    aimet_encoding_request* req = nullptr;
    const int rc = aimet_tq_get_encodings_launch(qs, nq, bw, sym, strict, unsign, stream, &req);
    if (rc != AIMET_OK)
        return rc;
    return aimet_tq_get_encodings_finish(req, out, valid);
}

int aimet_tq_get_stats_histogram(aimet_tensor_quantizer* q, int64_t channel, double* xleft, double* pdf, int* n,
                                 void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(q != nullptr && xleft != nullptr && pdf != nullptr && n != nullptr, "null argument");
        AIMET_REQUIRE(channel >= 0 && channel < q->C, "channel out of range");
        if (!q->hist)
            throw RuntimeError("the TF encoding analyzer keeps no histogram (TfEncodingAnalyzer.cpp:53-57)");
        if (q->kind == kKindEntropy)   // EntropyEncodingAnalyzer.cpp:56-78 returns a malformed PDF
            throw RuntimeError("getStatsHistogram is only defined for the PDF analyzers (TF-Enhanced, percentile, "
                               "MSE); v1/tensor_quantizer.py:366 allows it for TF-Enhanced only");
        DeviceGuard g(q->device);
        AIMET_HIP_CHECK(hipStreamSynchronize(as_stream(stream)));
        int32_t init = 0;
        AIMET_HIP_CHECK(hipMemcpy(&init, q->d.pdf_init + channel, sizeof(int32_t), hipMemcpyDeviceToHost));
        *n = 0;
        if (!init)
            return;
        float hmin = 0;
        double bs  = 0;
        AIMET_HIP_CHECK(hipMemcpy(&hmin, q->d.hist_min + channel, sizeof(float), hipMemcpyDeviceToHost));
        AIMET_HIP_CHECK(hipMemcpy(&bs, q->d.bucket_size + channel, sizeof(double), hipMemcpyDeviceToHost));
        AIMET_HIP_CHECK(hipMemcpy(pdf, q->d.pdf + kPdfSize * channel, sizeof(double) * kPdfSize,
                                  hipMemcpyDeviceToHost));
        histogram_xleft(hmin, bs, xleft);
        *n = kPdfSize;
    });
}

int aimet_tq_get_entropy_state(aimet_tensor_quantizer* q, int64_t channel, double* minmax, double* hist,
                               int* has_hist, int* iterations, void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(q && minmax && hist && has_hist && iterations, "null argument");
        AIMET_REQUIRE(channel >= 0 && channel < q->C, "channel out of range");
        AIMET_REQUIRE(q->kind == kKindEntropy, "not an entropy quantizer");
        DeviceGuard g(q->device);
        AIMET_HIP_CHECK(hipStreamSynchronize(as_stream(stream)));
        int32_t init = 0, it = 0;
        AIMET_HIP_CHECK(hipMemcpy(&init, q->d.pdf_init + channel, sizeof(int32_t), hipMemcpyDeviceToHost));
        AIMET_HIP_CHECK(hipMemcpy(&it, q->d.iterations + channel, sizeof(int32_t), hipMemcpyDeviceToHost));
        AIMET_HIP_CHECK(hipMemcpy(minmax, q->d.acc + 2 * channel, 2 * sizeof(double), hipMemcpyDeviceToHost));
        AIMET_HIP_CHECK(hipMemcpy(hist, q->d.pdf + kPdfSize * channel, kPdfSize * sizeof(double),
                                  hipMemcpyDeviceToHost));
        if (!init)   // a value-initialised TensorProfilingParams (the TF reset values live there)
            minmax[0] = minmax[1] = 0.0;
        *has_hist   = init;
        *iterations = it;
    });
}

int aimet_tq_num_channels(aimet_tensor_quantizer* q, int64_t* c)
{
    return guarded([&] {
        AIMET_REQUIRE(q && c, "null argument");
        *c = q->C;
    });
}

int aimet_tq_quant_scheme(aimet_tensor_quantizer* q, int* s)
{
    return guarded([&] {
        AIMET_REQUIRE(q && s, "null argument");
        *s = q->scheme;
    });
}

}   // extern "C"
