// calib_plan.cpp -- calibration plans: QuantizationSimModel.compute_encodings' work for a fixed
// set of quantizers and resident tensors (v1/quantsim.py:381-449: resetEncodingStats, updateStats
// of every quantizer, getEncoding of every quantizer), prepared once and launched many times.
//
// aimet_calibrate_launch builds and uploads every job table (statistics jobs, the parameters'
// channel jobs, the reset ranges, the TF-Enhanced search tables) on every call and copies the
// search results back after the search; a compute_encodings of ResNet-50's 109 quantizers spent
// ~170 us on the host before its first launch (profiles/r04/enc_timeline_api_after.txt). A plan
// keeps all of them in one device allocation made at creation, the per-tile min/max partials and
// the split search's hand-off buffers too, and the TF-Enhanced searches write their encodings
// straight into the plan's pinned host blocks: a launch is only kernel launches and stream joins.
//
// The same plan runs the sharded calibration in three stages with the caller's
// collectives between them (aimet_amd/distributed.py binds the packed exchange buffers first):
//   stage 1: resets, the parameters' statistics + search (side stream), the activations' min/max
//            pass -> {-min, max} per quantizer, and each rank's element counts into the packed
//            SUM buffer's tail                                          [all_reduce MAX]
//   stage 2: the PDF ranges from the global min/max + the histogram pass   [all_reduce SUM]
//   stage 4: the PDF fold with the global element counts + the activations' search
// stages = 7 is the single-device form (the fold fused into the min/max combine).
#include <algorithm>
#include <cstring>
#include <mutex>
#include <vector>

#include "tq_internal.hpp"

using namespace aimet_amd;

struct aimet_calib_plan
{
    int device = 0;
    std::vector<aimet_tensor_quantizer*> aq, pq;
    int32_t aset[4] = {}, pset[4] = {};
    // activations: statistics jobs (as reset / as continuing), their host copy for the walk rule
    std::vector<StatsJob> jobs;
    uint64_t mm = 0, hb = 0;
    StatsJob* dj_fresh = nullptr;
    StatsJob* dj_cont  = nullptr;
    bool all_pdf       = false;   // every activation quantizer is a PDF (non-entropy) scheme
    // reset tables (activations: the whole state; parameters: light, see reset_ranges)
    ZeroJob* dz_act  = nullptr;
    int nz_act       = 0;
    int64_t most_act = 0;
    ResetJob* dr_act = nullptr;
    ZeroJob* dz_par  = nullptr;
    int nz_par       = 0;
    int64_t most_par = 0;
    ResetJob* dr_par = nullptr;
    // parameters: channel statistics jobs
    ChannelJob* dch   = nullptr;
    uint64_t ch_blocks = 0;
    bool ch_hist      = false;
    // TF-Enhanced search tables (results into the pinned blocks)
    TfeTable tfe_act {}, tfe_par {};
    bool has_tfe_act = false, has_tfe_par = false;
    void* pinned_act = nullptr;
    void* pinned_par = nullptr;
    size_t pinned_act_bytes = 0, pinned_par_bytes = 0;
    int busy_act = 0, busy_par = 0;   // requests in flight (their pinned block is being written)
    void* dev_block = nullptr;        // every device table above
    hipEvent_t done = nullptr;        // recorded on the main stream after every launch
};

namespace
{

// The parameters' TF-Enhanced search runs beside the activations' min/max pass (another stream). At
// its own occupancy (~10 two-wave workgroups per CU) it held the wave slots the HBM-bound pass needs
// to keep its loads in flight: the pass took ~0.22 ms longer (profiles/r05/enc_plan_runs_c.jsonl:
// 3.70 vs 3.48 ms without the parameters). Held to a few workgroups per CU, it takes longer itself
// but finishes (and the host builds the 27,560 encodings) long before the activations' passes end.
constexpr int kParamSearchPerCu = 2;

// one device allocation holding many tables: offsets first, then one upload
struct Packer
{
    std::vector<unsigned char> host;
    size_t add(const void* p, size_t bytes)
    {
        const size_t off = (host.size() + 255) & ~size_t(255);
        host.resize(off + bytes);
        if (bytes && p)
            std::memcpy(host.data() + off, p, bytes);   // null: zero-filled space (e.g. tickets)
        return off;
    }
};

bool tfe_searched(const aimet_tensor_quantizer* q)
{
    return q->hist && q->scheme == AIMET_QUANTIZATION_TF_ENHANCED;
}

// the TF-E jobs of `qs` (in order), their outputs at `out` + the job's first channel
std::vector<TfeJob> tfe_jobs(const std::vector<aimet_tensor_quantizer*>& qs, int64_t* total)
{
    std::vector<TfeJob> jobs;
    int64_t t = 0;
    for (aimet_tensor_quantizer* q: qs)
        if (tfe_searched(q))
        {
            jobs.push_back(TfeJob {q->d.pdf_init, q->d.hist_min, q->d.bucket_size, q->d.pdf, nullptr, t});
            t += q->C;
        }
    *total = t;
    return jobs;
}

// Memory of destroyed plans, freed once the event recorded after their last launch has completed:
// destroying a plan (possibly from a garbage collection while another stream is being captured
// into a HIP graph) neither synchronises the device nor frees memory kernels may still read. The
// blocks are reaped when a plan is created (outside any capture).
struct DeadPlan
{
    int device;
    void* dev_block;
    void* pinned_act;
    void* pinned_par;
    hipEvent_t done;
};
struct Graveyard
{
    std::mutex m;
    std::vector<DeadPlan> items;
};
Graveyard& graveyard()
{
    static Graveyard* g = new Graveyard();   // never destroyed: reaped while the process runs
    return *g;
}

void reap_dead_plans()
{
    std::vector<DeadPlan> ready;
    {
        Graveyard& g = graveyard();
        std::lock_guard<std::mutex> lock(g.m);
        for (size_t i = 0; i < g.items.size();)
            if (g.items[i].done == nullptr || hipEventQuery(g.items[i].done) == hipSuccess)
            {
                ready.push_back(g.items[i]);
                g.items.erase(g.items.begin() + (std::ptrdiff_t) i);
            }
            else
                ++i;
    }
    for (const DeadPlan& d: ready)
    {
        DeviceGuard guard(d.device);
        if (d.dev_block)
            (void) hipFree(d.dev_block);
        if (d.pinned_act)
            (void) hipHostFree(d.pinned_act);
        if (d.pinned_par)
            (void) hipHostFree(d.pinned_par);
        if (d.done)
            (void) hipEventDestroy(d.done);
    }
}

void destroy_plan(aimet_calib_plan* p)
{
    if (p == nullptr)
        return;
    // a plan is destroyed only with no request in flight (aimet_calib_plan_destroy checks); its
    // device tables may still be read by launched kernels: freed once `done` has completed
    if (p->dev_block || p->pinned_act || p->pinned_par || p->done)
    {
        Graveyard& g = graveyard();
        std::lock_guard<std::mutex> lock(g.m);
        g.items.push_back(DeadPlan {p->device, p->dev_block, p->pinned_act, p->pinned_par, p->done});
    }
    delete p;
}

// the device's stream for the plan's one table upload: non-blocking, so the upload waits for no
// work queued on the legacy default stream (torch's current stream)
hipStream_t upload_stream(int device)
{
    static std::mutex m;
    static std::vector<hipStream_t> streams(64, nullptr);
    AIMET_REQUIRE(device >= 0 && device < 64, "device id out of range");
    std::lock_guard<std::mutex> lock(m);
    if (streams[(size_t) device] == nullptr)
        AIMET_HIP_CHECK(hipStreamCreateWithFlags(&streams[(size_t) device], hipStreamNonBlocking));
    return streams[(size_t) device];
}

// the requests of a launch: the plan's pinned block borrowed, the plan's in-flight count raised
void adopt(aimet_encoding_request* r, void* pinned, size_t bytes, bool has_tfe, int* busy)
{
    if (r == nullptr)
        return;
    if (has_tfe)
    {
        r->pinned          = pinned;
        r->pinned_bytes    = bytes;
        r->pinned_borrowed = true;
    }
    r->busy = busy;
    ++*busy;
}

}   // namespace

extern "C" {

int aimet_calib_plan_create(aimet_tensor_quantizer* const* act_qs, const float* const* act_x, const int64_t* act_n,
                            int64_t n_act, aimet_tensor_quantizer* const* par_qs, const float* const* par_x,
                            const int64_t* par_outer, const int64_t* par_C, const int64_t* par_K, int64_t n_par,
                            const int32_t* act_settings, const int32_t* par_settings, int64_t* elem_counts_dev,
                            aimet_calib_plan** out)
{
    aimet_calib_plan* p = nullptr;
    const int rc        = guarded([&] {
        AIMET_REQUIRE(out != nullptr && act_settings != nullptr && par_settings != nullptr, "null argument");
        AIMET_REQUIRE(n_act >= 0 && n_par >= 0, "negative quantizer count");
        AIMET_REQUIRE((n_act == 0 || (act_qs && act_x && act_n)) &&
                          (n_par == 0 || (par_qs && par_x && par_outer && par_C && par_K)),
                      "null argument");
        *out = nullptr;
        reap_dead_plans();
        p    = new aimet_calib_plan;
        std::copy(act_settings, act_settings + 4, p->aset);
        std::copy(par_settings, par_settings + 4, p->pset);
        p->aq.assign(act_qs, act_qs + n_act);
        p->pq.assign(par_qs, par_qs + n_par);
        AIMET_REQUIRE((n_act == 0 || act_qs[0] != nullptr) && (n_par == 0 || par_qs[0] != nullptr), "null quantizer");
        p->device = n_act ? act_qs[0]->device : (n_par ? par_qs[0]->device : 0);
        for (auto* q: p->pq)
            AIMET_REQUIRE(q != nullptr && q->device == p->device, "quantizers of one calibration share a device");
        if (elem_counts_dev)
            require_device_ptr(elem_counts_dev, "element counts");
        Packer pk;
        // activations
        size_t o_fresh = 0, o_cont = 0, o_parts = 0, o_zact = 0, o_ract = 0;
        std::vector<int64_t> part_offs;
        if (n_act)
        {
            p->jobs = make_jobs(act_qs, act_x, act_n, nullptr, n_act);
            int64_t k = 0;
            p->all_pdf = true;
            for (int64_t i = 0; i < n_act; ++i)
            {
                StatsJob& j = p->jobs[(size_t) i];
                p->all_pdf  = p->all_pdf && j.hist && !j.ent;
                if (elem_counts_dev && j.hist)
                {
                    j.count_dev = elem_counts_dev + k;
                    j.count_out = elem_counts_dev + k;
                    ++k;
                }
            }
            stats_layout(p->jobs, &p->mm, &p->hb);
            // the partials' offsets are fixed up below, once the block's address is known
            o_parts = pk.add(nullptr, sizeof(float) * 2 * p->mm);
            std::vector<StatsJob> fresh = p->jobs;
            for (auto& j: fresh)
            {
                j.fresh = 1;
                j.seen  = 0;
            }
            for (auto& j: p->jobs)
                j.fresh = 0;
            o_fresh = pk.add(fresh.data(), sizeof(StatsJob) * fresh.size());
            o_cont  = pk.add(p->jobs.data(), sizeof(StatsJob) * p->jobs.size());
            std::vector<ZeroJob> z;
            std::vector<ResetJob> r;
            for (auto* q: p->aq)
                reset_ranges(q, false, z, r);   // the PDF of an activation is rewritten by stage 4 only
            for (const ZeroJob& zj: z)
                p->most_act = std::max(p->most_act, zj.bytes);
            p->nz_act = (int) z.size();
            o_zact    = pk.add(z.data(), sizeof(ZeroJob) * z.size());
            o_ract    = pk.add(r.data(), sizeof(ResetJob) * r.size());
        }
        // parameters
        size_t o_zpar = 0, o_rpar = 0, o_ch = 0;
        if (n_par)
        {
            std::vector<ChannelJob> cj;
            for (int64_t i = 0; i < n_par; ++i)
                cj.push_back(make_channel_job(par_qs[i], par_x[i], par_outer[i], par_C[i], par_K[i]));
            p->ch_blocks = channel_layout(cj, &p->ch_hist);
            o_ch         = pk.add(cj.data(), sizeof(ChannelJob) * cj.size());
            std::vector<ZeroJob> z;
            std::vector<ResetJob> r;
            for (auto* q: p->pq)
                reset_ranges(q, true, z, r);   // stage 1 rewrites every parameter's statistics
            for (const ZeroJob& zj: z)
                p->most_par = std::max(p->most_par, zj.bytes);
            p->nz_par = (int) z.size();
            o_zpar    = pk.add(z.data(), sizeof(ZeroJob) * z.size());
            o_rpar    = pk.add(r.data(), sizeof(ResetJob) * r.size());
        }
        // TF-Enhanced search tables
        int64_t ta = 0, tp = 0;
        std::vector<TfeJob> ja = tfe_jobs(p->aq, &ta), jp = tfe_jobs(p->pq, &tp);
        DeviceGuard g(p->device);
        if (ta)
        {
            p->pinned_act_bytes = sizeof(aimet_tf_encoding) * (size_t) ta;
            AIMET_HIP_CHECK(hipHostMalloc(&p->pinned_act, p->pinned_act_bytes, hipHostMallocDefault));
            std::memset(p->pinned_act, 0, p->pinned_act_bytes);
        }
        if (tp)
        {
            p->pinned_par_bytes = sizeof(aimet_tf_encoding) * (size_t) tp;
            AIMET_HIP_CHECK(hipHostMalloc(&p->pinned_par, p->pinned_par_bytes, hipHostMallocDefault));
            std::memset(p->pinned_par, 0, p->pinned_par_bytes);
        }
        for (auto& j: ja)
            j.out = static_cast<aimet_tf_encoding*>(p->pinned_act) + j.start;
        for (auto& j: jp)
            j.out = static_cast<aimet_tf_encoding*>(p->pinned_par) + j.start;
        const int sa = ta ? tfe_splits(ta, p->aset[1] != 0) : 1, sp = tp ? tfe_splits(tp, p->pset[1] != 0) : 1;
        const size_t o_ja = pk.add(ja.data(), sizeof(TfeJob) * ja.size());
        const size_t o_jp = pk.add(jp.data(), sizeof(TfeJob) * jp.size());
        const size_t o_pa = sa > 1 ? pk.add(nullptr, sizeof(uint64_t) * 2 * ta * sa) : 0;
        const size_t o_ka = sa > 1 ? pk.add(nullptr, sizeof(unsigned) * ta) : 0;
        const size_t o_pp = sp > 1 ? pk.add(nullptr, sizeof(uint64_t) * 2 * tp * sp) : 0;
        const size_t o_kp = sp > 1 ? pk.add(nullptr, sizeof(unsigned) * tp) : 0;
        pk.add(nullptr, 0);
        if (pk.host.empty())
        {
            *out = p;
            p    = nullptr;
            return;
        }
        AIMET_HIP_CHECK(hipMalloc(&p->dev_block, pk.host.size()));
        char* base = static_cast<char*>(p->dev_block);
        // fix up the partials pointers in both statistics tables (host image) before the upload
        if (n_act)
        {
            float* parts = reinterpret_cast<float*>(base + o_parts);
            auto* hf     = reinterpret_cast<StatsJob*>(pk.host.data() + o_fresh);
            auto* hc     = reinterpret_cast<StatsJob*>(pk.host.data() + o_cont);
            for (int64_t i = 0; i < n_act; ++i)
            {
                float* mp         = parts + 2 * (int64_t) p->jobs[(size_t) i].mm_block0;
                hf[i].mm_part     = mp;
                hc[i].mm_part     = mp;
                p->jobs[(size_t) i].mm_part = mp;
            }
            p->dj_fresh = reinterpret_cast<StatsJob*>(base + o_fresh);
            p->dj_cont  = reinterpret_cast<StatsJob*>(base + o_cont);
            p->dz_act   = reinterpret_cast<ZeroJob*>(base + o_zact);
            p->dr_act   = reinterpret_cast<ResetJob*>(base + o_ract);
        }
        if (n_par)
        {
            p->dch    = reinterpret_cast<ChannelJob*>(base + o_ch);
            p->dz_par = reinterpret_cast<ZeroJob*>(base + o_zpar);
            p->dr_par = reinterpret_cast<ResetJob*>(base + o_rpar);
        }
        // hand-off buffers: partials need no initial value, the tickets start (and end) at zero
        hipStream_t up = upload_stream(p->device);
        AIMET_HIP_CHECK(hipMemcpyAsync(p->dev_block, pk.host.data(), pk.host.size(), hipMemcpyHostToDevice, up));
        AIMET_HIP_CHECK(hipStreamSynchronize(up));
        AIMET_HIP_CHECK(hipEventCreateWithFlags(&p->done, hipEventDisableTiming));
        if (ta)
        {
            p->has_tfe_act = true;
            p->tfe_act     = TfeTable {ja[0], reinterpret_cast<const TfeJob*>(base + o_ja), (int) ja.size(), ta,
                                   sa > 1 ? reinterpret_cast<uint64_t*>(base + o_pa) : nullptr,
                                   sa > 1 ? reinterpret_cast<unsigned*>(base + o_ka) : nullptr};
        }
        if (tp)
        {
            p->has_tfe_par = true;
            p->tfe_par     = TfeTable {jp[0], reinterpret_cast<const TfeJob*>(base + o_jp), (int) jp.size(), tp,
                                   sp > 1 ? reinterpret_cast<uint64_t*>(base + o_pp) : nullptr,
                                   sp > 1 ? reinterpret_cast<unsigned*>(base + o_kp) : nullptr,
                                   n_act ? kParamSearchPerCu : 0};
        }
        *out = p;
        p    = nullptr;
    });
    if (p)
        destroy_plan(p);
    return rc;
}

int aimet_calib_plan_launch(aimet_calib_plan* p, int stages, int reset, void* main_stream, void* side_stream,
                            aimet_encoding_request** act_req, aimet_encoding_request** par_req)
{
    aimet_encoding_request *ra = nullptr, *rp = nullptr;
    const int rc = guarded([&] {
        AIMET_REQUIRE(p != nullptr && act_req != nullptr && par_req != nullptr, "null argument");
        AIMET_REQUIRE(stages >= 1 && stages <= 7 && (stages == 7 || stages == 1 || stages == 2 || stages == 4),
                      "stages: 7 (the whole batch on one device) or 1, 2, 4 (the sharded calibration's steps)");
        *act_req = *par_req = nullptr;
        const int64_t n_act = (int64_t) p->aq.size(), n_par = (int64_t) p->pq.size();
        if (n_act == 0 && n_par == 0)
            return;
        if ((stages & 4) && p->has_tfe_act)
            AIMET_REQUIRE(p->busy_act == 0, "calibration plan: the previous activation request is not finished");
        if ((stages & 1) && p->has_tfe_par)
            AIMET_REQUIRE(p->busy_par == 0, "calibration plan: the previous parameter request is not finished");
        DeviceGuard g(p->device);
        hipStream_t ms = as_stream(main_stream), ss = as_stream(side_stream);
        const bool first = (stages & 1) != 0;
        // the side stream starts after everything already queued on the main stream (the inputs are
        // ordered there), before the activation passes are added to it
        if (first && ss != ms && (n_par || (reset && n_act)))
            stream_join(ss, ms);
        // enqueued right after the activations' min/max pass, so that pass starts at once: the
        // activations' reset (joined back into the main stream before the pass's combine; the pass
        // itself treats the quantizers as reset, StatsJob::fresh), then the parameters' reset,
        // statistics and search on the (high-priority) side stream beside the activation passes
        auto rest = [&] {
            if (reset && n_act)
            {
                launch_zero_table(p->dz_act, p->nz_act, p->most_act, ss);
                launch_reset_table(p->dr_act, (int) n_act, ss);
                for (auto* q: p->aq)
                    mark_reset(q);
                if (ss != ms)
                    stream_join(ms, ss);
            }
            if (n_par)
            {
                if (reset)
                {
                    launch_zero_table(p->dz_par, p->nz_par, p->most_par, ss);
                    launch_reset_table(p->dr_par, (int) n_par, ss);
                    for (auto* q: p->pq)
                        mark_reset(q);
                }
                launch_channel_table(p->dch, (int) n_par, p->ch_blocks, p->ch_hist, ss);
                for (auto* q: p->pq)
                    q->stats_updated = true;
                encodings_launch(p->pq.data(), n_par, (uint32_t) p->pset[0], p->pset[1], p->pset[2], p->pset[3], ss, rp,
                                 nullptr, p->has_tfe_par ? &p->tfe_par : nullptr);
                adopt(rp, p->pinned_par, p->pinned_par_bytes, p->has_tfe_par, &p->busy_par);
            }
        };
        if (n_act)
        {
            int phases = 0;
            if (stages & 1)
                phases |= kPhaseMinmax | (stages == 7 ? kPhaseFoldMinmax : 0);
            if (stages & 2)
                phases |= (stages == 7 ? 0 : kPhaseFoldMinmax) | kPhaseHistogram;
            if (stages & 4)
                phases |= kPhaseFoldHistogram;
            // the walk rule of launch_stats_many: every quantizer a PDF scheme that has seen a batch
            bool seen = !reset;
            for (auto* q: p->aq)
                seen = seen && q->stats_updated;
            const bool walk = n_act > 64 || (p->all_pdf && seen);
            const StatsJob* dj = (first && reset) ? p->dj_fresh : p->dj_cont;
            if (first)
                launch_stats_table(dj, (int) n_act, p->mm, p->hb, walk, phases, ms, rest);
            else
                launch_stats_table(dj, (int) n_act, p->mm, p->hb, walk, phases, ms);
            if (first)
                for (auto* q: p->aq)
                    q->stats_updated = true;
        }
        else if (first)
            rest();
        if (stages & 4)
        {
            encodings_launch(p->aq.data(), n_act, (uint32_t) p->aset[0], p->aset[1], p->aset[2], p->aset[3], ms, ra,
                             nullptr, p->has_tfe_act ? &p->tfe_act : nullptr);
            adopt(ra, p->pinned_act, p->pinned_act_bytes, p->has_tfe_act, &p->busy_act);
        }
        if (first && n_par && ss != ms)
            stream_join(ms, ss);   // later work on the main stream sees the parameters' state too
        if (p->done)
            AIMET_HIP_CHECK(hipEventRecord(p->done, ms));   // the plan's memory is in use until here
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

int aimet_calib_plan_destroy(aimet_calib_plan* p)
{
    return guarded([&] {
        if (p == nullptr)
            return;
        AIMET_REQUIRE(p->busy_act == 0 && p->busy_par == 0,
                      "calibration plan: finish (or discard) its requests before destroying it");
        destroy_plan(p);
    });
}

}   // extern "C"
