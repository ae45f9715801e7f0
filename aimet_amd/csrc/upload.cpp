// upload.cpp -- host -> device copies of small per-call tables (job / descriptor arrays) that
// never block the host, and the per-call device scratch they and a few kernels (learned-grid
// partial sums, blockwise re-layout) live in.
//
// Device scratch is a small caching allocator of its own rather than the stream-ordered pool
// (hipMallocAsync / hipFreeAsync): a released block carries an event recorded on the releasing
// stream after its consumers, and is handed out again only once that event has completed. The
// stream-ordered pool was measured to let a job table be reused while the kernel reading it still
// ran (tests/cpp/sanitize_host.cpp: an illegal access on the legacy null stream -- torch's default
// stream -- and, under ASan timing, on a created stream); this form needs no ordering guarantee
// beyond events. Inside a HIP-graph capture the pool IS used (its allocations become graph memory
// nodes).
//
// Host staging goes through a ring of pinned buffers, an event per slot guarding its reuse.
#include "common.hpp"

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <unordered_map>
#include <vector>

namespace aimet_amd
{
namespace
{

constexpr int kSlots   = 16;
constexpr int kDevices = 64;

struct Slot
{
    void* host    = nullptr;
    size_t cap    = 0;
    hipEvent_t ev = nullptr;
};

struct Ring
{
    std::mutex m;
    Slot slots[kSlots];
    int next = 0;
};

Ring& ring(int dev)
{
    static Ring rings[kDevices];
    return rings[dev];
}


bool capturing(hipStream_t s)
{
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    AIMET_HIP_CHECK(hipStreamIsCapturing(s, &st));
    return st != hipStreamCaptureStatusNone;
}

int current_device()
{
    int dev = 0;
    AIMET_HIP_CHECK(hipGetDevice(&dev));
    AIMET_REQUIRE(dev >= 0 && dev < kDevices, "device id out of range");
    return dev;
}

// released blocks, reusable once their event has completed
struct ScratchCache
{
    struct Block
    {
        int device;
        void* p;
        size_t bytes;
        hipEvent_t ev;
    };
    struct Live
    {
        int device;
        size_t bytes;
        int mode;   // 0: cached block, 1: stream-ordered pool (capture)
    };
    std::mutex m;
    std::vector<Block> free_blocks;
    std::vector<hipEvent_t> spare_events;
    std::unordered_map<void*, Live> live;
};
ScratchCache& cache()
{
    static ScratchCache* c = new ScratchCache();   // never destroyed: blocks live until process exit
    return *c;
}

constexpr size_t kMaxCachedBlocks = 64;

}   // namespace

void* scratch_alloc(size_t bytes, hipStream_t s)
{
    if (bytes == 0)
        bytes = 1;
    ScratchCache& c = cache();
    const int dev   = current_device();
    void* d         = nullptr;
    int mode        = 0;
    size_t real     = bytes;   // a reused block keeps its own (possibly larger) size
    if (s != nullptr && capturing(s))
    {
        AIMET_HIP_CHECK(hipMallocAsync(&d, bytes, s));
        mode = 1;
    }
    else
    {
        std::vector<void*> stale;
        {
            std::lock_guard<std::mutex> lock(c.m);
            size_t best = c.free_blocks.size();
            for (size_t i = 0; i < c.free_blocks.size(); ++i)
            {
                const ScratchCache::Block& b = c.free_blocks[i];
                if (b.device != dev || b.bytes < bytes || b.bytes > 4 * bytes + 4096)
                    continue;
                if (hipEventQuery(b.ev) != hipSuccess)   // its consumers still run (or an error)
                    continue;
                if (best == c.free_blocks.size() || b.bytes < c.free_blocks[best].bytes)
                    best = i;
            }
            if (best != c.free_blocks.size())
            {
                d    = c.free_blocks[best].p;
                real = c.free_blocks[best].bytes;
                c.spare_events.push_back(c.free_blocks[best].ev);
                c.free_blocks.erase(c.free_blocks.begin() + (std::ptrdiff_t) best);
            }
            else if (c.free_blocks.size() >= kMaxCachedBlocks)
            {
                // trim: completed blocks of this device go back to the driver
                for (size_t i = 0; i < c.free_blocks.size();)
                {
                    if (c.free_blocks[i].device == dev && hipEventQuery(c.free_blocks[i].ev) == hipSuccess)
                    {
                        stale.push_back(c.free_blocks[i].p);
                        c.spare_events.push_back(c.free_blocks[i].ev);
                        c.free_blocks.erase(c.free_blocks.begin() + (std::ptrdiff_t) i);
                    }
                    else
                        ++i;
                }
            }
        }
        for (void* p: stale)
            AIMET_HIP_CHECK(hipFree(p));
        if (d == nullptr)
            AIMET_HIP_CHECK(hipMalloc(&d, bytes));
    }
    std::lock_guard<std::mutex> lock(c.m);
    c.live[d] = ScratchCache::Live {dev, real, mode};
    return d;
}

void scratch_free(void* p, hipStream_t s)
{
    if (p == nullptr)
        return;
    ScratchCache& c = cache();
    ScratchCache::Live l {};
    hipEvent_t ev = nullptr;
    {
        std::lock_guard<std::mutex> lock(c.m);
        auto it = c.live.find(p);
        AIMET_REQUIRE(it != c.live.end(), "scratch_free of a pointer scratch_alloc did not return");
        l = it->second;
        c.live.erase(it);
        if (l.mode == 0 && !c.spare_events.empty())
        {
            ev = c.spare_events.back();
            c.spare_events.pop_back();
        }
    }
    if (l.mode == 1)
    {
        AIMET_HIP_CHECK(hipFreeAsync(p, s));
        return;
    }
    if (ev == nullptr)
        AIMET_HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    AIMET_HIP_CHECK(hipEventRecord(ev, s));   // after every launch that reads the block
    std::lock_guard<std::mutex> lock(c.m);
    c.free_blocks.push_back(ScratchCache::Block {l.device, p, l.bytes, ev});
}

// Completion tickets of the kernels that fold their per-workgroup partials in the last-arriving
// workgroup: `count` consecutive zeroed counters (one per group of workgroups that fold together),
// each left at zero again by the workgroup that folds.
// * Outside a HIP-graph capture, a ring per device: a counter is reused only after kTicketRing
//   later calls, so calls in flight on different streams never share one.
// * Inside a capture, a counter of its own that is never handed out again (the captured launch
//   keeps it for every replay; replays of one graph run one after the other).
// nullptr (the caller then launches its fold): a capture before any eager call made the pool (it
// cannot be allocated and zeroed inside a capture), or the capture counters used up.
namespace
{
constexpr unsigned kTicketRing = 1u << 16, kTicketCapture = 1u << 20;
constexpr size_t kCaptureArenaFloats = size_t(16) << 20;   // 64 MB of captured launches' partials
struct TicketPool
{
    std::mutex m;
    unsigned* dev = nullptr;
    unsigned next = 0, captured = 0;
    float* arena      = nullptr;   // partial-sum slots of captured launches, handed out once
    size_t arena_used = 0;
    size_t arena_cap  = kCaptureArenaFloats;   // aimet_capture_pool_limit (tests of the fallback)
};
TicketPool& ticket_pool(int dev)
{
    static TicketPool pools[kDevices];
    return pools[dev];
}
// the pool of the current device, created (and zeroed) on first use outside a capture
TicketPool* ready_pool(hipStream_t s, bool cap)
{
    TicketPool& p = ticket_pool(current_device());
    if (p.dev == nullptr)
    {
        if (cap)
            return nullptr;
        const size_t bytes = sizeof(unsigned) * (kTicketRing + kTicketCapture);
        unsigned* d        = nullptr;
        float* a           = nullptr;
        AIMET_HIP_CHECK(hipMalloc(&d, bytes));
        AIMET_HIP_CHECK(hipMalloc(&a, sizeof(float) * kCaptureArenaFloats));
        AIMET_HIP_CHECK(hipMemsetAsync(d, 0, bytes, s));
        AIMET_HIP_CHECK(hipStreamSynchronize(s));   // once per device: zero before any stream uses it
        p.dev   = d;
        p.arena = a;
    }
    return &p;
}
unsigned* take_tickets(TicketPool& p, bool cap, unsigned count)
{
    if (count == 0 || count > kTicketRing / 16)
        return nullptr;
    if (!cap)
    {
        if (p.next % kTicketRing + count > kTicketRing)   // consecutive counters: skip the ring's end
            p.next += kTicketRing - p.next % kTicketRing;
        unsigned* t = p.dev + p.next % kTicketRing;
        p.next += count;
        return t;
    }
    if (p.captured + count > kTicketCapture)
        return nullptr;
    unsigned* t = p.dev + kTicketRing + p.captured;
    p.captured += count;
    return t;
}
}   // namespace

unsigned* ticket_alloc(hipStream_t s, unsigned count)
{
    const bool cap = s != nullptr && capturing(s);
    std::lock_guard<std::mutex> lock(ticket_pool(current_device()).m);
    TicketPool* p = ready_pool(s, cap);
    return p ? take_tickets(*p, cap, count) : nullptr;
}

FoldBuffers fold_buffers(hipStream_t s, unsigned tickets, size_t part_floats)
{
    FoldBuffers f;
    const bool cap = s != nullptr && capturing(s);
    {
        std::lock_guard<std::mutex> lock(ticket_pool(current_device()).m);
        TicketPool* p = ready_pool(s, cap);
        if (p == nullptr)
            return f;
        if (cap)
        {
            // a captured launch keeps its partials slot for every replay: from the arena, never
            // handed out again (a graph memory node per replay cost ~10 us of every AdaRound iteration)
            const size_t n = (part_floats + 63) & ~size_t(63);
            if (p->arena_used + n > p->arena_cap)
                return f;   // used up: the caller folds in a launch of its own (same arithmetic)
            unsigned* t = take_tickets(*p, cap, tickets);
            if (t == nullptr)
                return f;
            f.ticket = t;
            f.part   = p->arena + p->arena_used;
            p->arena_used += n;
            return f;
        }
        f.ticket = take_tickets(*p, cap, tickets);
        if (f.ticket == nullptr)
            return f;
    }
    f.part    = static_cast<float*>(scratch_alloc(sizeof(float) * part_floats, s));
    f.scratch = true;
    return f;
}

size_t capture_pool_limit(size_t arena_floats)
{
    TicketPool& p = ticket_pool(current_device());
    std::lock_guard<std::mutex> lock(p.m);
    const size_t prev = p.arena_cap;
    p.arena_cap       = arena_floats < kCaptureArenaFloats ? arena_floats : kCaptureArenaFloats;
    return prev;
}

void fold_buffers_release(const FoldBuffers& f, hipStream_t s)
{
    if (f.scratch && f.part)
        scratch_free(f.part, s);
}

void* upload_async(const void* src, size_t bytes, hipStream_t s)
{
    // a captured copy would re-read the (reused) pinned slot at every replay
    AIMET_REQUIRE(s == nullptr || !capturing(s), "host tables cannot be uploaded inside a HIP-graph capture");
    void* d = scratch_alloc(bytes, s);
    Ring& r = ring(current_device());
    std::lock_guard<std::mutex> lock(r.m);
    Slot& slot = r.slots[r.next];
    r.next     = (r.next + 1) % kSlots;
    if (slot.ev)
        AIMET_HIP_CHECK(hipEventSynchronize(slot.ev));   // the previous copy out of this slot is done
    if (slot.cap < bytes)
    {
        // every slot holds at least kMinSlot: a slot the ring reaches with a large table is not
        // re-allocated (hipHostMalloc ~50 us + first-touch faults ~100 us per ViT-L/16 batch's
        // 318-job table, measured with --hip-trace)
        if (slot.host)
            AIMET_HIP_CHECK(hipHostFree(slot.host));
        slot.host = nullptr;
        slot.cap  = 0;
        constexpr size_t kMinSlot = size_t(256) << 10;
        size_t cap = bytes < kMinSlot ? kMinSlot : bytes * 2;
        AIMET_HIP_CHECK(hipHostMalloc(&slot.host, cap, hipHostMallocDefault));
        std::memset(slot.host, 0, cap);   // fault the pages in now, not in the first copy
        slot.cap = cap;
    }
    if (!slot.ev)
        AIMET_HIP_CHECK(hipEventCreateWithFlags(&slot.ev, hipEventDisableTiming));
    std::memcpy(slot.host, src, bytes);
    AIMET_HIP_CHECK(hipMemcpyAsync(d, slot.host, bytes, hipMemcpyHostToDevice, s));
    AIMET_HIP_CHECK(hipEventRecord(slot.ev, s));
    return d;
}

}   // namespace aimet_amd
