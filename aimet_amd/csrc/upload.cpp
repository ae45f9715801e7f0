// upload.cpp -- host -> device copies of small per-call tables (job / descriptor arrays) that
// never block the host. hipMemcpyAsync from pageable memory stages the data synchronously
// (the host waits for the stream); here the data goes through a ring of pinned staging buffers,
// an event per slot guarding its reuse, into a stream-ordered allocation.
#include "common.hpp"

#include <cstring>
#include <mutex>

namespace aimet_amd
{
namespace
{

constexpr int kSlots   = 16;
constexpr int kDevices = 64;

struct Slot
{
    void* host     = nullptr;
    size_t cap     = 0;
    hipEvent_t ev  = nullptr;
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

}   // namespace

void* upload_async(const void* src, size_t bytes, hipStream_t s)
{
    int dev = 0;
    AIMET_HIP_CHECK(hipGetDevice(&dev));
    AIMET_REQUIRE(dev >= 0 && dev < kDevices, "device id out of range");
    Ring& r = ring(dev);
    std::lock_guard<std::mutex> lock(r.m);
    Slot& slot = r.slots[r.next];
    r.next     = (r.next + 1) % kSlots;
    if (slot.ev)
        AIMET_HIP_CHECK(hipEventSynchronize(slot.ev));   // the previous copy out of this slot is done
    if (slot.cap < bytes)
    {
        if (slot.host)
            AIMET_HIP_CHECK(hipHostFree(slot.host));
        slot.host = nullptr;
        slot.cap  = 0;
        size_t cap = bytes < 4096 ? 4096 : bytes * 2;
        AIMET_HIP_CHECK(hipHostMalloc(&slot.host, cap, hipHostMallocDefault));
        slot.cap = cap;
    }
    if (!slot.ev)
        AIMET_HIP_CHECK(hipEventCreateWithFlags(&slot.ev, hipEventDisableTiming));
    std::memcpy(slot.host, src, bytes);
    void* d = nullptr;
    AIMET_HIP_CHECK(hipMallocAsync(&d, bytes, s));
    AIMET_HIP_CHECK(hipMemcpyAsync(d, slot.host, bytes, hipMemcpyHostToDevice, s));
    AIMET_HIP_CHECK(hipEventRecord(slot.ev, s));
    return d;
}

}   // namespace aimet_amd
