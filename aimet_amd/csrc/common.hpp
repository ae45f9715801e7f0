// common.hpp -- shared host/device helpers of the MI355X DlQuantization core.
//
// Numerics contract: every kernel reproduces the reference CPU arithmetic of
// DlQuantization bit for bit. That rules out fast-math: the library is compiled with
// -ffp-contract=off and correctly-rounded fp32 division (the reference GPU build used
// --use_fast_math, which is why its GPU output never matched its own CPU output).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>

#include "aimet_amd.h"

namespace aimet_amd
{

constexpr int kPdfSize     = 512;   // math_functions.hpp:80 PDF_SIZE
constexpr int kBlock       = 256;   // 4 waves of 64
constexpr int kMaxStreamBlocks = 2048;  // 256 CUs x 8 resident blocks (grid-stride beyond)

// ------------------------------------------------------------------------------------------
// Error plumbing: C++ exceptions are turned into status codes at the C-ABI.
// ------------------------------------------------------------------------------------------
struct InvalidArgument : std::invalid_argument
{
    using std::invalid_argument::invalid_argument;
};
struct RuntimeError : std::runtime_error
{
    using std::runtime_error::runtime_error;
};
struct HipError : std::runtime_error
{
    using std::runtime_error::runtime_error;
};

void set_last_error(const std::string& msg);

#define AIMET_HIP_CHECK(expr)                                                                            \
    do                                                                                                   \
    {                                                                                                    \
        hipError_t e_ = (expr);                                                                          \
        if (e_ != hipSuccess)                                                                            \
            throw ::aimet_amd::HipError(std::string(#expr) + ": " + hipGetErrorString(e_) + " (" +      \
                                        __FILE__ + ":" + std::to_string(__LINE__) + ")");                \
    } while (0)

#define AIMET_LAUNCH_CHECK() AIMET_HIP_CHECK(hipGetLastError())

#define AIMET_REQUIRE(cond, msg)                                                                         \
    do                                                                                                   \
    {                                                                                                    \
        if (!(cond))                                                                                     \
            throw ::aimet_amd::InvalidArgument(msg);                                                     \
    } while (0)

template <class F>
int guarded(F&& f)
{
    try
    {
        f();
        return AIMET_OK;
    }
    catch (const InvalidArgument& e)
    {
        set_last_error(e.what());
        return AIMET_ERR_INVALID_ARGUMENT;
    }
    catch (const HipError& e)
    {
        set_last_error(e.what());
        return AIMET_ERR_HIP;
    }
    catch (const std::exception& e)
    {
        set_last_error(e.what());
        return AIMET_ERR_RUNTIME;
    }
    catch (...)
    {
        set_last_error("unknown error");
        return AIMET_ERR_RUNTIME;
    }
}

inline hipStream_t as_stream(void* s)
{
    return reinterpret_cast<hipStream_t>(s);
}

// Reject host pointers: there is no CPU compute path in this library.
void require_device_ptr(const void* p, const char* what);

inline int64_t ceil_div(int64_t a, int64_t b)
{
    return (a + b - 1) / b;
}

inline int stream_blocks(int64_t work_items, int64_t items_per_block)
{
    int64_t b = ceil_div(work_items, items_per_block);
    if (b < 1)
        b = 1;
    if (b > kMaxStreamBlocks)
        b = kMaxStreamBlocks;
    return (int) b;
}

// ------------------------------------------------------------------------------------------
// Fast 32-bit division by a runtime-invariant divisor (dividends < 2^31).
// ------------------------------------------------------------------------------------------
struct FastDiv
{
    uint32_t d, mul, shr;
    FastDiv() = default;
    explicit FastDiv(uint32_t divisor) : d(divisor), mul(0), shr(0)
    {
        if (d > 1)
        {
            uint32_t l = 32 - __builtin_clz(d - 1);   // ceil(log2(d))
            uint32_t p = 31 + l;
            mul        = (uint32_t) (((1ull << p) + d - 1) / d);
            shr        = p - 32;
        }
    }
    __device__ __forceinline__ uint32_t div(uint32_t n) const
    {
        return d == 1 ? n : (__umulhi(n, mul) >> shr);
    }
};

// ------------------------------------------------------------------------------------------
// Reference element arithmetic (trim_functions.cpp:140-171, x86-64 glibc semantics).
// ------------------------------------------------------------------------------------------

// ---- hand-off of per-workgroup partials to the last-arriving workgroup (one launch) ------------
// The per-XCD L2s are not coherent and a CU's L1 is never refreshed by another CU's stores. The
// partials are stored write-through (agent-scope relaxed atomic store: a `global_store ... sc1`),
// the storing wave drains them (s_waitcnt vmcnt(0)) before its ticket add, and the last arriver
// reads them with agent-scope loads (`sc1`, past L1 and L2): no release fence (an agent release is
// a whole-L2 write-back, buffer_wbl2, per workgroup) and no acquire. MI355X_MICROARCH.md
// § visibility, cdna_hip_programming.md Guideline 16 (R1).
__device__ __forceinline__ void publish_f32(float* p, float v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float consume_f32(const float* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void publish_u64(uint64_t* p, uint64_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t consume_u64(const uint64_t* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// the calling lane's published partials drained, then its ticket: true for the last of
// `arrivals` (one call per workgroup, from the lane that published)
__device__ __forceinline__ bool arrive_is_last(unsigned* ticket, unsigned arrivals)
{
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == arrivals - 1;
}
// Arrival of every workgroup of the grid, two-level: a same-address atomic from each of thousands
// of workgroups finishing together serialises at the memory side (2048 of them added ~20 us to a
// 16-us kernel), so workgroup b counts on group counter b mod kTicketGroups, and each group's last
// arriver (which re-zeroes its group counter) on the top counter tickets[kTicketGroups]. True in
// the one workgroup that arrives last overall; its caller resets the top counter (ticket_reset).
// Needs kTicketGroups + 1 counters (ticket_alloc).
constexpr unsigned kTicketGroups = 32;
__device__ __forceinline__ bool arrive_is_last_grid(unsigned* tickets)
{
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned n = gridDim.x, G = n < kTicketGroups ? n : kTicketGroups;
    const unsigned g = blockIdx.x % G, members = (n - g + G - 1) / G;
    if (__hip_atomic_fetch_add(tickets + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != members - 1)
        return false;
    __hip_atomic_store(tickets + g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return __hip_atomic_fetch_add(tickets + kTicketGroups, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == G - 1;
}
// the last arriver leaves the ticket at zero for its next user (ticket_alloc)
__device__ __forceinline__ void ticket_reset(unsigned* ticket)
{
    __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// glibc fminf/fmaxf (x86-64): a NaN operand yields the other operand; otherwise
// minss/maxss, i.e. the SECOND operand on ties (matters for +-0).
__device__ __forceinline__ float glibc_fminf(float x, float y)
{
    return (x < y || __builtin_isnan(y)) ? x : y;
}
__device__ __forceinline__ float glibc_fmaxf(float x, float y)
{
    return (x > y || __builtin_isnan(y)) ? x : y;
}

// upload.cpp: stream-ordered device copy of a small host table without blocking the host
// (pinned staging ring); release with scratch_free(ptr, s) after the consuming launches.
void* upload_async(const void* src, size_t bytes, hipStream_t s);
// Stream-ordered device scratch without the stream-ordered pool: released blocks are reused once
// an event recorded after their consumers has completed (upload.cpp; the pool let a job table be
// reused under a running kernel: tests/cpp/sanitize_host.cpp).
void* scratch_alloc(size_t bytes, hipStream_t s);
// `count` consecutive zeroed completion counters for last-workgroup folds, or nullptr: upload.cpp
unsigned* ticket_alloc(hipStream_t s, unsigned count = 1);
// tickets + a partial-sum buffer of `part_floats` for one launch's last-workgroup fold; both null
// when there is no ticket (the caller then falls back). Inside a HIP-graph capture the buffer is a
// permanent slot of its own (no graph memory node); release with fold_buffers_release.
struct FoldBuffers
{
    unsigned* ticket = nullptr;
    float* part      = nullptr;
    bool scratch     = false;
};
FoldBuffers fold_buffers(hipStream_t s, unsigned tickets, size_t part_floats);
void fold_buffers_release(const FoldBuffers& f, hipStream_t s);
// aimet_capture_pool_limit: the capture arena's cap on the current device (returns the previous one)
size_t capture_pool_limit(size_t arena_floats);
void scratch_free(void* p, hipStream_t s);

struct QdqParams
{
    float min, max, delta, offset;
};

// quantizeValueCpu (ROUND_NEAREST): round(clamp(x)/delta - offset), half away from zero.
__device__ __forceinline__ float quantize_nearest(float x, const QdqParams& p)
{
    float o = glibc_fmaxf(glibc_fminf(x, p.max), p.min);
    o       = o / p.delta - p.offset;
    return __builtin_roundf(o);
}

// round(RN(RN(a / d) - off)) (half away from zero) without the IEEE division in the common case.
// q = RN(a * rcp) with rcp = RN(1/d) is within 3.0001 ulp(|a/d|) of RN(a/d), so v = RN(q - off)
// and the reference's v* = RN(RN(a/d) - off) differ by at most 6u(|q| + |off|) (u = 2^-24). Their
// roundings can only differ if a half-integer lies within that distance of v; when v is farther
// than 2^-21 (|q| + |off| + 1) (>= 8u(...)) from every half-integer, round(v) == round(v*).
// Otherwise -- and for every non-finite intermediate -- the exact IEEE division decides. The
// result is therefore bit-identical to the division form (and to the reference), signed zeros
// included (see below).
__device__ __forceinline__ float round_div_sub(float a, float d, float rcp, float off)
{
    const float q    = a * rcp;
    const float v    = q - off;
    const float h    = v - __builtin_floorf(v);             // exact fractional part, [0, 1)
    const float dist = __builtin_fabsf(h - 0.5f);
    const float thr  = (__builtin_fabsf(q) + __builtin_fabsf(off) + 1.0f) * 4.76837158203125e-7f;   // 2^-21
    // A zero result also needs the sign of v*: with off == +-0 it is the sign of a (as for v);
    // otherwise (v* = q* - off exactly) q' and q* may straddle off, so the division decides.
    if (dist > thr && (off == 0.0f || __builtin_fabsf(v) >= 0.5f))   // false for NaN / inf
        return __builtin_roundf(v);
    return __builtin_roundf(a / d - off);
}

// round_div_sub specialised for a quantize-DEQUANTIZE of a clamped value, with the threshold
// hoisted out of the element loop (VALU-bound 16-bit I/O kernels: ~9 fewer ops per element):
//  * |o| <= M = max(|min|, |max|) after the clamp, so |q| = |RN(o*rcp)| <= RN(M*rcp) and
//    qdq_round_thr() >= round_div_sub's per-element threshold (float ops are monotonic);
//  * away from half-integers rint(v) == roundf(v) (no tie to break), and round(v) == round(v*);
//  * a zero code's sign only reaches the output when off == +-0 (y = delta * (q + off)), where
//    round_div_sub already takes the fast path, so the |v| >= 0.5 test is not needed here.
// A NaN / inf threshold (non-finite encodings, overflowing o*rcp) sends every element to the
// exact division. Not for quantize-only output: there the sign of a zero code is observable.
__device__ __forceinline__ float qdq_round_thr(const QdqParams& p, float rcp)
{
    const float a = __builtin_fabsf(p.min), b = __builtin_fabsf(p.max);
    const float M = (a != a || b != b) ? __builtin_nanf("") : (a > b ? a : b);   // NaN bound -> exact path
    return (M * rcp + __builtin_fabsf(p.offset) + 1.0f) * 4.76837158203125e-7f;   // 2^-21
}
__device__ __forceinline__ float qdq_round_fast(float o, const QdqParams& p, float rcp, float thr)
{
    const float v = o * rcp - p.offset;
    if (__builtin_fabsf(__builtin_amdgcn_fractf(v) - 0.5f) > thr)   // false for NaN
        return __builtin_rintf(v);
    return __builtin_roundf(o / p.delta - p.offset);
}

// quantize_nearest with a per-thread reciprocal of delta (see round_div_sub): identical results
__device__ __forceinline__ float quantize_nearest_rcp(float x, const QdqParams& p, float rcp)
{
    float o = glibc_fmaxf(glibc_fminf(x, p.max), p.min);
    return round_div_sub(o, p.delta, rcp, p.offset);
}

// ROUND_STOCHASTIC: floor(v + U[0,1)). The reference draws rand() (CPU) or curand seeded by
// clock() (GPU) -- neither reproducible, so only the distribution is specified.
__device__ __forceinline__ float uniform01(uint64_t seed, uint64_t idx)
{
    uint64_t z = seed + 0x9E3779B97F4A7C15ull * (idx + 1);
    z          = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z          = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (float) (uint32_t) (z >> 40) * (1.0f / 16777216.0f);
}

__device__ __forceinline__ float quantize_stochastic(float x, const QdqParams& p, uint64_t seed, uint64_t idx)
{
    float o = glibc_fmaxf(glibc_fminf(x, p.max), p.min);
    o       = o / p.delta - p.offset;
    return __builtin_floorf(o + uniform01(seed, idx));
}

// dequantizeValueCpu
__device__ __forceinline__ float dequantize(float q, const QdqParams& p)
{
    return p.delta * (q + p.offset);
}

}   // namespace aimet_amd
