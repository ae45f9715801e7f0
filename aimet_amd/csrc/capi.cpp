// capi.cpp -- error state, device checks and the host encoding-math entry points of the C-ABI.
#include <map>
#include <string>

#include "encodings.hpp"

namespace aimet_amd
{

namespace
{
thread_local std::string g_last_error;
}

void set_last_error(const std::string& msg)
{
    g_last_error = msg;
}

// Device allocations already validated: [base, end) of the allocations (hipMemGetAddressRange)
// that earlier device pointers lay in, keyed by base. A batched call over ViT-L/16's 318
// activations (each its own torch segment) otherwise made 318 pointer queries per calibration
// batch on the critical path. A hit only skips a validation: kernels run on the pointer either way.
namespace
{
struct DeviceRanges
{
    std::map<uintptr_t, uintptr_t> r;   // base -> end
    bool hit(uintptr_t a) const
    {
        auto it = r.upper_bound(a);
        if (it == r.begin())
            return false;
        --it;
        return a < it->second;
    }
    void add(const void* p)
    {
        hipDeviceptr_t b = nullptr;
        size_t n         = 0;
        if (hipMemGetAddressRange(&b, &n, const_cast<void*>(p)) != hipSuccess || b == nullptr || n == 0)
        {
            (void) hipGetLastError();
            return;
        }
        if (r.size() >= 4096)
            r.clear();
        const uintptr_t base = reinterpret_cast<uintptr_t>(b);
        r[base]              = base + n;
    }
};
thread_local DeviceRanges t_ranges;
}   // namespace

void require_device_ptr(const void* p, const char* what)
{
    if (p == nullptr)
        throw InvalidArgument(std::string(what) + " pointer is null");
    if (t_ranges.hit(reinterpret_cast<uintptr_t>(p)))
        return;
    hipPointerAttribute_t attr;
    hipError_t e = hipPointerGetAttributes(&attr, p);
    if (e != hipSuccess)
    {
        (void) hipGetLastError();   // clear the sticky error of the failed query
        throw InvalidArgument(std::string(what) +
                              " is not device memory: aimet_amd has no CPU path (move the tensor to an MI355X)");
    }
    if (attr.type != hipMemoryTypeDevice && attr.type != hipMemoryTypeManaged)
        throw InvalidArgument(std::string(what) +
                              " is not device memory: aimet_amd has no CPU path (move the tensor to an MI355X)");
    if (attr.type == hipMemoryTypeDevice)
        t_ranges.add(p);
}

}   // namespace aimet_amd

using namespace aimet_amd;

extern "C" {

const char* aimet_last_error(void)
{
    return g_last_error.c_str();
}

const char* aimet_version(void)
{
    return "aimet_amd 0.1.0 gfx950";
}

int aimet_device_count(void)
{
    int n  = 0;
    int rc = guarded([&] { AIMET_HIP_CHECK(hipGetDeviceCount(&n)); });
    return rc == AIMET_OK ? n : rc;
}

int aimet_capture_pool_limit(int64_t arena_floats, int64_t* previous)
{
    return guarded([&] {
        AIMET_REQUIRE(arena_floats >= 0, "negative limit");
        const size_t prev = capture_pool_limit((size_t) arena_floats);
        if (previous)
            *previous = (int64_t) prev;
    });
}

int aimet_get_computed_encodings(int32_t bw, double mn, double mx, int sym, int strict, int unsign,
                                 aimet_tf_encoding* out)
{
    return guarded([&] {
        AIMET_REQUIRE(out != nullptr, "output is null");
        *out = computed_encoding((int32_t) (uint8_t) bw, mn, mx, sym != 0, strict != 0, unsign != 0);
    });
}

int aimet_fill_encoding_info(int32_t bw, double mn, double mx, aimet_tf_encoding* out)
{
    return guarded([&] {
        AIMET_REQUIRE(out != nullptr, "output is null");
        *out = fill_encoding_info(bw, mn, mx);
    });
}

int aimet_compute_partial_encoding(int32_t bw, aimet_tf_encoding* enc, int sym, int unsign, int strict)
{
    return guarded([&] {
        AIMET_REQUIRE(enc != nullptr, "encoding is null");
        std::string err;
        aimet_tf_encoding e = *enc;
        if (!partial_encoding((int32_t) (uint8_t) bw, e, sym != 0, unsign != 0, strict != 0, err))
        {
            if (err.find("Cannot determine") != std::string::npos)
                throw RuntimeError(err);
            throw InvalidArgument(err);
        }
        *enc = e;
    });
}

int aimet_encoding_from_minmax(double acc_min, double acc_max, int32_t bw, int sym, int strict, int unsign,
                               aimet_tf_encoding* out)
{
    return guarded([&] {
        AIMET_REQUIRE(out != nullptr, "output is null");
        *out = tf_encoding(acc_min, acc_max, (int32_t) (uint8_t) bw, sym != 0, strict != 0, unsign != 0);
    });
}

int aimet_encoding_from_histogram(int scheme, int initialized, int stats_updated, float hist_min, double bucket_size,
                                  const double* pdf, float percentile, int32_t bw, int sym, int strict, int unsign,
                                  aimet_tf_encoding* out)
{
    return guarded([&] {
        AIMET_REQUIRE(out != nullptr, "output is null");
        AIMET_REQUIRE(scheme == AIMET_QUANTIZATION_TF_ENHANCED || scheme == AIMET_QUANTIZATION_PERCENTILE ||
                          scheme == AIMET_QUANTIZATION_MSE,
                      "histogram encodings exist for TF-Enhanced, percentile and MSE only");
        AIMET_REQUIRE(!initialized || pdf != nullptr, "pdf is null");
        *out = histogram_encoding(scheme, initialized != 0, stats_updated != 0, hist_min, bucket_size, pdf, percentile,
                                  (int32_t) (uint8_t) bw, sym != 0, strict != 0, unsign != 0);
    });
}

int aimet_encoding_from_entropy_histogram(int has_histogram, int stats_updated, double tpp_min, double tpp_max,
                                          const double* hist, int32_t bw, int sym, int strict, int unsign,
                                          aimet_tf_encoding* out)
{
    return guarded([&] {
        AIMET_REQUIRE(out != nullptr, "output is null");
        AIMET_REQUIRE(!has_histogram || hist != nullptr, "histogram is null");
        *out = entropy_encoding(has_histogram != 0, stats_updated != 0, tpp_min, tpp_max, hist,
                                (int32_t) (uint8_t) bw, sym != 0, strict != 0, unsign != 0);
    });
}

}   // extern "C"
