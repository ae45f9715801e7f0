// sanitize_host.cpp -- ASan / UBSan driver for the HOST code of libaimet_amd.
//
// Built by `make -C aimet_amd/csrc sanitize` with every source's host side compiled under
// -fsanitize=address,undefined (device code is untouched: GPU sanitizers are not used on this pool).
// It drives:
//   * always (CPU only): the exact encoding math (getComputedEncodings, fillEncodingInfo,
//     computePartialEncoding) and the host analyzers (TF, TF-Enhanced, percentile, MSE from a PDF;
//     entropy KL search from a TensorProfilingParams histogram: tfe_core / mse_core / entropy_kl host
//     paths) over randomized and degenerate inputs (empty / one-bin / all-mass-in-one-bin / inf / nan
//     ranges), plus BroadcastShapeInfo;
//   * with argument "gpu" (a gfx950 device visible): the quantizer objects' life cycle -- create /
//     create_many, statistics, batched getEncodings (device search + the thread-pooled host entropy
//     re-search), the device-memory cache with deferred reuse, destroy in shuffled order.
// Exit status 0 and no sanitizer report = clean. tests/test_sanitize.py runs it.
#include "aimet_amd.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <random>
#include <vector>

#define CHECK(call)                                                                                  \
    do                                                                                               \
    {                                                                                                \
        int rc_ = (call);                                                                            \
        if (rc_ != AIMET_OK)                                                                         \
        {                                                                                            \
            std::fprintf(stderr, "%s:%d %s -> %d (%s)\n", __FILE__, __LINE__, #call, rc_,            \
                         aimet_last_error());                                                        \
            std::exit(2);                                                                            \
        }                                                                                            \
    } while (0)

static std::mt19937_64 rng(20251016);

static double uni(double a, double b)
{
    return std::uniform_real_distribution<double>(a, b)(rng);
}

static int g_scale = 1;   // argv "long": 10x the iterations

static void encoding_math()
{
    const double inf = std::numeric_limits<double>::infinity();
    const double nan = std::numeric_limits<double>::quiet_NaN();
    const double specials[] = {0.0, -0.0, 1e-30, -1e-30, 1e30, -1e30, inf, -inf, nan, 5.0, -5.0};
    const int bws[]         = {1, 2, 4, 8, 16, 31, 32};
    aimet_tf_encoding e;
    for (int it = 0; it < 3000 * g_scale; ++it)
    {
        double mn = (it % 7 == 0) ? specials[rng() % 11] : uni(-100, 100);
        double mx = (it % 5 == 0) ? specials[rng() % 11] : uni(-100, 100);
        int bw    = bws[rng() % 7];
        int sym = rng() & 1, strict = rng() & 1, uns = rng() & 1;
        aimet_get_computed_encodings(bw, mn, mx, sym, strict, uns, &e);
        aimet_fill_encoding_info(bw, mn, mx, &e);
        aimet_compute_partial_encoding(bw, &e, sym, uns, strict);
        aimet_encoding_from_minmax(mn, mx, bw, sym, strict, uns, &e);
    }
}

static void histogram_analyzers()
{
    const int schemes[] = {AIMET_QUANTIZATION_TF_ENHANCED, AIMET_QUANTIZATION_PERCENTILE, AIMET_QUANTIZATION_MSE};
    std::vector<double> pdf(512), hist(512);
    aimet_tf_encoding e;
    for (int it = 0; it < 48 * g_scale; ++it)
    {
        const int shape = it % 6;
        std::fill(pdf.begin(), pdf.end(), 0.0);
        if (shape == 0)
            pdf[rng() % 512] = 1.0;                               // one bin holds everything
        else if (shape == 1)
            for (auto& p: pdf)
                p = uni(0, 1);                                   // dense
        else if (shape == 2)
            for (int k = 0; k < 5; ++k)
                pdf[rng() % 512] += uni(0, 1);                   // sparse
        else if (shape == 3)
            ;                                                    // empty
        else
            for (int k = 200; k < 312; ++k)
                pdf[k] = std::exp(-0.001 * (k - 256) * (k - 256));
        double s = 0;
        for (double p: pdf)
            s += p;
        if (s > 0)
            for (auto& p: pdf)
                p /= s;
        float hmin     = (float) uni(-50, 0);
        double bucket  = uni(1e-6, 1.0);
        if (it % 37 == 0)
            hmin = -1e30f, bucket = 1e28;                        // beyond the bounded-range pruning
        const int bw   = (it % 3 == 0) ? 4 : 8;
        const float pc = (float) uni(90, 100);
        for (int sc: schemes)
            for (int flags = 0; flags < 4; ++flags)
                aimet_encoding_from_histogram(sc, it % 11 != 0, 1, hmin, bucket, pdf.data(), pc, bw, flags == 1 || flags == 2,
                                              flags == 2, flags == 3, &e);
        // entropy: TensorProfilingParams histogram (integer counts), 8-bit KL search
        for (int k = 0; k < 512; ++k)
            hist[k] = std::floor(pdf[k] * 1e6);
        double lo = uni(-10, 0), hi = lo + uni(0, 20);
        if (it % 29 == 0)
            lo = -std::numeric_limits<double>::infinity();
        for (int flags = 0; flags < 4; ++flags)
            aimet_encoding_from_entropy_histogram(it % 13 != 0, 1, lo, hi, hist.data(), 8, flags == 1 || flags == 2,
                                                  flags == 2, flags == 3, &e);
    }
}

static void shape_info()
{
    aimet_broadcast_shape_info info;
    const int64_t shapes[][4] = {{2, 3, 4, 1}, {16, 64, 1, 1}, {8, 6, 3, 3}, {1, 1, 1, 1}};
    for (auto& s: shapes)
        for (int ca = -1; ca < 4; ++ca)
            for (int ba = -1; ba < 4; ++ba)
                for (int bs: {0, 1, 2, 3})
                    aimet_broadcast_shape_info_init(s, 4, ca, ba, bs, &info);   // invalid combinations must fail cleanly
}

static hipStream_t g_stream = nullptr;   // argv "stream": a created stream instead of the null stream

static void device_lifecycle()
{
    const int schemes[] = {AIMET_QUANTIZATION_TF, AIMET_QUANTIZATION_TF_ENHANCED, AIMET_QUANTIZATION_PERCENTILE,
                           AIMET_QUANTIZATION_MSE, AIMET_QUANTIZATION_ENTROPY};
    const int64_t n     = 1 << 16;
    std::vector<float> host(n);
    for (auto& v: host)
        v = (float) uni(-3, 5);
    float* x = nullptr;
    CHECK(hipMalloc(&x, n * sizeof(float)) == hipSuccess ? AIMET_OK : 1);
    CHECK(hipMemcpy(x, host.data(), n * sizeof(float), hipMemcpyHostToDevice) == hipSuccess ? AIMET_OK : 1);
    for (int round = 0; round < 6; ++round)
    {
        // many per-tensor quantizers from one allocation, statistics in batched launches
        const int nq = 10;
        std::vector<int> sc(nq);
        std::vector<int64_t> ch(nq, 1), ns(nq);
        std::vector<const float*> xs(nq);
        for (int i = 0; i < nq; ++i)
        {
            sc[i] = schemes[i % 5];
            ns[i] = n - 97 * i;
            xs[i] = x + 13 * i;
        }
        std::vector<aimet_tensor_quantizer*> qs(nq);
        CHECK(aimet_tq_create_many(sc.data(), ch.data(), nq, 0, qs.data()));
        CHECK(aimet_tq_update_stats_many(qs.data(), xs.data(), ns.data(), nq, g_stream));
        CHECK(aimet_tq_update_stats_many(qs.data(), xs.data(), ns.data(), nq, g_stream));
        std::vector<aimet_tf_encoding> encs(nq);
        std::vector<int> valid(nq);
        for (int flags = 0; flags < 4; ++flags)
            CHECK(aimet_tq_get_encodings(qs.data(), nq, 8, flags == 1 || flags == 2, flags == 2, flags == 3, encs.data(),
                                         valid.data(), g_stream));
        // per-channel quantizers (device searches + host entropy re-search thread pool)
        aimet_tensor_quantizer* pc[3];
        for (int i = 0; i < 3; ++i)
        {
            CHECK(aimet_tq_create(schemes[(round + i) % 5], 64, 0, &pc[i]));
            CHECK(aimet_tq_update_stats(pc[i], x, 1, 64, n / 64, g_stream));
        }
        std::vector<aimet_tf_encoding> pe(3 * 64);
        int pv[3];
        CHECK(aimet_tq_get_encodings(pc, 3, 8, 1, 0, 0, pe.data(), pv, g_stream));
        // destroy in shuffled order (the slab of create_many is freed with its last quantizer)
        std::shuffle(qs.begin(), qs.end(), rng);
        for (auto* q: qs)
            CHECK(aimet_tq_destroy(q));
        for (auto* q: pc)
            CHECK(aimet_tq_destroy(q));
    }
    CHECK(hipDeviceSynchronize() == hipSuccess ? AIMET_OK : 1);
    (void) hipFree(x);
}

int main(int argc, char** argv)
{
    bool gpu = false;
    for (int i = 1; i < argc; ++i)
    {
        if (std::strcmp(argv[i], "long") == 0)
            g_scale = 10;
        if (std::strcmp(argv[i], "gpu") == 0)
            gpu = true;
        if (std::strcmp(argv[i], "stream") == 0)
            CHECK(hipStreamCreate(&g_stream) == hipSuccess ? AIMET_OK : 1);
    }
    encoding_math();
    histogram_analyzers();
    shape_info();
    if (gpu)
        device_lifecycle();
    std::printf("sanitize_host: clean\n");
    return 0;
}
