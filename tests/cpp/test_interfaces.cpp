// Exercises include/aimet_amd.hpp (the reference's C++ interfaces over the C-ABI).
//   test_interfaces host <out.txt>                    host-only entry points
//   test_interfaces gpu <in.f32> <n> <C> <out.f32> <encs.txt>   device path (MI355X)
// The Python side (tests/test_cpp_interfaces.py) writes the input and checks every output
// against the oracle.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

#include "aimet_amd.hpp"

using namespace aimet_amd;

static void put(FILE* f, const char* tag, const TfEncoding& e)
{
    std::fprintf(f, "%s %.17g %.17g %.17g %.17g %d\n", tag, e.min, e.max, e.delta, e.offset, e.bw);
}

static int host(const char* out)
{
    FILE* f = std::fopen(out, "w");
    TensorQuantizationSim sim;
    TfEncoding e {};
    sim.fillEncodingInfo(e, 8, -1.3, 2.7);
    put(f, "fill", e);
    double mn = -2.0, mx = 2.0, scale = 0, offset = 0;
    sim.generateScaleOffset(mn, mx, 4, scale, offset);
    TfEncoding g {mn, mx, scale, offset, 4};
    put(f, "gso", g);
    TensorQuantizer tq(QUANTIZATION_TF, ROUND_NEAREST);
    TfEncoding p {0, 0, 0.05, -128, 8};
    tq.computePartialEncoding(8, p, true, false, false);
    put(f, "partial", p);
    TfEncoding none = tq.computeEncoding(8, false);   // no statistics: zero encoding, not valid
    put(f, "unset", none);
    std::fprintf(f, "valid %d\n", (int) tq.isEncodingValid);
    bool threw = false;
    try
    {
        std::vector<float> hbuf(4);
        tq.updateStats(hbuf.data(), hbuf.size(), false);   // use_cuda == false: no CPU path
    }
    catch (const std::runtime_error&)
    {
        threw = true;
    }
    std::fprintf(f, "cpu_refused %d\n", (int) threw);
    std::fclose(f);
    return 0;
}

static int gpu(const char* in, long n, long C, const char* out, const char* encs)
{
    std::vector<float> h(n);
    FILE* fi = std::fopen(in, "rb");
    if (!fi || std::fread(h.data(), sizeof(float), n, fi) != (size_t) n)
        return 2;
    std::fclose(fi);
    float *x, *y, *tab;
    hipMalloc(&x, sizeof(float) * n);
    hipMalloc(&y, sizeof(float) * n * 3);
    hipMalloc(&tab, sizeof(float) * 4 * C);
    hipMemcpy(x, h.data(), sizeof(float) * n, hipMemcpyHostToDevice);
    FILE* fe = std::fopen(encs, "w");
    // every analyzer through the factory
    const QuantizationMode modes[] = {QUANTIZATION_TF, QUANTIZATION_TF_ENHANCED, QUANTIZATION_PERCENTILE,
                                      QUANTIZATION_MSE, QUANTIZATION_ENTROPY};
    const char* names[] = {"tf", "tfe", "pct", "mse", "ent"};
    for (int m = 0; m < 5; ++m)
    {
        auto a = getEncodingAnalyzerInstance<float>(modes[m]);
        a->updateStats(x, n / 2, COMP_MODE_GPU);
        a->updateStats(x + n / 2, n - n / 2, COMP_MODE_GPU);
        put(fe, names[m], a->computeEncoding(8, false, false, false));
        put(fe, names[m], a->computeEncoding(8, true, false, false));
    }
    // TensorQuantizer (the op facade): TF-E stats -> encoding -> QDQ
    TensorQuantizer tq(QUANTIZATION_TF_ENHANCED, ROUND_NEAREST);
    TensorQuantizerOpFacade& op = tq;
    op.updateStats(x, n, true);
    TfEncoding e = op.computeEncoding(8, false);
    put(fe, "facade", e);
    op.quantizeDequantize(x, n, y, e.min, e.max, 8, true);
    // per-channel QDQ with four device arrays (channel = (i / K) % C)
    std::vector<float> t(4 * C);
    for (long c = 0; c < C; ++c)
    {
        float d = 0.01f + 0.001f * (float) c;
        t[c] = -128 * d;
        t[C + c] = 127 * d;
        t[2 * C + c] = d;
        t[3 * C + c] = -128;
    }
    hipMemcpy(tab, t.data(), sizeof(float) * 4 * C, hipMemcpyHostToDevice);
    TensorQuantizationSim sim;
    sim.quantizeDequantizeTensorPerChannel(x, C, n, n / C, y + n, tab, tab + C, tab + 2 * C, tab + 3 * C,
                                           ROUND_NEAREST, true);
    sim.quantizeTensor(x, n, y + 2 * n, e.min, e.max, 8, ROUND_NEAREST, true, true);
    hipDeviceSynchronize();
    std::vector<float> r(3 * n);
    hipMemcpy(r.data(), y, sizeof(float) * 3 * n, hipMemcpyDeviceToHost);
    FILE* fo = std::fopen(out, "wb");
    std::fwrite(r.data(), sizeof(float), 3 * n, fo);
    std::fclose(fo);
    std::fclose(fe);
    hipFree(x);
    hipFree(y);
    hipFree(tab);
    return 0;
}

int main(int argc, char** argv)
{
    try
    {
        if (argc == 3 && !std::strcmp(argv[1], "host"))
            return host(argv[2]);
        if (argc == 7 && !std::strcmp(argv[1], "gpu"))
            return gpu(argv[2], std::atol(argv[3]), std::atol(argv[4]), argv[5], argv[6]);
    }
    catch (const std::exception& ex)
    {
        std::fprintf(stderr, "error: %s\n", ex.what());
        return 1;
    }
    std::fprintf(stderr, "usage: test_interfaces host <out> | gpu <in> <n> <C> <out> <encs>\n");
    return 2;
}
