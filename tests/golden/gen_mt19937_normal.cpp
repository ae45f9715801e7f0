// Regenerates the input data of the reference KATs TestTensorQuantizer.SanityTestCpu
// (ModelOptimizations/DlQuantization/test/TestTensorQuantizer.cpp:89-103, 6000 samples) and
// TestEntropyEncodingAnalyzer (TestEntropyEncodingAnalyzer.cpp:56-80, 100000 samples):
// std::normal_distribution<float>(2, 2) drawn from std::mt19937(1).
// libstdc++'s mt19937 and normal_distribution are deterministic, so the bytes written
// here are the exact tensor that KAT feeds to the TF-Enhanced analyzer.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

int main(int argc, char** argv)
{
    const char* path = argc > 1 ? argv[1] : "tfe_kat_data.f32";
    std::normal_distribution<float> distribution(2.0f, 2.0f);
    std::mt19937 generator(1);
    std::vector<float> data(argc > 2 ? std::atoi(argv[2]) : 6000);
    for (auto& v: data)
        v = distribution(generator);
    FILE* f = std::fopen(path, "wb");
    if (!f)
        return 1;
    std::fwrite(data.data(), sizeof(float), data.size(), f);
    std::fclose(f);
    return 0;
}
