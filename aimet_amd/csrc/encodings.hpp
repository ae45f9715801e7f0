// encodings.hpp -- host-side encoding math (see encodings.cpp for the reference map).
#pragma once

#include <string>
#include <vector>

#include "common.hpp"

namespace aimet_amd
{

aimet_tf_encoding computed_encoding(int32_t bw, double mn, double mx, bool sym, bool strict, bool unsign);
void gate_min_max(double& mn, double& mx);
aimet_tf_encoding fill_encoding_info(int32_t bw, double mn, double mx);
bool partial_encoding(int32_t bw, aimet_tf_encoding& e, bool sym, bool unsign, bool strict, std::string& err);
void per_channel_table_host(const aimet_tf_encoding* encs, int64_t C, float* table);

aimet_tf_encoding tf_encoding(double accMin, double accMax, int32_t bw, bool sym, bool strict, bool unsign);
aimet_tf_encoding histogram_encoding(int scheme, bool initialized, bool stats_updated, float hist_min,
                                     double bucket_size, const double* pdf, float percentile, int32_t bw, bool sym,
                                     bool strict, bool unsign);
// EntropyEncodingAnalyzer::computeEncoding from the TensorProfilingParams (min, max, 512 counts)
aimet_tf_encoding entropy_encoding(bool has_hist, bool stats_updated, double tmin, double tmax, const double* hist,
                                   int32_t bw, bool sym, bool strict, bool unsign);
// the tail of entropy_encoding for a _optimizeKL range found elsewhere (entropy_search.hip)
aimet_tf_encoding entropy_encoding_from_range(float kl_lo, float kl_hi, int32_t bw, bool sym, bool strict, bool unsign);
void histogram_xleft(float hist_min, double bucket_size, double* xleft);

}   // namespace aimet_amd
