/*
 * aimet_amd.h -- C-ABI of the MI355X-native DlQuantization hot path.
 *
 * This is the drop-in boundary that replaces the two pybind11 modules aimet_torch binds for
 * quantization simulation:
 *   - AimetTensorQuantizer          TrainingExtensions/torch/src/AimetTensorQuantizer.cpp:318-331
 *   - _libpymo (quantization subset) ModelOptimizations/PyModelOptimizations/PyModelOptimizations.cpp:147-261
 * Every entry point below names the reference interface it replaces (file:line, relative to the
 * reference repository root). Plain pointers and sizes only: no torch or pybind types cross it.
 *
 * Conventions
 *   - All float tensors are fp32 *device* pointers (HBM of an MI355X, gfx950) unless the name says
 *     _host. There is no CPU compute path: a host pointer is an error (the product fails loudly).
 *   - `stream` is a hipStream_t (nullptr = the legacy default stream). Every call is asynchronous on
 *     that stream unless documented otherwise; results stay device-resident until a get_* call.
 *   - Per-channel tensors are viewed as [outer][C][K] (channel = (i / K) % C), the reference's
 *     (numChannel, numElement, numElementPerChannel) triple (trim_functions.cpp:607-630).
 *   - Element counts are int64 (the reference uses int; results are identical below 2^31).
 *   - Return value: AIMET_OK (0) or a negative status; aimet_last_error() then holds the message.
 *     AIMET_ERR_INVALID_ARGUMENT mirrors std::invalid_argument (Python ValueError),
 *     AIMET_ERR_RUNTIME mirrors std::runtime_error (Python RuntimeError).
 */
#ifndef AIMET_AMD_H
#define AIMET_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AIMET_OK 0
#define AIMET_ERR_INVALID_ARGUMENT (-1)
#define AIMET_ERR_RUNTIME (-2)
#define AIMET_ERR_HIP (-3)

/* Quantization.hpp:84-106 QuantizationMode */
enum aimet_quantization_mode {
    AIMET_QUANTIZATION_TF = 0,
    AIMET_QUANTIZATION_TF_ENHANCED = 1,
    AIMET_QUANTIZATION_RANGE_LEARNING = 2,
    AIMET_QUANTIZATION_PERCENTILE = 3,
    AIMET_QUANTIZATION_MSE = 4,
    AIMET_QUANTIZATION_ENTROPY = 5
};

/* Quantization.hpp:140-144 RoundingMode */
enum aimet_rounding_mode { AIMET_ROUND_NEAREST = 0, AIMET_ROUND_STOCHASTIC = 1 };

/* Quantization.hpp:113-120 TfEncoding */
typedef struct aimet_tf_encoding {
    double min;
    double max;
    double delta;
    double offset;
    int32_t bw;
} aimet_tf_encoding;

/* Thread-local message of the last failing call. */
const char* aimet_last_error(void);
/* Library version string ("aimet_amd <semver> gfx950"). */
const char* aimet_version(void);
/* Number of gfx950 devices visible; negative status on HIP failure. */
int aimet_device_count(void);
/* Cap (in floats, at most its 64 MB size) on the current device's arena of partial-sum slots that
 * kernels captured into HIP graphs keep for every replay (the AdaRound round loss's last-workgroup
 * fold); *previous = the cap before. A launch captured once the arena is used up takes the same
 * fold as a launch of its own instead: the same values. For tests of that fallback. */
int aimet_capture_pool_limit(int64_t arena_floats, int64_t* previous);

/* ------------------------------------------------------------------------------------------ */
/* Encoding math (host, exact reference arithmetic)                                            */
/* ------------------------------------------------------------------------------------------ */

/* quantization_utils.cpp:58-143 getComputedEncodings */
int aimet_get_computed_encodings(int32_t bw, double min, double max, int use_symmetric, int use_strict_symmetric,
                                 int use_unsigned_symmetric, aimet_tf_encoding* out);
/* TensorQuantizationSim.cpp:62-92 fillEncodingInfo (gate, strict-symmetric detection, delta/offset) */
int aimet_fill_encoding_info(int32_t bw, double min, double max, aimet_tf_encoding* out);
/* TensorQuantizer.cpp:323-341 computePartialEncoding (in/out `enc`) */
int aimet_compute_partial_encoding(int32_t bw, aimet_tf_encoding* enc, int use_symmetric,
                                   int use_unsigned_symmetric, int use_strict_symmetric);

/* Host-side encoding analyzers applied to statistics already reduced (e.g. read back, or merged
 * from another process). They are what aimet_tq_get_encoding runs per channel.
 *   TF:        TfEncodingAnalyzer.cpp:80-101 from the running {min, max}
 *   histogram: TfEnhanced / Percentile / Mse computeEncoding from a PDF whose bucket edges are
 *              xLeft[i] = hist_min + i * bucket_size (InitializePdf, math_functions.cpp:207-241);
 *              initialized = 0 reproduces the "no histogram yet" branches. */
int aimet_encoding_from_minmax(double acc_min, double acc_max, int32_t bw, int use_symmetric,
                               int use_strict_symmetric, int use_unsigned_symmetric, aimet_tf_encoding* out);
int aimet_encoding_from_histogram(int quant_scheme, int initialized, int stats_updated, float hist_min,
                                  double bucket_size, const double* pdf_host, float percentile, int32_t bw,
                                  int use_symmetric, int use_strict_symmetric, int use_unsigned_symmetric,
                                  aimet_tf_encoding* out);
/* EntropyEncodingAnalyzer.cpp:97-435 computeEncoding (KL-divergence search, 8-bit) from the
 * analyzer's TensorProfilingParams (math_functions.hpp:71-77): the range {tpp_min, tpp_max} and the
 * 512 bin counts `hist_host`; has_histogram = 0 reproduces the "no histogram yet" branch. */
int aimet_encoding_from_entropy_histogram(int has_histogram, int stats_updated, double tpp_min, double tpp_max,
                                          const double* hist_host, int32_t bw, int use_symmetric,
                                          int use_strict_symmetric, int use_unsigned_symmetric,
                                          aimet_tf_encoding* out);

/* ------------------------------------------------------------------------------------------ */
/* Quantize-dequantize kernels                                                                 */
/* ------------------------------------------------------------------------------------------ */

/* AimetTensorQuantizer.cpp:129-155 quantizeDequantize -> TensorQuantizationSim.cpp:96-114 ->
 * trim_functions.cu:46-60. Uses enc->min/max/bw only (fillEncodingInfo is applied here).
 * `seed` is used by AIMET_ROUND_STOCHASTIC only. in == out is allowed. */
int aimet_qdq_per_tensor(const float* in, float* out, int64_t n, const aimet_tf_encoding* enc, int round_mode,
                         uint64_t seed, void* stream);

/* AimetTensorQuantizer.cpp:157-178 quantize -> trim_functions.cu:62-76 (float output holding integer
 * codes, shifted by 2^(bw-1) when shift_to_signed). */
int aimet_quantize_per_tensor(const float* in, float* out, int64_t n, const aimet_tf_encoding* enc, int round_mode,
                              int shift_to_signed, uint64_t seed, void* stream);

/* AimetTensorQuantizer.cpp:233-299 (gateMinMaxTensor / computeDeltaTensor / computeOffsetTensor):
 * builds the device table [4][C] = {min, max, delta, offset} (fp32, torch rounding semantics) from
 * `encs_host[C]`. The table depends only on the encodings: build it once per encoding change and
 * reuse it for every forward (the reference re-uploads it on every call). */
int aimet_per_channel_table(const aimet_tf_encoding* encs_host, int64_t C, float* table_dev, void* stream);

/* AimetTensorQuantizer.cpp:209-231 makeDeltaOffsetTensor: table_dev [2][C] = {(float)delta, (float)offset}. */
int aimet_make_delta_offset(const aimet_tf_encoding* encs_host, int64_t C, float* table_dev, void* stream);

/* AimetTensorQuantizer.cpp:233-307 quantizeDequantizePerChannel -> trim_functions.cu:78-92 with the
 * table from aimet_per_channel_table. N = outer*C*K elements. */
int aimet_qdq_per_channel(const float* in, float* out, int64_t outer, int64_t C, int64_t K, const float* table_dev,
                          int round_mode, uint64_t seed, void* stream);

/* Batched per-channel QDQ: every parameter quantizer of a model forward in ONE launch (the
 * reference loops over parameters in Python, one kernel + one table upload each:
 * v1/qc_quantize_op.py:753-798 -> AimetTensorQuantizer.cpp:233-307). A plan holds the device
 * copy of the descriptors; run it once per forward (graph-capturable). */
typedef struct aimet_qdq_channel_desc {
    const float* in;      /* [outer][C][K] fp32, device */
    float* out;           /* same shape, device (may equal in) */
    int64_t outer, C, K;
    const float* table;   /* [4][C] from aimet_per_channel_table */
} aimet_qdq_channel_desc;
typedef struct aimet_qdq_plan aimet_qdq_plan;
int aimet_qdq_channel_plan_create(const aimet_qdq_channel_desc* descs_host, int64_t count, int device,
                                  aimet_qdq_plan** out);
int aimet_qdq_channel_plan_run(aimet_qdq_plan* plan, int round_mode, uint64_t seed, void* stream);
int aimet_qdq_channel_plan_destroy(aimet_qdq_plan* plan);

/* quantsim_straight_through_grad.py:91-118 compute_dloss_by_dx: grad_in = grad * (min <= x <= max).
 * Per-tensor: C == 1, mins/maxs are one float each (device). */
int aimet_ste_backward(const float* x, const float* grad, float* grad_in, int64_t outer, int64_t C, int64_t K,
                       const float* mins_dev, const float* maxs_dev, void* stream);
/* Per-tensor STE with host scalars (the common activation case). */
int aimet_ste_backward_per_tensor(const float* x, const float* grad, float* grad_in, int64_t n, float enc_min,
                                  float enc_max, void* stream);

/* fp16 / bf16 I/O (io_dtype 1 = float16, 2 = bfloat16): the reference upcasts to fp32, runs the fp32
 * kernel and casts back (v1/tensor_quantizer.py:1116-1168, `.to(torch.float32)` ... `.to(dtype)`);
 * these fuse the casts (2 B in + 2 B out per element) with results identical to that sequence
 * (round-to-nearest-even downcast as torch). */
int aimet_qdq_per_tensor_16(const void* in, void* out, int64_t n, int io_dtype, const aimet_tf_encoding* enc,
                            int round_mode, uint64_t seed, void* stream);
int aimet_qdq_per_channel_16(const void* in, void* out, int64_t outer, int64_t C, int64_t K, int io_dtype,
                             const float* table_dev, int round_mode, uint64_t seed, void* stream);
/* grad_in = grad * (min <= float(x) <= max) in the grad dtype (x, grad, grad_in share io_dtype);
 * per-channel bounds mins_dev/maxs_dev[C], or per-tensor enc_min/enc_max when mins_dev is NULL. */
int aimet_ste_backward_16(const void* x, const void* grad, void* grad_in, int64_t outer, int64_t C, int64_t K,
                          int io_dtype, const float* mins_dev, const float* maxs_dev, float enc_min, float enc_max,
                          void* stream);

/* ------------------------------------------------------------------------------------------ */
/* Tensor quantizer: device-resident encoding statistics (AimetTensorQuantizer / TensorQuantizer) */
/* ------------------------------------------------------------------------------------------ */

typedef struct aimet_tensor_quantizer aimet_tensor_quantizer;

/* AimetTensorQuantizer.cpp:82-87 ctor(QuantizationMode); num_channels analyzers are held together
 * (the reference builds one AimetTensorQuantizer per channel, v1/tensor_quantizer.py:525).
 * QUANTIZATION_RANGE_LEARNING maps to TF (QuantizerFactory.cpp:93-96). `device` = HIP ordinal. */
int aimet_tq_create(int quant_scheme, int64_t num_channels, int device, aimet_tensor_quantizer** out);
int aimet_tq_destroy(aimet_tensor_quantizer* q);
/* count quantizers (schemes[i], num_channels[i]) on one device with ONE device allocation, one
 * memset and one initialisation launch (a model's quantizers are created together by
 * QuantizationSimModel; one aimet_tq_create each costs an allocation and a synchronisation).
 * Each out[i] is destroyed with aimet_tq_destroy as usual; the shared allocation is released
 * with the last of them. */
int aimet_tq_create_many(const int* schemes, const int64_t* num_channels, int64_t count, int device,
                         aimet_tensor_quantizer** out);
/* AimetTensorQuantizer.cpp:89-96 resetEncodingStats (synchronous w.r.t. `stream`). */
int aimet_tq_reset_encoding_stats(aimet_tensor_quantizer* q, void* stream);
/* resetEncodingStats of nq quantizers (one device) as two launches on `stream` (every state
 * range zeroed by one kernel, the running min/max re-initialised by another); no host
 * synchronisation (QuantizationSimModel.compute_encodings' reset of every quantizer,
 * v1/quantsim.py:387-399). */
int aimet_tq_reset_encoding_stats_many(aimet_tensor_quantizer* const* qs, int64_t nq, void* stream);
/* AimetTensorQuantizer.cpp:200-207 setPercentileValue (percentile scheme only). */
int aimet_tq_set_percentile_value(aimet_tensor_quantizer* q, float percentile);
int aimet_tq_get_percentile_value(aimet_tensor_quantizer* q, float* percentile);

/* AimetTensorQuantizer.cpp:98-127 updateStats -> TfEncodingAnalyzer.cpp:59-72 / UpdatePdf
 * (math_functions.cpp:243-288). x is [outer][C][K] with C == num_channels (per-tensor: outer=1,
 * C=1, K=n). All channels are reduced in one pass; no host synchronisation. */
int aimet_tq_update_stats(aimet_tensor_quantizer* q, const float* x, int64_t outer, int64_t C, int64_t K,
                          void* stream);

/* The same update split into phases, so a caller can exchange statistics between ranks
 * (sharded calibration):
 *   1. batch_minmax  -> q's device buffer of C pairs {-min, max} (float)   [all_reduce MAX]
 *   2. fold_minmax   -> TF: running min/max; histogram schemes: PDF range on first batch
 *   3. batch_histogram -> q's device buffer of C x 512 uint64 counts      [all_reduce SUM]
 *   4. fold_histogram(count_per_channel) -> PDF running average with the global element count */
int aimet_tq_batch_minmax(aimet_tensor_quantizer* q, const float* x, int64_t outer, int64_t C, int64_t K,
                          void* stream);
int aimet_tq_fold_minmax(aimet_tensor_quantizer* q, void* stream);
int aimet_tq_batch_histogram(aimet_tensor_quantizer* q, const float* x, int64_t outer, int64_t C, int64_t K,
                             void* stream);
int aimet_tq_fold_histogram(aimet_tensor_quantizer* q, int64_t count_per_channel, void* stream);
/* Device buffers exchanged between phases (owned by q). */
int aimet_tq_minmax_buffer(aimet_tensor_quantizer* q, float** dev, int64_t* num_floats);
int aimet_tq_counts_buffer(aimet_tensor_quantizer* q, uint64_t** dev, int64_t* num_counts);
/* Place the two exchange buffers in caller-owned device memory (e.g. one slice of a packed buffer
 * covering every quantizer, so one collective exchanges all of them). minmax_dev: 2*C floats,
 * counts_dev: 512*C uint64 (zeroed by the caller; histogram schemes only, may be NULL for TF).
 * The memory must outlive q or a later rebind. */
int aimet_tq_bind_exchange(aimet_tensor_quantizer* q, float* minmax_dev, uint64_t* counts_dev);
/* Marks statistics as updated without touching data (a rank whose shard was empty). */
int aimet_tq_mark_stats_updated(aimet_tensor_quantizer* q);

/* The statistics update of MANY per-tensor quantizers (num_channels == 1, one device) with one
 * launch per phase instead of ~5 per quantizer: a calibration batch of QuantizationSimModel
 * (v1/qc_quantize_op.py:837-897 calls updateStats once per activation quantizer). Equivalent to
 * aimet_tq_update_stats(qs[i], xs[i], 1, 1, ns[i], stream) for every i. */
int aimet_tq_update_stats_many(aimet_tensor_quantizer* const* qs, const float* const* xs, const int64_t* ns,
                               int64_t count, void* stream);
/* The phases of it for the sharded calibration (same semantics as the single-quantizer phases):
 * min/max (+ exchange buffer), fold, histogram (+ counts buffer), PDF fold with counts[i]. */
int aimet_tq_batch_minmax_many(aimet_tensor_quantizer* const* qs, const float* const* xs, const int64_t* ns,
                               int64_t count, void* stream);
int aimet_tq_fold_minmax_many(aimet_tensor_quantizer* const* qs, int64_t count, void* stream);
int aimet_tq_batch_histogram_many(aimet_tensor_quantizer* const* qs, const float* const* xs, const int64_t* ns,
                                  int64_t count, void* stream);
int aimet_tq_fold_histogram_many(aimet_tensor_quantizer* const* qs, const int64_t* counts, int64_t count,
                                 void* stream);
/* The same with the element counts read on the device from counts_dev[0..count) (int64 in HBM): the
 * sharded calibration sums them over ranks in the same all_reduce as the bin counts, so the fold
 * needs no host round trip. */
int aimet_tq_fold_histogram_many_dev(aimet_tensor_quantizer* const* qs, const int64_t* counts_dev, int64_t count,
                                     void* stream);
/* updateStats of many quantizers of any channel count, each tensor viewed as [outers[i]][Cs[i]][Ks[i]]
 * (Cs[i] == num_channels of qs[i]), in two launches with one workgroup per channel: the weight
 * quantizers of a model (v1/tensor_quantizer.py:535-571 per weight, batched). Equivalent to
 * aimet_tq_update_stats(qs[i], xs[i], outers[i], Cs[i], Ks[i], stream) for every i; meant for
 * per-channel quantizers (one workgroup streams a whole per-tensor quantizer's tensor). */
int aimet_tq_update_stats_channels_many(aimet_tensor_quantizer* const* qs, const float* const* xs,
                                        const int64_t* outers, const int64_t* Cs, const int64_t* Ks, int64_t count,
                                        void* stream);

/* AimetTensorQuantizer.cpp:180-192 getEncoding -> IQuantizationEncodingAnalyzer::computeEncoding.
 * Synchronises `stream`. out[num_channels]; *valid mirrors _isEncodingValid. */
int aimet_tq_get_encoding(aimet_tensor_quantizer* q, uint32_t bw, int use_symmetric, int use_strict_symmetric,
                          int use_unsigned_symmetric, aimet_tf_encoding* out, int* valid, void* stream);
/* getEncoding of nq quantizers (one device) with one stream synchronisation: every device-side
 * search is enqueued first (QuantizationSimModel.compute_encodings' per-quantizer loop,
 * v1/quantsim.py:425-449, batched). out = the quantizers' encodings concatenated
 * (sum of num_channels); valid[nq]. */
int aimet_tq_get_encodings(aimet_tensor_quantizer* const* qs, int64_t nq, uint32_t bw, int use_symmetric,
                           int use_strict_symmetric, int use_unsigned_symmetric, aimet_tf_encoding* out, int* valid,
                           void* stream);

/* aimet_tq_get_encodings in two halves, so the host can enqueue more work (another stream's
 * searches, the next batch) before it waits: _launch enqueues every device search on `stream`
 * and the copies of their results into pinned memory, and returns a request; _finish waits for
 * it, finishes the host-side encodings (TF, percentile, entropy near-ties) and frees the request
 * (always, also on error). out == valid == NULL discards the request: it waits for the request's
 * device work (so its pinned result block is idle) and frees it. */
typedef struct aimet_encoding_request aimet_encoding_request;
int aimet_tq_get_encodings_launch(aimet_tensor_quantizer* const* qs, int64_t nq, uint32_t bw, int use_symmetric,
                                  int use_strict_symmetric, int use_unsigned_symmetric, void* stream,
                                  aimet_encoding_request** request);
int aimet_tq_get_encodings_finish(aimet_encoding_request* request, aimet_tf_encoding* out, int* valid);

/* One calibration batch of tensors already resident in HBM, every quantizer in one call:
 * QuantizationSimModel.compute_encodings' resetEncodingStats (reset != 0) + updateStats of every
 * quantizer + getEncoding of every quantizer (v1/quantsim.py:381-449), enqueued with no host wait.
 * Activations (per-tensor, act_x[i] of act_n[i] floats) on `main_stream`: one launch per phase for
 * all of them + one search launch. Parameters (per channel of [outer][C][K]) first, on
 * `side_stream` (which waits for `main_stream`; `main_stream` then waits for it) or, when the two
 * are the same stream, ahead of the activations on it: two statistics launches + one search launch. act_settings / par_settings = {bw, symmetric, strict, unsigned}. The two
 * requests are finished (and freed) with aimet_tq_get_encodings_finish; on error neither exists.
 * Either count may be 0. aimet_amd's Python host issues two calls per batch: the activations
 * (n_par = 0; *par_req is then null) with the side stream already waiting for the inputs, then the
 * parameters (n_act = 0, both streams the side stream; *act_req is an empty request, finished like
 * any other), after which the main stream waits for the side stream -- the parameters' host
 * preparation then overlaps the activations' min/max pass. */
int aimet_calibrate_launch(aimet_tensor_quantizer* const* act_qs, const float* const* act_x, const int64_t* act_n,
                           int64_t n_act, aimet_tensor_quantizer* const* par_qs, const float* const* par_x,
                           const int64_t* par_outer, const int64_t* par_C, const int64_t* par_K, int64_t n_par,
                           const int32_t* act_settings, const int32_t* par_settings, int reset, void* main_stream,
                           void* side_stream, aimet_encoding_request** act_req, aimet_encoding_request** par_req);

/* A calibration plan: aimet_calibrate_launch's work for a FIXED set of quantizers and resident
 * tensors (the same arguments, the tensors' contents may change between launches), prepared once
 * -- every job table, the parameters' reset ranges, the TF-Enhanced search tables and hand-off
 * buffers in one device allocation, the TF-Enhanced results written by the searches straight into
 * the plan's pinned host blocks -- so that a launch is only kernel launches (QuantizationSimModel
 * .compute_encodings on an existing sim, v1/quantsim.py:381-449, repeated per batch or per
 * recalibration). elem_counts_dev (NULL on one device): the sharded calibration's element counts,
 * one int64 per histogram activation quantizer in order (the tail of the packed SUM buffer,
 * aimet_amd/distributed.py); the quantizers must already be bound to the packed exchange buffers
 * (aimet_tq_bind_exchange), and neither they nor the tensors may be re-bound, freed or destroyed
 * while the plan lives. */
typedef struct aimet_calib_plan aimet_calib_plan;
int aimet_calib_plan_create(aimet_tensor_quantizer* const* act_qs, const float* const* act_x, const int64_t* act_n,
                            int64_t n_act, aimet_tensor_quantizer* const* par_qs, const float* const* par_x,
                            const int64_t* par_outer, const int64_t* par_C, const int64_t* par_K, int64_t n_par,
                            const int32_t* act_settings, const int32_t* par_settings, int64_t* elem_counts_dev,
                            aimet_calib_plan** plan);
/* stages = 7: one batch on one device, as aimet_calibrate_launch (reset != 0: resetEncodingStats
 * first). The sharded calibration launches stage 1 (resets, the parameters'
 * statistics + search on side_stream, the activations' min/max pass and element counts), then,
 * after its all_reduce(MAX) of the packed {-min, max}, stage 2 (PDF ranges + histogram pass), then,
 * after its all_reduce(SUM) of the packed counts, stage 4 (PDF fold + the activations' search).
 * *par_req comes from the stage-1 launch, *act_req from the stage-4 launch (NULL otherwise); both
 * are finished with aimet_tq_get_encodings_finish, and the plan launches its next stage 1 / 4
 * only once the previous request of that kind is finished. A plan (like its quantizers) is used by
 * one host thread at a time. */
int aimet_calib_plan_launch(aimet_calib_plan* plan, int stages, int reset, void* main_stream, void* side_stream,
                            aimet_encoding_request** act_req, aimet_encoding_request** par_req);
/* Waits for the device, frees the plan (its requests must be finished first). */
int aimet_calib_plan_destroy(aimet_calib_plan* plan);

/* AimetTensorQuantizer.cpp:194-198 getStatsHistogram (histogram schemes): xleft/pdf[512] of
 * `channel`; *n = 0 when no histogram exists yet. Synchronises `stream`. */
int aimet_tq_get_stats_histogram(aimet_tensor_quantizer* q, int64_t channel, double* xleft, double* pdf, int* n,
                                 void* stream);
/* The entropy analyzer's TensorProfilingParams of `channel` (math_functions.hpp:71-77): minmax[2] =
 * {min, max}, hist[512] = bin counts, *has_histogram = histogram.size() != 0. Synchronises `stream`. */
int aimet_tq_get_entropy_state(aimet_tensor_quantizer* q, int64_t channel, double* minmax_host, double* hist_host,
                               int* has_histogram, int* iterations, void* stream);

int aimet_tq_num_channels(aimet_tensor_quantizer* q, int64_t* num_channels);
int aimet_tq_quant_scheme(aimet_tensor_quantizer* q, int* quant_scheme);

/* ------------------------------------------------------------------------------------------ */
/* Range-learning (LearnedGrid) QAT: quantsim_straight_through_grad.py:191-328,                  */
/* QuantizeDequantizeFunc v1/tensor_quantizer.py:896-986                                         */
/* ------------------------------------------------------------------------------------------ */

/* y = (clamp(round_half_even(x/delta) - offset, 0, num_steps) + offset) * delta, delta/offset per
 * channel of [outer][C][K] (C == 1: per-tensor), float32 device vectors. */
int aimet_lg_forward(const float* x, float* y, int64_t outer, int64_t C, int64_t K, const float* delta_dev,
                     const float* offset_dev, float num_steps, void* stream);
/* grad_x = mask * grad (grad_x may be NULL) and per-channel sums_dev[C][3] = {A, B, D} from which
 * the encoding-min/max gradients are assembled (asymmetric_gradients / symmetric_gradients, with
 * (A - B) as grad_scale's sum): with no range spec, or a symmetric one,
 * A = sum((x_quant+offset)*grad), B = sum((mask*(x/delta))*grad) (D = sum(!mask*grad) with no spec,
 * 0 with a symmetric one); with an asymmetric spec A = sum((x_quant+offset - x*mask/delta)*grad),
 * the reference's single grad_scale sum, B = 0 and D = sum(!mask*grad). NaN / inf inputs turn the
 * sums NaN where the reference's do. */
/* Optional epilogue of the learned-grid backward entry points: the encoding-min/max gradients
 * (aimet_lg_range_grads' arithmetic) written by the kernel that folds the sums, no extra launch.
 * null: the sums only. */
typedef struct
{
    const float* encoding_min;   /* [C] device */
    const float* encoding_max;   /* [C] device */
    const float* delta;          /* [C] device, as passed to the backward */
    float* grad_min;             /* [C] device out */
    float* grad_max;             /* [C] device out */
    int use_symmetric;
} aimet_lg_range_spec;
int aimet_lg_backward(const float* x, const float* grad, float* grad_x, float* sums_dev, int64_t outer, int64_t C,
                      int64_t K, const float* delta_dev, const float* offset_dev, float num_steps,
                      const aimet_lg_range_spec* range_spec, void* stream);
/* The learned-grid forward / backward for a per-tensor range on fp16 (io_dtype 1) or bf16 (2)
 * tensors with the casts in registers: results identical to x.to(float32) -> aimet_lg_forward /
 * aimet_lg_backward -> .to(dtype) (same arithmetic, same order of the backward's sums), 4 / 6 B
 * per element instead of 20 / 24 (QAT under autocast: bf16 activations quantized by 16-bit
 * output quantizers). sums_dev[3] as aimet_lg_backward's channel 0. */
int aimet_lg_forward_16(const void* x, void* y, int64_t n, int io_dtype, const float* delta_dev,
                        const float* offset_dev, float num_steps, void* stream);
int aimet_lg_backward_16(const void* x, const void* grad, void* grad_x, float* sums_dev, int64_t n, int io_dtype,
                         const float* delta_dev, const float* offset_dev, float num_steps,
                         const aimet_lg_range_spec* range_spec, void* stream);
/* A float32 weight consumed in 16 bits (a Linear under autocast): the forward writes the
 * quantize-dequantized weight cast to fp16 / bf16 in the same pass (== aimet_lg_forward then
 * .to(dtype), as autocast casts it for the matmul); the backward takes the matmul's 16-bit weight
 * gradient and upcasts it in registers (== aimet_lg_backward on grad.to(float32): same arithmetic,
 * same summation order; per-channel rows of a multiple of 1024 elements, see _supported). 6 B and
 * 10 B per element instead of 8 + 6 and 12 + 6 with the separate casts. */
/* The per-channel vectors around the learned-grid passes, one launch each, results equal to the
 * reference's torch ops bit for bit: _gate_range = set_encoding_min_max_gating_threshold
 * (v1/tensor_quantizer.py:1347-1359) in place; _encodings = get_computed_encodings
 * (quantsim_straight_through_grad.py:121-160) -> delta[C], offset[C]; _range_grads = the encoding
 * gradients of asymmetric_gradients / symmetric_gradients (:252-328) from aimet_lg_backward's sums. */
int aimet_lg_gate_range(float* emin_dev, float* emax_dev, int64_t C, void* stream);
/* The same gate over n <= 8 ranges (emin[r], emax[r] of C[r] floats each; host arrays of device
 * pointers) in one launch: QcQuantizeWrapper.apply_gating_logic (v1/qc_quantize_op.py:1019-1055)
 * over a wrapper's quantizers. */
int aimet_lg_gate_ranges(float* const* emin_dev, float* const* emax_dev, const int64_t* C, int n, void* stream);
int aimet_lg_encodings(const float* emin_dev, const float* emax_dev, int64_t C, int bitwidth, int use_symmetric,
                       int use_strict_symmetric, int is_unsigned_symmetric, float* delta_dev, float* offset_dev,
                       void* stream);
int aimet_lg_range_grads(const float* sums_dev, const float* emin_dev, const float* emax_dev, const float* delta_dev,
                         int64_t C, float num_steps, int use_symmetric, float* grad_min_dev, float* grad_max_dev,
                         void* stream);
/* The learned-grid forward with get_computed_encodings done in the same kernel: delta / offset of
 * every channel computed from the range (equal to aimet_lg_encodings) and stored to
 * delta_out / offset_out for the backward. range_out (optional, [2][C]): the range as the kernel
 * read it (min row, max row) -- the reference's encoding_min/max.clone() saved for the backward
 * (v1/tensor_quantizer.py:940-951), so an in-place gate between forward and backward (a module
 * called twice) leaves the saved range alone. out_dtype 0: float32 result (aimet_lg_forward), 1 / 2:
 * the fp16 / bf16 cast (aimet_lg_forward_cast); _16_range: aimet_lg_forward_16. */
int aimet_lg_forward_range(const float* x, void* y, int64_t outer, int64_t C, int64_t K, int out_dtype,
                           const float* encoding_min_dev, const float* encoding_max_dev, int bitwidth,
                           int use_symmetric, int use_strict_symmetric, int is_unsigned_symmetric, float* delta_out,
                           float* offset_out, float* range_out, void* stream);
int aimet_lg_forward_16_range(const void* x, void* y, int64_t n, int io_dtype, const float* encoding_min_dev,
                              const float* encoding_max_dev, int bitwidth, int use_symmetric,
                              int use_strict_symmetric, int is_unsigned_symmetric, float* delta_out,
                              float* offset_out, float* range_out, void* stream);
/* The float32-input forward passes of more than 2^30 elements run as sub-problems of whole rows /
 * channel ranges / row pieces (the reference's torch ops have no element limit,
 * quantsim_straight_through_grad.py:191-249). Testing hook: lower that bound to `elems`
 * (1024 .. 2^30; 0 restores the default) so the chunking is exercised on small tensors. */
int aimet_lg_set_chunk_limit(int64_t elems);
int aimet_lg_forward_cast(const float* x, void* y, int64_t outer, int64_t C, int64_t K, int out_dtype,
                          const float* delta_dev, const float* offset_dev, float num_steps, void* stream);
int aimet_lg_backward_grad16(const float* x, const void* grad, float* grad_x, float* sums_dev, int64_t outer,
                             int64_t C, int64_t K, int grad_dtype, const float* delta_dev, const float* offset_dev,
                             float num_steps, const aimet_lg_range_spec* range_spec, void* stream);
int aimet_lg_backward_grad16_supported(int64_t outer, int64_t C, int64_t K, const void* x, const void* grad,
                                       const void* grad_x);

/* ------------------------------------------------------------------------------------------ */
/* AdaRound soft rounding (v1/adaround/adaround_wrapper.py:124-149, adaround_loss.py:83-133)     */
/* ------------------------------------------------------------------------------------------ */

/* Wq = (clamp(floor(W/delta) + h(alpha) - offset, 0, 2^bw-1) + offset) * delta,
 * h = clamp(sigmoid(alpha)*(zeta-gamma)+gamma, 0, 1) (soft) or (alpha >= 0) (hard).
 * delta/offset broadcast along the channel axis of [outer][C][K] (per-tensor: C == 1).
 * Bit-identical to the reference's torch float32 ops on the CPU (torch's vectorized sigmoid). */
int aimet_adaround_forward(const float* w, const float* alpha, float* wq, int64_t outer, int64_t C, int64_t K,
                           const float* delta_dev, const float* offset_dev, int32_t bw, int use_soft_rounding,
                           void* stream);
/* dL/dalpha of the forward above (torch autograd of apply_adaround, op by op) plus, when
 * reg_param != 0, the round-loss gradient d/dalpha reg*sum(1-|2h-1|^beta) added as autograd adds
 * the two branches, and the round loss itself accumulated into round_loss_dev[0] (fp32,
 * atomically; caller zeroes it). reg_param / beta are the reference's python doubles (beta - 1 is
 * formed in double, as torch's pow_backward does). */
int aimet_adaround_backward(const float* w, const float* alpha, const float* grad_wq, float* grad_alpha,
                            int64_t outer, int64_t C, int64_t K, const float* delta_dev, const float* offset_dev,
                            int32_t bw, double reg_param, double beta, float* round_loss_dev, void* stream);
/* adaround_loss.py:70-80 compute_recon_loss + its autograd backward in one pass: grad[i] =
 * d/dq of mean(||act(q) - act(t)||^2 over dim 1) = 2 (act(q) - act(t)) act'(q) / (n / reduced),
 * where `reduced` is the size of dim 1 (channels / features) and act is 0 none, 1 ReLU,
 * 2 ReLU6 (the layer's following activation, applied to both outputs as the reference does). */
int aimet_adaround_recon_grad(const float* quant_out, const float* orig_out, float* grad, int64_t n, int64_t reduced,
                              int act, void* stream);
/* aimet_adaround_backward with {reg_param, beta, beta - 1} read from device memory
 * (reg_beta_dev[3], float32) when the kernel runs: the AdaRound iteration captured once in a HIP
 * graph and replayed with the annealed beta of each iteration (adaround_optimizer.py:115-222's
 * loop; aimet_amd.adaround_optimizer). */
int aimet_adaround_backward_dev(const float* w, const float* alpha, const float* grad_wq, float* grad_alpha,
                                int64_t outer, int64_t C, int64_t K, const float* delta_dev, const float* offset_dev,
                                int32_t bw, const float* reg_beta_dev, float* round_loss_dev, void* stream);
/* The single-process AdaRound loop's batch draw (adaround_optimizer.py:181-218: randperm'd
 * indices, index_select of the cached inputs and fp outputs) as one kernel: it = it_cur_dev[0];
 * rows idx_all_dev[it * nb + b] (int64, [iterations][nb]) of src_in / src_out ([N][row_in],
 * [N][row_out]) are copied to dst_in[b] / dst_out[b] (dst_out may be null: inputs only);
 * it_next_dev[0] = it + 1. For a HIP-graph replayed iteration (the counters live in device
 * memory). */
int aimet_adaround_gather(const float* src_in, const float* src_out, float* dst_in, float* dst_out,
                          const int64_t* idx_all_dev, const int64_t* it_cur_dev, int64_t* it_next_dev, int64_t nb,
                          int64_t row_in, int64_t row_out, void* stream);
/* aimet_adaround_recon_grad for the same replayed iteration with the fp target read in place:
 * sample b's target is row idx_all_dev[it * nb + b] of out_data ([N][C][hw]), it = it_cur_dev[0];
 * bias_dev (nullable, [C]) is added to quant_out first (a bias-free GEMM output). grad and
 * quant_out are the [nb][C][hw] batch. dst_out of aimet_adaround_gather may then be null. */
int aimet_adaround_recon_grad_indexed(const float* quant_out, const float* out_data, const int64_t* idx_all_dev,
                                      const int64_t* it_cur_dev, float* grad, int64_t nb, int64_t C, int64_t hw,
                                      const float* bias_dev, int act, void* stream);
/* Channel-major forms for a 1x1 layer's GEMM loop: aimet_adaround_gather_cm writes the batch's
 * inputs as dst[ci][b][hw] (rows idx_all_dev[it * nb + b] of src_in [N][Cin][hw]; it_next_dev[0] =
 * it + 1), so q = W x and dL/dW = g x^T are single GEMMs over all nb * hw positions;
 * aimet_adaround_recon_grad_indexed_cm is aimet_adaround_recon_grad_indexed for q / grad in the
 * [C][nb][hw] layout (targets read in place from out_data [N][C][hw]). */
int aimet_adaround_gather_cm(const float* src_in, float* dst, const int64_t* idx_all_dev, const int64_t* it_cur_dev,
                             int64_t* it_next_dev, int64_t nb, int64_t Cin, int64_t hw, void* stream);
int aimet_adaround_recon_grad_indexed_cm(const float* quant_out, const float* out_data, const int64_t* idx_all_dev,
                                         const int64_t* it_cur_dev, float* grad, int64_t nb, int64_t C, int64_t hw,
                                         const float* bias_dev, int act, void* stream);
/* aimet_adaround_backward + torch.optim.Adam(fused=True)'s update of alpha (no weight decay /
 * amsgrad) in one pass, for the same replayed iteration: step = it_next_dev[0] (1-based),
 * {reg, beta, beta - 1} = reg_beta_all_dev[3 * (step - 1) ..] (float32), alpha / exp_avg /
 * exp_avg_sq (the Adam moments, zero-initialised by the caller) updated in place with ATen's
 * per-element arithmetic (bias corrections 1 - beta^step in double); it_cur_dev[0] = step;
 * the round loss accumulated into round_loss_dev[0] when non-null; when wq_next_dev is non-null,
 * the next iteration's soft-quantized weight (aimet_adaround_forward of the updated alpha, same
 * arithmetic) is written there in the same pass. */
int aimet_adaround_backward_adam(const float* w, float* alpha, const float* grad_wq, float* exp_avg_dev,
                                 float* exp_avg_sq_dev, int64_t outer, int64_t C, int64_t K, const float* delta_dev,
                                 const float* offset_dev, int32_t bw, const float* reg_beta_all_dev,
                                 const int64_t* it_next_dev, int64_t* it_cur_dev, double lr, double beta1,
                                 double beta2, double eps, float* round_loss_dev, float* wq_next_dev, void* stream);

/* aimet_adaround_backward_adam with the weight gradient given as `nparts` slices added in slice
 * order (s = 0, 1, ...) element by element: part_kk == 0: grad_parts[s][n] (n = outer * C * K);
 * part_kk > 0: grad_parts[n / part_kk][s]
 * [part_kk] from +0 (the depthwise step's per-channel slices, aimet_adaround_dw_step with grad_w
 * NULL: the sum is its fold's, bit for bit). bias_corr_dev (nullable): the table of
 * aimet_adaround_adam_bias_corrections for beta1 / beta2, read at step instead of computing the
 * bias corrections in the kernel (same bits). nparts == 1 and bias_corr_dev == NULL is
 * aimet_adaround_backward_adam. */
int aimet_adaround_backward_adam_parts(const float* w, float* alpha, const float* grad_parts, int64_t nparts,
                                       int64_t part_kk, float* exp_avg_dev, float* exp_avg_sq_dev, int64_t outer, int64_t C, int64_t K,
                                       const float* delta_dev, const float* offset_dev, int32_t bw,
                                       const float* reg_beta_all_dev, const int64_t* it_next_dev, int64_t* it_cur_dev,
                                       double lr, double beta1, double beta2, double eps, float* round_loss_dev,
                                       float* wq_next_dev, const float* bias_corr_dev, void* stream);
/* Adam's bias corrections for step = 1 .. steps, as ATen's fused Adam computes them (1 - beta^step
 * in double, rounded to float; the second as its square root): bias_corr_dev[2 (step - 1)] =
 * bc1, [2 (step - 1) + 1] = sqrt(bc2) (float32, 2 * steps entries). */
int aimet_adaround_adam_bias_corrections(double beta1, double beta2, int64_t steps, float* bias_corr_dev,
                                         void* stream);
/* The rounding loss's pow(|2h - 1|, beta) / pow(|2h - 1|, beta - 1) (adaround_loss.py:83-110) of
 * every AdaRound backward launched afterwards, process-wide: 0 (default) a table-driven f32
 * evaluation within 1 ulp of torch's CPU pow (Sleef powf_u10) over every f32 input in (0, 1) and
 * the AdaRound beta schedules; 1 the bit-exact emulation of torch's pow (about 3x the arithmetic). Wq and the
 * reconstruction term of dL/dalpha do not depend on it. */
int aimet_adaround_set_exact_pow(int exact);
int aimet_adaround_get_exact_pow(int* exact);

/* Depthwise 2-D convolution (groups == C, weights [C][1][K][K], K = 3 or 5, square stride /
 * padding / dilation, NCHW fp32): the AdaRound loop's layer math on depthwise layers
 * (adaround_optimizer.py:257-286 runs the wrapped layer's forward and autograd's weight gradient;
 * no input gradient is needed). Forward: y = bias + sum w * x (bias may be null). Weight
 * gradient: grad_w[C][K][K] = sum over n, oh, ow of grad_y * x, in a fixed order (deterministic);
 * `workspace` (aimet_dwconv2d_grad_weight_workspace elements, device) may be null (internal
 * scratch) -- pass one to keep the call allocation-free inside a HIP-graph capture. */
int aimet_dwconv2d_forward(const float* x, const float* w, const float* bias, float* y, int64_t N, int64_t C,
                           int64_t H, int64_t W, int64_t OH, int64_t OW, int32_t K, int32_t stride, int32_t pad,
                           int32_t dilation, void* stream);
int aimet_dwconv2d_grad_weight_workspace(int64_t N, int64_t C, int64_t OH, int64_t OW, int32_t K, int64_t* elems);
int aimet_dwconv2d_grad_weight(const float* x, const float* grad_y, float* grad_w, float* workspace, int64_t N,
                               int64_t C, int64_t H, int64_t W, int64_t OH, int64_t OW, int32_t K, int32_t stride,
                               int32_t pad, int32_t dilation, void* stream);

/* The AdaRound iteration of a depthwise layer up to dL/dWq in one pass (no batch copy, no q / g
 * tensors): for iteration it = it_cur_dev[0], sample n of the batch is row idx_all_dev[it * N + n]
 * of x_cache ([rows][C][H][W]) and target_cache ([rows][C][OH][OW], the fp layer outputs); q =
 * aimet_dwconv2d_forward(x, w, bias), g = aimet_adaround_recon_grad_indexed's gradient of q
 * (act 0 none, 1 ReLU, 2 ReLU6) and grad_w = aimet_dwconv2d_grad_weight(x, g): bit-identical to
 * aimet_adaround_gather + those three calls. it_next_dev[0] = it + 1 (as aimet_adaround_gather).
 * `workspace` as aimet_dwconv2d_grad_weight. */
int aimet_adaround_dw_step(const float* x_cache, const float* target_cache, const int64_t* idx_all_dev,
                           const int64_t* it_cur_dev, int64_t* it_next_dev, const float* w, const float* bias,
                           float* grad_w, float* workspace, int64_t N, int64_t C, int64_t H, int64_t W, int64_t OH,
                           int64_t OW, int32_t K, int32_t stride, int32_t pad, int32_t dilation, int32_t act,
                           void* stream);
/* the slice count S of aimet_adaround_dw_step's [C][S][K K] weight-gradient partials (its
 * workspace, left unfolded when grad_w is NULL) for the same shape and target cache */
int aimet_adaround_dw_step_slices(const float* target_cache, int64_t N, int64_t C, int64_t OH, int64_t OW, int32_t K,
                                  int32_t stride, int32_t dilation, int64_t* slices);

/* The AdaRound iteration of a 1x1 convolution (or the unfolded stem) with few channels up to
 * dL/dWq in one pass: sample n of the batch is row idx_all_dev[it * N + n] (it = it_cur_dev[0])
 * of x_cache ([rows][Cin][HW]) and target_cache ([rows][Cout][HW]); q = W @ x (W [Cout][Cin],
 * sums over ci in order), g = aimet_adaround_recon_grad_indexed's gradient of q + bias (bias
 * nullable; act 0 none, 1 ReLU, 2 ReLU6), grad_w = sum over the batch positions of g x^T in a
 * fixed order (deterministic; fp32, not bit-identical to a library GEMM). it_next_dev[0] = it + 1.
 * Cin <= 192 (any Cout: row ranges of at most 6144 / Cin rows per workgroup), HW % 4 == 0, x_cache
 * and target_cache 16-B aligned. `workspace`
 * (aimet_adaround_pw_step_workspace elements, device) may be null (internal scratch). */
int aimet_adaround_pw_step_workspace(int64_t N, int64_t Cin, int64_t Cout, int64_t HW, int64_t* elems);
/* *uses = 1 when aimet_adaround_pw_step runs a (Cin, Cout) layer on the f32 matrix cores (C_in >= 32
 * and its staging fits in LDS), 0 for the VALU form: the loop's choice of the one-pass step for
 * projecting layers depends on it (adaround_optimizer.py). */
int aimet_adaround_pw_step_uses_mfma(int64_t Cin, int64_t Cout, int* uses);
int aimet_adaround_pw_step(const float* x_cache, const float* target_cache, const int64_t* idx_all_dev,
                           const int64_t* it_cur_dev, int64_t* it_next_dev, const float* w, const float* bias,
                           float* grad_w, float* workspace, int64_t N, int64_t Cin, int64_t Cout, int64_t HW,
                           int32_t act, void* stream);
/* aimet_adaround_pw_step with grad_w NULL leaves the weight gradient as ordered slices in its
 * workspace: elements [offset, offset + slices * C_in * C_out) hold [slices][C_out][C_in], which
 * aimet_adaround_backward_adam_parts adds with part_kk = C_in * C_out (from +0, the fold's sum) */
int aimet_adaround_pw_step_slices(int64_t N, int64_t Cin, int64_t Cout, int64_t HW, int64_t* offset, int64_t* slices);

/* ------------------------------------------------------------------------------------------ */
/* Blockwise (broadcast) quantization and the ONNX QcQuantizeOp                                */
/* ------------------------------------------------------------------------------------------ */

/* trim_functions.cpp:633-687 quantizeDequantizeBroadcast (Quantization.hpp:150-215): the E
 * encodings (device float arrays enc_*[E], used as given: no fillEncodingInfo) broadcast over a
 * contiguous tensor of n elements viewed with num_dims dims; input_strides_host = its row-major
 * strides, encoding_strides_host = the encodings' strides, 0 along broadcast dims. ROUND_NEAREST. */
int aimet_qdq_broadcast(const float* in, float* out, int64_t n, int64_t num_dims, const int64_t* input_strides_host,
                        const int64_t* encoding_strides_host, const float* enc_min, const float* enc_max,
                        const float* enc_delta, const float* enc_offset, void* stream);
/* onnx/src/QuantizeDequantizeUtils.cpp:64-95 permuteTensor: out[sum_d idx_d(i) * output_strides[d]] = in[i]. */
int aimet_permute_tensor(const float* in, float* out, int64_t n, int64_t num_dims, const int64_t* input_strides_host,
                         const int64_t* output_strides_host, void* stream);
/* quantizeDequantizeFp16 (onnx/src/AimetOpUtils.cpp:61-67, trim_functions.cu:135-148): out = (float)(half) in,
 * round to nearest even. */
int aimet_qdq_fp16(const float* in, float* out, int64_t n, void* stream);

#define AIMET_BCAST_MAX_DIMS 16
/* onnx/src/QuantizeDequantizeUtils.hpp:166-178 BroadcastShapeInfo: the input viewed with the block
 * axis split into (num_blocks, block_size) and the broadcastable encoding shape. */
typedef struct aimet_broadcast_shape_info {
    int64_t num_dims;
    int64_t tensor_shape[AIMET_BCAST_MAX_DIMS];
    int64_t encoding_shape[AIMET_BCAST_MAX_DIMS];
    int64_t tensor_strides[AIMET_BCAST_MAX_DIMS];
    int64_t encoding_strides[AIMET_BCAST_MAX_DIMS];
    int64_t num_elements;
    int64_t num_encodings;
    int contiguous_blocks; /* hasContiguousBlocks() */
} aimet_broadcast_shape_info;
/* QuantizeDequantizeUtils.cpp:100-170 (channel_axis / block_axis < 0: none). Host only. */
int aimet_broadcast_shape_info_init(const int64_t* input_shape, int64_t ndims, int channel_axis, int block_axis,
                                    int block_size, aimet_broadcast_shape_info* out);
/* QuantizeDequantizeUtils.cpp:173-213 copyToContiguousBlockLayout: every quantization block contiguous. */
int aimet_copy_to_contiguous_block_layout(const float* in, float* out, const aimet_broadcast_shape_info* info,
                                          void* stream);

/* TensorQuantizerOpMode (TensorQuantizerOpFacade.h:48-54) */
enum {
    AIMET_OP_UPDATE_STATS = 0,
    AIMET_OP_ONE_SHOT_QUANTIZE_DEQUANTIZE = 1,
    AIMET_OP_QUANTIZE_DEQUANTIZE = 2,
    AIMET_OP_PASS_THROUGH = 3
};
/* onnx/src/QcQuantizeInfo.h:46-73 with the TensorQuantizer settings its tensorQuantizerRef carry
 * (TensorQuantizer.h: roundingMode, strict / unsigned symmetric). The reference holds one
 * TensorQuantizer per encoding; here ONE aimet_tensor_quantizer with num_channels ==
 * num_encodings (1 per-tensor) holds all their analyzers. `encodings` is the caller's host array,
 * updated in place by oneShotQuantizeDequantize (min, max, offset, delta). */
typedef struct aimet_qc_quantize_info {
    int op_mode;
    int enabled;
    int is_int_data_type;
    int use_per_channel_mode;
    int channel_axis;
    int block_axis;
    int block_size;
    int use_symmetric_encoding;
    int use_strict_symmetric;
    int use_unsigned_symmetric;
    int rounding_mode;
    int64_t num_encodings;
    aimet_tf_encoding* encodings;
    aimet_tensor_quantizer* quantizer;
} aimet_qc_quantize_info;
/* onnx/src/QcQuantizeOp.cpp:62-113 QcQuantizeOp::computeImpl on a contiguous fp32 device tensor
 * of shape[ndims] (the ORT custom op's Compute; `stream` = the EP's compute stream). After a
 * oneShotQuantizeDequantize the info switches to quantizeDequantize. */
int aimet_qc_quantize_op_compute(aimet_qc_quantize_info* info, const float* in, float* out, const int64_t* shape,
                                 int64_t ndims, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* AIMET_AMD_H */
