"""ctypes binding of libaimet_amd.so (include/aimet_amd.h).

The library is the only compute path: there is no CPU or PyTorch fallback. If it is missing or
fails to load, every entry point raises immediately (`NativeLibraryError`).
"""
import ctypes
import os
import subprocess

import torch  # noqa: F401  -- load torch's HIP runtime first so libaimet_amd binds to the same one

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libaimet_amd.so")
CSRC = os.path.join(_HERE, "csrc")

AIMET_OK = 0
AIMET_ERR_INVALID_ARGUMENT = -1
AIMET_ERR_RUNTIME = -2
AIMET_ERR_HIP = -3


class NativeLibraryError(RuntimeError):
    """libaimet_amd.so is missing or unusable; aimet_amd has no fallback path."""


class HipError(RuntimeError):
    """A HIP runtime call inside libaimet_amd failed."""


class TfEncodingC(ctypes.Structure):
    _fields_ = [("min", ctypes.c_double), ("max", ctypes.c_double), ("delta", ctypes.c_double),
                ("offset", ctypes.c_double), ("bw", ctypes.c_int32)]


_fp = ctypes.POINTER(ctypes.c_float)
_dp = ctypes.POINTER(ctypes.c_double)
_vp = ctypes.c_void_p
_i64 = ctypes.c_int64
_i32 = ctypes.c_int32
_int = ctypes.c_int
_enc_p = ctypes.POINTER(TfEncodingC)


class ChannelDescC(ctypes.Structure):
    _fields_ = [("in_", ctypes.c_void_p), ("out", ctypes.c_void_p), ("outer", ctypes.c_int64),
                ("C", ctypes.c_int64), ("K", ctypes.c_int64), ("table", ctypes.c_void_p)]

AIMET_BCAST_MAX_DIMS = 16


class BroadcastShapeInfoC(ctypes.Structure):
    """aimet_broadcast_shape_info (onnx/src/QuantizeDequantizeUtils.hpp:166-178 BroadcastShapeInfo)."""
    _fields_ = [("num_dims", ctypes.c_int64),
                ("tensor_shape", ctypes.c_int64 * AIMET_BCAST_MAX_DIMS),
                ("encoding_shape", ctypes.c_int64 * AIMET_BCAST_MAX_DIMS),
                ("tensor_strides", ctypes.c_int64 * AIMET_BCAST_MAX_DIMS),
                ("encoding_strides", ctypes.c_int64 * AIMET_BCAST_MAX_DIMS),
                ("num_elements", ctypes.c_int64), ("num_encodings", ctypes.c_int64),
                ("contiguous_blocks", ctypes.c_int)]


class QcQuantizeInfoC(ctypes.Structure):
    """aimet_qc_quantize_info (onnx/src/QcQuantizeInfo.h:46-73 + the TensorQuantizer settings)."""
    _fields_ = [("op_mode", ctypes.c_int), ("enabled", ctypes.c_int), ("is_int_data_type", ctypes.c_int),
                ("use_per_channel_mode", ctypes.c_int), ("channel_axis", ctypes.c_int),
                ("block_axis", ctypes.c_int), ("block_size", ctypes.c_int),
                ("use_symmetric_encoding", ctypes.c_int), ("use_strict_symmetric", ctypes.c_int),
                ("use_unsigned_symmetric", ctypes.c_int), ("rounding_mode", ctypes.c_int),
                ("num_encodings", ctypes.c_int64), ("encodings", ctypes.POINTER(TfEncodingC)),
                ("quantizer", ctypes.c_void_p)]


_i64p = ctypes.POINTER(ctypes.c_int64)

# name -> argtypes (restype is int status unless listed in _RESTYPES)
_PROTOTYPES = {
    "aimet_last_error": [],
    "aimet_version": [],
    "aimet_device_count": [],
    "aimet_capture_pool_limit": [_i64, ctypes.POINTER(_i64)],
    "aimet_get_computed_encodings": [_i32, ctypes.c_double, ctypes.c_double, _int, _int, _int, _enc_p],
    "aimet_fill_encoding_info": [_i32, ctypes.c_double, ctypes.c_double, _enc_p],
    "aimet_compute_partial_encoding": [_i32, _enc_p, _int, _int, _int],
    "aimet_encoding_from_minmax": [ctypes.c_double, ctypes.c_double, _i32, _int, _int, _int, _enc_p],
    "aimet_encoding_from_histogram": [_int, _int, _int, ctypes.c_float, ctypes.c_double, _dp, ctypes.c_float, _i32,
                                      _int, _int, _int, _enc_p],
    "aimet_qdq_broadcast": [_vp, _vp, _i64, _i64, _i64p, _i64p, _vp, _vp, _vp, _vp, _vp],
    "aimet_permute_tensor": [_vp, _vp, _i64, _i64, _i64p, _i64p, _vp],
    "aimet_qdq_fp16": [_vp, _vp, _i64, _vp],
    "aimet_broadcast_shape_info_init": [_i64p, _i64, _int, _int, _int, ctypes.POINTER(BroadcastShapeInfoC)],
    "aimet_copy_to_contiguous_block_layout": [_vp, _vp, ctypes.POINTER(BroadcastShapeInfoC), _vp],
    "aimet_qc_quantize_op_compute": [ctypes.POINTER(QcQuantizeInfoC), _vp, _vp, _i64p, _i64, _vp],
    "aimet_encoding_from_entropy_histogram": [_int, _int, ctypes.c_double, ctypes.c_double, _dp, _i32, _int, _int,
                                              _int, _enc_p],
    "aimet_qdq_per_tensor": [_vp, _vp, _i64, _enc_p, _int, ctypes.c_uint64, _vp],
    "aimet_quantize_per_tensor": [_vp, _vp, _i64, _enc_p, _int, _int, ctypes.c_uint64, _vp],
    "aimet_per_channel_table": [_enc_p, _i64, _vp, _vp],
    "aimet_make_delta_offset": [_enc_p, _i64, _vp, _vp],
    "aimet_qdq_per_channel": [_vp, _vp, _i64, _i64, _i64, _vp, _int, ctypes.c_uint64, _vp],
    "aimet_qdq_channel_plan_create": [ctypes.POINTER(ChannelDescC), _i64, _int, ctypes.POINTER(_vp)],
    "aimet_qdq_channel_plan_run": [_vp, _int, ctypes.c_uint64, _vp],
    "aimet_qdq_channel_plan_destroy": [_vp],
    "aimet_ste_backward": [_vp, _vp, _vp, _i64, _i64, _i64, _vp, _vp, _vp],
    "aimet_ste_backward_per_tensor": [_vp, _vp, _vp, _i64, ctypes.c_float, ctypes.c_float, _vp],
    "aimet_qdq_per_tensor_16": [_vp, _vp, _i64, _int, _enc_p, _int, ctypes.c_uint64, _vp],
    "aimet_qdq_per_channel_16": [_vp, _vp, _i64, _i64, _i64, _int, _vp, _int, ctypes.c_uint64, _vp],
    "aimet_ste_backward_16": [_vp, _vp, _vp, _i64, _i64, _i64, _int, _vp, _vp, ctypes.c_float, ctypes.c_float,
                              _vp],
    "aimet_tq_create": [_int, _i64, _int, ctypes.POINTER(_vp)],
    "aimet_tq_destroy": [_vp],
    "aimet_tq_reset_encoding_stats": [_vp, _vp],
    "aimet_tq_set_percentile_value": [_vp, ctypes.c_float],
    "aimet_tq_get_percentile_value": [_vp, _fp],
    "aimet_tq_update_stats": [_vp, _vp, _i64, _i64, _i64, _vp],
    "aimet_tq_batch_minmax": [_vp, _vp, _i64, _i64, _i64, _vp],
    "aimet_tq_fold_minmax": [_vp, _vp],
    "aimet_tq_batch_histogram": [_vp, _vp, _i64, _i64, _i64, _vp],
    "aimet_tq_fold_histogram": [_vp, _i64, _vp],
    "aimet_tq_minmax_buffer": [_vp, ctypes.POINTER(_vp), ctypes.POINTER(_i64)],
    "aimet_tq_counts_buffer": [_vp, ctypes.POINTER(_vp), ctypes.POINTER(_i64)],
    "aimet_tq_bind_exchange": [_vp, _vp, _vp],
    "aimet_tq_mark_stats_updated": [_vp],
    "aimet_tq_get_encoding": [_vp, ctypes.c_uint32, _int, _int, _int, _enc_p, ctypes.POINTER(_int), _vp],
    "aimet_tq_update_stats_many": [ctypes.POINTER(_vp), ctypes.POINTER(_vp), ctypes.POINTER(_i64), _i64, _vp],
    "aimet_tq_batch_minmax_many": [ctypes.POINTER(_vp), ctypes.POINTER(_vp), ctypes.POINTER(_i64), _i64, _vp],
    "aimet_tq_fold_minmax_many": [ctypes.POINTER(_vp), _i64, _vp],
    "aimet_tq_batch_histogram_many": [ctypes.POINTER(_vp), ctypes.POINTER(_vp), ctypes.POINTER(_i64), _i64, _vp],
    "aimet_tq_fold_histogram_many": [ctypes.POINTER(_vp), ctypes.POINTER(_i64), _i64, _vp],
    "aimet_tq_fold_histogram_many_dev": [ctypes.POINTER(_vp), _vp, _i64, _vp],
    "aimet_tq_create_many": [ctypes.POINTER(ctypes.c_int), ctypes.POINTER(_i64), _i64, ctypes.c_int,
                             ctypes.POINTER(_vp)],
    "aimet_tq_update_stats_channels_many": [ctypes.POINTER(_vp), ctypes.POINTER(_vp), ctypes.POINTER(_i64),
                                            ctypes.POINTER(_i64), ctypes.POINTER(_i64), _i64, _vp],
    "aimet_tq_get_encodings": [ctypes.POINTER(_vp), _i64, ctypes.c_uint32, _int, _int, _int, _enc_p,
                               ctypes.POINTER(_int), _vp],
    "aimet_tq_reset_encoding_stats_many": [ctypes.POINTER(_vp), _i64, _vp],
    "aimet_tq_get_encodings_launch": [ctypes.POINTER(_vp), _i64, ctypes.c_uint32, _int, _int, _int, _vp,
                                      ctypes.POINTER(_vp)],
    "aimet_tq_get_encodings_finish": [_vp, _enc_p, ctypes.POINTER(_int)],
    "aimet_calibrate_launch": [ctypes.POINTER(_vp), ctypes.POINTER(_vp), ctypes.POINTER(_i64), _i64,
                               ctypes.POINTER(_vp), ctypes.POINTER(_vp), ctypes.POINTER(_i64), ctypes.POINTER(_i64),
                               ctypes.POINTER(_i64), _i64, ctypes.POINTER(ctypes.c_int32),
                               ctypes.POINTER(ctypes.c_int32), _int, _vp, _vp, ctypes.POINTER(_vp),
                               ctypes.POINTER(_vp)],
    "aimet_calib_plan_create": [ctypes.POINTER(_vp), ctypes.POINTER(_vp), ctypes.POINTER(_i64), _i64,
                                ctypes.POINTER(_vp), ctypes.POINTER(_vp), ctypes.POINTER(_i64), ctypes.POINTER(_i64),
                                ctypes.POINTER(_i64), _i64, ctypes.POINTER(ctypes.c_int32),
                                ctypes.POINTER(ctypes.c_int32), _vp, ctypes.POINTER(_vp)],
    "aimet_calib_plan_launch": [_vp, _int, _int, _vp, _vp, ctypes.POINTER(_vp), ctypes.POINTER(_vp)],
    "aimet_calib_plan_destroy": [_vp],
    "aimet_tq_get_stats_histogram": [_vp, _i64, _dp, _dp, ctypes.POINTER(_int), _vp],
    "aimet_tq_get_entropy_state": [_vp, _i64, _dp, _dp, ctypes.POINTER(_int), ctypes.POINTER(_int), _vp],
    "aimet_tq_num_channels": [_vp, ctypes.POINTER(_i64)],
    "aimet_tq_quant_scheme": [_vp, ctypes.POINTER(_int)],
    "aimet_lg_forward": [_vp, _vp, _i64, _i64, _i64, _vp, _vp, ctypes.c_float, _vp],
    "aimet_lg_backward": [_vp, _vp, _vp, _vp, _i64, _i64, _i64, _vp, _vp, ctypes.c_float, _vp, _vp],
    "aimet_lg_gate_range": [_vp, _vp, _i64, _vp],
    "aimet_lg_gate_ranges": [_vp, _vp, _vp, ctypes.c_int, _vp],
    "aimet_lg_encodings": [_vp, _vp, _i64, _int, _int, _int, _int, _vp, _vp, _vp],
    "aimet_lg_range_grads": [_vp, _vp, _vp, _vp, _i64, ctypes.c_float, _int, _vp, _vp, _vp],
    "aimet_lg_set_chunk_limit": [_i64],
    "aimet_lg_forward_range": [_vp, _vp, _i64, _i64, _i64, _int, _vp, _vp, _int, _int, _int, _int, _vp, _vp, _vp, _vp],
    "aimet_lg_forward_16_range": [_vp, _vp, _i64, _int, _vp, _vp, _int, _int, _int, _int, _vp, _vp, _vp, _vp],
    "aimet_lg_forward_cast": [_vp, _vp, _i64, _i64, _i64, _int, _vp, _vp, ctypes.c_float, _vp],
    "aimet_lg_backward_grad16": [_vp, _vp, _vp, _vp, _i64, _i64, _i64, _int, _vp, _vp, ctypes.c_float, _vp,
                                 _vp],
    "aimet_lg_backward_grad16_supported": [_i64, _i64, _i64, _vp, _vp, _vp],
    "aimet_lg_forward_16": [_vp, _vp, _i64, _int, _vp, _vp, ctypes.c_float, _vp],
    "aimet_lg_backward_16": [_vp, _vp, _vp, _vp, _i64, _int, _vp, _vp, ctypes.c_float, _vp, _vp],
    "aimet_adaround_forward": [_vp, _vp, _vp, _i64, _i64, _i64, _vp, _vp, _i32, _int, _vp],
    "aimet_adaround_backward": [_vp, _vp, _vp, _vp, _i64, _i64, _i64, _vp, _vp, _i32, ctypes.c_double,
                                ctypes.c_double, _vp, _vp],
    "aimet_adaround_backward_dev": [_vp, _vp, _vp, _vp, _i64, _i64, _i64, _vp, _vp, _i32, _vp, _vp, _vp],
    "aimet_adaround_recon_grad": [_vp, _vp, _vp, _i64, _i64, _int, _vp],
    "aimet_dwconv2d_forward": [_vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _i32, _i32, _i32, _i32, _vp],
    "aimet_dwconv2d_grad_weight_workspace": [_i64, _i64, _i64, _i64, _i32, _vp],
    "aimet_adaround_dw_step": [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64,
                               _i32, _i32, _i32, _i32, _i32, _vp],
    "aimet_adaround_pw_step_workspace": [_i64, _i64, _i64, _i64, _vp],
    "aimet_adaround_pw_step_uses_mfma": [_i64, _i64, ctypes.POINTER(_int)],
    "aimet_adaround_pw_step": [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i32, _vp],
    "aimet_dwconv2d_grad_weight": [_vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _i32, _i32, _i32, _i32,
                                   _vp],
    "aimet_adaround_gather": [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _vp],
    "aimet_adaround_gather_cm": [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _vp],
    "aimet_adaround_recon_grad_indexed_cm": [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _vp, _int, _vp],
    "aimet_adaround_recon_grad_indexed": [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _vp, _int, _vp],
    "aimet_adaround_backward_adam": [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _vp, _vp, _i32, _vp, _vp, _vp,
                                     ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double, _vp, _vp,
                                     _vp],
    "aimet_adaround_dw_step_slices": [_vp, _i64, _i64, _i64, _i64, _i32, _i32, _i32, _vp],
    "aimet_adaround_pw_step_slices": [_i64, _i64, _i64, _i64, _vp, _vp],
    "aimet_adaround_backward_adam_parts": [_vp, _vp, _vp, _i64, _i64, _vp, _vp, _i64, _i64, _i64, _vp, _vp, _i32, _vp, _vp,
                                           _vp, ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                           _vp, _vp, _vp, _vp],
    "aimet_adaround_adam_bias_corrections": [ctypes.c_double, ctypes.c_double, _i64, _vp, _vp],
    "aimet_adaround_set_exact_pow": [_int],
    "aimet_adaround_get_exact_pow": [ctypes.POINTER(_int)],
}
_RESTYPES = {"aimet_last_error": ctypes.c_char_p, "aimet_version": ctypes.c_char_p}

EXPORTED_SYMBOLS = tuple(_PROTOTYPES)

_lib = None
_load_error = None


def build(verbose=False):
    """Compile libaimet_amd.so for gfx950 with hipcc (make -C aimet_amd/csrc)."""
    jobs = str(min(16, os.cpu_count() or 4))
    subprocess.run(["make", "-s", "-j", jobs, "-C", CSRC], check=True,
                   stdout=None if verbose else subprocess.DEVNULL)


def load():
    """Return the loaded library or raise NativeLibraryError (never falls back)."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    if _load_error is not None:
        raise _load_error
    if not os.path.exists(LIB_PATH):
        _load_error = NativeLibraryError(
            "aimet_amd: %s not found. Build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(hipcc --offload-arch=gfx950). There is no CPU fallback." % LIB_PATH)
        raise _load_error
    try:
        lib = ctypes.CDLL(LIB_PATH)
    except OSError as e:
        _load_error = NativeLibraryError("aimet_amd: cannot load %s: %s" % (LIB_PATH, e))
        raise _load_error from e
    for name, args in _PROTOTYPES.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = _RESTYPES.get(name, ctypes.c_int)
    _lib = lib
    return lib


def check(rc):
    """Map a C-ABI status to the exception the reference's pybind layer would raise."""
    if rc == AIMET_OK:
        return
    msg = load().aimet_last_error().decode(errors="replace")
    if rc == AIMET_ERR_INVALID_ARGUMENT:
        raise ValueError(msg)
    if rc == AIMET_ERR_HIP:
        raise HipError(msg)
    raise RuntimeError(msg)


def call(name, *args):
    check(getattr(load(), name)(*args))
