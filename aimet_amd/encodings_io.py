"""Encoding dictionaries: export / import of quantizer encodings (the on-disk contract with
downstream runtimes).

Mirrors aimet_torch/utils.py:801-816 (create_encoding_from_dict), :1156-1196
(create_encoding_dict), :1273-1318 (validate_is_symmetric_flag, compute_partial_encoding) and
v1/qc_quantize_op.py:1514-1545 (get_encoding_by_quantizer, export_quantizer_encoding): same keys
('min', 'max', 'scale', 'offset', 'bitwidth', 'is_symmetric' as the strings 'True'/'False',
'dtype'), same partial-encoding completion (through the native computePartialEncoding).
"""
from typing import Dict, List, Optional

from aimet_amd.libpymo import TfEncoding, TensorQuantizer, QuantizationMode
from aimet_amd.quantizers import QuantizationDataType


def create_encoding_dict(encoding: TfEncoding, quantizer, propagate_encodings: bool) -> Optional[Dict]:
    """utils.py:1156-1186."""
    data_type, bitwidth = quantizer.data_type, quantizer.bitwidth
    if data_type == QuantizationDataType.float:
        return {"bitwidth": bitwidth, "dtype": "float"}
    if not encoding:
        return None
    if propagate_encodings:
        return {"bitwidth": encoding.bw, "dtype": "int"}
    return {"min": encoding.min, "max": encoding.max, "scale": encoding.delta, "offset": int(encoding.offset),
            "bitwidth": encoding.bw, "is_symmetric": str(bool(quantizer.use_symmetric_encodings)), "dtype": "int"}


def create_encoding_from_dict(encoding_dict: dict) -> TfEncoding:
    """utils.py:801-816."""
    if encoding_dict.get("is_symmetric") not in ("True", "False"):
        raise AssertionError("Unexpected value for is_symmetric: %r" % encoding_dict.get("is_symmetric"))
    enc = TfEncoding()
    enc.bw = encoding_dict.get("bitwidth")
    enc.max = encoding_dict.get("max")
    enc.min = encoding_dict.get("min")
    enc.delta = encoding_dict.get("scale")
    enc.offset = encoding_dict.get("offset")
    return enc


def _validate_is_symmetric_flag(quantizer, encoding_dict: Dict, strict: bool):
    if "is_symmetric" not in encoding_dict:
        return
    is_symmetric = encoding_dict["is_symmetric"] == "True"
    if quantizer.use_symmetric_encodings != is_symmetric:
        if strict:
            raise AttributeError("Provided quantizer use_symmetric_encodings flag does not match the is_symmetric "
                                 "flag of the encoding")
        quantizer.use_symmetric_encodings = is_symmetric


def validate_is_symmetric_flag(quantizer, encoding_dict: Dict, strict: bool = True):
    """utils.py:1273-1286: a full encoding must agree with the quantizer; a partial one sets it."""
    if not (encoding_dict.get("max", 0) == 0 and encoding_dict.get("min", 0) == 0) and \
            encoding_dict.get("delta", 0) != 0:
        _validate_is_symmetric_flag(quantizer, encoding_dict, strict=True)
    _validate_is_symmetric_flag(quantizer, encoding_dict, strict=strict)


def compute_partial_encoding(quantizer, encoding_dict: Dict) -> Dict:
    """utils.py:1289-1318: complete a partial encoding (e.g. only bitwidth + min or + scale)."""
    enc = TfEncoding()
    enc.bw = encoding_dict.get("bitwidth")
    enc.max = encoding_dict.get("max", 0)
    enc.min = encoding_dict.get("min", 0)
    enc.delta = encoding_dict.get("scale", 0)
    enc.offset = encoding_dict.get("offset", 0)
    if not (enc.max == 0 and enc.min == 0) and enc.delta != 0:
        return encoding_dict
    partial = TensorQuantizer(QuantizationMode.QUANTIZATION_TF, quantizer.round_mode)
    partial.computePartialEncoding(enc.bw, enc, quantizer.use_symmetric_encodings,
                                   quantizer.use_unsigned_symmetric, quantizer.use_strict_symmetric)
    encoding_dict["max"] = enc.max
    encoding_dict["min"] = enc.min
    encoding_dict["scale"] = enc.delta
    encoding_dict["offset"] = enc.offset
    encoding_dict["is_symmetric"] = "True" if quantizer.use_symmetric_encodings else "False"
    return encoding_dict


def get_encoding_by_quantizer(quantizer):
    """v1/qc_quantize_op.py:1514-1526 (learned-grid quantizers report their effective encoding)."""
    if hasattr(quantizer, "get_effective_encoding"):
        return quantizer.get_effective_encoding()
    return quantizer.encoding


def export_quantizer_encoding(quantizer) -> Optional[List[Dict]]:
    """v1/qc_quantize_op.py:1529-1545."""
    if not quantizer.enabled:
        return None
    encoding = get_encoding_by_quantizer(quantizer)
    if isinstance(encoding, list):
        return [create_encoding_dict(e, quantizer, False) for e in encoding]
    d = create_encoding_dict(encoding, quantizer, False)
    return [d] if d else None
