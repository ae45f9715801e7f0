"""TEST INFRASTRUCTURE: the drop-in QuantizationSimModel on the CPU with oracle-backed operators.

This container has no GPU, so the CPU tests of the sharded drop-in calibration replace the
quantizers' gfx950 operator (aimet_amd.tensor_quantizer.AimetTensorQuantizer) with OracleOp -- the
same duck-typed interface (per-call statistics, the phased statistics of aimet_amd.distributed,
encodings) on the CPU oracle analyzers (oracle/dlq_oracle.c, pinned to the reference C++) -- and the
QDQ of the ANALYSIS forwards with the oracle's. Everything above the operator is the product code:
QuantizationSimModel.compute_encodings, the wrappers, StatsBatch, the packed exchange and its
collectives. Never imported by the product package."""
import numpy as np
import torch

from oracle import oracle as O

from aimet_amd.libpymo import TfEncoding


def _tf(e) -> TfEncoding:
    t = TfEncoding()
    t.min, t.max, t.delta, t.offset, t.bw = e.as_tuple()
    return t


class OracleOp:
    """AimetTensorQuantizer's interface on the CPU oracle (one analyzer per channel)."""

    def __init__(self, scheme, num_channels=1):
        self._scheme = int(scheme)
        self._num_channels = int(num_channels)
        self._percentile = None
        self._device = None
        self.resetEncodingStats()

    @property
    def num_channels(self):
        return self._num_channels

    @property
    def uses_histogram(self):
        return self._scheme != O.QUANTIZATION_TF

    def resetEncodingStats(self):
        self.an = [O.Analyzer(self._scheme) for _ in range(self._num_channels)]
        if self._percentile is not None:
            for a in self.an:
                a.set_percentile(self._percentile)
        self.active = [False] * self._num_channels
        self.valid = False

    def setPercentileValue(self, p):
        if self._scheme == O.QUANTIZATION_PERCENTILE:
            self._percentile = float(p)
            for a in self.an:
                a.set_percentile(p)

    def _channels(self, t, ax=0):
        x = t.detach().float().cpu().numpy()
        if self._num_channels == 1:
            return [x.ravel()]
        return [np.ascontiguousarray(np.take(x, c, axis=ax)).ravel() for c in range(self._num_channels)]

    # per-call statistics (the non-sharded path)
    def updateStats(self, t, use_cuda=True):
        self.an[0].update(t.detach().float().cpu().numpy().ravel())
        self.valid = True

    def updateStatsPerChannel(self, t, ch_axis=0, use_cuda=True):
        for a, x in zip(self.an, self._channels(t, ch_axis)):
            a.update(x)
        self.valid = True

    # phased statistics (aimet_amd.distributed)
    def bind_exchange(self, minmax, counts=None):
        self.mm, self.cnt = minmax, counts

    def batch_minmax(self, t, ax=0):
        for c, x in enumerate(self._channels(t, ax)):
            self.mm[2 * c] = -O.get_min(x)
            self.mm[2 * c + 1] = O.get_max(x)
        self.valid = True

    def fold_minmax(self):
        for c, a in enumerate(self.an):
            self.active[c] = a.fold_minmax(-float(self.mm[2 * c]), float(self.mm[2 * c + 1]))

    def batch_histogram(self, t, ax=0):
        for c, x in enumerate(self._channels(t, ax)):
            if not self.active[c]:
                continue
            xl, _ = self.an[c].histogram()
            bucket = np.float32(xl[1] - xl[0])
            off = np.float32(np.float32(xl[0]) / bucket)
            self.cnt[512 * c:512 * (c + 1)] = torch.from_numpy(O.histogram(x, bucket, off).astype(np.int64))

    def fold_histogram(self, n):
        for c, a in enumerate(self.an):
            if self.active[c]:
                a.update_from_counts(self.cnt[512 * c:512 * (c + 1)].numpy().astype(np.uint64), n)
            self.cnt[512 * c:512 * (c + 1)] = 0

    # encodings
    def _get_encodings(self, bw, sym, strict, unsign):
        if not self.valid:
            return [TfEncoding() for _ in self.an], False
        return [_tf(a.compute(bw, sym, strict, unsign)) for a in self.an], True

    def getEncoding(self, bw, sym, strict, unsign):
        encs, valid = self._get_encodings(bw, sym, strict, unsign)
        return (encs[0] if self._num_channels == 1 else encs), valid


def _oracle_qdq(tensor, tq, round_mode):
    """QuantizeDequantize's values on the oracle (round to nearest: the ANALYSIS / eval forwards)."""
    from aimet_amd.quantizers import StaticGridPerChannelQuantizer
    from aimet_amd.tensor_quantizer import per_channel_view
    if not tq.enabled or tq.bitwidth == 32:
        return tensor
    x = tensor.detach().float().contiguous()
    if isinstance(tq, StaticGridPerChannelQuantizer):
        outer, C, K = per_channel_view(x.shape, tq.channel_axis)
        table = O.per_channel_table([e.to_tuple() for e in tq.encoding])
        xs = x.numpy().reshape(outer, C * K)
        y = np.stack([O.qdq_per_channel(xs[o], C, K, table) for o in range(outer)])
    else:
        e = tq.encoding
        y = O.qdq_per_tensor(x.numpy().ravel(), e.min, e.max, tq.bitwidth)
    return torch.from_numpy(np.asarray(y, np.float32).reshape(x.shape)).to(tensor.dtype)


def install(monkeypatch):
    """Route the sim's quantizers through OracleOp and the oracle QDQ (CPU only)."""
    import aimet_amd.quantizers as Q
    import aimet_amd.quantsim as QS

    def make_pt(self):
        self._cppOp = [OracleOp(Q._pymo_mode(self._quant_scheme))]

    def make_pc(self):
        self._cppOp = [OracleOp(Q._pymo_mode(self._quant_scheme), self._num_channels)]

    def batched(quantizers):
        for q in quantizers:
            q.compute_encoding()

    monkeypatch.setattr(Q.StaticGridPerTensorQuantizer, "_make_op", make_pt)
    monkeypatch.setattr(Q.StaticGridPerChannelQuantizer, "_make_op", make_pc)
    monkeypatch.setattr(Q, "_qdq_values", _oracle_qdq)
    # the batched GPU forms of the parameter encodings: per wrapper in the first forward instead
    monkeypatch.setattr(QS, "_precompute_param_encodings", lambda wrappers: [])
    monkeypatch.setattr(QS, "compute_encodings_batched", batched)
