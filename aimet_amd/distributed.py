"""Calibration (compute_encodings statistics) sharded per sample across ranks.

The reference forbids multi-GPU calibration (Docs/api_docs/torch_multi_gpu.rst:32) and runs
each quantizer's statistics on one device. Here every rank reduces its shard of the batch on its
own GPU and the ranks exchange only the reduced statistics, packed for ALL quantizers of the
batch into one buffer per phase:

  1. batch min/max          -> packed float32 {-min, max}   -> ONE all_reduce(MAX)
  2. fold: TF running min/max; histogram schemes fix the 512-bucket PDF range on the first batch
     from the GLOBAL min/max (so every rank bins identically)
  3. batch histogram        -> packed int64 counts, followed by every histogram quantizer's local
                               element count                 -> ONE all_reduce(SUM)
  4. fold: PDF running average with the GLOBAL element count, read by the fold kernel from the
     reduced buffer (no host round trip between the phases)

Every rank ends with statistics identical to one device processing the whole batch (integer
counts are order-independent; the double PDF recurrence sees the same inputs), hence identical
encodings. Collectives run over torch.distributed ("nccl" = RCCL over xGMI on MI355X; "gloo" on
CPU in the tests). Messages are tiny (8 B x C and 4 KiB x C per quantizer) and latency-bound, so
the packing (2 collectives per batch instead of 2 per quantizer) is what matters.

Quantizers are duck-typed: anything with ``num_channels``, ``uses_histogram``,
``bind_exchange``, ``batch_minmax``, ``fold_minmax``, ``batch_histogram``, ``fold_histogram``.
``AimetTensorQuantizer`` implements them on the gfx950 kernels.
"""
import torch
import torch.distributed as dist

PDF_SIZE = 512


class PackedExchange:
    """Packed exchange buffers for a fixed list of quantizers (bound once, reused every batch)."""

    def __init__(self, quantizers, device):
        self.quantizers = list(quantizers)
        if torch.device(device).type == "cuda":
            # device state of every native quantizer from one allocation (aimet_tq_create_many)
            from aimet_amd.tensor_quantizer import AimetTensorQuantizer
            native = [q for q in self.quantizers if isinstance(q, AimetTensorQuantizer)]
            if native:
                AimetTensorQuantizer._ensure_many(native, torch.device(device))
        chans = [q.num_channels for q in self.quantizers]
        self.minmax = torch.zeros(2 * sum(chans), dtype=torch.float32, device=device)
        hist_ch = sum(c for q, c in zip(self.quantizers, chans) if q.uses_histogram)
        n_hist = sum(1 for q in self.quantizers if q.uses_histogram)
        # bin counts of every histogram channel, then one element count per histogram quantizer:
        # the element counts ride the same SUM as the bins
        self.counts = torch.zeros(PDF_SIZE * hist_ch + n_hist, dtype=torch.int64, device=device)
        self.elem_counts = self.counts[PDF_SIZE * hist_ch:]
        m = h = 0
        for q, c in zip(self.quantizers, chans):
            mm = self.minmax[m:m + 2 * c]
            cc = self.counts[h:h + PDF_SIZE * c] if q.uses_histogram else None
            q.bind_exchange(mm, cc)
            m += 2 * c
            if q.uses_histogram:
                h += PDF_SIZE * c


def _world(group):
    return dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1


def _all_reduce(t, op, group):
    """all_reduce in place; a device tensor over a gloo group (no RCCL: e.g. several ranks sharing
    one GPU) is staged through host memory."""
    if t.is_cuda and dist.get_backend(group) == "gloo":
        h = t.cpu()
        dist.all_reduce(h, op=op, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=op, group=group)


def sharded_update_stats(quantizers, tensors, ch_axes=None, group=None, exchange=None, fused=True,
                         force_exchange=False):
    """One calibration batch: every rank passes ITS shard of each quantizer's tensor.

    Equivalent to ``q.updateStats(whole_batch_tensor)`` on one device for every quantizer.
    `force_exchange` runs both collectives even in a world of one rank (a world-size-1 RCCL group
    then executes the device-buffer all_reduces of the N-rank path on a single GPU)."""
    if not quantizers:
        return exchange
    device = tensors[0].device
    ch_axes = ch_axes or [0] * len(quantizers)
    world = _world(group)

    # per-tensor AimetTensorQuantizers: one launch per phase for all of them (aimet_tq_*_many)
    from aimet_amd.tensor_quantizer import AimetTensorQuantizer
    many = [i for i, q in enumerate(quantizers) if type(q) is AimetTensorQuantizer and q._num_channels == 1]
    many_set = set(many)
    rest = [i for i in range(len(quantizers)) if i not in many_set]
    mq = [quantizers[i] for i in many]
    mt = [tensors[i] for i in many]

    exchanging = world > 1 or force_exchange
    if not exchanging and not rest and fused:
        # nothing to exchange (no packed buffers either): the fused single-pass update, 4 launches
        # for all quantizers
        AimetTensorQuantizer.updateStatsMany(quantizers if len(mq) == len(quantizers) else mq,
                                             tensors if len(mq) == len(quantizers) else mt)
        return exchange

    if exchange is None or exchange.quantizers != list(quantizers):
        exchange = PackedExchange(quantizers, device)

    if mq:
        AimetTensorQuantizer.batch_minmax_many(mq, mt)
    for i in rest:
        quantizers[i].batch_minmax(tensors[i], ch_axes[i])
    if exchanging:
        # {-min, max}: a single MAX reduces both ends exactly
        _all_reduce(exchange.minmax, dist.ReduceOp.MAX, group)
    if mq:
        AimetTensorQuantizer.fold_minmax_many(mq)
    for i in rest:
        quantizers[i].fold_minmax()

    hist = [i for i in range(len(quantizers)) if quantizers[i].uses_histogram]
    if hist:
        hist_many = [i for i in many if quantizers[i].uses_histogram]
        hist_rest = [i for i in hist if i not in many_set]
        if hist_many:
            AimetTensorQuantizer.batch_histogram_many([quantizers[i] for i in hist_many],
                                                      [tensors[i] for i in hist_many])
        for i in hist_rest:
            quantizers[i].batch_histogram(tensors[i], ch_axes[i])
        local = [tensors[i].numel() // quantizers[i].num_channels for i in hist]
        # element counts, ordered as the histogram quantizers: the batched ones first (the fold
        # kernel reads its slice of the reduced buffer), then the others
        order = hist_many + hist_rest
        by_pos = {i: k for k, i in enumerate(hist)}
        if exchanging:
            host = torch.tensor([local[by_pos[i]] for i in order], dtype=torch.int64)
            if exchange.elem_counts.is_cuda:
                # a pinned staging buffer from torch's caching host allocator, which keeps it alive
                # until the stream-ordered copy has run
                exchange.elem_counts.copy_(host.pin_memory(), non_blocking=True)
            else:
                exchange.elem_counts.copy_(host)
            _all_reduce(exchange.counts, dist.ReduceOp.SUM, group)
            if hist_many:
                AimetTensorQuantizer.fold_histogram_many([quantizers[i] for i in hist_many],
                                                         exchange.elem_counts[:len(hist_many)])
            if hist_rest:
                rest_counts = exchange.elem_counts[len(hist_many):].tolist()
                for i, c in zip(hist_rest, rest_counts):
                    quantizers[i].fold_histogram(c)
        else:
            if hist_many:
                AimetTensorQuantizer.fold_histogram_many([quantizers[i] for i in hist_many],
                                                         [local[by_pos[i]] for i in hist_many])
            for i in hist_rest:
                quantizers[i].fold_histogram(local[by_pos[i]])
    return exchange
