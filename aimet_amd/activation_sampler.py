"""Activation sampling for AdaRound: a layer's input from the QuantSim model and its output from
the original model, for every cached batch.

Reference: aimet_torch/utils.py:106-190 (ModuleData.collect_inp_out_data) and
aimet_torch/v1/adaround/activation_sampler.py:198-301 (ActivationSampler). Same hooks, the same
early stop once the layer has run, eval mode and no_grad. The reference stacks the samples on the
host and then tries to move them to the device; here they stay in HBM where the forward left them
(288 GB per MI355X), concatenated there.
"""
from typing import Any, Callable, Tuple, Union

import torch

from aimet_amd.quantsim import _eval_mode


class StopForwardException(Exception):
    """Raised by the collection hook once the layer's data is in hand (aimet_torch/utils.py)."""


def _device_of(model: torch.nn.Module) -> torch.device:
    for p in model.parameters():
        return p.device
    return torch.device("cpu")


def _to_device(data, device):
    if isinstance(data, torch.Tensor):
        return data.to(device)
    if isinstance(data, (list, tuple)):
        return type(data)(_to_device(d, device) for d in data)
    if isinstance(data, dict):
        return {k: _to_device(v, device) for k, v in data.items()}
    return data


def _cast_floats(data, dtype):
    if isinstance(data, torch.Tensor):
        return data.to(dtype) if data.is_floating_point() else data
    if isinstance(data, (list, tuple)):
        return type(data)(_cast_floats(d, dtype) for d in data)
    return data


def default_forward_fn(model, inputs):
    """aimet_torch/utils.py ModuleData.default_forward_fn."""
    if isinstance(inputs, (list, tuple)):
        return model(*inputs)
    return model(inputs)


class ModuleData:
    """aimet_torch/utils.py:106-190."""

    def __init__(self, model: torch.nn.Module, module: torch.nn.Module,
                 forward_fn: Callable[[torch.nn.Module, Any], Any] = None):
        self._model = model
        self._module = module
        self._forward_fn = forward_fn or default_forward_fn

    def collect_inp_out_data(self, model_input: Union[torch.Tensor, list, tuple], collect_input: bool,
                             collect_output: bool) -> Tuple[torch.Tensor, torch.Tensor]:
        def adjust_input_dtype(module, inp):
            w = getattr(module, "weight", None)
            if isinstance(w, torch.Tensor):
                return _cast_floats(inp, w.dtype)
            return inp

        inp_list, out_list = [], []

        def hook(_, inp, out):
            if collect_input:
                inp_list.append(inp[0])
            if collect_output:
                out_list.append(out)
            raise StopForwardException

        handles = [m.register_forward_pre_hook(adjust_input_dtype) for m in self._model.modules()]
        handles.append(self._module.register_forward_hook(hook))
        model_input = _to_device(model_input, _device_of(self._model))
        try:
            with _eval_mode(self._model), torch.no_grad():
                self._forward_fn(self._model, model_input)
        except StopForwardException:
            pass
        finally:
            for h in handles:
                h.remove()
        inp = inp_list[0].detach() if inp_list and isinstance(inp_list[0], torch.Tensor) else None
        out = out_list[0].detach() if out_list and isinstance(out_list[0], torch.Tensor) else None
        return inp, out


class ActivationSampler:
    """activation_sampler.py:198-301: the quant module's input (from the QuantSim model) and the
    original module's output (from the original model)."""

    def __init__(self, orig_module: torch.nn.Module, quant_module: torch.nn.Module, orig_model: torch.nn.Module,
                 quant_model: torch.nn.Module, forward_fn: Callable[[torch.nn.Module, Any], Any]):
        self._orig_module = orig_module
        self._quant_module = quant_module
        self._orig_model = orig_model
        self._quant_model = quant_model
        self._orig_module_collector = ModuleData(orig_model, orig_module, forward_fn)
        self._quant_module_collector = ModuleData(quant_model, quant_module, forward_fn)

    def sample_acts(self, model_inputs, collect_input=True, collect_output=True):
        inp_data = out_data = None
        if collect_input:
            inp_data, _ = self._quant_module_collector.collect_inp_out_data(model_inputs, True, False)
        if collect_output:
            _, out_data = self._orig_module_collector.collect_inp_out_data(model_inputs, False, True)
        return inp_data, out_data

    def sample_all_acts(self, cached_dataset, cached_quant_dataset=None,
                        device=None) -> Tuple[torch.Tensor, torch.Tensor]:
        """sample_and_place_all_acts_on_cpu (activation_sampler.py:227-263) with the samples kept in
        device memory (`device`, default the layer's): every batch of the dataset, concatenated."""
        if cached_quant_dataset is not None:
            assert len(cached_dataset) == len(cached_quant_dataset)
        inps, outs = [], []
        for i in range(len(cached_dataset)):
            if cached_quant_dataset is not None:
                inp, _ = self.sample_acts(cached_quant_dataset[i], collect_input=True, collect_output=False)
                _, out = self.sample_acts(cached_dataset[i], collect_input=False, collect_output=True)
            else:
                inp, out = self.sample_acts(cached_dataset[i])
            if device is not None:
                inp, out = inp.to(device), out.to(device)
            inps.append(inp)
            outs.append(out)
        return torch.cat(inps, dim=0), torch.cat(outs, dim=0)

    def sample_and_place_all_acts_on_cpu(self, cached_dataset, cached_quant_dataset=None):
        """activation_sampler.py:227-263 (the samples on the host)."""
        inp, out = self.sample_all_acts(cached_dataset, cached_quant_dataset)
        return inp.cpu(), out.cpu()
