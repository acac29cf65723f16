"""Static post-training quantization. Reference: python/paddle/static/quantization/post_training_quantization.py
(PostTrainingQuantization, PostTrainingQuantizationProgram, WeightQuantization).

Calibration runs the program on the sample batches with a recorder around every quantizable op (conv2d / mul /
matmul whose weight is a program constant) that feeds its input activation to a threshold collector (KL,
hist, abs_max, avg, mse / emd -> percentile); quantize() then bakes channel-wise (or per-tensor) quantised
weights into the constants and inserts fixed-scale activation quant-dequant nodes, so the saved inference model
reproduces the int8 numerics."""
from __future__ import annotations

import os

import numpy as np
import torch

from .. import program as P
from . import _graph as G
from . import quant_ops as Q


def _collector(algo, bits, hist_percent):
    from ...quantization.imperative import AbsmaxQuantizer, HistQuantizer, KLQuantizer
    if algo == "KL":
        return KLQuantizer(quant_bits=bits)
    if algo in ("hist", "mse", "emd"):
        return HistQuantizer(quant_bits=bits, hist_percent=hist_percent)
    return AbsmaxQuantizer(quant_bits=bits)


class _Avg:
    def __init__(self, bits):
        self.quant_bits, self.vals, self.thresholds = bits, [], []

    def sample_data(self, layer, tensors):
        self.vals.append(float(tensors[0].detach().abs().max()))

    def cal_thresholds(self):
        self.thresholds = [float(np.mean(self.vals)) if self.vals else 0.0]


class PostTrainingQuantizationProgram:
    def __init__(self, executor, program, feed_list=None, fetch_list=None, scope=None, batch_generator=None,
                 sample_generator=None, data_loader=None, batch_size=10, batch_nums=None, algo="KL",
                 hist_percent=0.99999, quantizable_op_type=("conv2d", "depthwise_conv2d", "mul"), round_type="round",
                 learning_rate=0.001, is_full_quantize=False, bias_correction=False, activation_bits=8,
                 weight_bits=8, activation_quantize_type="range_abs_max",
                 weight_quantize_type="channel_wise_abs_max", onnx_format=False, freeze_model=True,
                 optimize_model=False, is_use_cache_file=False, skip_tensor_list=None, same_scale_tensor_list=None,
                 cache_dir=None, scale_dict=None, return_graph=False, deploy_backend=None):
        if algo not in ("KL", "hist", "avg", "mse", "emd", "abs_max", "min_max", "ptf"):
            raise ValueError(f"unsupported algo {algo}")
        if weight_quantize_type not in ("abs_max", "channel_wise_abs_max"):
            raise ValueError(f"unsupported weight_quantize_type {weight_quantize_type}")
        if sum(x is not None for x in (batch_generator, sample_generator, data_loader)) != 1:
            raise ValueError("give exactly one of batch_generator, sample_generator, data_loader")
        self._exe, self._program = executor, program
        self._feed_list = list(feed_list or [])
        self._fetch_list = list(fetch_list or [])
        self._batch_generator, self._sample_generator, self._data_loader = batch_generator, sample_generator, data_loader
        self._batch_size, self._batch_nums = batch_size, batch_nums
        self._algo, self._hist_percent = algo, hist_percent
        self._types = set(quantizable_op_type) | ({"mul", "matmul"} if is_full_quantize else set())
        self._abits, self._wbits = activation_bits, weight_bits
        self._wtype = weight_quantize_type
        self._scale_dict = dict(scale_dict or {})
        self._skip = set(skip_tensor_list or [])
        self.scales = {}

    # ---------------------------------------------------------------- calibration data
    def _batches(self):
        n = 0
        if self._data_loader is not None:
            src = self._data_loader() if callable(self._data_loader) else self._data_loader
        elif self._batch_generator is not None:
            src = self._batch_generator()
        else:
            def gen():
                buf = []
                for s in self._sample_generator():
                    buf.append(s if isinstance(s, (list, tuple)) else (s,))
                    if len(buf) == self._batch_size:
                        yield [np.stack([b[i] for b in buf]) for i in range(len(buf[0]))]
                        buf = []
            src = gen()
        for b in src:
            if self._batch_nums is not None and n >= self._batch_nums:
                break
            n += 1
            if isinstance(b, dict):
                yield b
            else:
                b = b if isinstance(b, (list, tuple)) else [b]
                yield {name: (v.numpy() if hasattr(v, "numpy") else np.asarray(v)) for name, v in
                       zip(self._feed_list, b)}

    def _calibrate(self, nodes):
        collectors = {}
        orig = {}
        for i, node, ref_type, w, axis in nodes:
            c = _Avg(self._abits) if self._algo == "avg" else _collector(self._algo, self._abits, self._hist_percent)
            collectors[id(node)] = c
            orig[id(node)] = node.func

            def rec(*a, _f=node.func, _c=c, **k):
                _c.sample_data(None, (a[0],))
                return _f(*a, **k)
            node.func = rec
        try:
            for feed in self._batches():
                self._exe.run(self._program, feed=feed, fetch_list=self._fetch_list)
        finally:
            for _, node, *_ in nodes:
                node.func = orig[id(node)]
        return collectors

    def quantize(self):
        prog = self._program
        nodes = G.quantizable_nodes(prog, self._types)
        collectors = self._calibrate(nodes)
        for i, node, ref_type, w, axis in nodes:
            c = collectors[id(node)]
            c.cal_thresholds()
            thr = self._scale_dict.get(node.name, c.thresholds[0] if c.thresholds else 0.0)
            self.scales[f"{ref_type}_{i}"] = float(thr)
            with torch.no_grad(), G.raw():
                w.t.copy_(Q.qat_fake_quant_weight(w.t.detach(), axis if self._wtype == "channel_wise_abs_max"
                                                  else None, self._wbits))
            G.insert_before(prog, node, Q.fake_quant_act, (float(thr), int(self._abits)), 0)
        return prog

    def save_quantized_model(self, save_model_path, model_filename=None, params_filename=None):
        from .. import io as sio
        prefix = os.path.join(save_model_path, (model_filename or "model").replace(".pdmodel", ""))
        fetch = [sio._slot_of(self._program, v) for v in self._fetch_list]
        sio.write_program(prefix, self._program, fetch)
        return prefix


class PostTrainingQuantization(PostTrainingQuantizationProgram):
    """Loads the inference model in ``model_dir`` (``model_filename`` / ``params_filename`` inside it) and
    calibrates it; the feed / fetch lists come from the model."""

    def __init__(self, executor, model_dir=None, scope=None, model_filename=None, params_filename=None,
                 batch_generator=None, sample_generator=None, data_loader=None, batch_size=10, batch_nums=None,
                 algo="KL", hist_percent=0.99999, quantizable_op_type=("conv2d", "depthwise_conv2d", "mul"),
                 round_type="round", learning_rate=0.001, is_full_quantize=False, bias_correction=False,
                 activation_bits=8, weight_bits=8, activation_quantize_type="range_abs_max",
                 weight_quantize_type="channel_wise_abs_max", onnx_format=False, freeze_model=True,
                 optimize_model=False, is_use_cache_file=False, skip_tensor_list=None, same_scale_tensor_list=None,
                 cache_dir=None, scale_dict=None, return_graph=False, deploy_backend=None):
        from .. import io as sio
        prefix = os.path.join(model_dir, (model_filename or "model").replace(".pdmodel", ""))
        prog, feeds, fetch = sio.load_inference_model(prefix, executor)
        if not isinstance(prog, P.Program):
            raise TypeError("PostTrainingQuantization calibrates this framework's programs (saved by "
                            "save_inference_model); reference ProgramDesc / PIR models run read-only")
        super().__init__(executor, prog, feeds, fetch, scope, batch_generator, sample_generator, data_loader,
                         batch_size, batch_nums, algo, hist_percent, quantizable_op_type, round_type, learning_rate,
                         is_full_quantize, bias_correction, activation_bits, weight_bits, activation_quantize_type,
                         weight_quantize_type, onnx_format, freeze_model, optimize_model, is_use_cache_file,
                         skip_tensor_list, same_scale_tensor_list, cache_dir, scale_dict, return_graph,
                         deploy_backend)


class WeightQuantization:
    """Weight-only quantization of a saved inference model (reference post_training_quantization.py
    WeightQuantization): the weights of the quantizable ops are replaced by their int-quantised values
    (abs max per tensor or channel-wise; ``threshold_rate`` clips the range to a percentile of |w|)."""

    def __init__(self, model_dir, model_filename=None, params_filename=None):
        self._dir, self._mf, self._pf = model_dir, model_filename, params_filename

    def quantize_weight_to_int(self, save_model_dir, save_model_filename=None, save_params_filename=None,
                               quantizable_op_type=("conv2d", "mul"), weight_bits=8,
                               weight_quantize_type="channel_wise_abs_max", generate_test_model=False,
                               threshold_rate=0.0):
        from .. import io as sio
        if weight_bits not in (8, 16):
            raise ValueError("weight_bits must be 8 or 16")
        prefix = os.path.join(self._dir, (self._mf or "model").replace(".pdmodel", ""))
        prog, fetch, _ = sio.read_program(prefix)
        for _, node, ref_type, w, axis in G.quantizable_nodes(prog, set(quantizable_op_type)):
            with torch.no_grad(), G.raw():
                t = w.t.detach()
                if threshold_rate > 0:
                    lim = torch.quantile(t.abs().float().reshape(-1)[:1 << 24], 1 - threshold_rate).to(t.dtype)
                    t = t.clamp(-lim, lim)
                w.t.copy_(Q.qat_fake_quant_weight(t, axis if weight_quantize_type == "channel_wise_abs_max"
                                                  else None, weight_bits))
        out = os.path.join(save_model_dir, (save_model_filename or "model").replace(".pdmodel", ""))
        sio.write_program(out, prog, fetch)
        return out
