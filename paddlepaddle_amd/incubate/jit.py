"""paddle.incubate.jit.inference: run a function / layer as a saved static inference model.

Reference: python/paddle/incubate/jit/inference_decorator.py:475 (inference), :116 (InferenceEngine). The first
call with a new input signature converts the layer with jit.to_static, saves it (optionally to save_model_dir,
reused when cache_static_model is set) and builds an inference Predictor; later calls run the Predictor."""
from __future__ import annotations

import functools
import os
import tempfile

from ..framework.tensor import Tensor

_INFER_FLAG = "__paddle_amd_inference__"


def is_inference_mode(function):
    return bool(getattr(function, _INFER_FLAG, False))


class InferenceEngine:
    def __init__(self, layer, save_model_dir=None, cache_static_model=False, precision_mode="float32",
                 use_gpu=True, **kw):
        self.layer = layer
        self.save_model_dir = save_model_dir
        self.cache_static_model = cache_static_model
        self.precision_mode = precision_mode
        self.use_gpu = use_gpu
        self._predictors = {}

    def _predictor(self, args):
        from .. import inference as pinf, jit
        from ..static import InputSpec
        sig = tuple((tuple(a.shape), str(a.dtype)) for a in args)
        pred = self._predictors.get(sig)
        if pred is not None:
            return pred
        root = self.save_model_dir or tempfile.mkdtemp(prefix="paddle_amd_infer_")
        prefix = os.path.join(root, "infer_%d" % len(self._predictors))
        if not (self.cache_static_model and os.path.exists(prefix + ".pdmodel")):
            specs = [InputSpec(list(a.shape), a.dtype) for a in args]
            patched = self.layer.__dict__.get("forward") is self
            if patched:  # trace the layer's own forward, not this engine
                del self.layer.__dict__["forward"]
            try:
                jit.save(self.layer, prefix, input_spec=specs)
            finally:
                if patched:
                    self.layer.forward = self
        cfg = pinf.Config(prefix + ".pdmodel", prefix + ".pdiparams")
        if not self.use_gpu:
            cfg.disable_gpu()
        pred = self._predictors[sig] = pinf.create_predictor(cfg)
        return pred

    def __call__(self, *args):
        tensors = [a for a in args if isinstance(a, Tensor)]
        outs = self._predictor(tensors).run(tensors)
        return outs[0] if len(outs) == 1 else outs


def inference(function=None, cache_static_model=False, save_model_dir=None, memory_pool_init_size_mb=1000,
              precision_mode="float32", switch_ir_optim=True, switch_ir_debug=False, enable_cinn=False,
              with_trt=False, trt_precision_mode="float32", trt_use_static=False, collect_shape=False,
              enable_new_ir=False, exp_enable_use_cutlass=False, delete_pass_lists=None, skip_prune_program=False):
    """Decorator (or direct call on a Layer): forward runs through a static inference Predictor."""
    from ..nn import Layer
    if with_trt or enable_cinn:
        raise NotImplementedError("incubate.jit.inference: TensorRT / CINN subgraphs are not part of this "
                                  "framework; the Predictor runs the program on the HIP kernels")

    def wrap(fn):
        if isinstance(fn, Layer):
            eng = InferenceEngine(fn, save_model_dir, cache_static_model, precision_mode)
            fn.forward = eng
            setattr(fn, _INFER_FLAG, True)
            return fn
        from ..nn import Layer as _L

        class _FnLayer(_L):
            def forward(self, *a):
                return fn(*a)
        eng = InferenceEngine(_FnLayer(), save_model_dir, cache_static_model, precision_mode)

        @functools.wraps(fn)
        def run(*a):
            return eng(*a)
        setattr(run, _INFER_FLAG, True)
        return run
    return wrap(function) if function is not None else wrap
