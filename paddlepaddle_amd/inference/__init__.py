"""paddle.inference: Config / create_predictor / Predictor / Tensor handles.

Reference: python/paddle/inference/__init__.py, paddle/fluid/inference/api/analysis_predictor.cc
(ZeroCopy input/output handles, Run). Our predictor loads a saved program (jit.save /
static.save_inference_model), replays it with the native-scheduled executor under no_grad, and — when
enabled and the input shapes repeat — captures the whole replay into a hipGraph so a request costs one
graph launch instead of one launch per op.
"""
from __future__ import annotations

import enum

import os

import numpy as np
import torch

from ..framework.tensor import _wrap
from ..static import program as P
from ..static import io as _sio


class PrecisionType(enum.IntEnum):
    Float32 = 0
    Int8 = 1
    Half = 2
    Bfloat16 = 3


class PlaceType(enum.IntEnum):
    UNK = -1
    CPU = 0
    GPU = 1


DataType = enum.IntEnum("DataType", "FLOAT32 INT64 INT32 UINT8 INT8 FLOAT16 BOOL FLOAT64 BFLOAT16")


class Config:
    def __init__(self, model_path=None, params_path=None):
        self._prefix = None
        self._params = params_path
        if model_path is not None:
            self.set_model(model_path, params_path)
        self._use_gpu = torch.cuda.is_available()
        self._device_id = 0
        self._hip_graph = False
        self._precision = PrecisionType.Float32
        self._ir_optim = True
        self._memory_optim = True
        self._threads = 1

    def set_model(self, model_path, params_path=None):
        p = model_path
        if p.endswith(".pdmodel"):
            p = p[:-len(".pdmodel")]
        elif p.endswith(".json"):
            p = p[:-len(".json")]
        self._prefix = p
        self._params = params_path

    def set_prog_file(self, f):
        self.set_model(f, self._params)

    def set_params_file(self, f):
        self._params = f

    def prog_file(self):
        return self._prefix + ".pdmodel"

    def params_file(self):
        return self._params or self._prefix + ".pdiparams"

    def model_dir(self):
        return self._prefix

    def enable_use_gpu(self, memory_pool_init_size_mb=100, device_id=0, precision_mode=PrecisionType.Float32):
        self._use_gpu = True
        self._device_id = device_id
        self._precision = precision_mode

    def disable_gpu(self):
        self._use_gpu = False

    def use_gpu(self):
        return self._use_gpu

    def gpu_device_id(self):
        return self._device_id

    def enable_hip_graph(self, enable=True):
        """Capture the replay into a hipGraph per input shape (MI355X-native extension)."""
        self._hip_graph = enable

    enable_cuda_graph = enable_hip_graph

    def switch_ir_optim(self, x=True):
        self._ir_optim = x

    def ir_optim(self):
        return self._ir_optim

    def enable_memory_optim(self, x=True):
        self._memory_optim = x

    def set_cpu_math_library_num_threads(self, n):
        self._threads = n

    def cpu_math_library_num_threads(self):
        return self._threads

    def enable_mkldnn(self):
        pass

    def disable_glog_info(self):
        pass

    def switch_use_feed_fetch_ops(self, x):
        pass

    def switch_specify_input_names(self, x=True):
        pass

    def enable_tensorrt_engine(self, *a, **k):
        raise NotImplementedError("TensorRT is not part of the MI355X build; use enable_hip_graph()")

    def summary(self):
        return f"Config(model={self._prefix}, gpu={self._use_gpu}:{self._device_id}, hip_graph={self._hip_graph})"


class _Handle:
    """ZeroCopy tensor handle (reference: paddle_infer::Tensor)."""

    def __init__(self, pred, name, is_input):
        self._pred = pred
        self._name = name
        self._is_input = is_input
        self._shape = None

    def name(self):
        return self._name

    def reshape(self, shape):
        self._shape = list(shape)

    def copy_from_cpu(self, data):
        self._pred._inputs[self._name] = np.ascontiguousarray(data)

    def share_external_data(self, tensor):
        self._pred._inputs[self._name] = tensor

    def copy_to_cpu(self):
        t = self._pred._outputs[self._name]
        return _wrap(t).numpy()

    def shape(self):
        if self._is_input:
            v = self._pred._inputs.get(self._name)
            return list(v.shape) if v is not None else list(self._shape or [])
        return list(self._pred._outputs[self._name].shape)

    def type(self):
        return DataType.FLOAT32


class Predictor:
    def __init__(self, config):
        self._config = config
        dev = torch.device(f"cuda:{config._device_id}") if (config._use_gpu and torch.cuda.is_available()) \
            else torch.device("cpu")
        self._dev = dev
        self._runner = None
        from ..framework import program_desc as _pd, pir_json as _pir
        pre = config._prefix
        if not os.path.exists(pre + ".pdmodel") and os.path.exists(pre + ".json") and _pir.is_pir_json(pre + ".json"):
            # Paddle 3.x PIR program (.json): run op by op over this framework's kernels
            self._runner = _pir.load(pre, dev)
            self._in_names = list(self._runner.feed_names)
            self._out_names = list(self._runner.fetch_names)
            self._inputs, self._outputs, self._graphs = {}, {}, {}
            return
        if os.path.exists(config._prefix + ".pdmodel") and _pd.is_program_desc(config._prefix + ".pdmodel"):
            # reference-format ProgramDesc: run op by op over this framework's kernels
            self._runner = _pd.load(config._prefix, dev)
            self._in_names = list(self._runner.program.feed_names)
            self._out_names = list(self._runner.program.fetch_names)
            self._inputs, self._outputs, self._graphs = {}, {}, {}
            return
        prog, fetch, _ = _sio.read_program(config._prefix, dev, config._params)
        self._prog = prog
        self._fetch = fetch
        self._plan = P.build_plan(prog, fetch)
        self._in_names = list(prog.feeds)
        self._out_names = [f"fetch_{i}" for i in range(len(fetch))]
        self._inputs = {}
        self._outputs = {}
        self._graphs = {}

    def get_input_names(self):
        return list(self._in_names)

    def get_output_names(self):
        return list(self._out_names)

    def get_input_handle(self, name):
        return _Handle(self, name, True)

    def get_output_handle(self, name):
        return _Handle(self, name, False)

    def _to_dev(self, name, v):
        slot, shape, dtype = self._prog.feeds[name]
        t = v if isinstance(v, torch.Tensor) else (v._t if hasattr(v, "_t") else torch.from_numpy(np.asarray(v)))
        return t.to(self._dev, getattr(torch, dtype), non_blocking=True)

    def _sym(self, env):
        if not self._prog._dyn:
            return None
        for name, (slot, shape, _) in self._prog.feeds.items():
            if -1 in shape:
                return int(env[slot].shape[list(shape).index(-1)])
        return None

    def _replay(self, env):
        P.run_plan(self._prog, self._plan, env, self._dev, None, self._sym(env))
        return [env[s] for s in self._fetch]

    def run(self, inputs=None):
        if inputs is not None:  # new-style API: list in, list out
            for n, v in zip(self._in_names, inputs):
                self._inputs[n] = v
        if self._runner is not None:
            def _t(v):
                v = v._t if hasattr(v, "_t") else v
                return (v if isinstance(v, torch.Tensor) else torch.from_numpy(np.asarray(v))).to(self._dev)
            feeds = {n: _wrap(_t(self._inputs[n])) for n in self._in_names}
            outs = [o._t for o in self._runner.run(feeds)]
            self._outputs = dict(zip(self._out_names, outs))
            return [_wrap(o) for o in outs] if inputs is not None else True
        tens = {n: self._to_dev(n, self._inputs[n]) for n in self._in_names}
        with torch.no_grad():
            if self._config._hip_graph and self._dev.type == "cuda":
                outs = self._graph_run(tens)
            else:
                env = {self._prog.feeds[n][0]: t for n, t in tens.items()}
                outs = self._replay(env)
        self._outputs = dict(zip(self._out_names, outs))
        if inputs is not None:
            return [_wrap(o.clone() if self._config._hip_graph else o) for o in outs]
        return True

    def _graph_run(self, tens):
        key = tuple((n, tuple(t.shape), t.dtype) for n, t in tens.items())
        ent = self._graphs.get(key)
        if ent is None:
            static_in = {n: t.clone() for n, t in tens.items()}
            env = {self._prog.feeds[n][0]: t for n, t in static_in.items()}
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                self._replay(dict(env))
            torch.cuda.current_stream().wait_stream(s)
            from ..device.cuda.graphs import CUDAGraph, capture
            g = CUDAGraph()
            with capture(g):
                outs = self._replay(dict(env))
            ent = self._graphs[key] = (g, static_in, outs)
        g, static_in, outs = ent
        for n, t in tens.items():
            static_in[n].copy_(t)
        g.replay()
        return outs

    def clone(self):
        return Predictor(self._config)

    def clear_intermediate_tensor(self):
        pass

    def try_shrink_memory(self):
        if torch.cuda.is_available():
            from ..device.cuda import empty_cache as _ec
            _ec()


def create_predictor(config):
    return Predictor(config)


def get_version():
    from .. import __version__
    return __version__


def convert_to_mixed_precision(*a, **k):
    raise NotImplementedError("mixed-precision model conversion: run the model under paddle.amp instead")


Tensor = _Handle


class PredictorPool:
    """A fixed pool of predictors built from one Config (reference inference PredictorPool)."""

    def __init__(self, config, size=1):
        self._preds = [create_predictor(config) for _ in range(max(1, size))]

    def retrive(self, idx):
        return self._preds[idx]

    retrieve = retrive


def get_num_bytes_of_data_type(dtype):
    return {DataType.FLOAT32: 4, DataType.FLOAT16: 2, DataType.BFLOAT16: 2, DataType.INT64: 8, DataType.INT32: 4,
            DataType.UINT8: 1, DataType.INT8: 1, DataType.BOOL: 1, DataType.FLOAT64: 8}.get(dtype, 4)


def get_trt_compile_version():
    return (0, 0, 0)


def get_trt_runtime_version():
    return (0, 0, 0)


class XpuConfig:
    def __init__(self, *a, **k):
        raise RuntimeError("XPU devices are not supported by this MI355X framework")


def _get_phi_kernel_name(op_name):
    return op_name
