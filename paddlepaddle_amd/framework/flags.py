"""Global flags. Reference: paddle/common/flags.cc, paddle.set_flags/get_flags."""
from __future__ import annotations

import os

_FLAGS = {
    "FLAGS_check_nan_inf": False,
    "FLAGS_check_nan_inf_level": 0,
    "FLAGS_use_hip_kernels": True,        # route hot ops to hand-written HIP kernels
    "FLAGS_cudnn_deterministic": False,
    "FLAGS_embedding_deterministic": 0,
    "FLAGS_fraction_of_gpu_memory_to_use": 0.92,
    "FLAGS_allocator_strategy": "auto_growth",
    "FLAGS_eager_delete_tensor_gb": 0.0,
    "FLAGS_use_cuda_graph": False,
    "FLAGS_enable_pir_api": False,
    "FLAGS_print_ir": False,
    "FLAGS_call_stack_level": 1,
    "FLAGS_dp_bucket_mb": 128,            # DataParallel fused all-reduce bucket (xGMI ring friendly)
    "FLAGS_sharding_bucket_mb": 256,
    "FLAGS_pir_native_interpreter": True,  # PIR programs run on the C++ interpreter (_C_interp) when every op maps
    "FLAGS_eager_backward_engine": "native",  # native (csrc/autograd/autograd_exec.cpp RunBackward) | torch
    "FLAGS_weight_only_dequant_cache_mb": 4096,  # weight-only / LLM.int8: bf16 images of quantized weights kept
                                                 # for the bf16 GEMM path (0 = dequantise per call)
    "FLAGS_fused_grad_accumulation": True,  # fleet pipeline engine: dW GEMMs / norm kernels add into .grad
    "FLAGS_static_native_executor": "auto",  # static training programs on the native executor (_C_train):
                                             # auto (GPU) | force (also CPU, ATen instructions only) | off
    "FLAGS_gemm_backend": "auto",         # per-shape GEMM / conv backend: auto (timed) | hip | blas
    "FLAGS_sharding_stage3_keep_params": "auto",  # stage 3: keep gathered params until the optimizer step
    "FLAGS_conv_per_direction": True,     # NHWC conv: forward / dgrad / wgrad each on the faster of ours and MIOpen
    "FLAGS_conv_bn_fusion": True,         # convs feeding a training BN write its statistics in their epilogue
    "FLAGS_use_autotune": True,           # time GEMM backends for shapes the tuning table does not hold
    "FLAGS_autotune_range_begin": 0,      # incubate.autotune kernel tuning_range (optimizer-step window)
    "FLAGS_autotune_range_end": 1 << 30,
    "FLAGS_layout_autotune": False,
    "FLAGS_dataloader_autotune": False,
    "FLAGS_dataloader_tuning_steps": 8,
    "FLAGS_static_engine_native": "auto",  # static auto-parallel stages on the native executor: auto (GPU) / force / 0
    "FLAGS_linear_wt_cache_mb": 0,        # [out,in] weight copies for TN-form forward GEMMs (0 = off;
                                          # measured no net gain on the 13B step, see ops/linear.py)
}

for _k in list(_FLAGS):
    if _k in os.environ:
        _v = os.environ[_k]
        _d = _FLAGS[_k]
        if isinstance(_d, bool):
            _FLAGS[_k] = _v.lower() in ("1", "true", "yes")
        elif isinstance(_d, int):
            _FLAGS[_k] = int(_v)
        elif isinstance(_d, float):
            _FLAGS[_k] = float(_v)
        else:
            _FLAGS[_k] = _v


def _norm(k):
    return k if k.startswith("FLAGS_") else "FLAGS_" + k


def set_flags(flags: dict):
    for k, v in flags.items():
        _FLAGS[_norm(k)] = v


def get_flags(flags):
    if isinstance(flags, str):
        flags = [flags]
    out = {}
    for k in flags:
        k = _norm(k)
        if k not in _FLAGS:
            raise ValueError(f"flag {k} not found")
        out[k] = _FLAGS[k]
    return out


def flag(k, default=None):
    return _FLAGS.get(_norm(k), default)
