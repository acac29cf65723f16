"""paddle.incubate.autotune. Reference: python/paddle/incubate/autotune.py:47 set_config.

What the switches drive here:
  kernel     -> the per-shape GEMM backend choice (ops/gemm.py choose(): hand-written MFMA kernels vs hipBLASLt,
                timed on first use, persisted in the tuning table). Disabled: shapes not in the table are not timed
                and take hipBLASLt; ``tuning_range`` bounds the step window in which new shapes may be timed.
  layout     -> FLAGS_layout_autotune: NCHW conv / batch-norm / max-pool calls on device tensors run the NHWC HIP
                kernels on channels-last views (framework/layout_autotune.py, read by nn/functional conv / norm /
                pooling).
  dataloader -> FLAGS_dataloader_autotune: io.DataLoader built with num_workers=0 times its first
                ``tuning_steps`` batches at 0, 2, 4, ... workers and keeps the cheapest (io/__init__.py
                _tune_num_workers).
"""
from __future__ import annotations

import json
import warnings

from ..framework.flags import set_flags

__all__ = ["set_config"]


def _kernel(cfg):
    if "enable" in cfg:
        if isinstance(cfg["enable"], bool):
            set_flags({"FLAGS_use_autotune": cfg["enable"]})
        else:
            warnings.warn("The auto-tuning configuration of the kernel is incorrect. The `enable` should be bool. "
                          "Use default parameter instead.")
    if "tuning_range" in cfg:
        r = cfg["tuning_range"]
        if isinstance(r, (list, tuple)) and len(r) == 2:
            set_flags({"FLAGS_autotune_range_begin": int(r[0]), "FLAGS_autotune_range_end": int(r[1])})
        else:
            warnings.warn("The auto-tuning configuration of the kernel is incorrect. The `tuning_range` should be "
                          "list. Use default parameter instead.")


def _bool_switch(cfg, flag, what):
    if "enable" in cfg:
        if isinstance(cfg["enable"], bool):
            set_flags({flag: cfg["enable"]})
        else:
            warnings.warn(f"The auto-tuning configuration of the {what} is incorrect. The `enable` should be bool. "
                          "Use default parameter instead.")


def set_config(config=None):
    if config is None:
        set_flags({"FLAGS_use_autotune": True, "FLAGS_layout_autotune": True, "FLAGS_dataloader_autotune": True})
        return
    cfg = {}
    if isinstance(config, dict):
        cfg = config
    elif isinstance(config, str):
        try:
            with open(config) as f:
                cfg = json.load(f)
        except Exception as e:  # the reference reports and keeps the defaults
            print(f"Load config error: {e}")
            warnings.warn("Use default configuration for auto-tuning.")
    if "kernel" in cfg:
        _kernel(cfg["kernel"])
    if "layout" in cfg:
        _bool_switch(cfg["layout"], "FLAGS_layout_autotune", "layout")
    if "dataloader" in cfg:
        _bool_switch(cfg["dataloader"], "FLAGS_dataloader_autotune", "dataloader")
        if "tuning_steps" in cfg["dataloader"]:
            ts = cfg["dataloader"]["tuning_steps"]
            if isinstance(ts, int) and ts > 0:
                set_flags({"FLAGS_dataloader_tuning_steps": ts})
            else:
                warnings.warn("The auto-tuning configuration of the dataloader is incorrect. The `tuning_steps` "
                              "should be int. Use default parameter instead.")
