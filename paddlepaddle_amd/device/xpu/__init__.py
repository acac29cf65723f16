"""paddle.device.xpu. Reference: python/paddle/device/xpu/__init__.py (synchronize, device_count,
set_debug_level). This framework targets MI355X; there are no XPU devices, so device_count() is 0 and the calls
that need one raise."""
from __future__ import annotations

__all__ = ["synchronize"]


def device_count() -> int:
    return 0


def synchronize(device=None) -> int:
    raise RuntimeError("paddle.device.xpu.synchronize: no XPU device (this build runs on MI355X / ROCm; use "
                       "paddle.device.synchronize)")


def set_debug_level(level: int = 1) -> None:
    raise RuntimeError("paddle.device.xpu.set_debug_level: no XPU device")
