"""Pooling layers. Reference: python/paddle/nn/layer/pooling.py."""
from __future__ import annotations

from .. import functional as F
from .layers import Layer


class _Pool(Layer):
    def __init__(self, **kw):
        super().__init__()
        self._kw = kw

    def extra_repr(self):
        kw = self._kw
        if "kernel_size" not in kw:  # adaptive pools
            keys = ["output_size"] + (["return_mask"] if "return_mask" in kw else [])
            return ", ".join(f"{k}={kw[k]}" for k in keys)
        head = f"norm_type={kw['norm_type']}, " if "norm_type" in kw else ""
        return head + f"kernel_size={kw['kernel_size']}, stride={kw.get('stride')}, padding={kw.get('padding', 0)}"


class MaxPool1D(_Pool):
    def __init__(self, kernel_size, stride=None, padding=0, return_mask=False, ceil_mode=False, name=None):
        super().__init__(kernel_size=kernel_size, stride=stride, padding=padding, return_mask=return_mask,
                         ceil_mode=ceil_mode)

    def forward(self, x):
        return F.max_pool1d(x, **self._kw)


class MaxPool2D(_Pool):
    def __init__(self, kernel_size, stride=None, padding=0, return_mask=False, ceil_mode=False, data_format="NCHW",
                 name=None):
        super().__init__(kernel_size=kernel_size, stride=stride, padding=padding, return_mask=return_mask,
                         ceil_mode=ceil_mode, data_format=data_format)

    def forward(self, x):
        return F.max_pool2d(x, **self._kw)


class MaxPool3D(_Pool):
    def __init__(self, kernel_size, stride=None, padding=0, return_mask=False, ceil_mode=False,
                 data_format="NCDHW", name=None):
        super().__init__(kernel_size=kernel_size, stride=stride, padding=padding, return_mask=return_mask,
                         ceil_mode=ceil_mode, data_format=data_format)

    def forward(self, x):
        return F.max_pool3d(x, **self._kw)


class AvgPool1D(_Pool):
    def __init__(self, kernel_size, stride=None, padding=0, exclusive=True, ceil_mode=False, name=None):
        super().__init__(kernel_size=kernel_size, stride=stride, padding=padding, exclusive=exclusive,
                         ceil_mode=ceil_mode)

    def forward(self, x):
        return F.avg_pool1d(x, **self._kw)


class AvgPool2D(_Pool):
    def __init__(self, kernel_size, stride=None, padding=0, ceil_mode=False, exclusive=True, divisor_override=None,
                 data_format="NCHW", name=None):
        super().__init__(kernel_size=kernel_size, stride=stride, padding=padding, ceil_mode=ceil_mode,
                         exclusive=exclusive, divisor_override=divisor_override, data_format=data_format)

    def forward(self, x):
        return F.avg_pool2d(x, **self._kw)


class AvgPool3D(_Pool):
    def __init__(self, kernel_size, stride=None, padding=0, ceil_mode=False, exclusive=True, divisor_override=None,
                 data_format="NCDHW", name=None):
        super().__init__(kernel_size=kernel_size, stride=stride, padding=padding, ceil_mode=ceil_mode,
                         exclusive=exclusive, divisor_override=divisor_override, data_format=data_format)

    def forward(self, x):
        return F.avg_pool3d(x, **self._kw)


class AdaptiveAvgPool1D(_Pool):
    def __init__(self, output_size, name=None):
        super().__init__(output_size=output_size)

    def forward(self, x):
        return F.adaptive_avg_pool1d(x, **self._kw)


class AdaptiveAvgPool2D(_Pool):
    def __init__(self, output_size, data_format="NCHW", name=None):
        super().__init__(output_size=output_size, data_format=data_format)

    def forward(self, x):
        return F.adaptive_avg_pool2d(x, **self._kw)


class AdaptiveAvgPool3D(_Pool):
    def __init__(self, output_size, data_format="NCDHW", name=None):
        super().__init__(output_size=output_size, data_format=data_format)

    def forward(self, x):
        return F.adaptive_avg_pool3d(x, **self._kw)


class AdaptiveMaxPool1D(_Pool):
    def __init__(self, output_size, return_mask=False, name=None):
        super().__init__(output_size=output_size, return_mask=return_mask)

    def forward(self, x):
        return F.adaptive_max_pool1d(x, **self._kw)


class AdaptiveMaxPool2D(_Pool):
    def __init__(self, output_size, return_mask=False, name=None):
        super().__init__(output_size=output_size, return_mask=return_mask)

    def forward(self, x):
        return F.adaptive_max_pool2d(x, **self._kw)


class AdaptiveMaxPool3D(_Pool):
    def __init__(self, output_size, return_mask=False, name=None):
        super().__init__(output_size=output_size, return_mask=return_mask)

    def forward(self, x):
        return F.adaptive_max_pool3d(x, **self._kw)


class LPPool1D(_Pool):
    def __init__(self, norm_type, kernel_size, stride=None, padding=0, ceil_mode=False, data_format="NCL", name=None):
        super().__init__(norm_type=norm_type, kernel_size=kernel_size, stride=stride, ceil_mode=ceil_mode)

    def forward(self, x):
        return F.lp_pool1d(x, **self._kw)


class LPPool2D(_Pool):
    def __init__(self, norm_type, kernel_size, stride=None, padding=0, ceil_mode=False, data_format="NCHW",
                 name=None):
        super().__init__(norm_type=norm_type, kernel_size=kernel_size, stride=stride, ceil_mode=ceil_mode,
                         data_format=data_format)

    def forward(self, x):
        return F.lp_pool2d(x, **self._kw)


class MaxUnPool1D(_Pool):
    def __init__(self, kernel_size, stride=None, padding=0, data_format="NCL", output_size=None, name=None):
        super().__init__(kernel_size=kernel_size, stride=stride, padding=padding, output_size=output_size)

    def forward(self, x, indices):
        return F.max_unpool1d(x, indices, **self._kw)


class MaxUnPool2D(_Pool):
    def __init__(self, kernel_size, stride=None, padding=0, data_format="NCHW", output_size=None, name=None):
        super().__init__(kernel_size=kernel_size, stride=stride, padding=padding, output_size=output_size)

    def forward(self, x, indices):
        return F.max_unpool2d(x, indices, **self._kw)


class MaxUnPool3D(_Pool):
    def __init__(self, kernel_size, stride=None, padding=0, data_format="NCDHW", output_size=None, name=None):
        super().__init__(kernel_size=kernel_size, stride=stride, padding=padding, output_size=output_size)

    def forward(self, x, indices):
        return F.max_unpool3d(x, indices, **self._kw)
