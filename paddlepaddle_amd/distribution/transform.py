"""Bijective / injective transforms. Reference: python/paddle/distribution/transform.py (Transform API:
forward, inverse, forward_log_det_jacobian, inverse_log_det_jacobian, forward_shape, inverse_shape)."""
from __future__ import annotations

import enum
import math

import torch

from ..framework.tensor import Tensor, _wrap
from .distribution import _shape, _t

__all__ = ["Transform", "AbsTransform", "AffineTransform", "ChainTransform", "ExpTransform", "IndependentTransform",
           "PowerTransform", "ReshapeTransform", "SigmoidTransform", "SoftmaxTransform", "StackTransform",
           "StickBreakingTransform", "TanhTransform"]


class Type(enum.Enum):
    BIJECTION = "bijection"
    INJECTION = "injection"
    SURJECTION = "surjection"
    OTHER = "other"

    @classmethod
    def is_injective(cls, _type):
        return _type in (cls.BIJECTION, cls.INJECTION)


def _v(x):
    t = _t(x)
    return t if t.is_floating_point() else t.float()


class Transform:
    """y = f(x). Subclasses implement _forward / _inverse / _forward_log_det_jacobian (on torch tensors);
    ``_event_rank``: number of trailing dims one application acts on jointly."""
    _type = Type.INJECTION
    _event_rank = 0

    def __init__(self):
        pass

    @classmethod
    def _is_injective(cls):
        return Type.is_injective(cls._type)

    def __call__(self, x):
        from .distribution import Distribution
        from .transformed_distribution import TransformedDistribution
        if isinstance(x, Distribution):
            return TransformedDistribution(x, [self])
        if isinstance(x, Transform):
            return ChainTransform([self, x])
        return self.forward(x)

    def forward(self, x):
        return _wrap(self._forward(_v(x)))

    def inverse(self, y):
        return _wrap(self._inverse(_v(y)))

    def forward_log_det_jacobian(self, x):
        return _wrap(self._forward_log_det_jacobian(_v(x)))

    def inverse_log_det_jacobian(self, y):
        yt = _v(y)
        return _wrap(-self._forward_log_det_jacobian(self._inverse(yt)))

    def forward_shape(self, shape):
        return tuple(_shape(shape))

    def inverse_shape(self, shape):
        return tuple(_shape(shape))

    def _forward(self, x):
        raise NotImplementedError

    def _inverse(self, y):
        raise NotImplementedError

    def _forward_log_det_jacobian(self, x):
        raise NotImplementedError


class AbsTransform(Transform):
    """y = |x| — not injective: the inverse returns both pre-images (-y, y)."""
    _type = Type.SURJECTION

    def _forward(self, x):
        return x.abs()

    def inverse(self, y):
        yt = _v(y)
        return _wrap(-yt), _wrap(yt)

    def inverse_log_det_jacobian(self, y):
        z = torch.zeros_like(_v(y))
        return _wrap(z), _wrap(z.clone())

    def forward_log_det_jacobian(self, x):
        raise NotImplementedError("AbsTransform is not injective")


class AffineTransform(Transform):
    _type = Type.BIJECTION

    def __init__(self, loc, scale):
        super().__init__()
        self.loc, self.scale = loc, scale
        self._loc, self._scale = _v(loc), _v(scale)

    def _forward(self, x):
        return self._loc + self._scale * x

    def _inverse(self, y):
        return (y - self._loc) / self._scale

    def _forward_log_det_jacobian(self, x):
        return torch.log(self._scale.abs())

    def inverse_log_det_jacobian(self, y):
        return _wrap(-torch.log(self._scale.abs()))

    def forward_shape(self, shape):
        return tuple(torch.broadcast_shapes(tuple(_shape(shape)), self._loc.shape, self._scale.shape))

    def inverse_shape(self, shape):
        return self.forward_shape(shape)


class ExpTransform(Transform):
    _type = Type.BIJECTION

    def _forward(self, x):
        return x.exp()

    def _inverse(self, y):
        return y.log()

    def _forward_log_det_jacobian(self, x):
        return x


class PowerTransform(Transform):
    """y = x ** power on x > 0."""
    _type = Type.BIJECTION

    def __init__(self, power):
        super().__init__()
        self.power = power
        self._power = _v(power)

    def _forward(self, x):
        return x.pow(self._power)

    def _inverse(self, y):
        return y.pow(1 / self._power)

    def _forward_log_det_jacobian(self, x):
        return torch.log((self._power * x.pow(self._power - 1)).abs())

    def forward_shape(self, shape):
        return tuple(torch.broadcast_shapes(tuple(_shape(shape)), self._power.shape))

    def inverse_shape(self, shape):
        return self.forward_shape(shape)


class SigmoidTransform(Transform):
    _type = Type.BIJECTION

    def _forward(self, x):
        return torch.sigmoid(x)

    def _inverse(self, y):
        return torch.log(y) - torch.log1p(-y)

    def _forward_log_det_jacobian(self, x):
        return -torch.nn.functional.softplus(-x) - torch.nn.functional.softplus(x)


class TanhTransform(Transform):
    _type = Type.BIJECTION

    def _forward(self, x):
        return torch.tanh(x)

    def _inverse(self, y):
        return torch.atanh(y)

    def _forward_log_det_jacobian(self, x):
        # log(1 - tanh(x)^2) = 2 (log 2 - x - softplus(-2x))
        return 2.0 * (math.log(2.0) - x - torch.nn.functional.softplus(-2.0 * x))


class SoftmaxTransform(Transform):
    """y = softmax(x) over the last axis (not injective: the inverse is log y up to a constant)."""
    _type = Type.OTHER
    _event_rank = 1

    def _forward(self, x):
        x = x - x.max(-1, keepdim=True).values
        e = x.exp()
        return e / e.sum(-1, keepdim=True)

    def _inverse(self, y):
        return y.log()

    def forward_shape(self, shape):
        s = tuple(_shape(shape))
        if len(s) < 1:
            raise ValueError(f"Expected length of shape is grater than 1, but got {len(s)}")
        return s

    def inverse_shape(self, shape):
        return self.forward_shape(shape)


class StickBreakingTransform(Transform):
    """R^{K-1} -> interior of the K-simplex by stick breaking."""
    _type = Type.BIJECTION
    _event_rank = 1

    def _forward(self, x):
        offset = x.shape[-1] + 1 - torch.ones(x.shape[-1], dtype=x.dtype, device=x.device).cumsum(-1)
        z = torch.sigmoid(x - offset.log())
        zc = (1 - z).cumprod(-1)
        return torch.nn.functional.pad(z, (0, 1), value=1.0) * torch.nn.functional.pad(zc, (1, 0), value=1.0)

    def _inverse(self, y):
        y_crop = y[..., :-1]
        offset = y.shape[-1] - torch.ones(y_crop.shape[-1], dtype=y.dtype, device=y.device).cumsum(-1)
        sf = 1 - y_crop.cumsum(-1)
        return torch.log(y_crop) - torch.log(sf.clamp_min(torch.finfo(y.dtype).tiny)) + offset.log()

    def _forward_log_det_jacobian(self, x):
        y = self._forward(x)
        offset = x.shape[-1] + 1 - torch.ones(x.shape[-1], dtype=x.dtype, device=x.device).cumsum(-1)
        xs = x - offset.log()
        return (-xs + torch.nn.functional.logsigmoid(xs) + torch.log(y[..., :-1])).sum(-1)

    def forward_shape(self, shape):
        s = tuple(_shape(shape))
        return s[:-1] + (s[-1] + 1,)

    def inverse_shape(self, shape):
        s = tuple(_shape(shape))
        return s[:-1] + (s[-1] - 1,)


class ReshapeTransform(Transform):
    """Reshape the event part of a tensor from ``in_event_shape`` to ``out_event_shape``."""
    _type = Type.BIJECTION

    def __init__(self, in_event_shape, out_event_shape):
        super().__init__()
        self.in_event_shape = tuple(_shape(in_event_shape))
        self.out_event_shape = tuple(_shape(out_event_shape))
        if math.prod(self.in_event_shape) != math.prod(self.out_event_shape):
            raise ValueError(f"The numel of 'in_event_shape' should be 'out_event_shape', but got "
                             f"{math.prod(self.in_event_shape)}!={math.prod(self.out_event_shape)}")
        self._event_rank = len(self.in_event_shape)

    def _forward(self, x):
        n = len(self.in_event_shape)
        return x.reshape(tuple(x.shape[:x.dim() - n]) + self.out_event_shape)

    def _inverse(self, y):
        n = len(self.out_event_shape)
        return y.reshape(tuple(y.shape[:y.dim() - n]) + self.in_event_shape)

    def _forward_log_det_jacobian(self, x):
        n = len(self.in_event_shape)
        return torch.zeros(x.shape[:x.dim() - n], dtype=x.dtype, device=x.device)

    def forward_shape(self, shape):
        s = tuple(_shape(shape))
        n = len(self.in_event_shape)
        if s[len(s) - n:] != self.in_event_shape:
            raise ValueError(f"Event shape mismatch, expected: {self.in_event_shape}, but got {s[len(s) - n:]}")
        return s[:len(s) - n] + self.out_event_shape

    def inverse_shape(self, shape):
        s = tuple(_shape(shape))
        n = len(self.out_event_shape)
        if s[len(s) - n:] != self.out_event_shape:
            raise ValueError(f"Event shape mismatch, expected: {self.out_event_shape}, but got {s[len(s) - n:]}")
        return s[:len(s) - n] + self.in_event_shape


class IndependentTransform(Transform):
    """Treat ``reinterpreted_batch_rank`` batch dims of ``base`` as event dims (log-det summed over them)."""

    def __init__(self, base, reinterpreted_batch_rank):
        super().__init__()
        if reinterpreted_batch_rank <= 0:
            raise ValueError(f"Expected 'reinterpreted_batch_rank' is grater than zero, but got "
                             f"{reinterpreted_batch_rank}")
        self._base = base
        self._rank = reinterpreted_batch_rank
        self._type = base._type
        self._event_rank = base._event_rank + reinterpreted_batch_rank

    def _forward(self, x):
        return self._base._forward(x)

    def _inverse(self, y):
        return self._base._inverse(y)

    def _forward_log_det_jacobian(self, x):
        ld = self._base._forward_log_det_jacobian(x)
        return ld.sum(list(range(-self._rank, 0))) if ld.dim() >= self._rank else ld

    def forward_shape(self, shape):
        return self._base.forward_shape(shape)

    def inverse_shape(self, shape):
        return self._base.inverse_shape(shape)


class ChainTransform(Transform):
    """Composition: forward applies transforms[0] first."""

    def __init__(self, transforms):
        super().__init__()
        self.transforms = list(transforms)
        self._type = Type.BIJECTION if all(t._is_injective() for t in self.transforms) else Type.OTHER
        self._event_rank = max([t._event_rank for t in self.transforms] or [0])

    def _forward(self, x):
        for t in self.transforms:
            x = t._forward(x)
        return x

    def _inverse(self, y):
        for t in reversed(self.transforms):
            y = t._inverse(y)
        return y

    def _forward_log_det_jacobian(self, x):
        total = 0.0
        rank = self._event_rank
        for t in self.transforms:
            ld = t._forward_log_det_jacobian(x)
            extra = rank - t._event_rank
            if extra > 0 and ld.dim() >= extra:
                ld = ld.sum(list(range(-extra, 0)))
            total = total + ld
            x = t._forward(x)
        return total

    def forward_shape(self, shape):
        for t in self.transforms:
            shape = t.forward_shape(shape)
        return shape

    def inverse_shape(self, shape):
        for t in reversed(self.transforms):
            shape = t.inverse_shape(shape)
        return shape


class StackTransform(Transform):
    """Apply transforms[i] to slice i of ``axis``."""

    def __init__(self, transforms, axis=0):
        super().__init__()
        self.transforms = list(transforms)
        self.axis = axis
        self._type = Type.BIJECTION if all(t._is_injective() for t in self.transforms) else Type.OTHER

    def _each(self, fn_name, x):
        parts = x.unbind(self.axis)
        if len(parts) != len(self.transforms):
            raise ValueError(f"Input size along axis {self.axis} ({len(parts)}) != number of transforms "
                             f"({len(self.transforms)})")
        return torch.stack([getattr(t, fn_name)(p) for t, p in zip(self.transforms, parts)], self.axis)

    def _forward(self, x):
        return self._each("_forward", x)

    def _inverse(self, y):
        return self._each("_inverse", y)

    def _forward_log_det_jacobian(self, x):
        return self._each("_forward_log_det_jacobian", x)
