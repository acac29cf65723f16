"""nn.Layer — the dygraph module base class.
Reference: python/paddle/nn/layer/layers.py:354 (class Layer), python/paddle/base/param_attr.py."""
from __future__ import annotations

import collections
import itertools
import re
import weakref

import numpy as np
import threading

import torch

from ...framework import dtype as _dt
from ...framework.place import to_torch_device
from ...framework.tensor import Parameter, Tensor, _wrap
from .. import initializer as I

_layer_name_counters = collections.defaultdict(itertools.count)
_param_name_counters = collections.defaultdict(itertools.count)


def _camel_to_snake(name):
    s1 = re.sub("(.)([A-Z][a-z]+)", r"\1_\2", name)
    return re.sub("([a-z0-9])([A-Z])", r"\1_\2", s1).lower()


class ParamAttr:
    """Reference: python/paddle/base/param_attr.py ParamAttr."""

    def __init__(self, name=None, initializer=None, learning_rate=1.0, regularizer=None, trainable=True,
                 do_model_average=True, need_clip=True):
        self.name = name
        self.initializer = initializer
        self.learning_rate = learning_rate
        self.regularizer = regularizer
        self.trainable = trainable
        self.do_model_average = do_model_average
        self.need_clip = need_clip

    @staticmethod
    def _to_attr(arg):
        if arg is None:
            return ParamAttr()
        if isinstance(arg, ParamAttr):
            return arg
        if isinstance(arg, str):
            return ParamAttr(name=arg)
        if isinstance(arg, I.Initializer):
            return ParamAttr(initializer=arg)
        if arg is False:
            return False
        if arg is True:
            return ParamAttr()
        raise TypeError(f"unsupported param attr {arg!r}")


class WeightNormParamAttr(ParamAttr):
    def __init__(self, dim=None, **kw):
        super().__init__(**kw)
        self.dim = dim


class HookRemoveHelper:
    _next_id = itertools.count()

    def __init__(self, hooks):
        self._hooks_ref = weakref.ref(hooks)
        self._hook_id = next(HookRemoveHelper._next_id)

    def remove(self):
        hooks = self._hooks_ref()
        if hooks is not None and self._hook_id in hooks:
            del hooks[self._hook_id]


class _LazyState(threading.local):
    depth = 0


_LAZY = _LazyState()  # > 0 inside paddle.LazyGuard


def create_parameter_tensor(shape, dtype, attr=None, is_bias=False, default_initializer=None, device=None):
    attr = ParamAttr._to_attr(attr)
    if attr is False:
        return None
    td = _dt.to_torch_dtype(dtype) if dtype is not None else _dt.default_dtype().torch_dtype
    dev = to_torch_device(device)
    lazy = _LAZY.depth > 0
    t = torch.empty([int(s) for s in shape], dtype=td, device="meta" if lazy else dev)
    init = attr.initializer or default_initializer
    if init is None:
        if is_bias:
            init = I._global_bias_init or I.Constant(0.0)
        else:
            init = I._global_weight_init or I.XavierUniform()
    if not lazy:
        with torch.no_grad():
            init._init(t)
    name = attr.name
    if name is None:
        name = f"create_parameter_{next(_param_name_counters['create_parameter'])}.{'b' if is_bias else 'w'}_0"
    p = Parameter(t, trainable=attr.trainable, name=name,
                  optimize_attr={"learning_rate": attr.learning_rate},
                  regularizer=attr.regularizer, need_clip=attr.need_clip,
                  do_model_average=attr.do_model_average)
    if lazy:
        p.__dict__["_lazy_init"] = (init, dev)
    return p


from ...framework.dy2static_state import ACTIVE as _D2S_ACTIVE  # noqa: E402


class Layer:
    """Base class of all layers (see module docstring)."""

    training = True

    def __init__(self, name_scope=None, dtype=None):
        if dtype is None:
            dtype = _dt.get_default_dtype()
        object.__setattr__(self, "_parameters", collections.OrderedDict())
        object.__setattr__(self, "_sub_layers", collections.OrderedDict())
        object.__setattr__(self, "_buffers", collections.OrderedDict())
        object.__setattr__(self, "_non_persistable_buffer_names_set", set())
        object.__setattr__(self, "_forward_pre_hooks", collections.OrderedDict())
        object.__setattr__(self, "_forward_post_hooks", collections.OrderedDict())
        object.__setattr__(self, "training", True)
        object.__setattr__(self, "_dtype", dtype)
        if name_scope is None:
            name_scope = _camel_to_snake(self.__class__.__name__)
        object.__setattr__(self, "_full_name", f"{name_scope}_{next(_layer_name_counters[name_scope])}")
        object.__setattr__(self, "_param_idx", itertools.count())
        object.__setattr__(self, "_casted_by_pure_fp16", False)
        object.__setattr__(self, "_state_dict_hooks", collections.OrderedDict())

    # ------------------------------------------------------------------ basics
    def full_name(self):
        return self._full_name

    def forward(self, *inputs, **kwargs):
        raise NotImplementedError

    def __call__(self, *inputs, **kwargs):
        if self._forward_pre_hooks:
            for hook in list(self._forward_pre_hooks.values()):
                r = hook(self, inputs)
                if r is not None:
                    inputs = r if isinstance(r, tuple) else (r,)
        if _D2S_ACTIVE[0] and "forward" not in self.__dict__:
            # recording a converted program: user sublayers' tensor-dependent control flow is converted too
            from ...jit.dy2static import convert_to_static
            out = convert_to_static(self.forward)(*inputs, **kwargs)
        else:
            out = self.forward(*inputs, **kwargs)
        if self._forward_post_hooks:
            for hook in list(self._forward_post_hooks.values()):
                r = hook(self, inputs, out)
                if r is not None:
                    out = r
        return out

    def register_forward_pre_hook(self, hook):
        h = HookRemoveHelper(self._forward_pre_hooks)
        self._forward_pre_hooks[h._hook_id] = hook
        return h

    def register_forward_post_hook(self, hook):
        h = HookRemoveHelper(self._forward_post_hooks)
        self._forward_post_hooks[h._hook_id] = hook
        return h

    def register_state_dict_hook(self, hook):
        h = HookRemoveHelper(self._state_dict_hooks)
        self._state_dict_hooks[h._hook_id] = hook
        return h

    def train(self):
        for l in self.sublayers(include_self=True):
            object.__setattr__(l, "training", True)
        return self

    def eval(self):
        for l in self.sublayers(include_self=True):
            object.__setattr__(l, "training", False)
        return self

    def extra_repr(self):
        return ""

    def __repr__(self):
        lines = []
        for name, l in self._sub_layers.items():
            r = repr(l).replace("\n", "\n  ")
            lines.append(f"({name}): {r}")
        main = self.__class__.__name__ + "(" + self.extra_repr()
        if lines:
            main += "\n  " + "\n  ".join(lines) + "\n"
        return main + ")"

    # ------------------------------------------------------------------ parameters
    def create_parameter(self, shape, attr=None, dtype=None, is_bias=False, default_initializer=None):
        dtype = dtype if dtype is not None else self._dtype
        p = create_parameter_tensor(shape, dtype, attr, is_bias, default_initializer)
        if p is not None and (ParamAttr._to_attr(attr) is None or getattr(ParamAttr._to_attr(attr), "name", None) is None):
            p.name = f"{self._full_name}.{'b' if is_bias else 'w'}_{next(self._param_idx)}"
        return p

    def create_variable(self, name=None, persistable=None, dtype=None):
        t = _wrap(torch.empty(0, dtype=_dt.to_torch_dtype(dtype or self._dtype)))
        t.persistable = bool(persistable)
        return t

    create_tensor = create_variable

    def add_parameter(self, name, parameter):
        if parameter is None:
            self._parameters[name] = None
        elif not isinstance(parameter, Parameter):
            raise TypeError("add_parameter expects a Parameter")
        else:
            self._parameters[name] = parameter
        return parameter

    def add_sublayer(self, name, sublayer):
        self._sub_layers[str(name)] = sublayer
        return sublayer

    def register_buffer(self, name, tensor, persistable=True):
        self._buffers[name] = tensor
        if not persistable:
            self._non_persistable_buffer_names_set.add(name)
        else:
            self._non_persistable_buffer_names_set.discard(name)

    def parameters(self, include_sublayers=True):
        return [p for _, p in self.named_parameters(include_sublayers=include_sublayers)]

    def named_parameters(self, prefix="", include_sublayers=True, remove_duplicate=True):
        seen = set()
        layers = self.named_sublayers(prefix=prefix, include_self=True) if include_sublayers else [(prefix, self)]
        for lp, l in layers:
            for n, p in l._parameters.items():
                if p is None or (remove_duplicate and id(p) in seen):
                    continue
                seen.add(id(p))
                yield (lp + "." + n if lp else n), p

    def named_sublayers(self, prefix="", include_self=False, layers_set=None):
        if layers_set is None:
            layers_set = set()
        if include_self and id(self) not in layers_set:
            layers_set.add(id(self))
            yield prefix, self
        for n, l in self._sub_layers.items():
            if l is None:
                continue
            p = prefix + "." + n if prefix else n
            if id(l) in layers_set:
                continue
            layers_set.add(id(l))
            yield p, l
            yield from l.named_sublayers(prefix=p, include_self=False, layers_set=layers_set)

    def sublayers(self, include_self=False):
        return [l for _, l in self.named_sublayers(include_self=include_self)]

    def children(self):
        return [l for _, l in self.named_children()]

    def named_children(self):
        seen = set()
        for n, l in self._sub_layers.items():
            if l is not None and id(l) not in seen:
                seen.add(id(l))
                yield n, l

    def buffers(self, include_sublayers=True):
        return [b for _, b in self.named_buffers(include_sublayers=include_sublayers)]

    def named_buffers(self, prefix="", include_sublayers=True):
        layers = self.named_sublayers(prefix=prefix, include_self=True) if include_sublayers else [(prefix, self)]
        seen = set()
        for lp, l in layers:
            for n, b in l._buffers.items():
                if b is None or id(b) in seen:
                    continue
                seen.add(id(b))
                yield (lp + "." + n if lp else n), b

    def clear_gradients(self, set_to_zero=True):
        for p in self.parameters():
            if p.trainable:
                p.clear_grad(set_to_zero)

    def apply(self, fn):
        for l in self.children():
            l.apply(fn)
        fn(self)
        return self

    # ------------------------------------------------------------------ attribute plumbing
    def __getattr__(self, name):
        d = self.__dict__
        if "_parameters" in d:
            if name in d["_parameters"]:
                return d["_parameters"][name]
            if name in d["_sub_layers"]:
                return d["_sub_layers"][name]
            if name in d["_buffers"]:
                return d["_buffers"][name]
        raise AttributeError(f"'{type(self).__name__}' object has no attribute '{name}'")

    def __setattr__(self, name, value):
        d = self.__dict__
        params = d.get("_parameters")
        if isinstance(value, Parameter):
            if params is None:
                raise RuntimeError("super().__init__() must be called before assigning parameters")
            for k in ("_sub_layers", "_buffers"):
                d[k].pop(name, None)
            d.pop(name, None)
            params[name] = value
        elif isinstance(value, Layer):
            if params is None:
                raise RuntimeError("super().__init__() must be called before assigning sublayers")
            params.pop(name, None)
            d["_buffers"].pop(name, None)
            d.pop(name, None)
            d["_sub_layers"][name] = value
        elif params is not None and name in params:
            if value is not None and not isinstance(value, Parameter):
                if isinstance(value, Tensor):
                    params[name]._t = value._t  # in-place re-bind of parameter storage
                    return
                raise TypeError(f"cannot assign {type(value)} to parameter {name}")
            params[name] = value
        elif params is not None and name in d["_sub_layers"]:
            d["_sub_layers"][name] = value
        elif params is not None and name in d["_buffers"]:
            d["_buffers"][name] = value
        else:
            object.__setattr__(self, name, value)

    def __delattr__(self, name):
        for k in ("_parameters", "_sub_layers", "_buffers"):
            if name in self.__dict__.get(k, {}):
                del self.__dict__[k][name]
                return
        object.__delattr__(self, name)

    def __dir__(self):
        return list(super().__dir__()) + list(self._parameters) + list(self._sub_layers) + list(self._buffers)

    # ------------------------------------------------------------------ state dict
    def state_dict(self, destination=None, include_sublayers=True, structured_name_prefix="", use_hook=True,
                   keep_vars=True):
        dest = collections.OrderedDict() if destination is None else destination
        for n, p in self.named_parameters(include_sublayers=include_sublayers):
            dest[structured_name_prefix + n] = p
        for lp, l in (self.named_sublayers(include_self=True) if include_sublayers else [("", self)]):
            for n, b in l._buffers.items():
                if b is None or n in l._non_persistable_buffer_names_set:
                    continue
                key = (lp + "." + n) if lp else n
                dest[structured_name_prefix + key] = b
        if use_hook:
            for hook in self._state_dict_hooks.values():
                r = hook(dest)
                if r is not None:
                    dest = r
        return dest

    to_static_state_dict = state_dict

    def set_state_dict(self, state_dict, use_structured_name=True):
        own = self.state_dict(use_hook=False)
        missing, unexpected = [], []
        if use_structured_name:
            mapping = own
        else:
            mapping = {v.name: v for v in own.values()}
        for k, target in mapping.items():
            if k not in state_dict:
                missing.append(k)
                continue
            v = state_dict[k]
            if isinstance(v, tuple) and len(v) == 2 and isinstance(v[1], np.ndarray):
                v = v[1]
            src = v._t if isinstance(v, Tensor) else torch.as_tensor(np.asarray(v))
            if list(src.shape) != list(target._t.shape):
                raise ValueError(f"shape mismatch for {k}: {list(src.shape)} vs {target.shape}")
            with torch.no_grad():
                target._t.copy_(src.to(target._t.device, target._t.dtype))
        for k in state_dict:
            if k not in mapping:
                unexpected.append(k)
        return missing, unexpected

    set_dict = set_state_dict
    load_dict = set_state_dict

    # ------------------------------------------------------------------ dtype / device
    def _apply_to_tensors(self, fn, include_buffers=True, floating_only=True):
        for l in self.sublayers(include_self=True):
            for p in l._parameters.values():
                if p is None:
                    continue
                if floating_only and not p._t.is_floating_point():
                    continue
                new = fn(p._t)
                if new is not p._t:
                    p._replace_data(new)
            if include_buffers:
                for n, b in list(l._buffers.items()):
                    if b is None or (floating_only and not b._t.is_floating_point()):
                        continue
                    b._t = fn(b._t)
        return self

    def to(self, device=None, dtype=None, blocking=None):
        if device is not None:
            dev = to_torch_device(device)
            self._apply_to_tensors(lambda t: t.to(dev), floating_only=False)
        if dtype is not None:
            td = _dt.to_torch_dtype(dtype)
            # floating parameters / buffers are cast (to any dtype: paddle's Layer.astype("int8") casts weights)
            self._apply_to_tensors(lambda t: t.to(td))
            for l in self.sublayers(include_self=True):
                object.__setattr__(l, "_dtype", _dt.convert_dtype(dtype).name)
        return self

    def astype(self, dtype=None):
        return self.to(dtype=dtype)

    def float(self, excluded_layers=None):
        return self.to(dtype="float32")

    def half(self, excluded_layers=None):
        return self.to(dtype="float16")

    def bfloat16(self, excluded_layers=None):
        return self.to(dtype="bfloat16")

    def float16(self, excluded_layers=None):
        return self.half()

    def cuda(self, device_id=None):
        return self.to(device=f"gpu:{device_id or 0}")

    def cpu(self):
        return self.to(device="cpu")
