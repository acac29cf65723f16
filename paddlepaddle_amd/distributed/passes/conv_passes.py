"""Convolution fusion passes over traced static Programs (static/program.py), reference
distributed/passes/cpp_pass.py:63 ``fuse_relu_depthwise_conv`` and :171 ``fuse_resunit`` (C++ IR passes there).

* ``fuse_relu_depthwise_conv``: ``relu(x)`` whose only consumer is a depthwise ``conv2d`` (groups == channels,
  one filter per channel; directly, or through the NHWC -> NCHW permute view of a channels-last layer) becomes ONE
  ``ops.fused_conv.relu_depthwise_conv2d`` node: on the NHWC HIP kernels the ReLU runs on the convolution's loads
  and as the data gradient's mask, so the ReLU output is neither written nor read back.
* ``fuse_resunit``: a channels-last convolution without bias (``permute -> conv2d -> permute``) whose only consumer
  is a batch_norm_act_nhwc node (training or inference, with the residual / ReLU that fuse_bn_act /
  fuse_bn_add_act folded into it) becomes ONE ``ops.fused_conv.conv_bn_unit`` node — the ResNet unit: the
  convolution writes the BN statistics from its epilogue and the BN apply kernel adds the residual and applies ReLU
  (incubate/operators/resnet_unit.py conv_bn_act).
"""
from __future__ import annotations

from .pass_base import PassBase, PassType, register_pass
from ...static import program as P
from .program_passes import _BN, _act_of, _bn_args, _keep_rc, _protected, _rewrite_until_fixed, _shape_of, _slot

__all__ = ["FuseReluDepthwiseConvPass", "FuseResUnitPass"]

_CONV = {"f:torch:conv2d", "f:torch.nn.functional:conv2d"}
_PERMUTE = {"m:permute", "f:torch:permute"}
_RELU_DW = "o:paddlepaddle_amd.ops.fused_conv:relu_depthwise_conv2d"
_UNIT = "o:paddlepaddle_amd.ops.fused_conv:conv_bn_unit"
_CONV_ARGS = ("input", "weight", "bias", "stride", "padding", "dilation", "groups")
_CONV_DEFAULTS = (None, None, None, 1, 0, 1, 1)


def _conv_args(n):
    """conv2d call as the 7 positional arguments, or None."""
    if n is None or n.name not in _CONV or len(n.args) > 7:
        return None
    a = list(n.args) + list(_CONV_DEFAULTS[len(n.args):])
    for k, v in n.kwargs.items():
        if k not in _CONV_ARGS:
            return None
        a[_CONV_ARGS.index(k)] = v
    return a


def _perm_of(n):
    """(source ref, dims) of a permute node, or (None, None)."""
    if n is None or n.name not in _PERMUTE or n.kwargs or not n.args:
        return None, None
    dims = n.args[1] if len(n.args) == 2 and isinstance(n.args[1], (list, tuple)) else n.args[1:]
    if not all(isinstance(d, int) for d in dims):
        return None, None
    return n.args[0], tuple(dims)


@register_pass("fuse_relu_depthwise_conv")
class FuseReluDepthwiseConvPass(PassBase):
    _after = ("auto_parallel_amp", "auto_parallel_fp16")

    def _type(self):
        return PassType.FUSION_OPT

    def _apply_single_impl(self, prog, startup, context):
        fn = P._resolve(_RELU_DW)

        def step(pr, j, n):
            a = _conv_args(n)
            if a is None or not isinstance(a[6], int) or a[6] < 2:
                return False
            xs, ws = _shape_of(prog, a[0]), _shape_of(prog, a[1])
            if xs is None or ws is None or len(xs) != 4 or len(ws) != 4:
                return False
            if not (xs[1] == a[6] == ws[0] and ws[1] == 1) or not pr.single(a[0]):
                return False  # not depthwise
            drop = []
            k, src = pr.of(a[0])
            cl = False
            s, dims = _perm_of(src)
            if s is not None:  # channels-last layer: relu(x_nhwc) -> permute(0, 3, 1, 2) -> conv
                if dims != (0, 3, 1, 2) or not pr.single(s):
                    return False
                drop.append(k)
                k, src = pr.of(s)
                cl = True
            if src is None or _act_of(src) != "relu" or src.kwargs.get("inplace", False):
                return False
            drop.append(k)
            x = src.args[0]
            if _slot(x) is None:
                return False
            pr.nodes[j] = _keep_rc(P.OpNode(fn, (x, a[1], a[2], a[3], a[4], a[5], a[6], cl), {}, n.outs, "op",
                                            _RELU_DW), n)
            for d in sorted(drop, reverse=True):
                del pr.nodes[d]
            return True

        n = _rewrite_until_fixed(prog, _protected(prog, self.get_attr("fetch_vars")), step)
        context.set_attr("fuse_relu_depthwise_conv.fused", context.get_attr("fuse_relu_depthwise_conv.fused", 0) + n)


@register_pass("fuse_resunit")
class FuseResUnitPass(PassBase):
    # after the BN passes, so the unit also takes the residual add and ReLU they folded into the BN node
    _after = ("auto_parallel_amp", "auto_parallel_fp16", "fuse_bn_act", "fuse_bn_add_act")

    def _type(self):
        return PassType.FUSION_OPT

    def _apply_single_impl(self, prog, startup, context):
        fn = P._resolve(_UNIT)

        def step(pr, j, n):
            b = _bn_args(n) if n.name == _BN else None
            if b is None or b[10] is not None or not pr.single(b[0]):
                return False
            k_out, pout = pr.of(b[0])
            c_ref, dims = _perm_of(pout)
            if c_ref is None or dims != (0, 2, 3, 1) or not pr.single(c_ref):
                return False
            k_conv, conv = pr.of(c_ref)
            a = _conv_args(conv)
            if a is None or a[2] is not None or isinstance(a[4], str):
                return False
            k_in, pin = pr.of(a[0])
            x, dims = _perm_of(pin)
            if x is None or dims != (0, 3, 1, 2) or _slot(x) is None:
                return False
            args = (x, a[1], a[3], a[4], a[5], a[6], b[1], b[2], b[3], b[4], b[5], b[6], b[7], b[8], b[9])
            pr.nodes[j] = _keep_rc(P.OpNode(fn, args, {}, n.outs, n.kind, _UNIT), n)
            drop = [k_out, k_conv] + ([k_in] if pr.single(a[0]) else [])
            for d in sorted(drop, reverse=True):
                del pr.nodes[d]
            return True

        n = _rewrite_until_fixed(prog, _protected(prog, self.get_attr("fetch_vars")), step)
        context.set_attr("fuse_resunit.fused", context.get_attr("fuse_resunit.fused", 0) + n)
