"""fuse_resnet_unit pass. Reference: python/paddle/incubate/passes/fuse_resnet_unit_pass.py:52 — a static-graph
rewrite of conv2d + batch_norm (+ elementwise_add) + relu into the resnet_unit op (cuDNN fused conv-BN).

In this framework the same fusion is a runtime rewrite that needs no graph pass: a convolution whose output a
training BN consumes writes the BN statistics in its epilogue and the add + relu run inside the BN apply pass
(ops/_conv_bn.py, csrc/kernels/bn.hip); programs replay through those ops. Applying this pass turns that
runtime fusion on (FLAGS_conv_bn_fusion) and returns the program unchanged."""
from __future__ import annotations


def fuse_resnet_unit(program=None):
    from ...framework.flags import set_flags
    set_flags({"FLAGS_conv_bn_fusion": True})
    return program
