"""paddle.jit.dy2static: AST conversion of Python control flow on tensors into static-program control flow.

Reference: python/paddle/jit/dy2static/__init__.py (the ``_jst`` names the rewritten code calls),
transformers/ifelse_transformer.py:57, loop_transformer.py:473, convert_operators.py:167,398.
"""
from __future__ import annotations

import sys

from .convert_operators import (  # noqa: F401
    Dygraph2StaticException, UndefinedVar, Vars, convert_assert as Assert, convert_attr as Attr,
    convert_ifelse as IfElse, convert_ifexp as IfExp, convert_len as Len, convert_load as Ld,
    convert_logical_and as And, convert_logical_not as Not, convert_logical_or as Or,
    convert_range_cond as RangeCond, convert_shape as Shape, convert_var_dtype as AsDtype,
    convert_while_loop as While, create_bool_as_type, indexable as Indexable, to_static_variable,
    unpack_by_structure as Unpack,
)
from .program_translator import (  # noqa: F401
    ast_to_source_code, conversion_scope, convert_to_static, converted_source, converting,
)
from .transformer import DygraphToStaticAst  # noqa: F401


def Call(fn):
    """convert_call: the converted version of a user function (framework functions pass through)."""
    return convert_to_static(fn)


def WrapSuper(super_fn):
    return super_fn


def saw(x):
    return x


def _runtime_namespace():
    return sys.modules[__name__]


__all__ = []
