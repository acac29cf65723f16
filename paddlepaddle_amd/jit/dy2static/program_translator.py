"""Source -> converted function (reference: python/paddle/jit/dy2static/program_translator.py
``convert_to_static``, convert_call_func.py ``convert_call``).

``convert_to_static(fn)`` reads ``fn``'s source, rewrites its body with transformer.DygraphToStaticAst and
compiles the result inside a factory function whose parameters are ``fn``'s free variables (so closures
keep working) plus ``_jst`` (this package) and ``__class__`` (for the rewritten zero-argument ``super()``).
Results are cached per function object. Functions without retrievable source, lambdas, generators and this
framework's own modules are returned unchanged.

While a converted program is being recorded (``converting()``), ``Layer.__call__`` also converts the
``forward`` of user-defined sublayers (the reference's convert_call over nested layer calls).
"""
from __future__ import annotations

import ast
import functools
import inspect
import textwrap
import types
import weakref

from .transformer import DygraphToStaticAst

_CACHE: "weakref.WeakKeyDictionary" = weakref.WeakKeyDictionary()
from ...framework.dy2static_state import ACTIVE as _ACTIVE  # noqa: E402
_SKIP_PREFIXES = ("paddlepaddle_amd.", "torch", "numpy")


def converting():
    return _ACTIVE[0] > 0


class _Converting:
    def __enter__(self):
        _ACTIVE[0] += 1

    def __exit__(self, *exc):
        _ACTIVE[0] -= 1


def conversion_scope():
    """Context: sublayer forwards called inside it are converted too."""
    return _Converting()


def _skip(fn):
    mod = getattr(fn, "__module__", "") or ""
    if mod == "paddlepaddle_amd" or mod.startswith(_SKIP_PREFIXES):
        return not mod.startswith("paddlepaddle_amd.tests")
    code = getattr(fn, "__code__", None)
    if code is None or code.co_flags & (inspect.CO_GENERATOR | inspect.CO_COROUTINE | inspect.CO_ASYNC_GENERATOR):
        return True
    return fn.__name__ == "<lambda>" or getattr(fn, "_not_to_static", False)


def convert_to_static(fn):
    """The converted version of ``fn`` (a function or bound method); ``fn`` itself when it cannot be
    converted."""
    if isinstance(fn, types.MethodType):
        conv = convert_to_static(fn.__func__)
        return fn if conv is fn.__func__ else types.MethodType(conv, fn.__self__)
    if not isinstance(fn, types.FunctionType) or _skip(fn):
        return fn
    hit = _CACHE.get(fn)
    if hit is not None:
        return hit
    try:
        conv = _convert(fn)
    except (OSError, TypeError, SyntaxError, IndentationError):
        conv = fn
    _CACHE[fn] = conv
    return conv


def _convert(fn):
    src = textwrap.dedent(inspect.getsource(fn))
    tree = ast.parse(src)
    fdef = next((n for n in tree.body if isinstance(n, (ast.FunctionDef, ast.AsyncFunctionDef))), None)
    if fdef is None or fdef.name != fn.__name__:
        raise TypeError("source is not a plain function definition")
    fdef.decorator_list = []  # to_static & co. must not re-apply to the converted function
    first = fdef.args.posonlyargs + fdef.args.args
    tr = DygraphToStaticAst(self_name=first[0].arg if first else None)
    fdef = tr.visit(fdef)
    if tr.converted == 0 and "super" not in fn.__code__.co_names:
        return fn  # nothing to rewrite: keep the original (exact tracebacks, no factory)
    free = list(fn.__code__.co_freevars)
    params = [f for f in free if f != "__class__"] + ["_jst", "__class__"]
    factory = ast.FunctionDef(
        name="__pa_factory",
        args=ast.arguments(posonlyargs=[], args=[ast.arg(arg=p) for p in params], vararg=None, kwonlyargs=[],
                           kw_defaults=[], kwarg=None, defaults=[]),
        body=[fdef, ast.Return(value=ast.Name(id=fdef.name, ctx=ast.Load()))], decorator_list=[], returns=None,
        type_comment=None)
    mod = ast.Module(body=[factory], type_ignores=[])
    ast.fix_missing_locations(mod)
    filename = f"<dy2static {fn.__module__}.{fn.__qualname__}>"
    code = compile(mod, filename, "exec")
    ns = {}
    exec(code, fn.__globals__, ns)  # the factory lands in ns; the function's globals stay untouched
    from . import _runtime_namespace
    cells = dict(zip(free, fn.__closure__ or ()))
    owner = _owner_class(fn, cells)
    args = [cells[f].cell_contents for f in params[:-2]] + [_runtime_namespace(), owner]
    new = ns["__pa_factory"](*args)
    new.__defaults__ = fn.__defaults__
    new.__kwdefaults__ = fn.__kwdefaults__
    functools.update_wrapper(new, fn)
    new.__wrapped__ = fn
    new._pa_dy2static_source = ast.unparse(fdef)
    return new


def _owner_class(fn, cells):
    c = cells.get("__class__")
    if c is not None:
        try:
            return c.cell_contents
        except ValueError:
            pass
    qual = fn.__qualname__.split(".")
    if len(qual) >= 2 and "<locals>" not in qual:
        obj = fn.__globals__.get(qual[0])
        for part in qual[1:-1]:
            obj = getattr(obj, part, None)
        return obj
    return None


def ast_to_source_code(node):
    return ast.unparse(node)


def converted_source(fn):
    """The rewritten source of ``fn`` (for inspection / debugging, like the reference's code printing)."""
    conv = convert_to_static(fn)
    return getattr(conv, "_pa_dy2static_source", None) or getattr(conv, "__func__", conv).__dict__.get(
        "_pa_dy2static_source")
