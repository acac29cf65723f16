"""AST rewriting of a function's source for dy2static (reference: python/paddle/jit/dy2static/transformers/:
ifelse_transformer.py:57, loop_transformer.py:473, logical_transformer.py, early_return_transformer.py,
return_transformer.py, assert_transformer.py, super_transformer.py).

Calling convention of the rewritten code (own design — one pure function per branch / loop part instead of the
reference's nonlocal getter / setter pairs):

    if <test>:                            def __pa_true_3(x, y):        def __pa_false_3(x, y):
        x = ...            ----->             x = ...                       y = ...
    else:                                     return (x, y)                 return (x, y)
        y = ...                           (x, y) = _jst.IfElse(<test'>, __pa_true_3, __pa_false_3,
                                                               _jst.Vars(locals(), ('x', 'y')), ('x', 'y'))

``while`` becomes a condition function and a body function over the variables the body assigns
(``_jst.While``); ``for i in range(a, b, s)`` becomes such a while loop over a hidden counter; ``and`` /
``or`` / ``not`` in tests become ``_jst.And`` / ``Or`` / ``Not`` (short-circuit kept for Python values);
``a if c else b`` becomes ``_jst.IfExp``; ``assert`` becomes ``_jst.Assert``; zero-argument ``super()`` becomes
``super(__class__, <self>)`` (the rewritten function is built outside its class body). ``break`` / ``continue``
of a ``while`` or ``for ... in range`` loop become boolean flags: the loop test gains ``not <break flag>`` and the
statements after a flag-setting ``if`` are guarded, so a tensor-dependent break ends a static while node.

Returns: an ``if`` whose body ends in ``return`` absorbs the statements after it as its ``else`` (early-return
normalisation); when both branches then end in ``return``, each return becomes an assignment to
``__pa_ret`` and one ``return __pa_ret`` follows the if. Statements the rewriting cannot express (``break`` /
``continue`` inside ``with`` / ``try`` or a non-range ``for``, ``return`` in non-tail positions, ``yield``, ``global`` / ``nonlocal``) keep their Python
form: they still run in dygraph and for Python predicates, and a tensor predicate there fails at trace time
with the usual graph-break path.
"""
from __future__ import annotations

import ast

_PREFIX = "__pa_"
RET = "__pa_ret"


def _names_assigned(stmts):
    """Names bound by ``stmts`` in the enclosing function scope, in first-binding order (not descending into
    nested function / class / lambda / comprehension scopes, whose own names are theirs)."""
    out = []

    def add(n):
        if n not in out and not (n.startswith(_PREFIX) and n != RET):
            out.append(n)

    class V(ast.NodeVisitor):
        def visit_Name(self, node):
            if isinstance(node.ctx, (ast.Store, ast.Del)):
                add(node.id)

        def visit_FunctionDef(self, node):
            add(node.name)

        visit_AsyncFunctionDef = visit_FunctionDef

        def visit_ClassDef(self, node):
            add(node.name)

        def visit_Lambda(self, node):
            pass

        def visit_ListComp(self, node):
            pass

        visit_SetComp = visit_DictComp = visit_GeneratorExp = visit_ListComp

        def visit_Import(self, node):
            for a in node.names:
                add((a.asname or a.name).split(".")[0])

        visit_ImportFrom = visit_Import

        def visit_ExceptHandler(self, node):
            if node.name:
                add(node.name)
            self.generic_visit(node)

        def visit_NamedExpr(self, node):
            add(node.target.id)
            self.generic_visit(node)

    v = V()
    for s in stmts:
        v.visit(s)
    return out


def _contains(stmts, types, into_loops=True):
    """Any node of ``types`` in ``stmts`` outside nested function scopes (and, with ``into_loops=False``,
    outside nested loops — for break / continue, which belong to the innermost loop)."""
    class V(ast.NodeVisitor):
        found = False

        def generic_visit(self, node):
            if isinstance(node, types):
                self.found = True
                return
            if isinstance(node, (ast.FunctionDef, ast.AsyncFunctionDef, ast.Lambda, ast.ClassDef)):
                return
            if not into_loops and isinstance(node, (ast.For, ast.While, ast.AsyncFor)):
                for s in node.orelse:
                    self.visit(s)
                return
            super().generic_visit(node)
    v = V()
    for s in stmts:
        v.visit(s)
        if v.found:
            return True
    return False


def _ends_in_return(stmts):
    if not stmts:
        return False
    last = stmts[-1]
    if isinstance(last, ast.Return):
        return True
    if isinstance(last, ast.If):
        return _ends_in_return(last.body) and _ends_in_return(last.orelse)
    return False


def _returns_only_in_tail(stmts):
    """Every return of ``stmts`` is the tail of a tail if-chain (so it can become ``__pa_ret = ...``)."""
    if not stmts:
        return True
    if _contains(stmts[:-1], (ast.Return,)):
        return False
    last = stmts[-1]
    if isinstance(last, ast.Return):
        return True
    if isinstance(last, ast.If):
        return _returns_only_in_tail(last.body) and _returns_only_in_tail(last.orelse)
    return not _contains([last], (ast.Return,))


def _tail_returns_to_assign(stmts):
    last = stmts[-1]
    if isinstance(last, ast.Return):
        val = last.value if last.value is not None else ast.Constant(value=None)
        stmts[-1] = ast.copy_location(ast.Assign(targets=[ast.Name(id=RET, ctx=ast.Store())], value=val), last)
    elif isinstance(last, ast.If):
        _tail_returns_to_assign(last.body)
        _tail_returns_to_assign(last.orelse)


def normalize_early_returns(stmts):
    """``if c: ...; return a`` followed by more statements -> ``if c: ...; return a  else: <the rest>``
    (recursively), so that a returning branch and the fall-through path become the two arms of one if."""
    out = []
    i = 0
    while i < len(stmts):
        s = stmts[i]
        for field in ("body", "orelse", "finalbody"):
            if isinstance(s, (ast.If, ast.While, ast.For, ast.With, ast.Try)) and hasattr(s, field):
                setattr(s, field, normalize_early_returns(getattr(s, field)))
        rest = stmts[i + 1:]
        if isinstance(s, ast.If) and rest:
            if _ends_in_return(s.body) and not _ends_in_return(s.orelse):
                s.orelse = normalize_early_returns(s.orelse + rest)
                out.append(s)
                return out
            if _ends_in_return(s.orelse) and not _ends_in_return(s.body) and s.orelse:
                s.body = normalize_early_returns(s.body + rest)
                out.append(s)
                return out
        out.append(s)
        i += 1
    return out


def _jst(attr):
    return ast.Attribute(value=ast.Name(id="_jst", ctx=ast.Load()), attr=attr, ctx=ast.Load())


def _names_tuple(names, ctx):
    return ast.Tuple(elts=[ast.Name(id=n, ctx=ctx()) for n in names], ctx=ctx())


def _str_tuple(names):
    return ast.Tuple(elts=[ast.Constant(value=n) for n in names], ctx=ast.Load())


def _vars_call(names):
    return ast.Call(func=_jst("Vars"), args=[ast.Call(func=ast.Name(id="locals", ctx=ast.Load()), args=[],
                                                      keywords=[]), _str_tuple(names)], keywords=[])


def _fdef(name, params, body):
    args = ast.arguments(posonlyargs=[], args=[ast.arg(arg=p) for p in params], vararg=None, kwonlyargs=[],
                         kw_defaults=[], kwarg=None, defaults=[])
    return ast.FunctionDef(name=name, args=args, body=body or [ast.Pass()], decorator_list=[], returns=None,
                           type_comment=None)


class _Logical(ast.NodeTransformer):
    """and / or / not / if-expressions inside a test expression (lambdas keep short-circuit evaluation)."""

    def visit_BoolOp(self, node):
        self.generic_visit(node)
        fn = "And" if isinstance(node.op, ast.And) else "Or"
        acc = node.values[0]
        for v in node.values[1:]:
            acc = ast.Call(func=_jst(fn), args=[_lam(acc), _lam(v)], keywords=[])
        return acc

    def visit_UnaryOp(self, node):
        self.generic_visit(node)
        if isinstance(node.op, ast.Not):
            return ast.Call(func=_jst("Not"), args=[node.operand], keywords=[])
        return node

    def visit_IfExp(self, node):
        self.generic_visit(node)
        return ast.Call(func=_jst("IfExp"), args=[node.test, _lam(node.body), _lam(node.orelse)], keywords=[])

    def visit_Lambda(self, node):
        return node


def _set_flag(name, value=True):
    """``name = _jst.create_bool_as_type(name, value)``: a Python bool, or a bool tensor once the flag is one."""
    return ast.Assign(targets=[ast.Name(id=name, ctx=ast.Store())],
                      value=ast.Call(func=_jst("create_bool_as_type"),
                                     args=[ast.Name(id=name, ctx=ast.Load()), ast.Constant(value=value)],
                                     keywords=[]))


def _lower_break_continue(stmts, brk, cnt):
    """A loop body with ``break`` / ``continue`` (of this loop) as straight-line flag code (reference:
    transformers/break_continue_transformer.py): ``break`` sets ``brk``, ``continue`` sets ``cnt``, and every
    statement after an ``if`` that may have set one runs under ``if not (brk or cnt)``. None when a break /
    continue sits in a statement other than ``if`` (``with`` / ``try``), which keeps the Python loop."""
    out = []
    for idx, s in enumerate(stmts):
        if isinstance(s, ast.Break):
            out.append(ast.copy_location(_set_flag(brk), s))
            return out
        if isinstance(s, ast.Continue):
            out.append(ast.copy_location(_set_flag(cnt), s))
            return out
        if not _contains([s], (ast.Break, ast.Continue), into_loops=False):
            out.append(s)
            continue
        if not isinstance(s, ast.If):
            return None
        body, orelse = _lower_break_continue(s.body, brk, cnt), _lower_break_continue(s.orelse, brk, cnt)
        if body is None or orelse is None:
            return None
        s.body, s.orelse = body or [ast.Pass()], orelse
        out.append(s)
        rest = _lower_break_continue(stmts[idx + 1:], brk, cnt)
        if rest is None:
            return None
        if rest:
            flags = [ast.Name(id=f, ctx=ast.Load()) for f in (brk, cnt) if f]
            test = flags[0] if len(flags) == 1 else ast.BoolOp(op=ast.Or(), values=flags)
            out.append(ast.If(test=ast.UnaryOp(op=ast.Not(), operand=test), body=rest, orelse=[]))
        return out
    return out


def _lam(expr):
    args = ast.arguments(posonlyargs=[], args=[], vararg=None, kwonlyargs=[], kw_defaults=[], kwarg=None,
                         defaults=[])
    return ast.Lambda(args=args, body=expr)


class DygraphToStaticAst(ast.NodeTransformer):
    """Rewrites one function body (see the module docstring). Nested function definitions are rewritten too."""

    def __init__(self, self_name=None):
        self.k = 0
        self.self_name = self_name
        self.converted = 0

    def _uid(self):
        self.k += 1
        return self.k

    # ---------------------------------------------------------------- statements lists
    def _block(self, stmts):
        stmts = normalize_early_returns(list(stmts))
        out = []
        for s in stmts:
            r = self.visit(s)
            if r is None:
                continue
            out.extend(r if isinstance(r, list) else [r])
        return out

    def visit_FunctionDef(self, node):
        node.body = self._block(node.body)
        return node

    visit_AsyncFunctionDef = visit_FunctionDef

    def visit_Lambda(self, node):
        return node

    def _generic_block_owner(self, node):
        for field in ("body", "orelse", "finalbody"):
            if hasattr(node, field) and isinstance(getattr(node, field), list):
                setattr(node, field, self._block(getattr(node, field)))
        if isinstance(node, ast.Try):
            for h in node.handlers:
                h.body = self._block(h.body)
        return node

    visit_With = visit_Try = _generic_block_owner

    # ---------------------------------------------------------------- expressions
    def visit_Call(self, node):
        self.generic_visit(node)
        if (isinstance(node.func, ast.Name) and node.func.id == "super" and not node.args and not node.keywords
                and self.self_name):
            node.args = [ast.Name(id="__class__", ctx=ast.Load()), ast.Name(id=self.self_name, ctx=ast.Load())]
        return node

    def visit_Assert(self, node):
        self.generic_visit(node)
        test = _Logical().visit(node.test)
        args = [test] + ([node.msg] if node.msg is not None else [])
        return ast.copy_location(ast.Expr(value=ast.Call(func=_jst("Assert"), args=args, keywords=[])), node)

    def visit_IfExp(self, node):
        self.generic_visit(node)
        return _Logical().visit(node)

    # ---------------------------------------------------------------- if / else
    def visit_If(self, node):
        body, orelse = node.body, node.orelse
        if (_contains(body + orelse, (ast.Break, ast.Continue), into_loops=False)
                or _contains(body + orelse, (ast.Yield, ast.YieldFrom, ast.Global, ast.Nonlocal, ast.Await))
                or not (_returns_only_in_tail(body) and _returns_only_in_tail(orelse))):
            return self._generic_block_owner(node)
        with_ret = _contains(body + orelse, (ast.Return,))
        if with_ret and not (_ends_in_return(body) and _ends_in_return(orelse)):
            return self._generic_block_owner(node)
        body, orelse = list(body), list(orelse)
        if with_ret:
            _tail_returns_to_assign(body)
            _tail_returns_to_assign(orelse)
        body = self._block(body)
        orelse = self._block(orelse)
        names = _names_assigned(body + orelse)
        k = self._uid()
        tname, fname = f"{_PREFIX}true_{k}", f"{_PREFIX}false_{k}"
        ret = ast.Return(value=_names_tuple(names, ast.Load))
        tdef = _fdef(tname, names, body + [ret])
        fdef = _fdef(fname, names, orelse + [ast.Return(value=_names_tuple(names, ast.Load))])
        call = ast.Call(func=_jst("IfElse"), args=[_Logical().visit(node.test), ast.Name(id=tname, ctx=ast.Load()),
                                                   ast.Name(id=fname, ctx=ast.Load()), _vars_call(names),
                                                   _str_tuple(names)], keywords=[])
        if names:
            stmt = ast.Assign(targets=[_names_tuple(names, ast.Store)], value=call)
        else:
            stmt = ast.Expr(value=call)
        out = [tdef, fdef, stmt]
        if with_ret:
            out.append(ast.Return(value=ast.Name(id=RET, ctx=ast.Load())))
        self.converted += 1
        return [ast.copy_location(s, node) for s in out]

    # ---------------------------------------------------------------- loops
    def _loop_ok(self, node):
        return not (node.orelse or _contains(node.body, (ast.Break, ast.Continue), into_loops=False)
                    or _contains(node.body, (ast.Return, ast.Yield, ast.YieldFrom, ast.Global, ast.Nonlocal,
                                             ast.Await)))

    def _break_flags(self, node):
        """(flag initialisers, lowered body, break flag or None) for a loop whose body breaks / continues, else
        None (see _lower_break_continue)."""
        import copy
        if node.orelse or not _contains(node.body, (ast.Break, ast.Continue), into_loops=False) or _contains(
                node.body, (ast.Return, ast.Yield, ast.YieldFrom, ast.Global, ast.Nonlocal, ast.Await)):
            return None
        k = self._uid()
        brk = f"_jst_brk_{k}" if _contains(node.body, (ast.Break,), into_loops=False) else None
        cnt = f"_jst_cnt_{k}" if _contains(node.body, (ast.Continue,), into_loops=False) else None
        body = _lower_break_continue(copy.deepcopy(node.body), brk, cnt)
        if body is None:
            return None
        pre = [ast.Assign(targets=[ast.Name(id=f, ctx=ast.Store())], value=ast.Constant(value=False))
               for f in (brk, cnt) if f]
        if cnt:
            body = [_set_flag(cnt, False)] + body
        return pre, body, brk

    @staticmethod
    def _and_not(brk, test):
        if brk is None:
            return test
        return ast.BoolOp(op=ast.And(), values=[ast.UnaryOp(op=ast.Not(), operand=ast.Name(id=brk, ctx=ast.Load())),
                                                test])

    def visit_While(self, node):
        bc = self._break_flags(node)
        if bc is not None:
            pre, body, brk = bc
            out = self.visit_While(ast.copy_location(ast.While(test=self._and_not(brk, node.test), body=body,
                                                               orelse=[]), node))
            return [ast.copy_location(s, node) for s in pre] + (out if isinstance(out, list) else [out])
        if not self._loop_ok(node):
            return self._generic_block_owner(node)
        body = self._block(node.body)
        names = _names_assigned(body)
        # names the test reads but the body never rebinds stay free (closure) reads
        k = self._uid()
        cname, bname = f"{_PREFIX}cond_{k}", f"{_PREFIX}body_{k}"
        cdef = _fdef(cname, names, [ast.Return(value=_Logical().visit(node.test))])
        bdef = _fdef(bname, names, body + [ast.Return(value=_names_tuple(names, ast.Load))])
        call = ast.Call(func=_jst("While"), args=[ast.Name(id=cname, ctx=ast.Load()), ast.Name(id=bname, ctx=ast.Load()),
                                                  _vars_call(names), _str_tuple(names)], keywords=[])
        stmt = ast.Assign(targets=[_names_tuple(names, ast.Store)], value=call) if names else ast.Expr(value=call)
        self.converted += 1
        return [ast.copy_location(s, node) for s in (cdef, bdef, stmt)]

    def visit_For(self, node):
        it = node.iter
        is_range = (isinstance(it, ast.Call) and isinstance(it.func, ast.Name) and it.func.id == "range"
                    and not it.keywords and 1 <= len(it.args) <= 3 and isinstance(node.target, ast.Name))
        # only a range loop is lowered: a Python iteration must keep rebinding its target until the real break
        bc = self._break_flags(node) if is_range else None
        flag_pre, brk = [], None
        if bc is not None:
            flag_pre, lowered, brk = bc
            node = ast.copy_location(ast.For(target=node.target, iter=node.iter, body=lowered, orelse=[],
                                             type_comment=None), node)
        if not (is_range and self._loop_ok(node)):
            return self._generic_block_owner(node)
        k = self._uid()
        ctr, stop, step = f"{_PREFIX}i_{k}", f"{_PREFIX}stop_{k}", f"{_PREFIX}step_{k}"
        a = it.args
        start_e = a[0] if len(a) >= 2 else ast.Constant(value=0)
        stop_e = a[1] if len(a) >= 2 else a[0]
        step_e = a[2] if len(a) == 3 else ast.Constant(value=1)
        name = lambda n, c=ast.Load: ast.Name(id=n, ctx=c())  # noqa: E731
        pre = [ast.Assign(targets=[name(ctr, ast.Store)], value=start_e),
               ast.Assign(targets=[name(stop, ast.Store)], value=stop_e),
               ast.Assign(targets=[name(step, ast.Store)], value=step_e)]
        body = [ast.Assign(targets=[ast.Name(id=node.target.id, ctx=ast.Store())], value=name(ctr))] + list(node.body)
        body.append(ast.Assign(targets=[name(ctr, ast.Store)],
                               value=ast.BinOp(left=name(ctr), op=ast.Add(), right=name(step))))
        test = self._and_not(brk, ast.Call(func=_jst("RangeCond"), args=[name(ctr), name(stop), name(step)],
                                           keywords=[]))
        w = ast.While(test=test, body=body, orelse=[])
        # the hidden counter is a loop variable too: _names_assigned skips the __pa_ prefix, so bind it by hand
        out = self.visit_While(w)
        if isinstance(out, list) and len(out) == 3:
            cdef, bdef, stmt = out
            for d in (cdef, bdef):
                d.args.args.insert(0, ast.arg(arg=ctr))
            bdef.body[-1] = ast.Return(value=ast.Tuple(elts=[name(ctr)] + list(bdef.body[-1].value.elts),
                                                       ctx=ast.Load()))
            call = stmt.value
            names = [ctr] + [e.value for e in call.args[3].elts]
            call.args[2] = _vars_call(names)
            call.args[3] = _str_tuple(names)
            if isinstance(stmt, ast.Expr):
                stmt = ast.Assign(targets=[_names_tuple(names, ast.Store)], value=call)
            else:
                stmt.targets = [_names_tuple(names, ast.Store)]
            out = [cdef, bdef, stmt]
        else:
            return self._generic_block_owner(node)
        return [ast.copy_location(s, node) for s in flag_pre + pre + out]
