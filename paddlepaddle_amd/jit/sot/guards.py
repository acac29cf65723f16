"""Sources and guards of the bytecode translator (reference: python/paddle/jit/sot/opcode_translator/executor/
guard.py, tracker.py — every value a translated frame reads from outside carries a tracker describing where it
came from; the compiled function is valid while guards over those trackers hold).

A Source is a path from a root the call can re-evaluate — a positional argument of the call, a module global,
a closure cell — through attribute and item accesses. A Guard is (source, kind, expected) with kind
"value" (==, for plain data), "id" (identity, for modules / functions / layers / tensors captured as
constants) or "len"."""
from __future__ import annotations

import types

_PLAIN = (int, float, bool, str, bytes, type(None), complex)


def is_plain(v, depth=0):
    if isinstance(v, _PLAIN):
        return True
    if isinstance(v, (tuple, frozenset)) and depth < 3:
        return all(is_plain(x, depth + 1) for x in v)
    return False


class Source:
    __slots__ = ("kind", "key", "parent")

    def __init__(self, kind, key, parent=None):
        self.kind, self.key, self.parent = kind, key, parent

    def attr(self, name):
        return Source("attr", name, self)

    def item(self, key):
        return Source("item", key, self)

    def get(self, args, fn):
        k = self.kind
        if k == "arg":
            return args[self.key]
        if k == "global":
            g, name = self.key
            if name in g:
                return g[name]
            b = g.get("__builtins__", __builtins__)
            return b[name] if isinstance(b, dict) else getattr(b, name)
        if k == "cell":
            return self.key.cell_contents
        if k == "const":
            return self.key
        base = self.parent.get(args, fn)
        if k == "attr":
            return getattr(base, self.key)
        return base[self.key]

    def __repr__(self):
        if self.kind == "arg":
            return f"arg:{self.key}"
        if self.kind == "global":
            return f"global:{self.key[1]}"
        if self.kind == "cell":
            return "cell"
        if self.kind == "const":
            return "const"
        return f"{self.parent!r}.{self.key}" if self.kind == "attr" else f"{self.parent!r}[{self.key!r}]"

    def key_tuple(self):
        k = self.key
        if self.kind == "global":
            k = (id(k[0]), k[1])
        elif self.kind in ("cell", "const"):
            k = id(k)
        return (self.kind, k, self.parent.key_tuple() if self.parent is not None else None)


class Guard:
    __slots__ = ("src", "kind", "expected")

    def __init__(self, src, kind, expected):
        self.src, self.kind, self.expected = src, kind, expected

    def check(self, args, fn):
        try:
            v = self.src.get(args, fn)
        except Exception:
            return False
        if self.kind == "id":
            return v is self.expected
        if self.kind == "len":
            try:
                return len(v) == self.expected
            except TypeError:
                return False
        return type(v) is type(self.expected) and v == self.expected

    def __repr__(self):
        return f"{self.src!r} {self.kind} {self.expected!r}" if self.kind != "id" else f"{self.src!r} is <{type(self.expected).__name__}>"


class GuardSet:
    def __init__(self):
        self.guards = {}

    def add(self, src, kind, expected):
        if src is None:
            return
        key = (src.key_tuple(), kind)
        if key not in self.guards:
            self.guards[key] = Guard(src, kind, expected)

    def add_for_value(self, src, v):
        """Guard a sourced value the trace specialised on: plain data by value, anything else by identity."""
        if src is None:
            return
        if is_plain(v):
            self.add(src, "value", v)
        elif isinstance(v, (types.ModuleType,)):
            return  # modules are stable; their attributes carry their own guards
        else:
            self.add(src, "id", v)

    def check(self, args, fn):
        return all(g.check(args, fn) for g in self.guards.values())

    def __iter__(self):
        return iter(self.guards.values())

    def __len__(self):
        return len(self.guards)
