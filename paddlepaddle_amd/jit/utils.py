"""paddle.jit.utils. Reference: python/paddle/jit/utils.py:25 OrderedSet (insertion-ordered set used by the
dy2static passes)."""
from __future__ import annotations


class OrderedSet:
    """A set that keeps insertion order (backed by a dict)."""

    def __init__(self, items=None):
        self._data = dict.fromkeys(items) if items is not None else {}

    def __iter__(self):
        return iter(self._data)

    def __or__(self, other):
        return OrderedSet(list(self) + list(other))

    def __ior__(self, other):
        for x in other:
            self._data[x] = None
        return self

    def __and__(self, other):
        return OrderedSet(x for x in self if x in other)

    def __iand__(self, other):
        self._data = {x: None for x in self if x in other}
        return self

    def __sub__(self, other):
        return OrderedSet(x for x in self if x not in other)

    def __isub__(self, other):
        self._data = {x: None for x in self if x not in other}
        return self

    def __xor__(self, other):
        return OrderedSet([x for x in self if x not in other] + [x for x in other if x not in self])

    def __ixor__(self, other):
        self._data = dict.fromkeys([x for x in self if x not in other] + [x for x in other if x not in self])
        return self

    def add(self, item):
        self._data[item] = None

    def remove(self, item):
        del self._data[item]

    def discard(self, item):
        self._data.pop(item, None)

    def __contains__(self, item):
        return item in self._data

    def __len__(self):
        return len(self._data)

    def __bool__(self):
        return bool(self._data)

    def __eq__(self, other):
        return isinstance(other, OrderedSet) and list(self._data) == list(other._data)

    def __hash__(self):
        return hash(tuple(self._data))

    def copy(self):
        return OrderedSet(self)

    def __repr__(self):
        return f"OrderedSet({', '.join(map(repr, self._data))})"
