"""Reference: python/paddle/utils/unique_name.py."""
from __future__ import annotations

import collections
import contextlib
import itertools

_counters = collections.defaultdict(itertools.count)
_prefix = [""]


def generate(key):
    return f"{_prefix[-1]}{key}_{next(_counters[key])}"


def generate_with_ignorable_key(key):
    return generate(key)


def switch(new_generator=None, new_para_name_checker=None):
    global _counters
    old = _counters
    _counters = collections.defaultdict(itertools.count) if new_generator is None else new_generator
    return old


@contextlib.contextmanager
def guard(new_generator=None):
    if isinstance(new_generator, str):
        _prefix.append(new_generator)
        old = None
    else:
        old = switch(new_generator)
    try:
        yield
    finally:
        if old is None:
            _prefix.pop()
        else:
            switch(old)
