"""paddle.base.dygraph: guard / to_variable / no_grad of the legacy dygraph API."""
import contextlib

from ..framework.grad_mode import no_grad  # noqa: F401
from ..framework.tensor import to_tensor


@contextlib.contextmanager
def guard(place=None):
    from ..static import disable_static
    disable_static()
    yield


def to_variable(value, name=None, zero_copy=None, dtype=None):
    return to_tensor(value, dtype=dtype)


def enabled():
    from ..framework import in_dynamic_mode
    return in_dynamic_mode()
