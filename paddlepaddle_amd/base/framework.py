"""paddle.base.framework: Program / dygraph-mode helpers."""
from ..static import Program, default_main_program, default_startup_program, program_guard  # noqa: F401
from ..framework import in_dynamic_mode  # noqa: F401
from ..framework.tensor import Tensor as Variable, Parameter  # noqa: F401

in_dygraph_mode = in_dynamic_mode


def _current_expected_place():
    from ..framework.place import get_device
    return get_device()
