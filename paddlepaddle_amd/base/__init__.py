"""paddle.base (formerly paddle.fluid): the legacy framework namespace that older code imports
(``paddle.base.core``, ``paddle.base.framework``, ``paddle.base.dygraph``). Reference:
python/paddle/base/__init__.py. Everything here re-exports the corresponding modern API."""
from __future__ import annotations

from .. import static as _static
from ..static import (Program, program_guard, Executor, global_scope, scope_guard, default_main_program,  # noqa
                      default_startup_program, CompiledProgram, BuildStrategy, ExecutionStrategy)
from ..framework.place import CPUPlace, CUDAPlace, CUDAPinnedPlace  # noqa: F401
from ..framework import in_dynamic_mode as in_dygraph_mode  # noqa: F401
from ..framework.tensor import Tensor as Variable  # noqa: F401
from ..framework.flags import set_flags, get_flags  # noqa: F401,E402
from . import core, framework, dygraph, io, layers  # noqa: F401,E402
from .data_feeder import DataFeeder  # noqa: F401,E402


def enable_dygraph(place=None):
    _static.disable_static(place)


def disable_dygraph():
    _static.enable_static()
