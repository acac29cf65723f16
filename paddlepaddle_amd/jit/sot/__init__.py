"""paddle.jit.sot — bytecode-level dynamic-to-static translation (reference python/paddle/jit/sot/).
See opcode_executor.py (the CPython 3.10 bytecode interpreter), guards.py and translate.py."""
from .opcode_executor import Unsupported, graph_break  # noqa: F401
from .translate import SOTFunction, symbolic_translate  # noqa: F401

__all__ = ["symbolic_translate"]
