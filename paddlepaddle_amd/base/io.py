"""paddle.base.io: the legacy io namespace — reader decorators plus the static-graph save / load API
(reference python/paddle/base/io.py re-exports both)."""
from ..reader import (cache, map_readers, shuffle, chain, compose, buffered, firstn,  # noqa: F401
                      xmap_readers, multiprocess_reader, ComposeNotAligned)
from ..static.io import (save_inference_model, load_inference_model, save_vars, load_vars,  # noqa: F401
                         save_persistables, load_persistables, get_program_persistable_vars,
                         get_program_parameter, is_persistable, is_parameter)
