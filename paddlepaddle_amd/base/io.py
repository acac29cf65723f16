"""paddle.base.io: the legacy io namespace — reader decorators plus the static-graph save / load API
(reference python/paddle/base/io.py re-exports both)."""
from ..reader import (cache, map_readers, shuffle, chain, compose, buffered, firstn,  # noqa: F401
                      xmap_readers, multiprocess_reader, ComposeNotAligned)
from ..static.io import (save_inference_model, load_inference_model, save_vars, load_vars,  # noqa: F401
                         save_persistables, load_persistables, get_program_persistable_vars,
                         get_program_parameter, is_persistable, is_parameter)

import os as _os

from ..static import io as _sio


def _legacy_prefix(dirname, model_filename):
    return _os.path.join(dirname, model_filename or "__model__")


def save_inference_model(path_prefix=None, feed_vars=None, fetch_vars=None, executor=None, *args, dirname=None,
                         feeded_var_names=None, target_vars=None, main_program=None, model_filename=None,
                         params_filename=None, **kwargs):
    """Modern signature (path_prefix, feed_vars, fetch_vars, executor) or the fluid one (dirname,
    feeded_var_names, target_vars, executor, main_program, model_filename): the program is written under
    ``dirname/<model_filename or __model__>``."""
    if dirname is not None or feeded_var_names is not None:
        _os.makedirs(dirname, exist_ok=True)
        return _sio.save_inference_model(_legacy_prefix(dirname, model_filename), list(feeded_var_names),
                                         target_vars, executor, program=main_program, **kwargs)
    return _sio.save_inference_model(path_prefix, feed_vars, fetch_vars, executor, *args, **kwargs)


def load_inference_model(path_prefix=None, executor=None, *, dirname=None, model_filename=None,
                         params_filename=None, pserver_endpoints=None, **kwargs):
    if dirname is not None:
        path_prefix = _legacy_prefix(dirname, model_filename)
    return _sio.load_inference_model(path_prefix, executor, **kwargs)
