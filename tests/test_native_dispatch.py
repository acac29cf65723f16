"""The native launch module (csrc/dispatch, generated from ops/_sigs.py): argument conversion and parity
with the ctypes path on launchers that do not touch the GPU."""
import ctypes
import os

import numpy as np
import pytest
import torch

from paddlepaddle_amd.ops import _loader as L
from paddlepaddle_amd.ops import _sigs

D = pytest.importorskip("paddlepaddle_amd._C_dispatch")


def test_every_exported_launcher_has_an_entry_point():
    lib = L.lib()
    exported = [n for n in _sigs.SIGS if hasattr(lib, n)]
    assert exported and all(hasattr(D, n) for n in exported)


def test_host_only_launchers_match_ctypes():
    lib = L.lib()
    for R, C in ((1024, 64), (802816, 256), (3136, 2048)):
        assert D.pa_bn_chunks(R, C) == lib.pa_bn_chunks(R, C)
        assert D.pa_bn_chunks(np.int64(R), ctypes.c_int(C)) == lib.pa_bn_chunks(R, C)  # numpy / ctypes scalars
    old = D.pa_bn_set_target_wgs(777)
    assert lib.pa_bn_set_target_wgs(old) == 777
    assert D.pa_version() == lib.pa_version()


def test_argument_errors_are_python_exceptions():
    with pytest.raises(TypeError, match="takes 9 arguments"):
        D.pa_rms_norm_fwd(1, 2)
    with pytest.raises(TypeError, match="pointer"):
        D.pa_rms_norm_fwd("x", None, None, None, 1, 1, 1.0, 0, L.CURRENT_STREAM)
    with pytest.raises(TypeError):
        D.pa_bn_chunks(1.5j, 3)


def test_loader_hands_objects_through_on_the_native_path():
    if not L.native_launch():
        pytest.skip("PADDLE_AMD_CTYPES_LAUNCH=1")
    t = torch.zeros(3)
    assert L.ptr(t) is t and L.ptr(None) is None
    assert L.stream_ptr() is L.CURRENT_STREAM
    assert os.environ.get("PADDLE_AMD_CTYPES_LAUNCH", "0") != "1"
