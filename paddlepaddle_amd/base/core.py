"""paddle.base.core: build / device queries of the native core."""
from ..framework.place import CPUPlace, CUDAPlace, CUDAPinnedPlace, is_compiled_with_cuda, is_compiled_with_rocm  # noqa


def is_compiled_with_xpu():
    return False


def is_compiled_with_custom_device(name=""):
    return False


def is_compiled_with_distribute():
    return True


def get_cuda_device_count():
    import torch
    return torch.cuda.device_count() if torch.cuda.is_available() else 0


def globals():
    from ..framework.flags import get_flags
    return get_flags([])
