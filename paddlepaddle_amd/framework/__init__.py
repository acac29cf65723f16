from . import dtype, place, flags, grad_mode, random  # noqa: F401
from .tensor import Tensor, Parameter, EagerParamBase, to_tensor, is_tensor  # noqa: F401
from .place import (CPUPlace, CUDAPlace, CUDAPinnedPlace, set_device, get_device,  # noqa: F401
                    is_compiled_with_cuda, is_compiled_with_rocm)
from .grad_mode import no_grad, enable_grad, set_grad_enabled, is_grad_enabled  # noqa: F401
from .random import seed, get_rng_state, set_rng_state, get_cuda_rng_state, set_cuda_rng_state  # noqa: F401
from .flags import set_flags, get_flags  # noqa: F401


def in_dynamic_mode():
    from ..static import _static_mode
    return not _static_mode.enabled


in_dygraph_mode = in_dynamic_mode
