"""paddle.static — Program / Executor static graph (see static/program.py for the design)."""
from .executor import (_static_mode, enable_static, disable_static, default_main_program,  # noqa: F401
                       default_startup_program, program_guard, data, InputSpec, append_backward, gradients,
                       Executor, global_scope, scope_guard, Scope, BuildStrategy, ExecutionStrategy,
                       CompiledProgram, cpu_places, cuda_places, device_guard, name_scope, Print, create_global_var,
                       create_parameter)
from .program import Program, OpNode  # noqa: F401
from .io import (save_inference_model, load_inference_model, save, load, load_program_state,  # noqa: F401
                 set_program_state, serialize_program, serialize_persistables, deserialize_program,
                 save_to_file, load_from_file, normalize_program, save_persistables, load_persistables)
from . import nn  # noqa: F401
from .extras import *  # noqa: F401,F403
from .io import (deserialize_persistables, save_vars, load_vars, get_program_persistable_vars,  # noqa: F401,E402
                 get_program_parameter, is_persistable, is_parameter)
from . import io, log_helper  # noqa: F401,E402
from ..framework.tensor import Tensor as Variable  # noqa: F401
from ..framework.place import CPUPlace, CUDAPlace  # noqa: F401,E402

ParallelExecutor = Executor
