from .....parallel.tensor_parallel import _c_identity, _mp_allreduce, _c_split, _c_concat  # noqa: F401
