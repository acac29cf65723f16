from .....parallel.tensor_parallel import get_rng_state_tracker, RNGStatesTracker, model_parallel_random_seed  # noqa: F401
