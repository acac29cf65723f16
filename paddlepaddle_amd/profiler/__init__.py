"""paddle.profiler (in progress)."""
