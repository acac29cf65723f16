"""paddle.jit (in progress)."""
