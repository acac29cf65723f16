"""paddle.inference (in progress)."""
