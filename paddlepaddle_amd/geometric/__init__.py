"""paddle.geometric (in progress)."""
