"""paddle.distribution (in progress)."""
