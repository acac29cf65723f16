"""paddle.incubate (in progress)."""
