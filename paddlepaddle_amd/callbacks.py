"""paddle.callbacks."""
