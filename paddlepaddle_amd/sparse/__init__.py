"""paddle.sparse (in progress)."""
