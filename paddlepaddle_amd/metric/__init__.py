"""paddle.metric."""
