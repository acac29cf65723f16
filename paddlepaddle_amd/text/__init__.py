"""paddle.text (in progress)."""
