"""paddle.audio (in progress)."""
