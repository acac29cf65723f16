"""paddle.quantization (in progress)."""
