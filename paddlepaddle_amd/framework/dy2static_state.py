"""Depth of dy2static program recordings in flight (read on every Layer call, so it lives in a leaf module
without imports; jit/dy2static/program_translator.py owns the counter's meaning)."""
ACTIVE = [0]
