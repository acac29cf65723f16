"""Reference: python/paddle/distribution/exponential_family.py."""
from .distribution import ExponentialFamily  # noqa: F401
