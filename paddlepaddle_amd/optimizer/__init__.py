"""paddle.optimizer. Reference: python/paddle/optimizer/__init__.py."""
from . import lr  # noqa: F401
from .optimizer import Optimizer, L1Decay, L2Decay  # noqa: F401
from .adam import Adam, AdamW  # noqa: F401
from .others import (SGD, Momentum, Adamax, Adagrad, Adadelta, RMSProp, Lamb, NAdam, RAdam, ASGD,  # noqa: F401
                     Rprop, LBFGS)
