"""paddle.vision. Reference: python/paddle/vision/."""
from . import models  # noqa: F401
from .models import *  # noqa: F401,F403
