"""paddle.callbacks (re-export of hapi.callbacks)."""
from .hapi.callbacks import (Callback, ProgBarLogger, ModelCheckpoint, LRScheduler, EarlyStopping,  # noqa: F401
                             ReduceLROnPlateau, VisualDL, WandbCallback)
