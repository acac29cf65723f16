"""Loggers that do not touch logging.basicConfig. Reference: python/paddle/base/log_helper.py:20 get_logger,
python/paddle/static/log_helper.py."""
from __future__ import annotations

import logging


def get_logger(name, level, fmt=None):
    logger = logging.getLogger(name)
    logger.setLevel(level)
    handler = logging.StreamHandler()
    if fmt:
        handler.setFormatter(logging.Formatter(fmt=fmt, datefmt="%a %b %d %H:%M:%S"))
    logger.addHandler(handler)
    # keep records out of the root logger so a user's basicConfig does not print them twice
    logger.propagate = False
    return logger
