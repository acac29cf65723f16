"""Reference: python/paddle/distributed/utils/log_utils.py:18."""
import logging


def get_logger(log_level, name="root"):
    logger = logging.getLogger(name)
    logger.setLevel(log_level)
    if not logger.handlers:
        h = logging.StreamHandler()
        h.setFormatter(logging.Formatter("%(levelname)s %(asctime)s %(filename)s:%(lineno)d] %(message)s"))
        logger.addHandler(h)
    return logger
