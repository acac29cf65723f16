"""Reference: python/paddle/distributed/utils/stream_utils.py."""
from enum import Enum


class ExecutionStreamType(Enum):
    DefaultStream = "DefaultStream"
    CalcStream = "CalcStream"
    CommStream = "CommStream"
