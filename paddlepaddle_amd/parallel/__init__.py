"""MI355X-native parallelism engines (DP buckets, ZeRO sharding, TP layers, 1F1B pipeline)."""
from .data_parallel import DataParallel  # noqa: F401
