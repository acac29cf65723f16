"""paddle.io.dataloader. Reference: python/paddle/io/dataloader/__init__.py (the dataset / sampler / collate
classes the paddle.io namespace re-exports)."""
from .. import (BatchSampler, ChainDataset, ComposeDataset, ConcatDataset, DataLoader, Dataset,  # noqa: F401
                DistributedBatchSampler, IterableDataset, RandomSampler, Sampler, SequenceSampler, Subset,
                SubsetRandomSampler, TensorDataset, WeightedRandomSampler, default_collate_fn, default_convert_fn,
                get_worker_info, random_split)

__all__ = []
