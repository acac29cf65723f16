"""paddle.distributed.auto_tuner: search the hybrid-parallel configuration (dp / mp / pp / vpp / sharding /
micro-batch / recompute) of a training job by launching short trials and keeping the best measured one.

Reference: python/paddle/distributed/auto_tuner/ (tuner.py AutoTuner, search.py GridSearch /
CustomizeSearch, prune.py pruning rules, memory_cost_model.py, recorder.py HistoryRecorder, utils.py
default_candidates / search_all). Driven from the launcher:
``python -m paddlepaddle_amd.distributed.launch --nproc_per_node 8 --auto_tuner_json tuner.json train.py ...``.

MI355X sizing: the memory pruning rule prices a decoder LM per GPU against ``max_mem_usage`` (default 288 GB
HBM3E minus 10 %), and tensor parallelism is capped at one node's 8 xGMI-connected GPUs."""
from .tuner import AutoTuner  # noqa: F401
from .recorder import HistoryRecorder  # noqa: F401
from .search import GridSearch, CustomizeSearch  # noqa: F401
from .utils import default_candidates, search_all, gen_new_args, parse_metric  # noqa: F401
from .memory_cost_model import estimate_memory_gb  # noqa: F401
from . import prune  # noqa: F401
