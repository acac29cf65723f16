"""Search algorithms (reference auto_tuner/search.py)."""
from __future__ import annotations

from . import prune as P
from .utils import search_all


class SearchAlgo:
    def __init__(self, tuner_cfg):
        self.tuner_cfg = tuner_cfg
        self.pruned_cfgs = []

    def search_once(self, history_cfgs):
        raise NotImplementedError


class GridSearch(SearchAlgo):
    """Walk the candidate grid; ``schedule_mode="performance"`` orders it by the cost model first
    (fewest pipeline stages / least tensor parallelism / largest micro-batch that fits), "memory" (default)
    starts from the configurations with the most headroom."""

    def __init__(self, tuner_cfg):
        super().__init__(tuner_cfg)
        from .memory_cost_model import estimate_memory_gb
        tasks = search_all(tuner_cfg)
        model = tuner_cfg.get("model_cfg", {})
        if tuner_cfg.get("schedule_mode", "memory") == "performance":
            tasks.sort(key=lambda c: (c["pp_degree"], c["mp_degree"], c["use_recompute"], -c["micro_batch_size"],
                                      c["sharding_stage"]))
        elif "hidden_size" in model and "num_layers" in model:
            tasks.sort(key=lambda c: estimate_memory_gb(c, model))
        self.all_tasks = tasks
        self.idx = 0

    def search_once(self, history_cfgs):
        while self.idx < len(self.all_tasks):
            cfg = dict(self.all_tasks[self.idx])
            self.idx += 1
            if P.prune(self.tuner_cfg, cfg, history_cfgs):
                self.pruned_cfgs.append(cfg)
                continue
            return cfg
        return None


class CustomizeSearch(SearchAlgo):
    """Run exactly the configurations listed in ``tuner_cfg["configs"]`` (in order)."""

    def __init__(self, tuner_cfg):
        super().__init__(tuner_cfg)
        self.configs = list(tuner_cfg.get("configs", []))
        self.idx = 0

    def search_once(self, history_cfgs):
        if self.idx >= len(self.configs):
            return None
        cfg = dict(self.configs[self.idx])
        self.idx += 1
        return cfg
