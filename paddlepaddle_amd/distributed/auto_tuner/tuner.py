"""AutoTuner (reference auto_tuner/tuner.py): hands out one trial configuration at a time."""
from __future__ import annotations

from .utils import default_candidates


class AutoTuner:
    def __init__(self, tuner_cfg):
        self.cur_task_id = 1
        self.task_limit = int(tuner_cfg.get("task_limit", 100))
        name = tuner_cfg.get("search_algo", {"name": "grid"})["name"]
        if name == "grid":
            from .search import GridSearch
            tuner_cfg["candidates"] = default_candidates(tuner_cfg)
            self.algo = GridSearch(tuner_cfg)
        elif name == "customize":
            from .search import CustomizeSearch
            self.algo = CustomizeSearch(tuner_cfg)
        else:
            raise NotImplementedError(f"auto tuner search algorithm {name!r} (grid / customize)")
        self.history_cfgs = []
        self.tuner_cfg = tuner_cfg

    def search_once(self):
        if self.cur_task_id > self.task_limit:
            return None
        cfg = self.algo.search_once(self.history_cfgs)
        self.cur_task_id += 1
        return cfg

    def add_cfg(self, cfg):
        self.history_cfgs.append(cfg)

    def resume_from_history(self, rows):
        self.history_cfgs.extend(rows)

    resume_form_history = resume_from_history  # the reference's spelling
