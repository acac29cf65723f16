"""Trial history (reference auto_tuner/recorder.py): every run's config + metric, best-so-far, CSV store."""
from __future__ import annotations

import csv
import os


class HistoryRecorder:
    def __init__(self, tuner_cfg):
        self.tuner_cfg = tuner_cfg
        self.history = []
        m = tuner_cfg.get("metric_cfg", {})
        self.metric = m.get("name", "metric")
        self.maximize = str(m.get("OptimizationDirection", "Maximize")).lower().startswith("max")

    def add_cfg(self, **cfg):
        self.history.append(dict(cfg))

    def sort_metric(self):
        ok = [h for h in self.history if h.get(self.metric) is not None and not h.get("error")]
        ok.sort(key=lambda h: h[self.metric], reverse=self.maximize)
        return ok

    def get_best(self):
        ok = self.sort_metric()
        return (ok[0], False) if ok else (None, True)

    def store_history(self, path="./history.csv"):
        if not self.history:
            return
        keys = []
        for h in self.history:
            for k in h:
                if k not in keys:
                    keys.append(k)
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=keys)
            w.writeheader()
            for h in self.history:
                w.writerow(h)

    def load_history(self, path="./history.csv"):
        if not os.path.exists(path):
            return [], True
        with open(path) as f:
            rows = list(csv.DictReader(f))
        for r in rows:
            for k, v in list(r.items()):
                if v in ("True", "False"):
                    r[k] = v == "True"
                elif v == "":
                    r[k] = None
                else:
                    try:
                        r[k] = int(v)
                    except ValueError:
                        try:
                            r[k] = float(v)
                        except ValueError:
                            pass
        return rows, False

    def clean_history(self):
        self.history = []
