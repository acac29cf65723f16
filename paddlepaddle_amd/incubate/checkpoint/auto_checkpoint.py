"""Auto checkpoint: ``train_epoch_range`` resumes an interrupted job at the epoch it stopped in.

Reference: python/paddle/base/incubate/checkpoint/auto_checkpoint.py:615 (train_epoch_range), :70
(AutoCheckpointChecker: PADDLE_RUNNING_ENV=PADDLE_EDL_AUTO_CHECKPOINT, PADDLE_JOB_ID,
PADDLE_EDL_HDFS_CHECKPOINT_PATH, PADDLE_TRAINER_ID, PADDLE_EDL_SAVE_CHECKPOINT_INTER). The checkpoint path is a
file-system directory here (HDFS clients are not part of this framework); what is saved is the parameters of the
default static main program plus every object registered with ``register(name, obj)`` (anything with
state_dict / set_state_dict: layers, optimizers, LR schedulers, data loaders)."""
from __future__ import annotations

import json
import os
import time

_REGISTERED: dict = {}
g_train_epoch_range = None


class AutoCheckpointChecker:
    def __init__(self):
        self.run_env = os.getenv("PADDLE_RUNNING_ENV")
        self.job_id = os.getenv("PADDLE_JOB_ID", "job")
        self.checkpoint_path = os.getenv("PADDLE_EDL_HDFS_CHECKPOINT_PATH")
        self.trainer_id = int(os.getenv("PADDLE_TRAINER_ID", "0"))
        self.save_checkpoint_inter = int(os.getenv("PADDLE_EDL_SAVE_CHECKPOINT_INTER", "900"))

    def valid(self):
        return self.run_env == "PADDLE_EDL_AUTO_CHECKPOINT" and bool(self.checkpoint_path)

    def range_dir(self, name):
        return os.path.join(self.checkpoint_path, self.job_id, name)


def register(name, obj):
    """Save / restore ``obj`` (state_dict / set_state_dict) with the epoch range checkpoints."""
    _REGISTERED[name] = obj


def _static_params():
    try:
        from ...static import default_main_program
        prog = default_main_program()
        return prog.state_dict() if hasattr(prog, "state_dict") else {}
    except Exception:  # noqa: BLE001 - no static program in this process
        return {}


class TrainEpochRange:
    def __init__(self, max_epoch_num, name, checkpoint_inter=None, checker=None):
        self._max = max_epoch_num
        self._checker = checker or AutoCheckpointChecker()
        self._dir = self._checker.range_dir(name)
        self._inter = checkpoint_inter if checkpoint_inter is not None else self._checker.save_checkpoint_inter
        self._epoch_no = -1
        self._last_save = time.time()
        self.restored_from = None
        self._restore()

    def _status_file(self):
        return os.path.join(self._dir, f"status.{self._checker.trainer_id}.json")

    def _restore(self):
        from ... import framework
        f = self._status_file()
        if not os.path.exists(f):
            return
        with open(f) as fh:
            st = json.load(fh)
        self._epoch_no = int(st["epoch_no"])
        state = framework.io.load(os.path.join(self._dir, f"state.{self._checker.trainer_id}.pdparams"))
        for name, obj in _REGISTERED.items():
            if name in state:
                obj.set_state_dict(state[name])
        static = state.get("__static__")
        if static:
            from ...static import default_main_program
            default_main_program().set_state_dict(static)
        self.restored_from = "checkpoint"

    def save_checkpoint(self):
        from ... import framework
        os.makedirs(self._dir, exist_ok=True)
        state = {name: obj.state_dict() for name, obj in _REGISTERED.items()}
        static = _static_params()
        if static:
            state["__static__"] = static
        tmp = os.path.join(self._dir, f"state.{self._checker.trainer_id}.pdparams.tmp")
        framework.io.save(state, tmp)
        os.replace(tmp, os.path.join(self._dir, f"state.{self._checker.trainer_id}.pdparams"))
        with open(self._status_file() + ".tmp", "w") as fh:
            json.dump({"epoch_no": self._epoch_no, "max_epoch_num": self._max, "time": time.time()}, fh)
        os.replace(self._status_file() + ".tmp", self._status_file())
        self._last_save = time.time()

    def get(self):
        return self._epoch_no

    def next(self):
        start = self._epoch_no + 1
        for i in range(start, self._max if self._max >= 0 else 1 << 62):
            self._epoch_no = i
            yield i
            # an epoch finished: persist it (the interval bounds how often a long epoch list writes)
            if time.time() - self._last_save >= self._inter or i == self._max - 1 or self._inter <= 0:
                self.save_checkpoint()


def train_epoch_range(max_epoch_num, save_checkpoint_inter=None):
    global g_train_epoch_range
    checker = AutoCheckpointChecker()
    if not checker.valid():
        yield from range(0, max_epoch_num if max_epoch_num >= 0 else 1 << 62)
        return
    try:
        g_train_epoch_range = TrainEpochRange(max_epoch_num, "range_0", save_checkpoint_inter, checker)
        yield from g_train_epoch_range.next()
    finally:
        g_train_epoch_range = None
