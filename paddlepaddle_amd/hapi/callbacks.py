"""hapi callbacks. Reference: python/paddle/hapi/callbacks.py (Callback, CallbackList, ProgBarLogger,
ModelCheckpoint, LRScheduler, EarlyStopping, ReduceLROnPlateau, VisualDL, WandbCallback)."""
from __future__ import annotations

import copy
import numbers
import os
import sys
import time
import warnings

import numpy as np


class Callback:
    def __init__(self):
        self.model = None
        self.params = {}

    def set_params(self, params):
        self.params = params

    def set_model(self, model):
        self.model = model

    def on_train_begin(self, logs=None): ...
    def on_train_end(self, logs=None): ...
    def on_eval_begin(self, logs=None): ...
    def on_eval_end(self, logs=None): ...
    def on_predict_begin(self, logs=None): ...
    def on_predict_end(self, logs=None): ...
    def on_epoch_begin(self, epoch, logs=None): ...
    def on_epoch_end(self, epoch, logs=None): ...
    def on_train_batch_begin(self, step, logs=None): ...
    def on_train_batch_end(self, step, logs=None): ...
    def on_eval_batch_begin(self, step, logs=None): ...
    def on_eval_batch_end(self, step, logs=None): ...
    def on_predict_batch_begin(self, step, logs=None): ...
    def on_predict_batch_end(self, step, logs=None): ...


class CallbackList:
    def __init__(self, callbacks=None):
        self.callbacks = list(callbacks or [])
        self.params = {}
        self.model = None

    def append(self, cb):
        self.callbacks.append(cb)

    def set_params(self, params):
        self.params = params
        for c in self.callbacks:
            c.set_params(params)

    def set_model(self, model):
        self.model = model
        for c in self.callbacks:
            c.set_model(model)

    def _call(self, name, *args):
        for c in self.callbacks:
            getattr(c, name)(*args)

    def __getattr__(self, name):
        if name.startswith("on_"):
            return lambda *a: self._call(name, *a)
        raise AttributeError(name)


def config_callbacks(callbacks=None, model=None, batch_size=None, epochs=None, steps=None, log_freq=2, verbose=2,
                     save_freq=1, save_dir=None, metrics=None, mode="train"):
    cbks = list(callbacks or [])
    if not any(isinstance(k, ProgBarLogger) for k in cbks) and verbose:
        cbks = [ProgBarLogger(log_freq, verbose=verbose)] + cbks
    if not any(isinstance(k, ModelCheckpoint) for k in cbks):
        cbks = cbks + [ModelCheckpoint(save_freq, save_dir)]
    if not any(isinstance(k, LRScheduler) for k in cbks):
        cbks = cbks + [LRScheduler()]
    cl = CallbackList(cbks)
    cl.set_model(model)
    metrics = metrics or ([] if mode != "train" else ["loss"])
    cl.set_params({"batch_size": batch_size, "epochs": epochs, "steps": steps, "verbose": verbose,
                   "metrics": metrics})
    return cl


class ProgBarLogger(Callback):
    def __init__(self, log_freq=1, verbose=2):
        super().__init__()
        self.log_freq = log_freq
        self.verbose = verbose
        self.epochs = None

    def _fmt(self, logs):
        parts = []
        for k, v in (logs or {}).items():
            if k in ("batch_size", "step", "samples"):
                continue
            if isinstance(v, (list, tuple)):
                v = v[0] if len(v) == 1 else v
            if isinstance(v, numbers.Number):
                parts.append(f"{k}: {v:.4f}")
            elif isinstance(v, (list, tuple)):
                parts.append(f"{k}: " + ", ".join(f"{x:.4f}" for x in v if isinstance(x, numbers.Number)))
        return " - ".join(parts)

    def on_train_begin(self, logs=None):
        self.epochs = self.params.get("epochs")
        self._t0 = time.time()

    def on_epoch_begin(self, epoch, logs=None):
        self.epoch = epoch
        self.steps = self.params.get("steps")
        if self.verbose and self.epochs:
            print(f"Epoch {epoch + 1}/{self.epochs}")
        self._tick = time.time()

    def on_train_batch_end(self, step, logs=None):
        if self.verbose and step % self.log_freq == 0:
            tot = f"/{self.steps}" if self.steps else ""
            print(f"step {step + 1}{tot} - {self._fmt(logs)}")

    def on_epoch_end(self, epoch, logs=None):
        if self.verbose == 1:
            print(f"epoch {epoch + 1} - {self._fmt(logs)} - {time.time() - self._tick:.2f}s")

    def on_eval_begin(self, logs=None):
        if self.verbose:
            print("Eval begin...")

    def on_eval_end(self, logs=None):
        if self.verbose:
            print(f"Eval samples: {logs.get('samples', '')} - {self._fmt(logs)}")


class ModelCheckpoint(Callback):
    def __init__(self, save_freq=1, save_dir=None):
        super().__init__()
        self.save_freq = save_freq
        self.save_dir = save_dir

    def on_epoch_end(self, epoch, logs=None):
        if self.save_dir and (epoch + 1) % self.save_freq == 0:
            self.model.save(os.path.join(self.save_dir, str(epoch)))

    def on_train_end(self, logs=None):
        if self.save_dir:
            self.model.save(os.path.join(self.save_dir, "final"))


class LRScheduler(Callback):
    def __init__(self, by_step=True, by_epoch=False):
        super().__init__()
        if by_step and by_epoch:
            raise ValueError("by_step and by_epoch are mutually exclusive")
        self.by_step = by_step
        self.by_epoch = by_epoch

    def _sched(self):
        opt = getattr(self.model, "_optimizer", None)
        from ..optimizer.lr import LRScheduler as _S
        lr = getattr(opt, "_learning_rate", None)
        return lr if isinstance(lr, _S) else None

    def on_epoch_end(self, epoch, logs=None):
        s = self._sched()
        if self.by_epoch and s is not None:
            s.step()

    def on_train_batch_end(self, step, logs=None):
        s = self._sched()
        if self.by_step and s is not None:
            s.step()


class EarlyStopping(Callback):
    def __init__(self, monitor="loss", mode="auto", patience=0, verbose=1, min_delta=0, baseline=None,
                 save_best_model=True):
        super().__init__()
        self.monitor = monitor
        self.patience = patience
        self.verbose = verbose
        self.baseline = baseline
        self.min_delta = abs(min_delta)
        self.save_best_model = save_best_model
        if mode not in ("auto", "min", "max"):
            mode = "auto"
        if mode == "min" or (mode == "auto" and "acc" not in monitor):
            self.monitor_op, self.min_delta = np.less, -self.min_delta
        else:
            self.monitor_op = np.greater
        self.wait_epoch = 0
        self.best_weights = None
        self.stopped_epoch = 0

    def on_train_begin(self, logs=None):
        self.wait_epoch = 0
        self.best_value = self.baseline if self.baseline is not None else \
            (np.inf if self.monitor_op == np.less else -np.inf)
        self.model.stop_training = False

    def on_eval_end(self, logs=None):
        if logs is None or self.monitor not in logs:
            warnings.warn(f"EarlyStopping: monitor {self.monitor} not in eval logs")
            return
        cur = logs[self.monitor]
        cur = cur[0] if isinstance(cur, (list, tuple)) else cur
        if self.monitor_op(cur - self.min_delta, self.best_value):
            self.best_value = cur
            self.wait_epoch = 0
            if self.save_best_model and getattr(self.model, "_save_dir", None):
                self.model.save(os.path.join(self.model._save_dir, "best_model"))
        else:
            self.wait_epoch += 1
        if self.wait_epoch > self.patience:
            self.model.stop_training = True
            if self.verbose:
                print(f"Epoch stopped early: best {self.monitor} = {self.best_value:.5f}")


class ReduceLROnPlateau(Callback):
    def __init__(self, monitor="loss", factor=0.1, patience=10, verbose=1, mode="auto", min_delta=1e-4, cooldown=0,
                 min_lr=0):
        super().__init__()
        self.monitor, self.factor, self.patience = monitor, factor, patience
        self.verbose, self.min_delta, self.cooldown, self.min_lr = verbose, min_delta, cooldown, min_lr
        self.mode = "max" if (mode == "max" or (mode == "auto" and "acc" in monitor)) else "min"
        self.best = np.inf if self.mode == "min" else -np.inf
        self.wait = 0
        self.cooldown_counter = 0

    def on_eval_end(self, logs=None):
        if not logs or self.monitor not in logs:
            return
        cur = logs[self.monitor]
        cur = cur[0] if isinstance(cur, (list, tuple)) else cur
        better = cur < self.best - self.min_delta if self.mode == "min" else cur > self.best + self.min_delta
        if self.cooldown_counter > 0:
            self.cooldown_counter -= 1
            self.wait = 0
        if better:
            self.best = cur
            self.wait = 0
        elif self.cooldown_counter <= 0:
            self.wait += 1
            if self.wait >= self.patience:
                opt = self.model._optimizer
                old = opt.get_lr()
                new = max(old * self.factor, self.min_lr)
                if old > new:
                    opt.set_lr(new)
                    if self.verbose:
                        print(f"ReduceLROnPlateau: lr {old:.3e} -> {new:.3e}")
                self.cooldown_counter = self.cooldown
                self.wait = 0


class VisualDL(Callback):
    """Scalar logger writing CSV (VisualDL itself is not available in this environment)."""

    def __init__(self, log_dir):
        super().__init__()
        self.log_dir = log_dir
        self._step = 0

    def on_train_batch_end(self, step, logs=None):
        os.makedirs(self.log_dir, exist_ok=True)
        with open(os.path.join(self.log_dir, "train.csv"), "a") as f:
            for k, v in (logs or {}).items():
                if isinstance(v, (list, tuple)):
                    v = v[0]
                if isinstance(v, numbers.Number):
                    f.write(f"{self._step},{k},{v}\n")
        self._step += 1


class WandbCallback(Callback):
    def __init__(self, *a, **k):
        raise NotImplementedError("wandb is not available in this environment")
