"""Learning-rate schedulers. Reference: python/paddle/optimizer/lr.py."""
from __future__ import annotations

import math
import warnings


class LRScheduler:
    def __init__(self, learning_rate=0.1, last_epoch=-1, verbose=False):
        self.base_lr = float(learning_rate)
        self.last_lr = float(learning_rate)
        self.last_epoch = last_epoch
        self.verbose = verbose
        self._var_name = None
        self.step()

    def __call__(self):
        return self.last_lr

    def _register_device_lr(self, t, ratio=1.0):
        """A device scalar (hyper[0] of a hipGraph-captured optimizer step) that follows this schedule: every
        step() writes last_lr * ratio into it, outside the graph, before the next replay reads it."""
        import weakref
        self.__dict__.setdefault("_device_lrs", []).append((weakref.ref(t), float(ratio)))

    @property
    def last_lr(self):
        return self.__dict__.get("_last_lr")

    @last_lr.setter
    def last_lr(self, v):
        # every schedule (including subclasses with their own step()) sets last_lr: push it to the device
        # scalars of captured optimizer steps
        self.__dict__["_last_lr"] = v
        sinks = self.__dict__.get("_device_lrs")
        if sinks:
            live = []
            for ref, ratio in sinks:
                t = ref()
                if t is not None:
                    t[0].fill_(float(v) * ratio)
                    live.append((ref, ratio))
            self._device_lrs = live

    def step(self, epoch=None):
        if epoch is None:
            self.last_epoch += 1
            self.last_lr = self.get_lr()
        else:
            self.last_epoch = epoch
            if hasattr(self, "_get_closed_form_lr"):
                self.last_lr = self._get_closed_form_lr()
            else:
                self.last_lr = self.get_lr()
        if self.verbose:
            print(f"Epoch {self.last_epoch}: {self.__class__.__name__} set learning rate to {self.last_lr}.")

    def get_lr(self):
        raise NotImplementedError

    def state_keys(self):
        self.keys = ["last_epoch", "last_lr"]

    def state_dict(self):
        self.state_keys()
        return {k: getattr(self, k) for k in self.keys}

    def set_state_dict(self, state_dict):
        self.state_keys()
        for k in self.keys:
            if k in state_dict:
                setattr(self, k, state_dict[k])

    set_dict = set_state_dict


class NoamDecay(LRScheduler):
    def __init__(self, d_model, warmup_steps, learning_rate=1.0, last_epoch=-1, verbose=False):
        self.d_model, self.warmup_steps = d_model, warmup_steps
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        a = 1 if self.last_epoch == 0 else self.last_epoch ** -0.5
        b = self.warmup_steps ** -1.5 * (1 if self.last_epoch == 0 else self.last_epoch)
        return self.base_lr * (self.d_model ** -0.5) * min(a, b)


class PiecewiseDecay(LRScheduler):
    def __init__(self, boundaries, values, last_epoch=-1, verbose=False):
        self.boundaries, self.values = boundaries, values
        super().__init__(last_epoch=last_epoch, verbose=verbose)

    def get_lr(self):
        for i, b in enumerate(self.boundaries):
            if self.last_epoch < b:
                return self.values[i]
        return self.values[len(self.values) - 1]


class NaturalExpDecay(LRScheduler):
    def __init__(self, learning_rate, gamma, last_epoch=-1, verbose=False):
        self.gamma = gamma
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        return self.base_lr * math.exp(-1 * self.gamma * self.last_epoch)


class InverseTimeDecay(LRScheduler):
    def __init__(self, learning_rate, gamma, last_epoch=-1, verbose=False):
        self.gamma = gamma
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        return self.base_lr / (1 + self.gamma * self.last_epoch)


class PolynomialDecay(LRScheduler):
    def __init__(self, learning_rate, decay_steps, end_lr=0.0001, power=1.0, cycle=False, last_epoch=-1,
                 verbose=False):
        self.decay_steps, self.end_lr, self.power, self.cycle = decay_steps, end_lr, power, cycle
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        t = self.last_epoch
        ds = self.decay_steps
        if self.cycle:
            div = math.ceil(t / float(ds)) if t > 0 else 1
            ds = ds * div
        else:
            t = min(t, ds)
        return (self.base_lr - self.end_lr) * ((1 - float(t) / float(ds)) ** self.power) + self.end_lr


class LinearWarmup(LRScheduler):
    def __init__(self, learning_rate, warmup_steps, start_lr, end_lr, last_epoch=-1, verbose=False):
        self.learning_rate = learning_rate
        self.warmup_steps, self.start_lr, self.end_lr = warmup_steps, start_lr, end_lr
        base = learning_rate if not isinstance(learning_rate, LRScheduler) else learning_rate.base_lr
        super().__init__(base, last_epoch, verbose)

    def state_dict(self):
        d = super().state_dict()
        if isinstance(self.learning_rate, LRScheduler):
            d["LinearWarmup_LR"] = self.learning_rate.state_dict()
        return d

    def set_state_dict(self, state_dict):
        super().set_state_dict(state_dict)
        if isinstance(self.learning_rate, LRScheduler) and "LinearWarmup_LR" in state_dict:
            self.learning_rate.set_state_dict(state_dict["LinearWarmup_LR"])

    def get_lr(self):
        if self.last_epoch < self.warmup_steps:
            return (self.end_lr - self.start_lr) * float(self.last_epoch) / float(self.warmup_steps) + self.start_lr
        if isinstance(self.learning_rate, LRScheduler):
            self.learning_rate.step(self.last_epoch - self.warmup_steps)
            return self.learning_rate()
        return self.learning_rate


class ExponentialDecay(LRScheduler):
    def __init__(self, learning_rate, gamma, last_epoch=-1, verbose=False):
        self.gamma = gamma
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        return self.base_lr * (self.gamma ** self.last_epoch)


class MultiStepDecay(LRScheduler):
    def __init__(self, learning_rate, milestones, gamma=0.1, last_epoch=-1, verbose=False):
        self.milestones, self.gamma = milestones, gamma
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        for i, m in enumerate(self.milestones):
            if self.last_epoch < m:
                return self.base_lr * (self.gamma ** i)
        return self.base_lr * (self.gamma ** len(self.milestones))


class StepDecay(LRScheduler):
    def __init__(self, learning_rate, step_size, gamma=0.1, last_epoch=-1, verbose=False):
        self.step_size, self.gamma = step_size, gamma
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        return self.base_lr * (self.gamma ** (self.last_epoch // self.step_size))


class LambdaDecay(LRScheduler):
    def __init__(self, learning_rate, lr_lambda, last_epoch=-1, verbose=False):
        self.lr_lambda = lr_lambda
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        return self.base_lr * self.lr_lambda(self.last_epoch)


class MultiplicativeDecay(LRScheduler):
    def __init__(self, learning_rate, lr_lambda, last_epoch=-1, verbose=False):
        self.lr_lambda = lr_lambda
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        cur = self.base_lr
        for e in range(1, self.last_epoch + 1):
            cur = cur * self.lr_lambda(e)
        return cur


class ReduceOnPlateau(LRScheduler):
    def __init__(self, learning_rate, mode="min", factor=0.1, patience=10, threshold=1e-4, threshold_mode="rel",
                 cooldown=0, min_lr=0, epsilon=1e-8, verbose=False):
        self.mode, self.factor, self.patience = mode, factor, patience
        self.threshold, self.threshold_mode = threshold, threshold_mode
        self.cooldown, self.min_lr, self.epsilon = cooldown, min_lr, epsilon
        self.cooldown_counter = 0
        self.best = None
        self.num_bad_epochs = 0
        self.last_epoch = 0
        self.base_lr = float(learning_rate)
        self.last_lr = float(learning_rate)
        self.verbose = verbose

    def state_keys(self):
        self.keys = ["cooldown_counter", "best", "num_bad_epochs", "last_epoch", "last_lr"]

    def _is_better(self, cur, best):
        if self.mode == "min" and self.threshold_mode == "rel":
            return cur < best - best * self.threshold
        if self.mode == "min":
            return cur < best - self.threshold
        if self.threshold_mode == "rel":
            return cur > best + best * self.threshold
        return cur > best + self.threshold

    def step(self, metrics=None, epoch=None):
        if metrics is None:
            return
        self.last_epoch = self.last_epoch + 1 if epoch is None else epoch
        m = float(metrics.item() if hasattr(metrics, "item") else metrics)
        if self.cooldown_counter > 0:
            self.cooldown_counter -= 1
        else:
            if self.best is None or self._is_better(m, self.best):
                self.best = m
                self.num_bad_epochs = 0
            else:
                self.num_bad_epochs += 1
            if self.num_bad_epochs > self.patience:
                self.cooldown_counter = self.cooldown
                self.num_bad_epochs = 0
                new = max(self.last_lr * self.factor, self.min_lr)
                if self.last_lr - new > self.epsilon:
                    self.last_lr = new


class CosineAnnealingDecay(LRScheduler):
    def __init__(self, learning_rate, T_max, eta_min=0, last_epoch=-1, verbose=False):
        self.T_max, self.eta_min = T_max, eta_min
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        if self.last_epoch == 0:
            return self.base_lr
        if (self.last_epoch - 1 - self.T_max) % (2 * self.T_max) == 0:
            return self.last_lr + (self.base_lr - self.eta_min) * (1 - math.cos(math.pi / self.T_max)) / 2
        return (1 + math.cos(math.pi * self.last_epoch / self.T_max)) / (
            1 + math.cos(math.pi * (self.last_epoch - 1) / self.T_max)) * (self.last_lr - self.eta_min) + self.eta_min

    def _get_closed_form_lr(self):
        return self.eta_min + (self.base_lr - self.eta_min) * (1 + math.cos(math.pi * self.last_epoch / self.T_max)) / 2


class CosineAnnealingWarmRestarts(LRScheduler):
    def __init__(self, learning_rate, T_0, T_mult=1, eta_min=0, last_epoch=-1, verbose=False):
        self.T_0, self.T_mult, self.eta_min = T_0, T_mult, eta_min
        self.T_i, self.T_cur = T_0, last_epoch
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        return self.eta_min + (self.base_lr - self.eta_min) * (1 + math.cos(math.pi * self.T_cur / self.T_i)) / 2

    def step(self, epoch=None):
        if epoch is None:
            self.last_epoch += 1
            self.T_cur = self.T_cur + 1
            if self.T_cur >= self.T_i:
                self.T_cur -= self.T_i
                self.T_i *= self.T_mult
        else:
            if epoch >= self.T_0:
                if self.T_mult == 1:
                    self.T_cur = epoch % self.T_0
                else:
                    n = int(math.log(epoch / self.T_0 * (self.T_mult - 1) + 1, self.T_mult))
                    self.T_cur = epoch - self.T_0 * (self.T_mult ** n - 1) / (self.T_mult - 1)
                    self.T_i = self.T_0 * self.T_mult ** n
            else:
                self.T_i, self.T_cur = self.T_0, epoch
            self.last_epoch = epoch
        self.last_lr = self.get_lr()


class OneCycleLR(LRScheduler):
    def __init__(self, max_learning_rate, total_steps, divide_factor=25.0, end_learning_rate=0.0001,
                 phase_pct=0.3, anneal_strategy="cos", three_phase=False, last_epoch=-1, verbose=False):
        self.max_lr, self.total_steps = max_learning_rate, total_steps
        self.initial_lr = max_learning_rate / divide_factor
        self.end_lr = end_learning_rate
        self.anneal = anneal_strategy
        if three_phase:
            self.phases = [(float(phase_pct * total_steps) - 1, self.initial_lr, self.max_lr),
                           (float(2 * phase_pct * total_steps) - 2, self.max_lr, self.initial_lr),
                           (total_steps - 1, self.initial_lr, self.end_lr)]
        else:
            self.phases = [(float(phase_pct * total_steps) - 1, self.initial_lr, self.max_lr),
                           (total_steps - 1, self.max_lr, self.end_lr)]
        super().__init__(self.initial_lr, last_epoch, verbose)

    def _interp(self, start, end, pct):
        if self.anneal == "cos":
            return end + (start - end) / 2.0 * (math.cos(math.pi * pct) + 1)
        return (end - start) * pct + start

    def get_lr(self):
        step = self.last_epoch
        start_step = 0
        for i, (end_step, s, e) in enumerate(self.phases):
            if step <= end_step or i == len(self.phases) - 1:
                pct = (step - start_step) / max(end_step - start_step, 1)
                return self._interp(s, e, min(pct, 1.0))
            start_step = end_step
        return self.end_lr


class CyclicLR(LRScheduler):
    def __init__(self, base_learning_rate, max_learning_rate, step_size_up, step_size_down=None, mode="triangular",
                 exp_gamma=1.0, scale_fn=None, scale_mode="cycle", last_epoch=-1, verbose=False):
        self.max_lr = max_learning_rate
        up = float(step_size_up)
        down = float(step_size_down) if step_size_down is not None else up
        self.cycle_size = up + down
        self.step_up_pct = up / self.cycle_size
        self.mode, self.gamma = mode, exp_gamma
        if scale_fn is None:
            if mode == "triangular":
                self.scale_fn, self.scale_mode = (lambda x: 1.0), "cycle"
            elif mode == "triangular2":
                self.scale_fn, self.scale_mode = (lambda x: 1 / (2.0 ** (x - 1))), "cycle"
            else:
                self.scale_fn, self.scale_mode = (lambda x: self.gamma ** x), "iterations"
        else:
            self.scale_fn, self.scale_mode = scale_fn, scale_mode
        super().__init__(base_learning_rate, last_epoch, verbose)

    def get_lr(self):
        it = self.last_epoch
        cycle = 1 + it // self.cycle_size
        pct = 1.0 + it / self.cycle_size - cycle
        sf = pct / self.step_up_pct if pct <= self.step_up_pct else (pct - 1) / (self.step_up_pct - 1)
        h = (self.max_lr - self.base_lr) * sf
        x = cycle if self.scale_mode == "cycle" else it
        return self.base_lr + h * self.scale_fn(x)


class LinearLR(LRScheduler):
    def __init__(self, learning_rate, total_steps, start_factor=1.0 / 3, end_factor=1.0, last_epoch=-1,
                 verbose=False):
        self.total_steps, self.start_factor, self.end_factor = total_steps, start_factor, end_factor
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        t = min(self.last_epoch, self.total_steps)
        f = self.start_factor + (self.end_factor - self.start_factor) * t / self.total_steps
        return self.base_lr * f


class ConstantLR(LRScheduler):
    def __init__(self, learning_rate, factor=1.0 / 3, total_steps=5, last_epoch=-1, verbose=False):
        self.factor, self.total_steps = factor, total_steps
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        return self.base_lr * (self.factor if self.last_epoch < self.total_steps else 1.0)


# ---------------------------------------------------------------------------------------------------------------
# Legacy step-based decay functions (reference: python/paddle/optimizer/lr.py:2636-3150, the fluid-era API).
# The reference builds a global-step counter variable in static mode and returns an LRScheduler in dygraph
# (where its decay_steps / staircase arguments are dropped). Here every mode gets a scheduler that evaluates the
# legacy formula of the global step exactly (decay_steps, staircase, cycle honoured); optimizers step it like any
# other LRScheduler.
class _LegacyStepDecay(LRScheduler):
    def __init__(self, fn, learning_rate=1.0):
        self._fn = fn
        super().__init__(learning_rate, -1, False)

    def get_lr(self):
        return float(self._fn(max(self.last_epoch, 0)))


class _StepCounter:
    """autoincreased_step_counter: value = begin + step * (number of increments)."""

    def __init__(self, name, begin, step):
        self.name, self.begin, self.step_size, self.n = name, begin, step, 0

    def increment(self):
        self.n += 1
        return self.value

    @property
    def value(self):
        return self.begin + self.step_size * self.n

    def __int__(self):
        return int(self.value)

    def __repr__(self):
        return f"StepCounter({self.name}={self.value})"


_COUNTERS = {}


def autoincreased_step_counter(counter_name=None, begin=1, step=1):
    name = counter_name or "@STEP_COUNTER@"
    c = _COUNTERS.get(name)
    if c is None:
        c = _COUNTERS[name] = _StepCounter(name, begin, step)
    return c


def noam_decay(d_model, warmup_steps, learning_rate=1.0):
    return NoamDecay(d_model, warmup_steps, learning_rate)


def _div(step, decay_steps, staircase):
    d = step / decay_steps
    return math.floor(d) if staircase else d


def exponential_decay(learning_rate, decay_steps, decay_rate, staircase=False):
    return _LegacyStepDecay(lambda s: learning_rate * decay_rate ** _div(s, decay_steps, staircase), learning_rate)


def natural_exp_decay(learning_rate, decay_steps, decay_rate, staircase=False):
    return _LegacyStepDecay(lambda s: learning_rate * math.exp(-decay_rate * _div(s, decay_steps, staircase)),
                            learning_rate)


def inverse_time_decay(learning_rate, decay_steps, decay_rate, staircase=False):
    return _LegacyStepDecay(lambda s: learning_rate / (1 + decay_rate * _div(s, decay_steps, staircase)),
                            learning_rate)


def polynomial_decay(learning_rate, decay_steps, end_learning_rate=0.0001, power=1.0, cycle=False):
    def f(s):
        ds = decay_steps
        if cycle:
            ds = decay_steps * max(math.ceil(s / decay_steps), 1)
        else:
            s = min(s, decay_steps)
        return (learning_rate - end_learning_rate) * (1 - s / ds) ** power + end_learning_rate
    return _LegacyStepDecay(f, learning_rate)


def piecewise_decay(boundaries, values):
    return PiecewiseDecay(boundaries, values)


def cosine_decay(learning_rate, step_each_epoch, epochs):
    return _LegacyStepDecay(
        lambda s: learning_rate * 0.5 * (math.cos(math.floor(s / step_each_epoch) * math.pi / epochs) + 1),
        learning_rate)


def linear_lr_warmup(learning_rate, warmup_steps, start_lr, end_lr):
    if isinstance(learning_rate, LRScheduler):
        return LinearWarmup(learning_rate, warmup_steps, start_lr, end_lr)

    def f(s):
        if s < warmup_steps:
            return start_lr + (end_lr - start_lr) * (s / warmup_steps)
        return learning_rate
    return _LegacyStepDecay(f, learning_rate)
