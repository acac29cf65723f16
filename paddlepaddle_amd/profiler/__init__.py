"""paddle.profiler. Reference: python/paddle/profiler/ (profiler.py: Profiler, make_scheduler,
export_chrome_tracing, ProfilerState/Target; utils.py: RecordEvent; profiler_statistic.py: summary
tables; timer.py: step timer / ips).

Device activity comes from the ROCm tracer behind torch.profiler (HIP kernels incl. ours, RCCL,
memcpy); host ranges from RecordEvent. ``timer_only=True`` skips tracing and reports step time /
throughput (the reference's benchmark timer)."""
from __future__ import annotations

import enum
import json
import os
import time

import torch


class ProfilerState(enum.Enum):
    CLOSED = 0
    READY = 1
    RECORD = 2
    RECORD_AND_RETURN = 3


class ProfilerTarget(enum.Enum):
    CPU = 0
    GPU = 1
    XPU = 2
    CUSTOM_DEVICE = 3


class SortedKeys(enum.Enum):
    CPUTotal = 0
    CPUAvg = 1
    CPUMax = 2
    CPUMin = 3
    GPUTotal = 4
    GPUAvg = 5
    GPUMax = 6
    GPUMin = 7


class SummaryView(enum.Enum):
    DeviceView = 0
    OverView = 1
    ModelView = 2
    DistributedView = 3
    KernelView = 4
    OperatorView = 5
    MemoryView = 6
    MemoryManipulationView = 7
    UDFView = 8


def make_scheduler(*, closed, ready, record, repeat=0, skip_first=0):
    def sched(step):
        if step < skip_first:
            return ProfilerState.CLOSED
        s = step - skip_first
        period = closed + ready + record
        if repeat > 0 and s >= period * repeat:
            return ProfilerState.CLOSED
        m = s % period
        if m < closed:
            return ProfilerState.CLOSED
        if m < closed + ready:
            return ProfilerState.READY
        return ProfilerState.RECORD_AND_RETURN if m == period - 1 else ProfilerState.RECORD
    return sched


def _default_sched(step):
    return ProfilerState.RECORD


def export_chrome_tracing(dir_name, worker_name=None):
    def handler(prof):
        os.makedirs(dir_name, exist_ok=True)
        name = worker_name or f"host_{os.uname().nodename}_pid_{os.getpid()}"
        path = os.path.join(dir_name, f"{name}_time_{time.strftime('%Y_%m_%d_%H_%M_%S')}.paddle_trace.json")
        prof.export(path)
    return handler


def export_protobuf(dir_name, worker_name=None):
    return export_chrome_tracing(dir_name, worker_name)


class RecordEvent:
    """Host range visible in the trace (and as an roctx range on the device timeline)."""

    def __init__(self, name, event_type=None):
        self.name = name
        self._ctx = None

    def begin(self):
        self._ctx = torch.profiler.record_function(self.name)
        self._ctx.__enter__()

    def end(self):
        if self._ctx is not None:
            self._ctx.__exit__(None, None, None)
            self._ctx = None

    def __enter__(self):
        self.begin()
        return self

    def __exit__(self, *a):
        self.end()


class _StepTimer:
    def __init__(self):
        self.reset()

    def reset(self):
        self.times, self.samples, self._t = [], [], None

    def begin(self):
        self._t = time.perf_counter()

    def step(self, num_samples=None):
        now = time.perf_counter()
        if self._t is not None:
            self.times.append(now - self._t)
            self.samples.append(num_samples)
        self._t = now

    def info(self, unit="samples"):
        if not self.times:
            return "no steps recorded"
        ts = self.times
        avg = sum(ts) / len(ts)
        s = f"avg batch_cost: {avg:.5f} s, max: {max(ts):.5f} s, min: {min(ts):.5f} s"
        if all(n is not None for n in self.samples):
            ips = sum(self.samples) / sum(ts)
            s += f", ips: {ips:.3f} {unit}/s"
        return s


class Profiler:
    def __init__(self, *, targets=None, scheduler=None, on_trace_ready=None, record_shapes=False,
                 profile_memory=False, timer_only=False, emit_nvtx=False, custom_device_types=None,
                 with_flops=False):
        targets = targets or [ProfilerTarget.CPU, ProfilerTarget.GPU]
        acts = [torch.profiler.ProfilerActivity.CPU]
        if ProfilerTarget.GPU in targets and torch.cuda.is_available():
            acts.append(torch.profiler.ProfilerActivity.CUDA)
        if isinstance(scheduler, tuple):
            lo, hi = scheduler
            scheduler = make_scheduler(closed=max(lo, 0), ready=0, record=hi - lo, repeat=1)
        self._sched = scheduler or _default_sched
        self._on_ready = on_trace_ready
        self._timer_only = timer_only
        self._acts, self._shapes, self._mem, self._flops = acts, record_shapes, profile_memory, with_flops
        self._prof = None
        self.step_num = 0
        self._timer = _StepTimer()
        self._state = ProfilerState.CLOSED
        self._events = None

    def _start_trace(self):
        self._prof = torch.profiler.profile(activities=self._acts, record_shapes=self._shapes,
                                            profile_memory=self._mem, with_flops=self._flops)
        self._prof.__enter__()

    def _stop_trace(self):
        if self._prof is not None:
            self._prof.__exit__(None, None, None)
            self._events = self._prof
            if self._on_ready is not None:
                self._on_ready(self)
            self._prof = None

    def start(self):
        self._timer.begin()
        if self._timer_only:
            return
        self._state = self._sched(self.step_num)
        if self._state in (ProfilerState.RECORD, ProfilerState.RECORD_AND_RETURN, ProfilerState.READY):
            self._start_trace()

    def step(self, num_samples=None):
        self._timer.step(num_samples)
        self.step_num += 1
        if self._timer_only:
            return
        prev = self._state
        self._state = self._sched(self.step_num)
        recording = prev in (ProfilerState.RECORD, ProfilerState.READY)
        if prev == ProfilerState.RECORD_AND_RETURN or (recording and self._state == ProfilerState.CLOSED):
            self._stop_trace()
        if self._prof is None and self._state in (ProfilerState.RECORD, ProfilerState.READY,
                                                  ProfilerState.RECORD_AND_RETURN):
            self._start_trace()

    def stop(self):
        if not self._timer_only:
            self._stop_trace()
        self._state = ProfilerState.CLOSED

    def __enter__(self):
        self.start()
        return self

    def __exit__(self, *a):
        self.stop()

    def step_info(self, unit="samples"):
        return self._timer.info(unit)

    def export(self, path, format="json"):
        src = self._prof or self._events
        if src is None:
            raise RuntimeError("nothing recorded")
        src.export_chrome_trace(path)

    def summary(self, sorted_by=SortedKeys.CPUTotal, op_detail=True, thread_sep=False, time_unit="ms", views=None):
        src = self._events
        if src is None:
            print(self.step_info())
            return None
        key = {SortedKeys.CPUTotal: "cpu_time_total", SortedKeys.GPUTotal: "device_time_total",
               SortedKeys.CPUAvg: "cpu_time", SortedKeys.GPUAvg: "device_time"}.get(sorted_by, "cpu_time_total")
        try:
            table = src.key_averages().table(sort_by=key, row_limit=40)
        except Exception:
            table = src.key_averages().table(row_limit=40)
        print(table)
        return table


def load_profiler_result(filename):
    with open(filename) as f:
        return json.load(f)


def get_profiler(config_path=None):
    return Profiler()
