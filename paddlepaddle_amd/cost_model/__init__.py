"""paddle.cost_model (reference python/paddle/cost_model/cost_model.py:33-110).

``static_cost_data()`` serves a per-op forward / backward time table measured on MI355X by
tools/gen_op_cost_table.py (mi355x_op_benchmark.json next to this file), in the reference table's record
format (op, config, gpu_time, gpu_time_backward). ``profile_measure`` times every node of a static program
on the device (one synchronised timing per node, summed per op type) — the per-program counterpart the
reference gets from its C++ CostModel over the profiler.
"""
from __future__ import annotations

import json
import os
import time

import numpy as np
import torch

__all__ = ["CostModel"]

_TABLE = os.path.join(os.path.dirname(__file__), "mi355x_op_benchmark.json")


class CostModel:
    def __init__(self):
        self._static_cost_data = None

    def build_program(self):
        """A tiny fc + SGD program pair (startup, main), as the reference's example."""
        import paddlepaddle_amd as paddle
        paddle.enable_static()
        main, startup = paddle.static.Program(), paddle.static.Program()
        with paddle.static.program_guard(main, startup):
            data = paddle.static.data(name="X", shape=[None, 1], dtype="float32")
            hidden = paddle.static.nn.fc(data, 10)
            loss = paddle.mean(hidden)
            paddle.optimizer.SGD(learning_rate=0.01).minimize(loss)
        return startup, main

    def profile_measure(self, startup_program, main_program, device="gpu", fetch_cost_list=("time",),
                        feed=None, repeat=3):
        """Run ``main_program`` and return {op type: total ms per run} (median over ``repeat`` runs)."""
        import paddlepaddle_amd as paddle
        from ..static import program as P
        from ..static.executor import Executor, CompiledProgram
        on_gpu = device == "gpu" and torch.cuda.is_available()
        place = paddle.CUDAPlace(0) if on_gpu else paddle.CPUPlace()
        exe = Executor(place)
        exe.run(startup_program)
        prog = main_program._program if isinstance(main_program, CompiledProgram) else main_program
        if feed is None:
            feed = {}
            for name, (slot, shape, dtype) in prog.feeds.items():
                shp = [10 if d is None or d < 0 else d for d in shape]
                feed[name] = np.random.random(shp).astype(dtype)
        dev = torch.device("cuda", 0) if on_gpu else torch.device("cpu")
        env = exe._feed(prog, feed, dev)
        sync = torch.cuda.synchronize if on_gpu else (lambda: None)
        per_run = []
        for _ in range(max(1, repeat)):
            e = dict(env)
            cost = {}
            with torch.no_grad():
                for n in prog.nodes:
                    sync()
                    t = time.perf_counter()
                    P._exec_node(n, e, None, dev, None)
                    sync()
                    key = n.name.rsplit(":", 1)[-1]
                    cost[key] = cost.get(key, 0.0) + (time.perf_counter() - t) * 1e3
            per_run.append(cost)
        return {k: float(np.median([c.get(k, 0.0) for c in per_run])) for k in per_run[0]}

    def static_cost_data(self):
        if not os.path.exists(_TABLE):
            raise FileNotFoundError(f"{_TABLE} missing: generate it with tools/gen_op_cost_table.py on the GPU")
        with open(_TABLE) as f:
            self._static_cost_data = json.load(f)
        return self._static_cost_data

    def get_static_op_time(self, op_name, forward=True, dtype="float32"):
        if op_name is None:
            raise ValueError("op_name should not be empty when you want to get static op time")
        if self._static_cost_data is None:
            self.static_cost_data()
        cost = {}
        for rec in self._static_cost_data:
            if rec["op"] == op_name and f"dtype: {dtype}" in rec["config"]:
                cost["op_time"] = rec["gpu_time"] if forward else rec["gpu_time_backward"]
                cost["config"] = rec["config"]
        return cost
