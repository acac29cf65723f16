"""Auto tuner (distributed/auto_tuner): candidate grid, pruning (degrees tile the GPUs, TP in one node, layers
per stage, micro-batch split, MI355X memory estimate, OOM history), history recorder, and the launcher's
``--auto_tuner_json`` trial loop end to end on CPU (2 worker processes per trial, metric read from rank 0's
log, best config written). Reference: python/paddle/distributed/auto_tuner/."""
import json
import os
import subprocess
import sys

import pytest

from paddlepaddle_amd.distributed import auto_tuner as AT

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cfg(**kw):
    c = {"num_gpus": 8, "gpus_per_node": 8,
         "model_cfg": {"num_layers": 40, "hidden_size": 5120, "num_attention_heads": 40, "vocab_size": 50304,
                       "seq_length": 2048, "global_batch_size": 16}}
    c.update(kw)
    return c


def test_grid_covers_valid_tilings_only():
    tasks = AT.search_all(_cfg())
    assert tasks
    for t in tasks:
        assert t["dp_degree"] * t["mp_degree"] * t["pp_degree"] == 8
        assert t["dp_degree"] % t["sharding_degree"] == 0
        assert 16 % (t["dp_degree"] * t["micro_batch_size"]) == 0 and 40 % t["pp_degree"] == 0
    assert {t["mp_degree"] for t in tasks} <= {1, 2, 4, 8}


def test_memory_model_and_pruning():
    m = _cfg()["model_cfg"]
    big = dict(dp_degree=1, mp_degree=1, pp_degree=1, sharding_degree=1, sharding_stage=1, micro_batch_size=16,
               use_recompute=False, acc_steps=1, vpp_degree=1)
    small = dict(big, dp_degree=8, sharding_degree=8, sharding_stage=3, micro_batch_size=1, use_recompute=True)
    assert AT.estimate_memory_gb(big, m) > 288 > AT.estimate_memory_gb(small, m)
    cfg = _cfg(num_gpus=1, gpus_per_node=1)
    assert AT.prune.prune(cfg, dict(big))          # 13B with no sharding at mbs 16 does not fit
    oom = dict(small, oom=True)
    cand = dict(small, micro_batch_size=2)         # same layout, bigger micro-batch than an OOM run
    assert AT.prune.prune_by_oom_history(_cfg(), cand, [oom])
    assert AT.prune.prune_by_mp(_cfg(gpus_per_node=4), dict(small, mp_degree=8))


def test_tuner_and_recorder(tmp_path):
    t = AT.AutoTuner(_cfg(task_limit=5, metric_cfg={"name": "tps", "OptimizationDirection": "Maximize"}))
    rec = AT.HistoryRecorder(t.tuner_cfg)
    seen = []
    while True:
        c = t.search_once()
        if c is None:
            break
        c["tps"] = 100.0 / (c["pp_degree"] + c["mp_degree"])
        rec.add_cfg(**c)
        t.add_cfg(c)
        seen.append(c)
    assert len(seen) == 5
    best, none = rec.get_best()
    assert not none and best["tps"] == max(s["tps"] for s in seen)
    rec.store_history(str(tmp_path / "h.csv"))
    rows, _ = rec.load_history(str(tmp_path / "h.csv"))
    assert len(rows) == 5 and isinstance(rows[0]["dp_degree"], int)
    args = AT.gen_new_args(["--tp", "1", "--x"], {"mp_degree": 2, "use_recompute": True},
                           {"run_cmd": {"mp_degree": ["--tp", "{value}"], "use_recompute": ["--rc", "{value}"]}})
    assert args == ["--tp", "2", "--x", "--rc", "1"]


def test_launch_auto_tuner_end_to_end(tmp_path):
    script = tmp_path / "train.py"
    script.write_text(
        "import argparse, os\n"
        "p = argparse.ArgumentParser(); p.add_argument('--mp', type=int, default=1)\n"
        "p.add_argument('--mbs', type=int, default=1); a = p.parse_args()\n"
        "if os.environ.get('RANK') == '0':\n"
        "    print(f'step done tokens/s={1000 * a.mbs / a.mp:.1f}', flush=True)\n")
    cfg = {"search_algo": {"name": "grid"}, "dp_degree": "auto", "mp_degree": [1, 2], "pp_degree": [1],
           "sharding_degree": [1], "sharding_stage": [1], "micro_batch_size": [1, 2], "use_recompute": [False],
           "model_cfg": {"num_layers": 2, "global_batch_size": 4},
           "run_cmd": {"mp_degree": ["--mp", "{value}"], "micro_batch_size": ["--mbs", "{value}"]},
           "metric_cfg": {"name": "tokens/s", "OptimizationDirection": "Maximize"}}
    (tmp_path / "tuner.json").write_text(json.dumps(cfg))
    env = dict(os.environ, PYTHONPATH=ROOT, PADDLE_AMD_FORCE_CPU="1")
    r = subprocess.run([sys.executable, "-m", "paddlepaddle_amd.distributed.launch", "--nproc_per_node", "2",
                        "--log_dir", str(tmp_path / "log"), "--auto_tuner_json", str(tmp_path / "tuner.json"),
                        str(script)], env=env, capture_output=True, timeout=300, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    best = json.loads((tmp_path / "log" / "best_cfg.json").read_text())
    assert best["mp_degree"] == 1 and best["micro_batch_size"] == 2 and best["tokens/s"] == 2000.0
    hist = (tmp_path / "log" / "history.csv").read_text().splitlines()
    assert len(hist) == 1 + 4   # header + the 4 trials (dp = 2 / mp, mbs in {1, 2})
