"""bench.py driver contract on CPU: torchrun with 2 ranks (gloo), bf16 GPT (sharding stage 3 with
no_sync accumulation) + ResNet-50 DP, exactly one JSON line from rank 0 with the required fields."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_two_ranks_json_line():
    env = dict(os.environ, PADDLE_AMD_FORCE_CPU="1", PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--tp", "1",
           "--model", "tiny", "--steps", "2", "--warmup", "1", "--seq-len", "64", "--micro-batch", "2", "--accum", "2",
           "--resnet-batch", "2", "--resnet-steps", "1"]
    r = subprocess.run(cmd, env=env, capture_output=True, timeout=600, cwd="/tmp")
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    lines = [l for l in r.stdout.decode().splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in d
    assert d["n_gpus"] == 2 and d["steps"] == 2 and d["value"] > 0 and d["dtype"] == "bf16"
    assert d["config"]["parallelism"] == "sharding_stage3_degree2"
    assert d["secondary"]["value"] > 0


def test_bench_llama_pipeline_x_tp_four_ranks():
    env = dict(os.environ, PADDLE_AMD_FORCE_CPU="1", PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"), "--gpus", "4", "--model",
           "llama-tiny", "--pp", "2", "--tp", "2", "--steps", "2", "--warmup", "1", "--seq-len", "32",
           "--micro-batch", "1", "--accum", "4", "--llama-engine", "fleet"]
    r = subprocess.run(cmd, env=env, capture_output=True, timeout=600, cwd="/tmp")
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    lines = [l for l in r.stdout.decode().splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 4 and d["value"] > 0 and d["config"]["parallelism"] == "pp2_tp2_dp1"


def test_bench_llama_static_auto_parallel_pp4_tp2_eight_ranks():  # collective-sequence checker on
    """The BASELINE LLaMA-2 layout (PP4 x TP2, static-graph auto-parallel) on 8 gloo ranks: `bench.py --model
    llama-tiny --pp 4 --tp 2` distributes a plain LLaMA with dist.parallelize and trains it through
    dist.to_static (traced program, per-rank partition, 1F1B)."""
    env = dict(os.environ, PADDLE_AMD_FORCE_CPU="1", PYTHONPATH=ROOT, OMP_NUM_THREADS="1",
               PADDLE_AMD_CHECK_COLLECTIVES="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"), "--gpus", "8", "--model",
           "llama-tiny", "--pp", "4", "--tp", "2", "--steps", "2", "--warmup", "1", "--seq-len", "32",
           "--micro-batch", "1", "--accum", "4"]
    r = subprocess.run(cmd, env=env, capture_output=True, timeout=900, cwd="/tmp")
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    lines = [l for l in r.stdout.decode().splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8 and d["value"] > 0
    assert d["config"]["parallelism"] == "pp4_tp2_dp1_static_auto_parallel"
    assert "[llama-static]" in r.stderr.decode() + r.stdout.decode()
    assert "sequence checks passed" in r.stderr.decode()  # every rank's collective sequence matched its peers' 


def test_bench_self_launch_sharding_x_tp_four_ranks():
    """`bench.py --gpus 4 --tp 2` with no launcher starts the 4 ranks itself; GPT runs fleet's hybrid
    topology (sharding stage 3 over 2 ranks x tensor parallel 2)."""
    env = dict(os.environ, PADDLE_AMD_FORCE_CPU="1", PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--tp", "2", "--model", "tiny",
           "--steps", "2", "--warmup", "1", "--seq-len", "64", "--micro-batch", "2", "--accum", "2", "--resnet", "0"]
    r = subprocess.run(cmd, env=env, capture_output=True, timeout=600, cwd="/tmp")
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    lines = [l for l in r.stdout.decode().splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 4 and d["value"] > 0
    assert d["config"]["parallelism"] == "sharding_stage3_degree2_tp2_sp"
    assert d["config"]["global_batch"] == 2 * 2 * 2


def test_bench_eight_ranks_sharding4_x_tp2_sp():
    """The 8-GPU flagship layout on 8 gloo ranks: `bench.py --gpus 8 --tp 2` (sharding stage 3 over 4 ranks x
    tensor parallel 2 with sequence parallelism), self-launched, with the collective-sequence checker on."""
    env = dict(os.environ, PADDLE_AMD_FORCE_CPU="1", PYTHONPATH=ROOT, OMP_NUM_THREADS="1",
               PADDLE_AMD_CHECK_COLLECTIVES="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--tp", "2", "--model", "tiny",
           "--steps", "2", "--warmup", "1", "--seq-len", "64", "--micro-batch", "2", "--accum", "2", "--resnet", "0"]
    r = subprocess.run(cmd, env=env, capture_output=True, timeout=900, cwd="/tmp")
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    lines = [l for l in r.stdout.decode().splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8 and d["value"] > 0
    assert d["config"]["parallelism"] == "sharding_stage3_degree4_tp2_sp"
    assert d["config"]["global_batch"] == 2 * 2 * 4
    assert "sequence checks passed" in r.stderr.decode()


def test_bench_rejects_world_mismatch():
    env = dict(os.environ, PADDLE_AMD_FORCE_CPU="1", PYTHONPATH=ROOT, WORLD_SIZE="1", RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--resnet", "0"], env=env,
                       capture_output=True, timeout=300, cwd="/tmp")
    assert r.returncode != 0 and b"WORLD_SIZE" in r.stderr
