"""Semi-auto parallel (ProcessMesh / shard_tensor / reshard / shard_layer / shard_optimizer),
distributed checkpoint with reshard-on-load, launcher failure detection — gloo, 2 ranks on CPU.
Reference test strategy: test/auto_parallel/semi_auto_parallel_*.py (dist result == single-card result),
test/auto_parallel/test_dist_checkpoint*.py."""
import os
import subprocess
import sys
import textwrap

import numpy as np
import torch

from test_distributed_cpu import ROOT, _setup, _spawn


def _ap_worker(rank, world, port, q):
    paddle = _setup(rank, world, port)
    import paddlepaddle_amd.distributed as dist
    mesh = dist.ProcessMesh([0, 1], dim_names=["x"])
    a = np.arange(24, dtype="float32").reshape(4, 6)
    t = dist.shard_tensor(paddle.to_tensor(a), mesh, [dist.Shard(0)])
    out = {"local": t._local_value().numpy(), "is_dist": t.is_dist(), "pl": repr(t.placements)}
    r = dist.reshard(t, mesh, [dist.Replicate()])
    out["replicated"] = r._local_value().numpy()
    s1 = dist.reshard(t, mesh, [dist.Shard(1)])
    out["shard1"] = s1._local_value().numpy()
    # an op on sharded inputs: (row-sharded A) @ (replicated B) stays row-sharded, values correct
    b = np.ones((6, 3), dtype="float32")
    y = paddle.matmul(t, dist.shard_tensor(paddle.to_tensor(b), mesh, [dist.Replicate()]))
    out["mm"] = dist.unshard_dtensor(y).numpy()
    # data-parallel training through sharding propagation == single-process full batch
    paddle.seed(0)
    net = paddle.nn.Sequential(paddle.nn.Linear(6, 8), paddle.nn.Tanh(), paddle.nn.Linear(8, 2))
    dist.shard_layer(net, mesh)
    opt = dist.shard_optimizer(paddle.optimizer.AdamW(0.05, parameters=net.parameters()),
                               dist.ShardingStage1(mesh))
    rng = np.random.RandomState(1)
    X, Y = rng.randn(8, 6).astype("float32"), rng.randn(8, 2).astype("float32")
    xs = dist.shard_tensor(paddle.to_tensor(X), mesh, [dist.Shard(0)])
    ys = dist.shard_tensor(paddle.to_tensor(Y), mesh, [dist.Shard(0)])
    losses = []
    for _ in range(3):
        loss = ((net(xs) - ys) ** 2).mean()
        loss.backward()
        opt.step()
        opt.clear_grad()
        losses.append(float(dist.unshard_dtensor(loss).numpy()))
    out["losses"] = losses
    out["w"] = dist.unshard_dtensor(net[0].weight).numpy()
    # distributed checkpoint: save row-sharded, load into column-sharded + into a plain tensor
    ck = os.environ["CKPT_DIR"]
    dist.save_state_dict({"t": t, "w": net[0].weight}, ck)
    tgt = dist.shard_tensor(paddle.zeros([4, 6]), mesh, [dist.Shard(1)])
    plain = paddle.zeros([4, 6])
    dist.load_state_dict({"t": tgt, "w": paddle.zeros([6, 8])}, ck)
    dist.load_state_dict({"t": plain}, ck)
    out["ckpt_col"] = tgt._local_value().numpy()
    out["ckpt_plain"] = plain.numpy()
    q.put((rank, out))
    dist.barrier()


def test_semi_auto_parallel_and_dist_checkpoint(tmp_path):
    os.environ["CKPT_DIR"] = str(tmp_path / "ck")
    res = _spawn(_ap_worker)
    a = np.arange(24, dtype="float32").reshape(4, 6)
    for rank, out in res:
        assert out["is_dist"] and "Shard(dim=0)" in out["pl"]
        np.testing.assert_array_equal(out["local"], a[2 * rank:2 * rank + 2])
        np.testing.assert_array_equal(out["replicated"], a)
        np.testing.assert_array_equal(out["shard1"], a[:, 3 * rank:3 * rank + 3])
        np.testing.assert_allclose(out["mm"], a @ np.ones((6, 3), "float32"))
        np.testing.assert_array_equal(out["ckpt_col"], a[:, 3 * rank:3 * rank + 3])
        np.testing.assert_array_equal(out["ckpt_plain"], a)
    # single-process reference of the DP training
    sys.path.insert(0, ROOT)
    os.environ["PADDLE_AMD_FORCE_CPU"] = "1"
    import paddlepaddle_amd as paddle
    paddle.seed(0)
    net = paddle.nn.Sequential(paddle.nn.Linear(6, 8), paddle.nn.Tanh(), paddle.nn.Linear(8, 2))
    opt = paddle.optimizer.AdamW(0.05, parameters=net.parameters())
    rng = np.random.RandomState(1)
    X, Y = rng.randn(8, 6).astype("float32"), rng.randn(8, 2).astype("float32")
    ref = []
    for _ in range(3):
        loss = ((net(paddle.to_tensor(X)) - paddle.to_tensor(Y)) ** 2).mean()
        loss.backward()
        opt.step()
        opt.clear_grad()
        ref.append(float(loss))
    for _, out in res:
        np.testing.assert_allclose(out["losses"], ref, rtol=1e-5, atol=1e-6)
    # the checkpoint is in the reference layout and reshards onto a single process
    ck = os.environ["CKPT_DIR"]
    assert sorted(os.listdir(ck)) == ["0.metadata", "0_0.distcp", "1_0.distcp"]
    with open(os.path.join(ck, "0.metadata"), "rb") as f:
        assert b"paddle.distributed.checkpoint.metadata" in f.read()
    md = paddle.load(os.path.join(ck, "0.metadata"))
    assert [m.global_offset for m in md.state_dict_metadata["t"]] == [(0, 0), (2, 0)]
    assert md.state_dict_metadata["t"][0].dtype == "float32"
    part0 = paddle.load(os.path.join(ck, "0_0.distcp"), return_numpy=True)
    part1 = paddle.load(os.path.join(ck, "1_0.distcp"), return_numpy=True)
    np.testing.assert_array_equal(part0["t"], a[:2])
    np.testing.assert_array_equal(part1["t"], a[2:])
    whole = paddle.zeros([4, 6])
    paddle.distributed.load_state_dict({"t": whole}, ck)
    np.testing.assert_array_equal(whole.numpy(), a)
    w = part0["w"] if "w" in part0 else part1["w"]  # replicated: stored once
    assert ("w" in part0) != ("w" in part1)
    np.testing.assert_allclose(w, res[0][1]["w"], rtol=1e-6)
    for _, out in res:
        np.testing.assert_allclose(out["w"], net[0].weight.numpy(), rtol=1e-5, atol=1e-6)


def test_launch_runs_workers_and_detects_failure(tmp_path):
    script = tmp_path / "w.py"
    script.write_text(textwrap.dedent("""
        import os, sys
        r = int(os.environ["RANK"])
        print("hello from", r, os.environ["WORLD_SIZE"], os.environ["LOCAL_RANK"])
        sys.exit(3 if (r == 1 and len(sys.argv) > 1) else 0)
    """))
    env = dict(os.environ, PYTHONPATH=ROOT, PADDLE_AMD_FORCE_CPU="1")
    logd = tmp_path / "log"
    ok = subprocess.run([sys.executable, "-m", "paddlepaddle_amd.distributed.launch", "--nproc_per_node", "2",
                         "--log_dir", str(logd), str(script)], env=env, capture_output=True, timeout=120)
    assert ok.returncode == 0, ok.stderr.decode()
    assert "hello from 1 2 1" in (logd / "workerlog.1").read_text()
    bad = subprocess.run([sys.executable, "-m", "paddlepaddle_amd.distributed.launch", "--nproc_per_node", "2",
                          "--log_dir", str(logd), str(script), "fail"], env=env, capture_output=True, timeout=120)
    assert bad.returncode == 3 and b"rank 1 exited with code 3" in bad.stderr
