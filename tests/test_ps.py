"""Parameter-server training (distributed/ps, distributed/rpc, native SparseTable).

Reference test strategy: test/legacy_test/test_dist_fleet_ps*.py / test_fleet_*ps* (trainers + pservers as
local processes on a CTR-style model with sparse_embedding; sync and async modes; save / load) and
test/cpp/fluid/.../memory_sparse_table_test.cc (pull creates, push updates with the sgd rule, save / load,
shrink). Everything here runs on the CPU; the cross-process parts use TensorPipe RPC over 127.0.0.1.
"""
import os
import socket
import threading

import numpy as np
import pytest

from paddlepaddle_amd import _C_runtime as R


def _table(dim=4, **kw):
    return R.ps.SparseTable(dim, **kw)


def _pull(t, ids, training=True):
    ids = np.asarray(ids, dtype=np.int64)
    out = np.empty((ids.size, t.dim()), np.float32)
    t.pull(ids, out, training)
    return out


def test_sparse_table_sgd_rule_and_lazy_create():
    t = _table(4, rule=0, lr=0.5, init=2)  # zeros init
    assert t.size() == 0
    np.testing.assert_array_equal(_pull(t, [7, 9]), 0)
    assert t.size() == 2
    g = np.arange(8, dtype=np.float32).reshape(2, 4)
    t.push(np.array([7, 9], np.int64), g)
    np.testing.assert_allclose(_pull(t, [9, 7]), -0.5 * g[::-1])
    # unknown ids in a push are ignored, inference pulls do not create
    t.push(np.array([123], np.int64), np.ones((1, 4), np.float32))
    np.testing.assert_array_equal(_pull(t, [55], training=False), 0)
    assert t.size() == 2


def test_sparse_table_adagrad_and_adam_match_numpy():
    rng = np.random.default_rng(0)
    w0 = None
    for rule in (1, 2):
        t = _table(6, rule=rule, lr=0.1, init=0, init_range=0.3, seed=5)
        w = _pull(t, [3]).astype(np.float64)[0]
        w0 = w.copy() if w0 is None else w0
        np.testing.assert_allclose(w, w0)  # the initial value is a function of (seed, id)
        g2, m, v, b1p, b2p = 0.0, np.zeros(6), np.zeros(6), 0.9, 0.999
        for _ in range(5):
            g = rng.standard_normal(6).astype(np.float32)
            t.push(np.array([3], np.int64), g[None])
            if rule == 1:
                w -= 0.1 * g * np.sqrt(3.0 / (3.0 + g2))
                g2 += float((g.astype(np.float64) ** 2).sum()) / 6
            else:
                m = 0.9 * m + 0.1 * g
                v = 0.999 * v + 0.001 * g * g
                w -= 0.1 * np.sqrt(1 - b2p) / (1 - b1p) * m / (np.sqrt(v) + 1e-8)
                b1p *= 0.9
                b2p *= 0.999
        np.testing.assert_allclose(_pull(t, [3])[0], w, rtol=1e-4, atol=1e-6)


def test_sparse_table_entry_admission_and_stats():
    t = _table(2, rule=0, lr=1.0, init=0, init_range=0.5, entry=1, entry_param=3)  # count filter: 3 shows
    ids = np.array([11], np.int64)
    for i in range(2):
        np.testing.assert_array_equal(_pull(t, ids), 0)
        t.push(ids, np.ones((1, 2), np.float32))  # counted, not applied
    show, click, unseen, admitted = t.stat(11)
    assert show == 2 and not admitted
    t.push(ids, np.ones((1, 2), np.float32), np.array([1.0], np.float32), np.array([1.0], np.float32))
    w = _pull(t, ids)
    assert np.abs(w).max() > 0 and t.stat(11)[3]
    assert t.stat(11)[1] == 1.0
    # probability entry: the admitted fraction follows p, and the decision is stable per id
    tp = _table(2, entry=2, entry_param=0.25, seed=1)
    n = 4000
    out = _pull(tp, np.arange(n))
    frac = float((np.abs(out).sum(1) > 0).mean())
    assert 0.2 < frac < 0.3, frac
    np.testing.assert_array_equal(_pull(tp, np.arange(n)), out)


def test_sparse_table_shrink_save_load(tmp_path):
    t = _table(3, rule=1, lr=0.1, seed=2)
    _pull(t, np.arange(10))
    t.push(np.arange(5, dtype=np.int64), np.ones((5, 3), np.float32))
    full = str(tmp_path / "full.txt")
    assert t.save(full, 0) == 10
    assert t.save(str(tmp_path / "delta.txt"), 1) == 0  # deltas were cleared by the first save
    t.push(np.array([2], np.int64), np.ones((1, 3), np.float32))
    assert t.save(str(tmp_path / "delta2.txt"), 1) == 1
    t2 = _table(3, rule=1, lr=0.1, seed=99)
    assert t2.load(full) == 10
    ref = _pull(t, np.arange(10))
    got = _pull(t2, np.arange(10))
    keep = [0, 1, 3, 4, 5, 6, 7, 8, 9]
    np.testing.assert_allclose(got[keep], ref[keep], rtol=1e-6)
    # the optimizer state came along: the same push moves both tables identically
    g = np.full((1, 3), 0.5, np.float32)
    t.push(np.array([0], np.int64), g)
    t2.push(np.array([0], np.int64), g)
    np.testing.assert_allclose(_pull(t2, [0]), _pull(t, [0]), rtol=1e-6)
    # shrink: ages every feature; those not pulled (training) for more than `threshold` passes are dropped
    assert t.shrink(5) == 0
    _pull(t, [1, 2])
    for _ in range(4):
        t.shrink(5)
    assert t.shrink(5) == 8 and t.size() == 2


def test_sparse_table_concurrent_pushes_are_atomic():
    t = _table(8, rule=0, lr=1.0, init=2)
    ids = np.arange(20000, dtype=np.int64)  # large batches take the multi-threaded shard path
    _pull(t, ids)
    g = np.ones((ids.size, 8), np.float32)

    def work():
        for _ in range(5):
            t.push(ids, g)
    th = [threading.Thread(target=work) for _ in range(4)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    np.testing.assert_array_equal(_pull(t, ids), -20.0)


# ------------------------------------------------------------------------------------------- multi-process
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _ps_proc(role, index, n_servers, n_trainers, port, a_sync, outdir, q):
    import torch  # noqa: F401
    os.environ.update({"TRAINING_ROLE": role, "PADDLE_PSERVERS_IP_PORT_LIST":
                       ",".join(f"127.0.0.1:{port + i}" for i in range(n_servers)),
                       "PADDLE_TRAINERS_NUM": str(n_trainers), "PADDLE_TRAINER_ID": str(index),
                       "POD_IP": "127.0.0.1", "PADDLE_PORT": str(port + index)})
    try:
        import paddlepaddle_amd as paddle
        from paddlepaddle_amd.distributed import fleet
        strategy = fleet.DistributedStrategy()
        strategy.a_sync = a_sync
        fleet.init(fleet.PaddleCloudRoleMaker(), strategy=strategy)
        if fleet.is_server():
            fleet.init_server()
            fleet.run_server()
            q.put(("server", index, None))
            return
        paddle.seed(1234)
        slots, dim = 3, 8
        fc = paddle.nn.Linear(slots * dim, 1)
        opt = fleet.distributed_optimizer(paddle.optimizer.SGD(learning_rate=1.0, parameters=fc.parameters()),
                                          strategy)
        fleet.init_worker()
        rng = np.random.default_rng(100 + index)
        losses = []
        for step in range(60):
            ids = rng.integers(0, 50, size=(32, slots))
            label = ((ids % 2).sum(1, keepdims=True) >= 2).astype(np.float32)  # depends on the features only
            emb = paddle.static.nn.sparse_embedding(paddle.to_tensor(ids), size=[1000, dim],
                                                    param_attr=paddle.ParamAttr(name="ctr_emb"))
            logit = fc(emb.reshape([32, slots * dim]))
            loss = paddle.nn.functional.binary_cross_entropy_with_logits(logit, paddle.to_tensor(label))
            loss.backward()
            opt.step()
            opt.clear_grad()
            losses.append(float(loss))
        fleet.barrier_worker()
        n_saved = fleet.save_persistables(None, outdir) if index == 0 else None
        fleet.barrier_worker()
        from paddlepaddle_amd.distributed.communicator import Communicator
        comm = Communicator(mode="ASYNC" if a_sync else "SYNC")
        comm.start()
        assert comm.create_client_to_client_connection() and comm.is_running()
        # the servers' dense tables back into the parameters: after the barrier both trainers read one value
        n_pulled = comm.pull_dense([fc.weight]) + comm.recv()
        comm.stop()
        w = fc.weight.numpy().copy()
        fleet.stop_worker()
        q.put(("trainer", index, (losses, w, n_saved, n_pulled)))
    except Exception as e:  # pragma: no cover - surfaced by the parent
        import traceback
        q.put(("error", index, traceback.format_exc() + repr(e)))


def _run_ps(a_sync, tmp_path, n_servers=2, n_trainers=2):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ps_proc, args=("PSERVER", i, n_servers, n_trainers, port, a_sync,
                                                 str(tmp_path), q)) for i in range(n_servers)]
    procs += [ctx.Process(target=_ps_proc, args=("TRAINER", i, n_servers, n_trainers, port, a_sync,
                                                  str(tmp_path), q)) for i in range(n_trainers)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in procs:
            kind, idx, val = q.get(timeout=240)
            assert kind != "error", val
            res[(kind, idx)] = val
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return res


@pytest.mark.timeout(300)
def test_ps_sync_training_two_servers_two_trainers(tmp_path):
    res = _run_ps(False, tmp_path)
    (l0, w0, n_saved, _), (l1, w1, _, _) = res[("trainer", 0)], res[("trainer", 1)]
    # sync mode: one averaged dense update per step, so both trainers hold identical dense weights
    np.testing.assert_allclose(w0, w1, rtol=0, atol=0)
    for losses in (l0, l1):
        assert np.mean(losses[-8:]) < np.mean(losses[:8]) - 0.05, losses
    # the sparse table (ids 0..49 seen by the trainers) is sharded over both servers and saved per shard
    assert n_saved == 50
    files = sorted(os.listdir(tmp_path))
    assert "ctr_emb.shard0.txt" in files and "ctr_emb.shard1.txt" in files
    with open(tmp_path / "ctr_emb.shard1.txt") as f:
        ids = [int(line.split("\t")[0]) for line in f]
    assert ids and all(i % 2 == 1 for i in ids)


@pytest.mark.timeout(300)
def test_ps_async_training(tmp_path):
    res = _run_ps(True, tmp_path, n_servers=1, n_trainers=2)
    for i in range(2):
        losses = res[("trainer", i)][0]
        assert np.mean(losses[-8:]) < np.mean(losses[:8]), losses
    # Communicator.pull_dense / recv: one weight, then both dense tables (weight, bias); after the final barrier
    # the pulled values are the servers' and agree between the trainers although their async steps did not
    assert res[("trainer", 0)][3] == 1 + 2
    np.testing.assert_allclose(res[("trainer", 0)][1], res[("trainer", 1)][1], rtol=0, atol=0)


def test_rpc_api_single_worker():
    import paddlepaddle_amd.distributed.rpc as rpc
    rpc.init_rpc("solo", rank=0, world_size=1, master_endpoint=f"127.0.0.1:{_free_port()}")
    try:
        assert rpc.rpc_sync("solo", max, args=(3, 9)) == 9
        fut = rpc.rpc_async("solo", divmod, args=(17, 5))
        assert fut.wait() == (3, 2)
        info = rpc.get_current_worker_info()
        assert info.name == "solo" and info.rank == 0
        assert [w.name for w in rpc.get_all_worker_infos()] == ["solo"]
        assert rpc.get_worker_info("solo").rank == 0
    finally:
        rpc.shutdown()


def test_communicator_handle_without_ps_worker():
    """No parameter-server worker: the handle tracks its run state and the table calls raise instead of
    silently doing nothing (reference communicator.py:129-201)."""
    from paddlepaddle_amd.distributed.communicator import Communicator
    c = Communicator(mode="SYNC")
    assert c.mode == "sync" and not c.is_running()
    c.start()
    assert c.is_running()
    with pytest.raises(RuntimeError, match="init_worker"):
        c.pull_dense(None)
    with pytest.raises(RuntimeError, match="init_worker"):
        c.create_client_to_client_connection()
    c.stop()
    assert not c.is_running()
