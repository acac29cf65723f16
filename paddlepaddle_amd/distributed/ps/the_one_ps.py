"""Parameter-server training: sparse / dense tables on server processes, trainers pulling and pushing.

Reference: python/paddle/distributed/ps/the_one_ps.py (TheOnePSRuntime: init_server / run_server /
init_worker / stop_worker, table configs, save / load / shrink), paddle/fluid/distributed/ps/service/
(brpc PS client / server, communicator with sync / async push), ps/table/ (memory_sparse_table,
memory_dense_table, ctr accessor, sgd rules), python/paddle/distributed/fleet/base/role_maker.py (role and
endpoints from TRAINING_ROLE / PADDLE_PSERVERS_IP_PORT_LIST / PADDLE_TRAINERS_NUM / PADDLE_TRAINER_ID /
POD_IP / PADDLE_PORT) and python/paddle/static/nn/common.py sparse_embedding.

Design (the CTR / huge-embedding workload a PS exists for):
* Servers hold the tables. A sparse table is the native ``_C_runtime.ps.SparseTable`` (sharded hash map,
  lazily created rows, show / click statistics, SGD / AdaGrad / Adam rules, entry admission, shrink, text
  save / load). Dense tables are flat fp32 tensors with an SGD / Adam rule.
* Transport is paddle.distributed.rpc (TensorPipe): a server answers calls on a thread pool, so trainers
  are served concurrently; arrays travel as CPU tensors.
* Sparse ids are sharded over servers by ``id % n_servers``; a dense table lives on one server (chosen by
  name). Trainers pull rows for the unique ids of a batch, gather them on the device, and push the
  per-unique-id gradient sums in backward.
* Communicator modes: ``sync`` (a_sync False) — sparse pushes are sent in backward and dense gradients
  are averaged over all trainers on the server before one update per step (every trainer then pulls the
  same version); ``async`` (a_sync True) — sparse and dense pushes go through a background thread that
  merges gradients of the same ids, and trainers pull whatever version is current (Hogwild-style).
"""
from __future__ import annotations

import os
import queue
import threading
import zlib

import numpy as np
import torch

from .. import rpc as _rpc

# ----------------------------------------------------------------------------------------------- server side
_SRV = {"sparse": {}, "dense": {}, "cfg": {}, "lock": threading.Lock(), "cv": threading.Condition(),
        "load_dir": None, "barriers": {}, "n_trainers": 1, "index": 0}

_RULES = {"sgd": 0, "naive": 0, "adagrad": 1, "adam": 2}
_INITS = {"uniform": 0, "normal": 1, "zeros": 2}


def _native():
    from ... import _C_runtime
    return _C_runtime.ps


def _srv_setup(index, n_trainers, load_dir):
    _SRV["index"], _SRV["n_trainers"], _SRV["load_dir"] = index, n_trainers, load_dir


def _table_file(dirname, name, index):
    return os.path.join(dirname, f"{name}.shard{index}.txt")


def _srv_create_sparse(name, cfg):
    with _SRV["lock"]:
        if name in _SRV["sparse"]:
            return _SRV["sparse"][name].size()
        entry, entry_param = cfg.get("entry", (0, 0.0))
        t = _native().SparseTable(int(cfg["dim"]), rule=_RULES[cfg.get("rule", "adagrad")],
                                  lr=float(cfg.get("lr", 0.05)), init_range=float(cfg.get("init_range", 0.01)),
                                  init=_INITS[cfg.get("init", "uniform")], seed=int(cfg.get("seed", 0)),
                                  entry=int(entry), entry_param=float(entry_param),
                                  initial_g2sum=float(cfg.get("initial_g2sum", 3.0)),
                                  beta1=float(cfg.get("beta1", 0.9)), beta2=float(cfg.get("beta2", 0.999)),
                                  eps=float(cfg.get("eps", 1e-8)), min_bound=float(cfg.get("min_bound", -1e30)),
                                  max_bound=float(cfg.get("max_bound", 1e30)))
        ld = _SRV["load_dir"]
        if ld and os.path.exists(_table_file(ld, name, _SRV["index"])):
            t.load(_table_file(ld, name, _SRV["index"]))
        _SRV["sparse"][name] = t
        _SRV["cfg"][name] = dict(cfg)
        return t.size()


def _srv_pull_sparse(name, ids, training):
    t = _SRV["sparse"][name]
    out = np.empty((ids.numel(), t.dim()), dtype=np.float32)
    t.pull(ids.numpy(), out, bool(training))
    return torch.from_numpy(out)


def _srv_push_sparse(name, ids, grads, shows, clicks):
    _SRV["sparse"][name].push(ids.numpy(), grads.numpy(), None if shows is None else shows.numpy(),
                              None if clicks is None else clicks.numpy())


class _DenseTable:
    def __init__(self, value, rule, lr, beta1=0.9, beta2=0.999, eps=1e-8, sync_trainers=1):
        self.w = value.detach().float().reshape(-1).clone()
        self.rule, self.lr, self.b1, self.b2, self.eps = rule, lr, beta1, beta2, eps
        self.m = torch.zeros_like(self.w) if rule == "adam" else None
        self.v = torch.zeros_like(self.w) if rule == "adam" else None
        self.t = 0
        self.version = 0
        self.sync = sync_trainers
        self.acc = torch.zeros_like(self.w)
        self.count = 0
        self.cv = threading.Condition()

    def apply(self, g):
        if self.rule == "adam":
            self.t += 1
            self.m.mul_(self.b1).add_(g, alpha=1 - self.b1)
            self.v.mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
            lr_t = self.lr * (1 - self.b2 ** self.t) ** 0.5 / (1 - self.b1 ** self.t)
            self.w.addcdiv_(self.m, self.v.sqrt().add_(self.eps), value=-lr_t)
        else:
            self.w.add_(g, alpha=-self.lr)
        self.version += 1

    def push(self, g):
        with self.cv:
            if self.sync <= 1:
                self.apply(g)
            else:  # average the gradients of all trainers, then one update for this step
                self.acc.add_(g)
                self.count += 1
                if self.count == self.sync:
                    self.apply(self.acc.div_(self.sync))
                    self.acc.zero_()
                    self.count = 0
                    self.cv.notify_all()

    def pull(self, min_version):
        with self.cv:
            if not self.cv.wait_for(lambda: self.version >= min_version, timeout=600):
                raise TimeoutError(f"dense table: version {min_version} not reached (at {self.version}); "
                                   f"a trainer stopped pushing")
            return self.w.clone(), self.version


def _srv_create_dense(name, value, cfg):
    with _SRV["lock"]:
        if name not in _SRV["dense"]:
            ld = _SRV["load_dir"]
            path = os.path.join(ld, f"{name}.dense.pt") if ld else None
            if path and os.path.exists(path):
                value = torch.load(path, weights_only=True).reshape(-1)
            _SRV["dense"][name] = _DenseTable(value, cfg.get("rule", "sgd"), float(cfg.get("lr", 0.01)),
                                              sync_trainers=int(cfg.get("sync_trainers", 1)))
        return _SRV["dense"][name].version


def _srv_push_dense(name, grad):
    _SRV["dense"][name].push(grad)


def _srv_pull_dense(name, min_version):
    return _SRV["dense"][name].pull(min_version)


def _srv_barrier(key, n):
    cv = _SRV["cv"]
    with cv:
        _SRV["barriers"][key] = _SRV["barriers"].get(key, 0) + 1
        cv.notify_all()
        if not cv.wait_for(lambda: _SRV["barriers"][key] >= n, timeout=900):
            raise TimeoutError(f"barrier {key}: {_SRV['barriers'][key]} of {n} trainers arrived")
    return True


def _srv_save(dirname, mode):
    os.makedirs(dirname, exist_ok=True)
    n = 0
    for name, t in list(_SRV["sparse"].items()):
        n += t.save(_table_file(dirname, name, _SRV["index"]), int(mode))
    for name, d in list(_SRV["dense"].items()):
        torch.save(d.w, os.path.join(dirname, f"{name}.dense.pt"))
    return n


def _srv_load(dirname):
    n = 0
    for name, t in list(_SRV["sparse"].items()):
        p = _table_file(dirname, name, _SRV["index"])
        if os.path.exists(p):
            n += t.load(p)
    for name, d in list(_SRV["dense"].items()):
        p = os.path.join(dirname, f"{name}.dense.pt")
        if os.path.exists(p):
            d.w.copy_(torch.load(p, weights_only=True))
    return n


def _srv_shrink(threshold, decay):
    return sum(t.shrink(int(threshold), float(decay)) for t in _SRV["sparse"].values())


def _srv_sizes():
    return {k: t.size() for k, t in _SRV["sparse"].items()}


def _srv_set_lr(lr):
    for t in _SRV["sparse"].values():
        t.set_lr(float(lr))
    for d in _SRV["dense"].values():
        d.lr = float(lr)


# ----------------------------------------------------------------------------------------------- trainer side
class PsClient:
    """Routes table calls to the servers: sparse ids by ``id % n``, dense tables by a hash of the name."""

    def __init__(self, server_names):
        self.servers = list(server_names)
        self.n = len(self.servers)

    def _dense_server(self, name):
        return self.servers[zlib.crc32(name.encode()) % self.n]

    def _split(self, ids):
        owner = np.mod(ids, self.n)
        return [np.nonzero(owner == s)[0] for s in range(self.n)]

    def create_sparse(self, name, cfg):
        futs = [_rpc.rpc_async(s, _srv_create_sparse, args=(name, cfg)) for s in self.servers]
        return sum(f.wait() for f in futs)

    def pull_sparse(self, name, ids, dim, training=True):
        ids = np.ascontiguousarray(ids, dtype=np.int64)
        out = np.empty((ids.size, dim), dtype=np.float32)
        parts = self._split(ids)
        futs = [(p, _rpc.rpc_async(self.servers[s], _srv_pull_sparse,
                                   args=(name, torch.from_numpy(ids[p]), training)))
                for s, p in enumerate(parts) if p.size]
        for p, f in futs:
            out[p] = f.wait().numpy()
        return out

    def push_sparse_async(self, name, ids, grads, shows=None, clicks=None):
        ids = np.ascontiguousarray(ids, dtype=np.int64)
        grads = np.ascontiguousarray(grads, dtype=np.float32)
        futs = []
        for s, p in enumerate(self._split(ids)):
            if not p.size:
                continue
            sh = None if shows is None else torch.from_numpy(np.ascontiguousarray(shows[p], dtype=np.float32))
            ck = None if clicks is None else torch.from_numpy(np.ascontiguousarray(clicks[p], dtype=np.float32))
            futs.append(_rpc.rpc_async(self.servers[s], _srv_push_sparse,
                                       args=(name, torch.from_numpy(ids[p]), torch.from_numpy(grads[p]), sh, ck)))
        return futs

    def push_sparse(self, name, ids, grads, shows=None, clicks=None):
        for f in self.push_sparse_async(name, ids, grads, shows, clicks):
            f.wait()

    def create_dense(self, name, value, cfg):
        return _rpc.rpc_sync(self._dense_server(name), _srv_create_dense, args=(name, value.detach().cpu().float(),
                                                                                cfg))

    def push_dense(self, name, grad):
        return _rpc.rpc_async(self._dense_server(name), _srv_push_dense, args=(name, grad.detach().cpu().float()))

    def pull_dense(self, name, min_version=0):
        return _rpc.rpc_sync(self._dense_server(name), _srv_pull_dense, args=(name, min_version))

    def barrier(self, key, n):
        _rpc.rpc_sync(self.servers[0], _srv_barrier, args=(key, n))

    def save(self, dirname, mode=0):
        return sum(f.wait() for f in [_rpc.rpc_async(s, _srv_save, args=(dirname, mode)) for s in self.servers])

    def load(self, dirname):
        return sum(f.wait() for f in [_rpc.rpc_async(s, _srv_load, args=(dirname,)) for s in self.servers])

    def shrink(self, threshold, decay=0.98):
        return sum(f.wait() for f in [_rpc.rpc_async(s, _srv_shrink, args=(threshold, decay))
                                      for s in self.servers])

    def sizes(self):
        tot = {}
        for s in self.servers:
            for k, v in _rpc.rpc_sync(s, _srv_sizes).items():
                tot[k] = tot.get(k, 0) + v
        return tot

    def set_lr(self, lr):
        for f in [_rpc.rpc_async(s, _srv_set_lr, args=(lr,)) for s in self.servers]:
            f.wait()


class Communicator:
    """Trainer-side push path. ``sync``: pushes are sent (and awaited) in place. ``async``: pushes are queued to
    a background thread that merges gradients of repeated ids over up to ``max_merge`` queued pushes of the same
    table before sending (reference communicator.h AsyncCommunicator / MergeVars)."""

    def __init__(self, client, mode="sync", max_merge=20):
        self.client, self.mode, self.max_merge = client, mode, max_merge
        self._q = queue.Queue()
        self._err = None
        self._th = None
        if mode == "async":
            self._th = threading.Thread(target=self._loop, daemon=True)
            self._th.start()

    def push_sparse(self, name, ids, grads, shows=None, clicks=None):
        if self.mode != "async":
            self.client.push_sparse(name, ids, grads, shows, clicks)
            return
        self._raise()
        self._q.put(("sparse", name, ids, grads, shows, clicks))

    def push_dense(self, name, grad):
        if self.mode != "async":
            return self.client.push_dense(name, grad)
        self._raise()
        self._q.put(("dense", name, grad.detach().cpu().float().clone()))
        return None

    def _loop(self):
        while True:
            item = self._q.get()
            if item is None:
                self._q.task_done()
                return
            batch = [item]
            while len(batch) < self.max_merge:
                try:
                    nxt = self._q.get_nowait()
                except queue.Empty:
                    break
                batch.append(nxt)
            stop = batch[-1] is None
            if stop:
                batch.pop()
            try:
                self._send(batch)
            except Exception as e:  # surfaced on the trainer's next push / flush
                self._err = e
            for _ in range(len(batch) + int(stop)):
                self._q.task_done()
            if stop:
                return

    def _send(self, batch):
        sparse, dense = {}, {}
        for it in batch:
            if it[0] == "sparse":
                sparse.setdefault(it[1], []).append(it[2:])
            else:
                dense.setdefault(it[1], []).append(it[2])
        futs = []
        for name, items in sparse.items():
            ids = np.concatenate([i[0] for i in items])
            grads = np.concatenate([i[1] for i in items])
            uniq, inv = np.unique(ids, return_inverse=True)
            merged = np.zeros((uniq.size, grads.shape[1]), dtype=np.float32)
            np.add.at(merged, inv, grads)
            shows = clicks = None
            if items[0][2] is not None:
                shows = np.zeros(uniq.size, np.float32)
                np.add.at(shows, inv, np.concatenate([i[2] for i in items]))
            if items[0][3] is not None:
                clicks = np.zeros(uniq.size, np.float32)
                np.add.at(clicks, inv, np.concatenate([i[3] for i in items]))
            futs += self.client.push_sparse_async(name, uniq, merged, shows, clicks)
        for name, gs in dense.items():
            for g in gs:  # each trainer step is one update
                futs.append(self.client.push_dense(name, g))
        for f in futs:
            f.wait()

    def _raise(self):
        if self._err is not None:
            e, self._err = self._err, None
            raise RuntimeError(f"parameter-server async push failed: {e}") from e

    def flush(self):
        if self._th is not None:
            self._q.join()
        self._raise()

    def stop(self):
        if self._th is not None:
            self._q.put(None)
            self._th.join(timeout=600)
            self._th = None
        self._raise()


# ----------------------------------------------------------------------------------------------- runtime
class PsRuntime:
    """The process's PS role (reference TheOnePSRuntime + PaddleCloudRoleMaker in PS mode)."""

    def __init__(self, role_maker=None, strategy=None):
        rm = role_maker
        env = os.environ
        eps = (getattr(rm, "_server_endpoints", None) or env.get("PADDLE_PSERVERS_IP_PORT_LIST", "")).split(",")
        self.server_endpoints = [e for e in eps if e]
        if not self.server_endpoints:
            raise ValueError("parameter-server mode needs PADDLE_PSERVERS_IP_PORT_LIST (or a role maker with "
                             "server_endpoints)")
        self.n_servers = len(self.server_endpoints)
        self.n_trainers = int(getattr(rm, "_worker_num", None) or env.get("PADDLE_TRAINERS_NUM", "1"))
        role = getattr(rm, "_role", None) or env.get("TRAINING_ROLE", "TRAINER")
        self.role = "PSERVER" if str(role).upper() in ("PSERVER", "SERVER", "2") else "TRAINER"
        if self.role == "PSERVER":
            idx = getattr(rm, "_current_id", None)
            if idx is None:
                me = f"{env.get('POD_IP', '127.0.0.1')}:{env.get('PADDLE_PORT', '')}"
                idx = self.server_endpoints.index(me) if me in self.server_endpoints else int(
                    env.get("PADDLE_PSERVER_ID", "0"))
            self.index = int(idx)
        else:
            idx = getattr(rm, "_current_id", None)
            self.index = int(env.get("PADDLE_TRAINER_ID", "0") if idx is None else idx)
        self.master = env.get("PADDLE_PS_MASTER_ENDPOINT") or self.server_endpoints[0]
        strategy = strategy
        self.a_sync = bool(getattr(strategy, "a_sync", False))
        self.client = None
        self.comm = None
        self._started = False
        self._barrier_count = 0
        self.sparse_rule = {"rule": "adagrad", "lr": 0.05}
        self.dense_rule = {"rule": "sgd", "lr": 0.01}
        self._sparse_created = set()
        self._dense = {}  # name -> (param, version)

    # names / ranks in the RPC world: servers first, then trainers
    def _server_names(self):
        return [f"ps{i}" for i in range(self.n_servers)]

    def _my_name(self):
        return f"ps{self.index}" if self.role == "PSERVER" else f"trainer{self.index}"

    def _my_rank(self):
        return self.index if self.role == "PSERVER" else self.n_servers + self.index

    def _start_rpc(self):
        if not self._started:
            _rpc.init_rpc(self._my_name(), rank=self._my_rank(), world_size=self.n_servers + self.n_trainers,
                          master_endpoint=self.master)
            self._started = True

    # ------------------------------------------------------------ server
    def init_server(self, dirname=None, var_names=None, **kwargs):
        _srv_setup(self.index, self.n_trainers, dirname)
        self._start_rpc()

    def run_server(self):
        """Serve until every trainer has called stop_worker()."""
        self._start_rpc()
        _rpc.shutdown()
        self._started = False

    # ------------------------------------------------------------ worker
    def init_worker(self, scopes=None):
        self._start_rpc()
        self.client = PsClient(self._server_names())
        self.comm = Communicator(self.client, "async" if self.a_sync else "sync")

    def stop_worker(self):
        if self.comm is not None:
            self.comm.stop()
        self.barrier_worker()
        _rpc.shutdown()
        self._started = False

    def barrier_worker(self):
        if self.comm is not None:
            self.comm.flush()
        self._barrier_count += 1
        self.client.barrier(f"worker_barrier_{self._barrier_count}", self.n_trainers)

    def ensure_sparse(self, name, dim, cfg=None):
        if name in self._sparse_created:
            return
        c = dict(self.sparse_rule)
        c.update(cfg or {})
        c["dim"] = dim
        self.client.create_sparse(name, c)
        self._sparse_created.add(name)

    def register_dense(self, params):
        """Create a dense table per parameter, seeded by trainer 0's values so every trainer starts equal."""
        cfg = dict(self.dense_rule)
        cfg["sync_trainers"] = 1 if self.a_sync else self.n_trainers
        if self.index == 0:
            for p in params:
                self.client.create_dense(p.name, p._t, cfg)
        self.barrier_worker()
        for p in params:
            if self.index != 0:
                self.client.create_dense(p.name, p._t, cfg)
            w, ver = self.client.pull_dense(p.name, 0)
            with torch.no_grad():
                p._t.copy_(w.view_as(p._t).to(p._t.dtype))
            self._dense[p.name] = [p, ver]

    def dense_step(self, params):
        futs = []
        for p in params:
            if p.name not in self._dense:
                continue
            g = p._t.grad
            if g is None:
                if self.a_sync:
                    continue
                g = torch.zeros_like(p._t)  # sync mode: every trainer contributes to every step's average
            futs.append(self.comm.push_dense(p.name, g.reshape(-1)))
        for f in futs:
            if f is not None:
                f.wait()
        for p in params:
            if p.name not in self._dense:
                continue
            ent = self._dense[p.name]
            want = 0 if self.a_sync else ent[1] + 1
            w, ver = self.client.pull_dense(p.name, want)
            with torch.no_grad():
                p._t.copy_(w.view_as(p._t).to(p._t.dtype))
            ent[1] = ver

    def pull_dense(self, names=None):
        """Overwrite the registered dense parameters (all, or ``names``) with the servers' current values; returns
        how many were pulled (reference communicator.cc PullDense / RecvNoBarrier)."""
        n = 0
        for name, ent in self._dense.items():
            if names is not None and name not in names:
                continue
            w, ver = self.client.pull_dense(name, 0)
            with torch.no_grad():
                ent[0]._t.copy_(w.view_as(ent[0]._t).to(ent[0]._t.dtype))
            ent[1] = max(ent[1], ver)
            n += 1
        return n

    def save(self, dirname, mode=0):
        if self.comm is not None:
            self.comm.flush()
        return self.client.save(dirname, mode)

    def load(self, dirname):
        return self.client.load(dirname)

    def shrink(self, threshold, decay=0.98):
        return self.client.shrink(threshold, decay)


_RUNTIME = {"rt": None}


def get_runtime():
    return _RUNTIME["rt"]


def set_runtime(rt):
    _RUNTIME["rt"] = rt


# ----------------------------------------------------------------------------------------------- sparse lookup
class _PullPush(torch.autograd.Function):
    @staticmethod
    def forward(ctx, anchor, ids, rt, name, dim, training, shows, clicks):
        flat = ids.reshape(-1)
        uniq, inv = torch.unique(flat, return_inverse=True)
        uniq_np = uniq.cpu().numpy()
        rows = rt.client.pull_sparse(name, uniq_np, dim, training)
        table = torch.from_numpy(rows).to(device=anchor.device, dtype=anchor.dtype)
        ctx.rt, ctx.name, ctx.uniq, ctx.shape = rt, name, uniq_np, ids.shape
        ctx.save_for_backward(inv)
        ctx.n = uniq_np.size
        ctx.shows = None if shows is None else shows.reshape(-1)
        ctx.clicks = None if clicks is None else clicks.reshape(-1)
        return table[inv].view(*ids.shape, dim)

    @staticmethod
    def backward(ctx, dy):
        (inv,) = ctx.saved_tensors
        dim = dy.shape[-1]
        g = torch.zeros(ctx.n, dim, dtype=torch.float32, device=dy.device)
        g.index_add_(0, inv, dy.reshape(-1, dim).float())
        shows = torch.zeros(ctx.n, dtype=torch.float32, device=dy.device)
        shows.index_add_(0, inv, torch.ones_like(inv, dtype=torch.float32) if ctx.shows is None
                         else ctx.shows.float().to(dy.device))
        clicks = None
        if ctx.clicks is not None:
            clicks = torch.zeros(ctx.n, dtype=torch.float32, device=dy.device)
            clicks.index_add_(0, inv, ctx.clicks.float().to(dy.device))
            clicks = clicks.cpu().numpy()
        ctx.rt.comm.push_sparse(ctx.name, ctx.uniq, g.cpu().numpy(), shows.cpu().numpy(), clicks)
        return None, None, None, None, None, None, None, None


def sparse_lookup(ids, name, dim, training=True, padding_idx=None, cfg=None, shows=None, clicks=None,
                  dtype=torch.float32):
    """Rows of PS sparse table ``name`` for integer ``ids`` (any shape) -> ids.shape + [dim]; the backward
    pushes the summed gradient of every unique id. ``padding_idx`` rows are zeros and get no update."""
    rt = get_runtime()
    if rt is None or rt.client is None:
        raise RuntimeError("sparse_embedding needs an initialised parameter-server worker "
                           "(fleet.init(role_maker) in PS mode + fleet.init_worker())")
    rt.ensure_sparse(name, dim, cfg)
    anchor = torch.zeros((), dtype=dtype, device=ids.device, requires_grad=training and torch.is_grad_enabled())
    out = _PullPush.apply(anchor, ids, rt, name, dim, training, shows, clicks)
    if padding_idx is not None:
        out = out * (ids != padding_idx).unsqueeze(-1).to(out.dtype)
    return out
