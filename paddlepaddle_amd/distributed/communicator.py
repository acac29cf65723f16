"""paddle.distributed.communicator (reference: python/paddle/distributed/communicator.py): the trainer-side
parameter-server communicator handle of a static program, plus LargeScaleKV.

``Communicator`` fronts this framework's PS runtime (distributed/ps/the_one_ps.py: sync pushes in place, async
pushes merged by a background thread, dense tables pulled back into the parameters). Without a parameter-server
worker (collective or single-process jobs) start / stop / is_running track the run state and the table calls
raise.
"""
from __future__ import annotations

import numpy as np

__all__ = ["Communicator", "FLCommunicator", "LargeScaleKV"]


def _names(context):
    """A pull / init context as parameter names: None (every registered table), a name, a parameter, or a
    list / dict of either (the reference passes a {var_name: CommContext} map)."""
    if context is None:
        return None
    if isinstance(context, dict):
        context = list(context)
    if not isinstance(context, (list, tuple, set)):
        context = [context]
    return {c if isinstance(c, str) else c.name for c in context}


class Communicator:
    """Reference: communicator.py:41-214 over core.DistCommunicator. Here the handle drives this framework's
    PS runtime (distributed/ps/the_one_ps.py): ``init_params`` creates the dense tables (trainer 0 seeds them),
    ``pull_dense`` / ``recv`` overwrite the local parameters with the servers' values (after draining queued
    async pushes), ``push_sparse_param`` drains the sparse push queue. The RPC world is fully connected once
    ``init_worker`` ran, so client-to-client connection set-up only checks that."""

    def __init__(self, program=None, mode=None, kwargs=None, envs=None):
        self.program = program
        self.mode = {None: "async", "ASYNC": "async", "SYNC": "sync", "GEO": "async", "HALF_ASYNC": "async"}.get(
            str(mode).upper() if mode is not None else None, str(mode).lower() if mode else "async")
        self.kwargs = dict(kwargs or {})
        self.envs = dict(envs or {})
        self._running = False
        self._impl = None
        self._rt = None
        self._clients = []

    def init_with_ctx(self, send_ctx=None, recv_ctx=None, proto_txt=None, unit64_hosts=None, scope=None):
        from .ps import the_one_ps as _ps
        rt = _ps.get_runtime()
        if rt is not None and getattr(rt, "client", None) is not None:
            self._rt = rt
            # the worker's own push path when its mode matches, else a handle of the requested mode
            own = rt.comm is not None and rt.comm.mode == self.mode
            self._impl = rt.comm if own else _ps.Communicator(rt.client, mode=self.mode)
        return self

    def _need(self):
        if self._impl is None:
            self.init_with_ctx()
        if self._rt is None:
            raise RuntimeError("Communicator: no parameter-server worker is running (fleet.init_worker() first)")
        return self._rt

    def create_client_to_client_connection(self, pserver_timeout_ms=500000, pserver_connect_timeout_ms=10000,
                                           max_retry=3):
        self._need()  # init_rpc already connected every pair of workers
        return True

    def get_client_info(self):
        from .ps import the_one_ps as _ps
        rt = _ps.get_runtime()
        return list(getattr(rt, "server_endpoints", []) if rt is not None else [])

    def set_clients(self, host_list):
        self._clients = list(host_list)

    def start(self):
        if self._impl is None:
            self.init_with_ctx()
        self._running = True

    def stop(self):
        if self._impl is not None and (self._rt is None or self._impl is not self._rt.comm):
            self._impl.stop()  # the worker's own push path is stopped by stop_worker()
        self._running = False

    def is_running(self):
        return self._running

    def init_params(self, context):
        params = list(context.values()) if isinstance(context, dict) else list(context)
        self._need().register_dense([p for p in params if not isinstance(p, str)])

    def pull_dense(self, context=None):
        rt = self._need()
        self._impl.flush()
        return rt.pull_dense(_names(context))

    def recv(self):
        return self.pull_dense(None)

    def push_sparse_param(self, var_name, table_id=-1, scope=None):
        self._need()
        self._impl.flush()


class FLCommunicator(Communicator):
    """Federated-learning communicator handle (reference: communicator.py FLCommunicator)."""

    def __init__(self, ps_hosts=None, kwargs=None):
        super().__init__(None, "SYNC", kwargs)
        self.ps_hosts = list(ps_hosts or [])

    def start_coordinator(self, self_endpoint=None, trainer_endpoints=None):
        self._running = True

    def save_fl_strategy(self, mp):
        self._strategy = dict(mp)

    def query_fl_clients_info(self):
        return dict(getattr(self, "_strategy", {}))


class LargeScaleKV:
    """A host-side id -> row table (reference: communicator.py LargeScaleKV over the C++ sparse table):
    save / load of named tables and their sizes."""

    def __init__(self):
        self._tables = {}

    def table(self, varname):
        return self._tables.setdefault(varname, {})

    def save(self, varname, dirname):
        import os
        t = self._tables.get(varname, {})
        os.makedirs(dirname, exist_ok=True)
        ids = np.array(sorted(t), dtype=np.int64)
        rows = np.stack([t[i] for i in ids]) if len(ids) else np.zeros((0, 0), np.float32)
        np.savez(os.path.join(dirname, varname + ".npz"), ids=ids, rows=rows)

    def load(self, varname, dirname):
        import os
        d = np.load(os.path.join(dirname, varname + ".npz"))
        self._tables[varname] = {int(i): r for i, r in zip(d["ids"], d["rows"])}

    def size(self, varname):
        return len(self._tables.get(varname, {}))
