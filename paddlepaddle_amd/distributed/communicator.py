"""paddle.distributed.communicator (reference: python/paddle/distributed/communicator.py): the trainer-side
parameter-server communicator handle of a static program, plus LargeScaleKV.

``Communicator`` fronts this framework's PS push path (distributed/ps/the_one_ps.py Communicator: sync pushes in
place, async pushes merged by a background thread). Without a parameter-server runtime (collective or
single-process jobs) it is a local handle whose start / stop / is_running track the run state only, as the
reference's communicator does before a PS context is attached.
"""
from __future__ import annotations

import numpy as np

__all__ = ["Communicator", "FLCommunicator", "LargeScaleKV"]


class Communicator:
    def __init__(self, program=None, mode=None, kwargs=None, envs=None):
        self.program = program
        self.mode = {None: "async", "ASYNC": "async", "SYNC": "sync", "GEO": "async", "HALF_ASYNC": "async"}.get(
            str(mode).upper() if mode is not None else None, str(mode).lower() if mode else "async")
        self.kwargs = dict(kwargs or {})
        self.envs = dict(envs or {})
        self._running = False
        self._impl = None

    def init_with_ctx(self, send_ctx=None, recv_ctx=None, proto_txt=None, unit64_hosts=None, scope=None):
        from .ps import the_one_ps as _ps
        rt = _ps.get_runtime()
        if rt is not None and getattr(rt, "client", None) is not None:
            self._impl = _ps.Communicator(rt.client, mode=self.mode)
        return self

    def create_client_to_client_connection(self, *a, **k):
        return None

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
        if self._impl is not None:
            self._impl.stop()
        self._running = False

    def is_running(self):
        return self._running

    def recv(self):
        if self._impl is not None:
            self._impl.flush()

    def push_sparse_param(self, var_name, table_id=-1, scope=None):
        if self._impl is not None:
            self._impl.flush()

    def pull_dense(self, context):
        return None


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
