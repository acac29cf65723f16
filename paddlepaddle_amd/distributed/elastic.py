"""Elastic job control: read / change the desired worker count of a running elastic job.

Reference: python/paddle/distributed/elastic.py (``Command`` over etcd: set_np / scale_np / clean, CLI
``--elastic_server --job_id --np <action>``) and fleet/elastic/manager.py (launchers watch the np key and
restart the job at the new size). Here the store is a c10d TCPStore at ``--elastic_server``: the node-0
launcher hosts it (``host=True``), this CLI and other launchers connect to it — no etcd dependency.

    python -m paddlepaddle_amd.distributed.elastic --elastic_server 127.0.0.1:2379 --job_id j --np 4 scale
"""
from __future__ import annotations

import argparse
from datetime import timedelta


class Command:
    def __init__(self, server, name, host=False, timeout=30):
        from torch.distributed import TCPStore
        srv, port = server.rsplit(":", 1)
        self.store = TCPStore(srv, int(port), is_master=bool(host), timeout=timedelta(seconds=timeout),
                              wait_for_workers=False)
        self.prefix = "/paddle/" + name
        self.np_path = self.prefix + "/np"

    def get_np(self):
        if not self.store.check([self.np_path]):
            return None
        v = self.store.get(self.np_path).decode()
        return int(v) if v else None

    def set_np(self, np):
        self.store.set(self.np_path, str(int(np)))

    def scale_np(self, np):
        if self.get_np() is not None:
            self.set_np(np)
            return True
        return False

    def clean(self):
        if self.store.check([self.np_path]):
            self.store.delete_key(self.np_path)

    def close(self):
        self.store = None


def main(argv=None):
    p = argparse.ArgumentParser(description="Elastic Command")
    p.add_argument("--elastic_server", type=str, help="key-value store host:port")
    p.add_argument("--job_id", type=str, help="job unique id")
    p.add_argument("--np", type=str, help="job worker number")
    p.add_argument("action", type=str, help="scale | clean")
    a = p.parse_args(argv)
    cmd = Command(a.elastic_server, a.job_id)
    if a.action == "scale":
        ok = cmd.scale_np(int(str(a.np).split(":")[0]))
        print("scale np {} {}".format(a.np, "ok" if ok else "failed: job not running"))
    elif a.action == "clean":
        cmd.clean()
    cmd.close()


if __name__ == "__main__":
    main()
