"""fleet.utils file-system helpers (reference: python/paddle/distributed/fleet/utils/fs.py): LocalFS is
the real implementation; HDFSClient keeps the API and shells out to a `hadoop` binary when present."""
from __future__ import annotations

import os
import shutil
import subprocess


class FS:
    pass


class LocalFS(FS):
    def ls_dir(self, fs_path):
        if not self.is_exist(fs_path):
            return [], []
        dirs, files = [], []
        for f in os.listdir(fs_path):
            (dirs if os.path.isdir(os.path.join(fs_path, f)) else files).append(f)
        return dirs, files

    def mkdirs(self, fs_path):
        os.makedirs(fs_path, exist_ok=True)

    def rename(self, fs_src_path, fs_dst_path):
        os.rename(fs_src_path, fs_dst_path)

    def delete(self, fs_path):
        if os.path.isdir(fs_path):
            shutil.rmtree(fs_path)
        elif os.path.exists(fs_path):
            os.remove(fs_path)

    def need_upload_download(self):
        return False

    def is_file(self, fs_path):
        return os.path.isfile(fs_path)

    def is_dir(self, fs_path):
        return os.path.isdir(fs_path)

    def is_exist(self, fs_path):
        return os.path.exists(fs_path)

    def touch(self, fs_path, exist_ok=True):
        if os.path.exists(fs_path) and not exist_ok:
            raise FileExistsError(fs_path)
        open(fs_path, "a").close()

    def mv(self, src_path, dst_path, overwrite=False, test_exists=False):
        if overwrite and self.is_exist(dst_path):
            self.delete(dst_path)
        shutil.move(src_path, dst_path)

    def list_dirs(self, fs_path):
        return self.ls_dir(fs_path)[0]

    def upload(self, local_path, fs_path):
        shutil.copy(local_path, fs_path)

    def download(self, fs_path, local_path):
        shutil.copy(fs_path, local_path)

    def cat(self, fs_path=None):
        with open(fs_path) as f:
            return f.read()


class HDFSClient(FS):
    def __init__(self, hadoop_home, configs, time_out=5 * 60 * 1000, sleep_inter=1000):
        self._bin = os.path.join(hadoop_home, "bin", "hadoop")
        self._cfg = " ".join(f"-D{k}={v}" for k, v in (configs or {}).items())
        self._timeout = time_out / 1000.0

    def _run(self, *args):
        if not os.path.exists(self._bin):
            raise RuntimeError(f"hadoop binary not found at {self._bin}")
        cmd = [self._bin, "fs"] + self._cfg.split() + list(args)
        return subprocess.run(cmd, capture_output=True, text=True, timeout=self._timeout)

    def is_exist(self, fs_path):
        return self._run("-test", "-e", fs_path).returncode == 0

    def is_dir(self, fs_path):
        return self._run("-test", "-d", fs_path).returncode == 0

    def is_file(self, fs_path):
        return self.is_exist(fs_path) and not self.is_dir(fs_path)

    def ls_dir(self, fs_path):
        r = self._run("-ls", fs_path)
        dirs, files = [], []
        for line in r.stdout.splitlines():
            parts = line.split()
            if len(parts) >= 8:
                (dirs if parts[0].startswith("d") else files).append(os.path.basename(parts[-1]))
        return dirs, files

    def mkdirs(self, fs_path):
        self._run("-mkdir", "-p", fs_path)

    def delete(self, fs_path):
        self._run("-rm", "-r", "-f", fs_path)

    def upload(self, local_path, fs_path, multi_processes=1, overwrite=False):
        self._run("-put", *(["-f"] if overwrite else []), local_path, fs_path)

    def download(self, fs_path, local_path, multi_processes=1, overwrite=False):
        self._run("-get", fs_path, local_path)

    def need_upload_download(self):
        return True


class DistributedInfer:
    """Inference helper of the PS mode: in collective mode it simply runs the given program / layer."""

    def __init__(self, main_program=None, startup_program=None):
        self.main_program, self.startup_program = main_program, startup_program

    def init_distributed_infer_env(self, exe, loss, role_maker=None, dirname=None):
        return None

    def get_dist_infer_program(self):
        return self.main_program
