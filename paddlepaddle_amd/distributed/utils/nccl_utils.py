"""Reference: python/paddle/distributed/utils/nccl_utils.py (version checks; RCCL here)."""
import torch


def _version():
    try:
        v = torch.cuda.nccl.version()
    except Exception:  # noqa: BLE001 - no RCCL in this build
        return 0
    if isinstance(v, tuple):
        return v[0] * 10000 + v[1] * 100 + v[2]
    return int(v)


def get_nccl_version_str(ver):
    if ver >= 10000:
        major, rest = divmod(ver, 10000)
        minor, patch = divmod(rest, 100)
    else:
        major, rest = divmod(ver, 1000)
        minor, patch = divmod(rest, 100)
    return f"{major}.{minor}.{patch}"


def check_nccl_version_for_p2p():
    return _version() >= 20804


def check_nccl_version_for_bf16():
    return _version() >= 21000
