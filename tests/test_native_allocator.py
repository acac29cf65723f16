"""Native auto-growth best-fit allocator (csrc/runtime/allocator.h). CPU: the core on host memory (best fit,
split / coalesce, chunk growth, per-stream pools, cross-stream reuse, release, stats). GPU: a training loop
in a child process with the allocator installed for every device buffer. Reference:
paddle/phi/core/memory/allocation/auto_growth_best_fit_allocator.cc, stream_safe_cuda_allocator.cc
(test/cpp/.../auto_growth_best_fit_allocator_test.cc)."""
import json
import os
import subprocess
import sys

import pytest

from paddlepaddle_amd.utils import native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MB = 1 << 20


def _alloc(min_chunk=4 * MB):
    m = native.module()
    if m is None or not hasattr(m, "HostAllocator"):
        pytest.skip("native runtime not built")
    return m.HostAllocator(min_chunk)


def test_growth_split_and_best_fit():
    a = _alloc()
    p1 = a.allocate(1000)
    s = a.stats()
    assert s["n_chunks"] == 1 and s["reserved"] == 4 * MB and s["allocated"] == 1024  # 512-B granules
    p2 = a.allocate(3000)
    assert p2 == p1 + 1024  # carved from the same chunk, right after p1
    big = a.allocate(6 * MB)  # larger than a chunk: its own region
    assert a.stats()["n_chunks"] == 2
    a.free(p1)
    # best fit: a 512-B request takes the freed 1 KiB hole, not the chunk tail
    p3 = a.allocate(512)
    assert p3 == p1
    for p in (p2, p3, big):
        assert a.free(p)
    assert a.stats()["allocated"] == 0
    assert a.free_blocks() == 2  # every chunk coalesced back into one free block


def test_coalesce_both_neighbours():
    a = _alloc()
    ps = [a.allocate(4096) for _ in range(3)]
    a.free(ps[0])
    a.free(ps[2])
    n_before = a.free_blocks()
    a.free(ps[1])  # merges with the free blocks on both sides and the chunk tail
    assert n_before == 2 and a.free_blocks() == 1
    assert a.stats()["allocated"] == 0


def test_streams_keep_own_pools_and_cross_stream_reuse():
    a = _alloc(min_chunk=1 * MB)
    p = a.allocate(1 * MB, stream=1)  # fills a whole chunk of stream 1
    a.free(p)
    q = a.allocate(4096, stream=2)    # stream 2 may take stream 1's free block (after an event wait)
    s = a.stats()
    assert q == p and s["n_cross_stream"] == 1 and s["n_chunks"] == 1
    r = a.allocate(4096, stream=2)    # the remainder now belongs to stream 2: no further cross-stream take
    assert a.stats()["n_cross_stream"] == 1 and r == q + 4096
    a.free(q)
    a.free(r)


def test_release_free_chunks_and_peaks():
    a = _alloc()
    ps = [a.allocate(3 * MB) for _ in range(4)]
    s = a.stats()
    assert s["peak_allocated"] == 12 * MB and s["n_raw_alloc"] == 4
    for p in ps[:3]:
        a.free(p)
    freed = a.release()
    s = a.stats()
    assert freed == 3 * 4 * MB and s["n_chunks"] == 1 and s["reserved"] == 4 * MB
    assert not a.free(12345)  # not ours
    a.free(ps[3])


_CHILD = r"""
import json, os, sys
sys.path.insert(0, os.environ["REPO"])
import paddlepaddle_amd as paddle
from paddlepaddle_amd.device import allocator as A
assert A.is_enabled()
paddle.seed(0)
net = paddle.nn.Sequential(paddle.nn.Linear(256, 1024), paddle.nn.GELU(), paddle.nn.Linear(1024, 256))
opt = paddle.optimizer.AdamW(1e-3, parameters=net.parameters())
x = paddle.randn([64, 256])
losses = []
for _ in range(5):
    loss = (net(x) ** 2).mean()
    loss.backward()
    opt.step()
    opt.clear_grad()
    losses.append(float(loss))
s = A.stats()
s["losses"] = losses
s["api_allocated"] = paddle.device.cuda.memory_allocated()
s["api_peak"] = paddle.device.cuda.max_memory_allocated()
print("JSON" + json.dumps(s))
"""


@pytest.mark.gpu
def test_native_allocator_drives_training_gpu():
    env = dict(os.environ, PADDLE_AMD_ALLOCATOR="auto_growth", REPO=ROOT)
    env.pop("PADDLE_AMD_FORCE_CPU", None)  # a CPU-parity test earlier in the same process may have set it
    r = subprocess.run([sys.executable, "-c", _CHILD], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    s = json.loads(r.stdout.split("JSON", 1)[1])
    assert s["n_alloc"] > 50 and s["n_chunks"] >= 1 and s["reserved"] >= s["peak_allocated"] > 0
    assert s["api_allocated"] == s["allocated"] and s["api_peak"] == s["peak_allocated"]
    assert s["losses"][-1] < s["losses"][0]


def test_graph_pool_isolation_and_release():
    a = _alloc(min_chunk=1 * MB)
    a.begin_pool(5, 1)                 # stream 5 is being captured into graph pool 1
    p = a.allocate(4096, stream=5)
    a.free(p)                          # freed during capture: stays in the graph's pool
    a.end_pool(5)
    q = a.allocate(4096, stream=5)     # after capture: ordinary allocations never reuse graph memory
    assert q != p
    r = a.allocate(4096, stream=9)
    assert r != p
    a.release_pool(1)                  # graph destroyed: its blocks rejoin stream 5's pool
    s = a.allocate(4096, stream=5)
    assert s == p
    for t in (q, r, s):
        a.free(t)
    assert a.stats()["allocated"] == 0


def test_graph_pool_chunks_survive_release_free_chunks():
    """empty_cache / OOM release must not hand a live graph pool's memory back to the driver."""
    a = _alloc(min_chunk=1 * MB)
    a.begin_pool(5, 7)
    p = a.allocate(4096, stream=5)     # the pool grows its own chunk during the capture
    a.free(p)                          # graph intermediates are freed once the capture ends
    a.end_pool(5)
    before = a.stats()["reserved"]
    a.release()                        # release_free_chunks: the pool chunk is free but still in use by replays
    assert a.stats()["reserved"] == before
    a.release_pool(7)                  # graph gone: now the chunk is idle and can go
    a.release()
    assert a.stats()["reserved"] == 0


def test_graph_pool_shared_by_two_graphs_is_refcounted():
    a = _alloc(min_chunk=1 * MB)
    a.begin_pool(5, 3)                 # graph A captures into pool 3
    p = a.allocate(4096, stream=5)
    a.free(p)
    a.end_pool(5)
    a.begin_pool(6, 3)                 # graph B shares pool 3
    q = a.allocate(4096, stream=6)
    a.free(q)
    a.end_pool(6)
    a.release_pool(3)                  # graph A reset: B still replays into the pool
    r = a.allocate(4096, stream=5)
    assert r not in (p, q)
    a.release_pool(3)                  # graph B reset: the pool's memory is ordinary again
    a.free(r)
    a.begin_pool(5, 3)                 # the id reused by a new capture: frees stay reserved for it
    s = a.allocate(4096, stream=5)
    a.free(s)
    a.end_pool(5)
    t = a.allocate(4096, stream=5)
    assert t != s
    a.free(t)


_CHILD_LOADER = r"""
import os, sys
sys.path.insert(0, os.environ["REPO"])
import numpy as np
import torch
import paddlepaddle_amd as paddle
from paddlepaddle_amd.device import allocator as A
assert A.is_enabled()

class DS(paddle.io.Dataset):
    def __len__(self):
        return 64
    def __getitem__(self, i):
        return np.full([1 << 16], float(i), dtype="float32")

loader = paddle.io.DataLoader(DS(), batch_size=4, shuffle=False)
sums = []
for b in loader:
    torch.cuda._sleep(5_000_000)          # a slow consumer: the batch is read long after it was yielded
    sums.append(b._t.sum())
    del b
got = torch.stack(sums).cpu().numpy()
want = np.array([sum(range(4 * k, 4 * k + 4)) * (1 << 16) for k in range(16)], dtype="float64")
assert np.allclose(got, want), (got, want)
print("LOADER_OK")
"""


@pytest.mark.gpu
def test_dataloader_slow_consumer_native_allocator_gpu():
    """Batches staged on the DataLoader's side stream are never overwritten while the compute stream still reads
    them, under the native allocator (which receives no record_stream calls)."""
    env = dict(os.environ, PADDLE_AMD_ALLOCATOR="auto_growth", REPO=ROOT)
    r = subprocess.run([sys.executable, "-c", _CHILD_LOADER], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "LOADER_OK" in r.stdout, r.stderr[-3000:]
