"""Native pinned-host pool (csrc/runtime/pinned_pool.cpp) and the double-buffered DataLoader that
stages batches through it."""
import gc

import numpy as np
import pytest
import torch

import paddlepaddle_amd as paddle
from paddlepaddle_amd.device import pinned as P
from paddlepaddle_amd.utils import native


def test_best_fit_split_coalesce_cpu():
    pool = native.module().PinnedPool(1 << 20, 256, False)
    a = pool.allocate(1000)      # rounds to 1024
    b = pool.allocate(5000)
    c = pool.allocate(300)
    st = pool.stats()
    assert st["allocated"] == 1024 + 5120 + 512 and st["chunks"] == 1
    pool.deallocate(b)
    d = pool.allocate(4000)      # best fit reuses b's block
    assert d == b and pool.stats()["chunks"] == 1 and pool.stats()["reuse_hits"] == 3  # served from free blocks
    for p in (a, c, d):
        pool.deallocate(p)
    st = pool.stats()
    assert st["allocated"] == 0 and st["free_blocks"] == 1  # fully coalesced
    big = pool.allocate(3 << 20)  # larger than a chunk: dedicated chunk
    assert pool.stats()["chunks"] == 2
    pool.deallocate(big)
    assert pool.release_idle() == (1 << 20) + (3 << 20) and pool.stats()["reserved"] == 0
    with pytest.raises(ValueError):
        pool.deallocate(12345)


def test_pooled_tensor_lifetime_cpu():
    a = P.empty([4, 8], torch.float32)
    a.fill_(1.5)
    view = a[1:]
    live0 = P.stats()["live_blocks"]
    del a
    gc.collect()
    assert P.stats()["live_blocks"] == live0 and float(view.sum()) == 1.5 * 24
    del view
    gc.collect()
    assert P.stats()["live_blocks"] == live0 - 1
    t = paddle.to_tensor(np.arange(6, dtype="float32")).pin_memory()
    assert P.is_pooled(t._t) and t.numpy().tolist() == list(range(6))


@pytest.mark.gpu
def test_dataloader_double_buffered_h2d_gpu():
    paddle.set_device("gpu")
    data = np.random.RandomState(0).rand(64, 3, 8, 8).astype("float32")
    labels = np.arange(64).astype("int64")

    class DS(paddle.io.Dataset):
        def __getitem__(self, i):
            return data[i], labels[i]

        def __len__(self):
            return 64

    loader = paddle.io.DataLoader(DS(), batch_size=16, shuffle=False)
    seen = []
    for x, y in loader:
        assert x.place.is_gpu_place() if hasattr(x.place, "is_gpu_place") else x._t.is_cuda
        x._t.mul_(2)  # compute on the main stream while the next batch is staged
        seen.append((x.numpy(), y.numpy()))
    assert len(seen) == 4
    np.testing.assert_allclose(np.concatenate([s[0] for s in seen]), data * 2)
    np.testing.assert_array_equal(np.concatenate([s[1] for s in seen]), labels)
    st = P.stats()
    assert st["pinned"] and st["num_allocs"] >= 8
