"""paddle.dataset: legacy reader creators (reference python/paddle/dataset/). There is no network here:
each creator reads the standard files from a local directory (``data_dir`` / PADDLE_AMD_DATA_HOME) through
the paddle.vision / paddle.text dataset classes and yields the legacy sample tuples."""
from __future__ import annotations

import os

__all__ = []


def _home(data_dir):
    return data_dir or os.environ.get("PADDLE_AMD_DATA_HOME", os.path.expanduser("~/.cache/paddle/dataset"))


class mnist:
    @staticmethod
    def _reader(mode, data_dir=None):
        def reader():
            from ..vision.datasets import MNIST
            d = _home(data_dir)
            ds = MNIST(image_path=os.path.join(d, f"{'train' if mode == 'train' else 't10k'}-images-idx3-ubyte.gz"),
                       label_path=os.path.join(d, f"{'train' if mode == 'train' else 't10k'}-labels-idx1-ubyte.gz"),
                       mode=mode)
            for img, lab in ds:
                import numpy as np
                x = np.asarray(img, dtype="float32").reshape(-1) / 255.0 * 2.0 - 1.0
                yield x, int(np.asarray(lab).reshape(-1)[0])
        return reader

    @staticmethod
    def train(data_dir=None):
        return mnist._reader("train", data_dir)

    @staticmethod
    def test(data_dir=None):
        return mnist._reader("test", data_dir)


class cifar:
    @staticmethod
    def _reader(mode, cls, data_dir=None):
        def reader():
            import numpy as np
            from ..vision import datasets as D
            ds = getattr(D, cls)(data_file=os.path.join(_home(data_dir), "cifar-10-python.tar.gz" if cls == "Cifar10"
                                                        else "cifar-100-python.tar.gz"), mode=mode)
            for img, lab in ds:
                yield np.asarray(img, dtype="float32").reshape(-1) / 255.0, int(np.asarray(lab).reshape(-1)[0])
        return reader

    @staticmethod
    def train10(data_dir=None):
        return cifar._reader("train", "Cifar10", data_dir)

    @staticmethod
    def test10(data_dir=None):
        return cifar._reader("test", "Cifar10", data_dir)

    @staticmethod
    def train100(data_dir=None):
        return cifar._reader("train", "Cifar100", data_dir)

    @staticmethod
    def test100(data_dir=None):
        return cifar._reader("test", "Cifar100", data_dir)


class uci_housing:
    """13 features -> price; reads housing.data (whitespace separated), features normalised like the
    reference (x - mean) / (max - min), 80 / 20 train / test split."""

    @staticmethod
    def _load(data_dir=None):
        import numpy as np
        path = os.path.join(_home(data_dir), "housing.data")
        data = np.fromfile(path, sep=" ").reshape(-1, 14).astype("float32")
        mx, mn, avg = data.max(0), data.min(0), data.mean(0)
        data[:, :13] = (data[:, :13] - avg[:13]) / (mx[:13] - mn[:13])
        cut = int(data.shape[0] * 0.8)
        return data[:cut], data[cut:]

    @staticmethod
    def train(data_dir=None):
        def reader():
            for row in uci_housing._load(data_dir)[0]:
                yield row[:-1], row[-1:]
        return reader

    @staticmethod
    def test(data_dir=None):
        def reader():
            for row in uci_housing._load(data_dir)[1]:
                yield row[:-1], row[-1:]
        return reader


class common:
    DATA_HOME = _home(None)

    @staticmethod
    def download(url, module_name, md5sum, save_name=None):
        raise RuntimeError("paddle.dataset.common.download: no network access; place the file under "
                           f"{_home(None)}/{module_name}")
