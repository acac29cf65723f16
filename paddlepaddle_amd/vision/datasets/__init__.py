"""paddle.vision.datasets. Reference: python/paddle/vision/datasets/{mnist,cifar,flowers,voc2012,folder}.py.

There is no network: every dataset reads local files in the upstream formats (IDX for MNIST,
CIFAR python / binary tarballs, Flowers jpg tarball + .mat labels, VOC2012 tarball, image folders).
CIFAR python batches are read with a restricted unpickler that only builds plain containers and
numpy arrays (no code execution). ``download=True`` without local files raises.
"""
from __future__ import annotations

import gzip
import io
import os
import pickle
import struct
import tarfile

import numpy as np

from ...io import Dataset

IMG_EXTENSIONS = (".jpg", ".jpeg", ".png", ".ppm", ".bmp", ".pgm", ".tif", ".tiff", ".webp")


def _need(path, what):
    if path is None or not os.path.exists(path):
        raise FileNotFoundError(f"{what}: local file {path!r} not found (no network; downloads are disabled)")


def _pil_loader(path_or_bytes):
    from PIL import Image
    f = io.BytesIO(path_or_bytes) if isinstance(path_or_bytes, bytes) else open(path_or_bytes, "rb")
    with f:
        img = Image.open(f)
        return img.convert("RGB")


def _backend_out(img, backend):
    if backend == "cv2" or backend == "numpy":
        return np.asarray(img)
    return img


# ---------------------------------------------------------------------------- MNIST
class MNIST(Dataset):
    NAME = "mnist"

    def __init__(self, image_path=None, label_path=None, mode="train", transform=None, download=False, backend=None):
        assert mode in ("train", "test")
        _need(image_path, f"{self.NAME} images")
        _need(label_path, f"{self.NAME} labels")
        self.mode, self.transform, self.backend = mode, transform, backend or "pil"
        self.images = self._read_idx(image_path).astype("float32")
        self.labels = self._read_idx(label_path).astype("int64").reshape(-1, 1)

    @staticmethod
    def _read_idx(path):
        op = gzip.open if path.endswith(".gz") else open
        with op(path, "rb") as f:
            data = f.read()
        zero, dtype_code, nd = struct.unpack(">HBB", data[:4])
        dims = struct.unpack(">" + "I" * nd, data[4:4 + 4 * nd])
        arr = np.frombuffer(data, dtype=np.uint8, offset=4 + 4 * nd)
        return arr.reshape(dims)

    def __getitem__(self, idx):
        img, label = self.images[idx], self.labels[idx]
        if self.backend == "pil":
            from PIL import Image
            img = Image.fromarray(img.astype("uint8"), mode="L")
        if self.transform is not None:
            img = self.transform(img)
        if self.backend == "pil" and not hasattr(img, "shape"):
            img = np.asarray(img, dtype="float32")
        return img, label

    def __len__(self):
        return len(self.labels)


class FashionMNIST(MNIST):
    NAME = "fashion-mnist"


# ---------------------------------------------------------------------------- CIFAR
class _RestrictedUnpickler(pickle.Unpickler):
    _OK = {("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
           ("numpy", "ndarray"), ("numpy", "dtype"), ("numpy.core.multiarray", "scalar"),
           ("numpy._core.multiarray", "scalar")}

    def find_class(self, module, name):
        if (module, name) in self._OK:
            import importlib
            return getattr(importlib.import_module(module), name)
        raise pickle.UnpicklingError(f"refusing to load {module}.{name} from a dataset file")


class Cifar10(Dataset):
    _N_CLASSES = 10
    _TRAIN = "data_batch"
    _TEST = "test_batch"
    _LABEL = b"labels"

    def __init__(self, data_file=None, mode="train", transform=None, download=False, backend=None):
        assert mode in ("train", "test")
        _need(data_file, f"cifar-{self._N_CLASSES}")
        self.mode, self.transform, self.backend = mode, transform, backend or "pil"
        self.data = []
        key = self._TRAIN if mode == "train" else self._TEST
        with tarfile.open(data_file, "r:*") as tf:
            names = sorted(m.name for m in tf.getmembers() if m.isfile())
            for n in names:
                base = os.path.basename(n)
                if n.endswith(".bin") and (("test" in base) == (mode == "test")):
                    self._read_binary(tf.extractfile(n).read())
                elif base.startswith(key):
                    d = _RestrictedUnpickler(io.BytesIO(tf.extractfile(n).read()), encoding="bytes").load()
                    imgs = d[b"data"].reshape(-1, 3, 32, 32)
                    labels = d.get(self._LABEL, d.get(b"labels"))
                    for im, lb in zip(imgs, labels):
                        self.data.append((im, int(lb)))

    def _read_binary(self, raw):
        rec = 1 + 3072 if self._N_CLASSES == 10 else 2 + 3072
        a = np.frombuffer(raw, np.uint8).reshape(-1, rec)
        lab = a[:, 0] if self._N_CLASSES == 10 else a[:, 1]
        for row, lb in zip(a[:, rec - 3072:], lab):
            self.data.append((row.reshape(3, 32, 32), int(lb)))

    def __getitem__(self, idx):
        img, label = self.data[idx]
        img = np.transpose(img, (1, 2, 0))
        if self.backend == "pil":
            from PIL import Image
            img = Image.fromarray(img)
        if self.transform is not None:
            img = self.transform(img)
        if self.backend == "pil" and not hasattr(img, "shape"):
            img = np.asarray(img, dtype="float32")
        return img, np.array(label).astype("int64")

    def __len__(self):
        return len(self.data)


class Cifar100(Cifar10):
    _N_CLASSES = 100
    _TRAIN = "train"
    _TEST = "test"
    _LABEL = b"fine_labels"


# ---------------------------------------------------------------------------- Flowers
class Flowers(Dataset):
    def __init__(self, data_file=None, label_file=None, setid_file=None, mode="train", transform=None,
                 download=False, backend=None):
        for p, w in ((data_file, "flowers images"), (label_file, "flowers labels"), (setid_file, "flowers setid")):
            _need(p, w)
        import scipy.io
        self.transform, self.backend = transform, backend or "pil"
        self.labels = scipy.io.loadmat(label_file)["labels"][0]
        key = {"train": "tstid", "valid": "valid", "test": "trnid"}[mode]  # reference swaps train/test sizes
        self.indexes = scipy.io.loadmat(setid_file)[key][0]
        self.tar = tarfile.open(data_file, "r:*")
        self.names = {os.path.basename(m.name): m for m in self.tar.getmembers() if m.isfile()}

    def __getitem__(self, idx):
        i = int(self.indexes[idx])
        m = self.names[f"image_{i:05d}.jpg"]
        img = _pil_loader(self.tar.extractfile(m).read())
        img = _backend_out(img, self.backend)
        if self.transform is not None:
            img = self.transform(img)
        return img, np.array([self.labels[i - 1]]).astype("int64")

    def __len__(self):
        return len(self.indexes)


# ---------------------------------------------------------------------------- VOC2012
class VOC2012(Dataset):
    def __init__(self, data_file=None, mode="train", transform=None, download=False, backend=None):
        _need(data_file, "VOC2012")
        self.transform, self.backend = transform, backend or "pil"
        self.tar = tarfile.open(data_file, "r:*")
        self.members = {m.name: m for m in self.tar.getmembers() if m.isfile()}
        split = {"train": "train", "valid": "val", "test": "val"}[mode]
        lst = [k for k in self.members if k.endswith(f"ImageSets/Segmentation/{split}.txt")]
        if not lst:
            raise FileNotFoundError(f"VOC2012: no ImageSets/Segmentation/{split}.txt in {data_file}")
        root = lst[0].split("ImageSets/")[0]
        self.root = root
        self.ids = [l.strip() for l in self.tar.extractfile(self.members[lst[0]]).read().decode().split() if l.strip()]

    def __getitem__(self, idx):
        from PIL import Image
        i = self.ids[idx]
        img = _pil_loader(self.tar.extractfile(self.members[f"{self.root}JPEGImages/{i}.jpg"]).read())
        lab = Image.open(io.BytesIO(self.tar.extractfile(self.members[f"{self.root}SegmentationClass/{i}.png"]).read()))
        img, lab = _backend_out(img, self.backend), _backend_out(lab, self.backend)
        if self.transform is not None:
            img = self.transform(img)
        return img, np.asarray(lab)

    def __len__(self):
        return len(self.ids)


# ---------------------------------------------------------------------------- folders
def has_valid_extension(filename, extensions):
    return filename.lower().endswith(tuple(extensions))


def make_dataset(dir, class_to_idx, extensions=IMG_EXTENSIONS, is_valid_file=None):
    out = []
    check = is_valid_file or (lambda p: has_valid_extension(p, extensions))
    for target in sorted(class_to_idx):
        d = os.path.join(dir, target)
        for root, _, fnames in sorted(os.walk(d, followlinks=True)):
            for f in sorted(fnames):
                p = os.path.join(root, f)
                if check(p):
                    out.append((p, class_to_idx[target]))
    return out


class DatasetFolder(Dataset):
    def __init__(self, root, loader=None, extensions=None, transform=None, is_valid_file=None):
        self.root = root
        classes = sorted(d.name for d in os.scandir(root) if d.is_dir())
        self.classes = classes
        self.class_to_idx = {c: i for i, c in enumerate(classes)}
        exts = extensions if extensions is not None else (None if is_valid_file else IMG_EXTENSIONS)
        self.samples = make_dataset(root, self.class_to_idx, exts or IMG_EXTENSIONS, is_valid_file)
        if not self.samples:
            raise RuntimeError(f"found 0 files in subfolders of {root}")
        self.targets = [s[1] for s in self.samples]
        self.loader = loader or _pil_loader
        self.transform = transform

    def __getitem__(self, index):
        path, target = self.samples[index]
        sample = self.loader(path)
        if self.transform is not None:
            sample = self.transform(sample)
        return sample, target

    def __len__(self):
        return len(self.samples)


class ImageFolder(Dataset):
    """Flat (unlabelled) image folder."""

    def __init__(self, root, loader=None, extensions=None, transform=None, is_valid_file=None):
        self.root = root
        check = is_valid_file or (lambda p: has_valid_extension(p, extensions or IMG_EXTENSIONS))
        self.samples = [os.path.join(r, f) for r, _, fs in sorted(os.walk(root, followlinks=True)) for f in sorted(fs)
                        if check(os.path.join(r, f))]
        if not self.samples:
            raise RuntimeError(f"found 0 files in {root}")
        self.loader = loader or _pil_loader
        self.transform = transform

    def __getitem__(self, index):
        s = self.loader(self.samples[index])
        if self.transform is not None:
            s = self.transform(s)
        return [s]

    def __len__(self):
        return len(self.samples)
