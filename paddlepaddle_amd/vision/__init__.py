"""paddle.vision. Reference: python/paddle/vision/ (models, transforms, datasets, ops, image)."""
from . import models  # noqa: F401
from .models import *  # noqa: F401,F403
from . import transforms, datasets, ops  # noqa: F401
from .datasets import (MNIST, VOC2012, Cifar10, Cifar100, DatasetFolder, FashionMNIST,  # noqa: F401
                       Flowers, ImageFolder)
from .transforms import (  # noqa: F401
    BaseTransform,
    BrightnessTransform,
    CenterCrop,
    ColorJitter,
    Compose,
    ContrastTransform,
    Grayscale,
    HueTransform,
    Normalize,
    Pad,
    RandomCrop,
    RandomHorizontalFlip,
    RandomResizedCrop,
    RandomRotation,
    RandomVerticalFlip,
    Resize,
    SaturationTransform,
    ToTensor,
    Transpose,
    adjust_brightness,
    adjust_contrast,
    adjust_hue,
    center_crop,
    crop,
    hflip,
    normalize,
    pad,
    resize,
    rotate,
    to_grayscale,
    to_tensor,
    vflip,
)

_image_backend = "pil"


def set_image_backend(backend):
    global _image_backend
    if backend not in ("pil", "cv2", "tensor"):
        raise ValueError(f"unknown image backend {backend}")
    _image_backend = backend


def get_image_backend():
    return _image_backend


def image_load(path, backend=None):
    from PIL import Image
    import numpy as np
    backend = backend or _image_backend
    img = Image.open(path)
    if backend == "pil":
        return img
    a = np.asarray(img.convert("RGB"))
    if backend == "cv2":
        return a[..., ::-1].copy()  # BGR like OpenCV
    from ..framework.tensor import to_tensor
    return to_tensor(a.transpose(2, 0, 1).copy())
