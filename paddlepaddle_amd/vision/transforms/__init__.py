"""paddle.vision.transforms."""
from .transforms import (Compose, BaseTransform, ToTensor, Resize, RandomResizedCrop, CenterCrop,  # noqa: F401
                         RandomHorizontalFlip, RandomVerticalFlip, Normalize, Transpose, BrightnessTransform,
                         ContrastTransform, SaturationTransform, HueTransform, ColorJitter, RandomCrop, Pad,
                         RandomAffine, RandomRotation, RandomPerspective, Grayscale, RandomErasing)
from .functional import (to_tensor, resize, pad, crop, center_crop, hflip, vflip, adjust_brightness,  # noqa: F401
                         adjust_contrast, adjust_saturation, adjust_hue, affine, rotate, perspective, to_grayscale,
                         normalize, erase)
from . import functional  # noqa: F401
