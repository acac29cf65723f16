"""Transform classes. Reference: python/paddle/vision/transforms/transforms.py."""
from __future__ import annotations

import math
import numbers
import random

import numpy as np

from . import functional as F


def _get_image_size(img):
    return F._size(img)


class Compose:
    def __init__(self, transforms):
        self.transforms = list(transforms)

    def __call__(self, data):
        for t in self.transforms:
            data = t(data)
        return data

    def __repr__(self):
        return "Compose(" + ", ".join(type(t).__name__ for t in self.transforms) + ")"


class BaseTransform:
    def __init__(self, keys=None):
        self.keys = keys if keys is not None else ("image",)

    def _get_params(self, inputs):
        return None

    def __call__(self, inputs):
        if isinstance(inputs, tuple):
            self.params = self._get_params(inputs)
            out = []
            for k, x in zip(self.keys, inputs):
                fn = getattr(self, f"_apply_{k}", None)
                out.append(fn(x) if fn is not None else x)
            return tuple(out) + tuple(inputs[len(self.keys):])
        self.params = self._get_params((inputs,))
        return self._apply_image(inputs)

    def _apply_image(self, img):
        return img


class ToTensor(BaseTransform):
    def __init__(self, data_format="CHW", keys=None):
        super().__init__(keys)
        self.data_format = data_format

    def _apply_image(self, img):
        return F.to_tensor(img, self.data_format)


class Resize(BaseTransform):
    def __init__(self, size, interpolation="bilinear", keys=None):
        super().__init__(keys)
        self.size, self.interpolation = size, interpolation

    def _apply_image(self, img):
        return F.resize(img, self.size, self.interpolation)


class RandomResizedCrop(BaseTransform):
    def __init__(self, size, scale=(0.08, 1.0), ratio=(3.0 / 4, 4.0 / 3), interpolation="bilinear", keys=None):
        super().__init__(keys)
        self.size = (size, size) if isinstance(size, int) else size
        self.scale, self.ratio, self.interpolation = scale, ratio, interpolation

    def _get_param(self, img, attempts=10):
        w, h = _get_image_size(img)
        area = h * w
        for _ in range(attempts):
            ta = random.uniform(*self.scale) * area
            lr = (math.log(self.ratio[0]), math.log(self.ratio[1]))
            ar = math.exp(random.uniform(*lr))
            cw = int(round(math.sqrt(ta * ar)))
            ch = int(round(math.sqrt(ta / ar)))
            if 0 < cw <= w and 0 < ch <= h:
                return random.randint(0, h - ch), random.randint(0, w - cw), ch, cw
        r = w / h
        if r < min(self.ratio):
            cw, ch = w, int(round(w / min(self.ratio)))
        elif r > max(self.ratio):
            ch, cw = h, int(round(h * max(self.ratio)))
        else:
            cw, ch = w, h
        return (h - ch) // 2, (w - cw) // 2, ch, cw

    def _apply_image(self, img):
        i, j, h, w = self._get_param(img)
        return F.resize(F.crop(img, i, j, h, w), self.size, self.interpolation)


class CenterCrop(BaseTransform):
    def __init__(self, size, keys=None):
        super().__init__(keys)
        self.size = size

    def _apply_image(self, img):
        return F.center_crop(img, self.size)


class RandomHorizontalFlip(BaseTransform):
    def __init__(self, prob=0.5, keys=None):
        super().__init__(keys)
        self.prob = prob

    def _apply_image(self, img):
        return F.hflip(img) if random.random() < self.prob else img


class RandomVerticalFlip(BaseTransform):
    def __init__(self, prob=0.5, keys=None):
        super().__init__(keys)
        self.prob = prob

    def _apply_image(self, img):
        return F.vflip(img) if random.random() < self.prob else img


class Normalize(BaseTransform):
    def __init__(self, mean=0.0, std=1.0, data_format="CHW", to_rgb=False, keys=None):
        super().__init__(keys)
        self.mean = [mean] * 3 if isinstance(mean, numbers.Number) else mean
        self.std = [std] * 3 if isinstance(std, numbers.Number) else std
        self.data_format, self.to_rgb = data_format, to_rgb

    def _apply_image(self, img):
        return F.normalize(img, self.mean, self.std, self.data_format, self.to_rgb)


class Transpose(BaseTransform):
    def __init__(self, order=(2, 0, 1), keys=None):
        super().__init__(keys)
        self.order = order

    def _apply_image(self, img):
        if F._is_tensor_image(img):
            return img.transpose(list(self.order))
        a = np.asarray(img)
        if a.ndim == 2:
            a = a[..., None]
        return a.transpose(self.order)


class BrightnessTransform(BaseTransform):
    def __init__(self, value, keys=None):
        super().__init__(keys)
        self.value = value

    def _apply_image(self, img):
        if not self.value:
            return img
        return F.adjust_brightness(img, random.uniform(max(0, 1 - self.value), 1 + self.value))


class ContrastTransform(BaseTransform):
    def __init__(self, value, keys=None):
        super().__init__(keys)
        self.value = value

    def _apply_image(self, img):
        if not self.value:
            return img
        return F.adjust_contrast(img, random.uniform(max(0, 1 - self.value), 1 + self.value))


class SaturationTransform(BaseTransform):
    def __init__(self, value, keys=None):
        super().__init__(keys)
        self.value = value

    def _apply_image(self, img):
        if not self.value:
            return img
        return F.adjust_saturation(img, random.uniform(max(0, 1 - self.value), 1 + self.value))


class HueTransform(BaseTransform):
    def __init__(self, value, keys=None):
        super().__init__(keys)
        self.value = value

    def _apply_image(self, img):
        if not self.value:
            return img
        return F.adjust_hue(img, random.uniform(-self.value, self.value))


class ColorJitter(BaseTransform):
    def __init__(self, brightness=0, contrast=0, saturation=0, hue=0, keys=None):
        super().__init__(keys)
        self.ts = [BrightnessTransform(brightness), ContrastTransform(contrast), SaturationTransform(saturation),
                   HueTransform(hue)]

    def _apply_image(self, img):
        order = list(range(4))
        random.shuffle(order)
        for i in order:
            img = self.ts[i]._apply_image(img)
        return img


class RandomCrop(BaseTransform):
    def __init__(self, size, padding=None, pad_if_needed=False, fill=0, padding_mode="constant", keys=None):
        super().__init__(keys)
        self.size = (int(size), int(size)) if isinstance(size, numbers.Number) else size
        self.padding, self.pad_if_needed, self.fill, self.padding_mode = padding, pad_if_needed, fill, padding_mode

    def _apply_image(self, img):
        if self.padding is not None:
            img = F.pad(img, self.padding, self.fill, self.padding_mode)
        w, h = _get_image_size(img)
        th, tw = self.size
        if self.pad_if_needed and w < tw:
            img = F.pad(img, (tw - w, 0), self.fill, self.padding_mode)
        if self.pad_if_needed and h < th:
            img = F.pad(img, (0, th - h), self.fill, self.padding_mode)
        w, h = _get_image_size(img)
        i = random.randint(0, h - th)
        j = random.randint(0, w - tw)
        return F.crop(img, i, j, th, tw)


class Pad(BaseTransform):
    def __init__(self, padding, fill=0, padding_mode="constant", keys=None):
        super().__init__(keys)
        self.padding, self.fill, self.padding_mode = padding, fill, padding_mode

    def _apply_image(self, img):
        return F.pad(img, self.padding, self.fill, self.padding_mode)


class RandomAffine(BaseTransform):
    def __init__(self, degrees, translate=None, scale=None, shear=None, interpolation="nearest", fill=0, center=None,
                 keys=None):
        super().__init__(keys)
        self.degrees = (-degrees, degrees) if isinstance(degrees, numbers.Number) else degrees
        self.translate, self.scale, self.interpolation, self.fill, self.center = translate, scale, interpolation, \
            fill, center
        if shear is None or isinstance(shear, numbers.Number):
            self.shear = None if shear is None else (-shear, shear, 0, 0)
        else:
            self.shear = tuple(shear) + (0, 0) if len(shear) == 2 else tuple(shear)

    def _apply_image(self, img):
        w, h = _get_image_size(img)
        angle = random.uniform(*self.degrees)
        tx = ty = 0
        if self.translate is not None:
            tx = round(random.uniform(-self.translate[0] * w, self.translate[0] * w))
            ty = round(random.uniform(-self.translate[1] * h, self.translate[1] * h))
        sc = random.uniform(*self.scale) if self.scale is not None else 1.0
        sh = (0.0, 0.0)
        if self.shear is not None:
            sh = (random.uniform(self.shear[0], self.shear[1]), random.uniform(self.shear[2], self.shear[3]))
        return F.affine(img, angle, (tx, ty), sc, sh, self.interpolation, self.fill, self.center)


class RandomRotation(BaseTransform):
    def __init__(self, degrees, interpolation="nearest", expand=False, center=None, fill=0, keys=None):
        super().__init__(keys)
        self.degrees = (-degrees, degrees) if isinstance(degrees, numbers.Number) else degrees
        self.interpolation, self.expand, self.center, self.fill = interpolation, expand, center, fill

    def _apply_image(self, img):
        return F.rotate(img, random.uniform(*self.degrees), self.interpolation, self.expand, self.center, self.fill)


class RandomPerspective(BaseTransform):
    def __init__(self, prob=0.5, distortion_scale=0.5, interpolation="nearest", fill=0, keys=None):
        super().__init__(keys)
        self.prob, self.distortion_scale, self.interpolation, self.fill = prob, distortion_scale, interpolation, fill

    def _apply_image(self, img):
        if random.random() >= self.prob:
            return img
        w, h = _get_image_size(img)
        dx, dy = int(self.distortion_scale * w / 2), int(self.distortion_scale * h / 2)
        tl = [random.randint(0, dx), random.randint(0, dy)]
        tr = [w - 1 - random.randint(0, dx), random.randint(0, dy)]
        br = [w - 1 - random.randint(0, dx), h - 1 - random.randint(0, dy)]
        bl = [random.randint(0, dx), h - 1 - random.randint(0, dy)]
        start = [[0, 0], [w - 1, 0], [w - 1, h - 1], [0, h - 1]]
        return F.perspective(img, start, [tl, tr, br, bl], self.interpolation, self.fill)


class Grayscale(BaseTransform):
    def __init__(self, num_output_channels=1, keys=None):
        super().__init__(keys)
        self.num_output_channels = num_output_channels

    def _apply_image(self, img):
        return F.to_grayscale(img, self.num_output_channels)


class RandomErasing(BaseTransform):
    def __init__(self, prob=0.5, scale=(0.02, 0.33), ratio=(0.3, 3.3), value=0, inplace=False, keys=None):
        super().__init__(keys)
        self.prob, self.scale, self.ratio, self.value, self.inplace = prob, scale, ratio, value, inplace

    def _apply_image(self, img):
        if random.random() >= self.prob:
            return img
        if F._is_tensor_image(img):
            c, h, w = img.shape[-3:]
        else:
            h, w = np.asarray(img).shape[:2]
        for _ in range(10):
            ea = random.uniform(*self.scale) * h * w
            ar = math.exp(random.uniform(math.log(self.ratio[0]), math.log(self.ratio[1])))
            eh, ew = int(round(math.sqrt(ea * ar))), int(round(math.sqrt(ea / ar)))
            if eh < h and ew < w:
                i, j = random.randint(0, h - eh), random.randint(0, w - ew)
                return F.erase(img, i, j, eh, ew, self.value, self.inplace)
        return img
