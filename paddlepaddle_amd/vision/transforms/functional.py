"""Image transforms (functional). Reference: python/paddle/vision/transforms/functional.py
(+ functional_pil / functional_cv2 / functional_tensor backends).

One implementation for all input kinds: PIL images and HWC numpy arrays are converted to a CHW torch
tensor, transformed (resize / affine / perspective via interpolate / grid_sample), and converted back
to the input's kind, so PIL, numpy and Tensor inputs give the same pixels. Tensors are CHW (or NCHW).
"""
from __future__ import annotations

import math
import numbers

import numpy as np
import torch
import torch.nn.functional as TF

from ...framework.tensor import Tensor, _wrap

try:
    from PIL import Image
except ImportError:  # pragma: no cover
    Image = None


def _is_pil_image(img):
    return Image is not None and isinstance(img, Image.Image)


def _is_tensor_image(img):
    return isinstance(img, Tensor)


def _is_numpy_image(img):
    return isinstance(img, np.ndarray) and img.ndim in (2, 3)


class _Img:
    """CHW torch view of any supported image + how to convert back."""

    def __init__(self, img, data_format="CHW"):
        self.kind = "pil" if _is_pil_image(img) else ("tensor" if _is_tensor_image(img) else "numpy")
        self.mode = img.mode if self.kind == "pil" else None
        if self.kind == "pil":
            a = np.asarray(img)
        elif self.kind == "numpy":
            a = img
        if self.kind in ("pil", "numpy"):
            self.dtype = a.dtype
            self.gray2d = a.ndim == 2
            a = a[:, :, None] if a.ndim == 2 else a
            self.t = torch.from_numpy(np.ascontiguousarray(a)).permute(2, 0, 1)
            self.hwc = True
        else:
            t = img._t
            self.hwc = data_format == "HWC"
            self.t = t.permute(2, 0, 1) if self.hwc else t
            self.dtype = None
            self.gray2d = False

    def out(self, t):
        if self.kind == "tensor":
            return _wrap(t.permute(1, 2, 0) if self.hwc else t)
        a = t.permute(1, 2, 0).cpu().numpy()
        if np.issubdtype(self.dtype, np.integer):
            a = np.clip(np.round(a), 0, 255).astype(self.dtype)
        else:
            a = a.astype(self.dtype)
        if self.gray2d:
            a = a[:, :, 0]
        if self.kind == "pil":
            return Image.fromarray(a, mode=None if a.ndim == 3 else "L")
        return a


def _float(t):
    return t.float() if not t.is_floating_point() else t


def _size(img):
    """(w, h)"""
    if _is_pil_image(img):
        return img.size
    if _is_tensor_image(img):
        return img.shape[-1], img.shape[-2]
    return img.shape[1], img.shape[0]


def to_tensor(pic, data_format="CHW"):
    if _is_tensor_image(pic):
        return pic
    im = _Img(pic)
    t = im.t
    if t.dtype == torch.uint8:
        t = t.float() / 255.0
    else:
        t = t.float()
    if data_format == "HWC":
        t = t.permute(1, 2, 0)
    return _wrap(t.contiguous())


_INTERP = {"nearest": "nearest", "bilinear": "bilinear", "bicubic": "bicubic", "area": "area", "lanczos": "bicubic"}


def resize(img, size, interpolation="bilinear"):
    w, h = _size(img)
    if isinstance(size, int):
        if w < h:
            ow, oh = size, int(size * h / w)
        else:
            oh, ow = size, int(size * w / h)
    else:
        oh, ow = size
    if _is_pil_image(img):
        m = {"nearest": Image.NEAREST, "bilinear": Image.BILINEAR, "bicubic": Image.BICUBIC,
             "lanczos": Image.LANCZOS, "box": Image.BOX, "hamming": Image.HAMMING}[interpolation]
        return img.resize((ow, oh), m)
    im = _Img(img)
    t = _float(im.t)[None]
    mode = _INTERP.get(interpolation, "bilinear")
    kw = {"align_corners": False} if mode in ("bilinear", "bicubic") else {}
    return im.out(TF.interpolate(t, size=(oh, ow), mode=mode, **kw)[0])


def pad(img, padding, fill=0, padding_mode="constant"):
    if isinstance(padding, numbers.Number):
        l = r = t_ = b = int(padding)
    elif len(padding) == 2:
        l, t_ = padding
        r, b = padding
    else:
        l, t_, r, b = padding
    im = _Img(img)
    x = _float(im.t)[None]
    mode = {"constant": "constant", "edge": "replicate", "reflect": "reflect", "symmetric": "reflect"}[padding_mode]
    if mode == "constant":
        y = TF.pad(x, (l, r, t_, b), mode="constant", value=float(fill) if isinstance(fill, numbers.Number) else 0.0)
    elif padding_mode == "symmetric":
        y = torch.cat([x[..., :, :l].flip(-1), x, x[..., :, x.shape[-1] - r:].flip(-1)], -1) if (l or r) else x
        y = torch.cat([y[..., :t_, :].flip(-2), y, y[..., y.shape[-2] - b:, :].flip(-2)], -2) if (t_ or b) else y
    else:
        y = TF.pad(x, (l, r, t_, b), mode=mode)
    return im.out(y[0])


def crop(img, top, left, height, width):
    if _is_pil_image(img):
        return img.crop((left, top, left + width, top + height))
    im = _Img(img)
    return im.out(im.t[:, top:top + height, left:left + width])


def center_crop(img, output_size):
    if isinstance(output_size, numbers.Number):
        output_size = (int(output_size), int(output_size))
    w, h = _size(img)
    th, tw = output_size
    return crop(img, int(round((h - th) / 2.0)), int(round((w - tw) / 2.0)), th, tw)


def hflip(img):
    if _is_pil_image(img):
        return img.transpose(Image.FLIP_LEFT_RIGHT)
    im = _Img(img)
    return im.out(im.t.flip(-1))


def vflip(img):
    if _is_pil_image(img):
        return img.transpose(Image.FLIP_TOP_BOTTOM)
    im = _Img(img)
    return im.out(im.t.flip(-2))


def _blend(a, b, ratio, bound):
    return (ratio * a + (1.0 - ratio) * b).clamp(0, bound)


def _bound(t):
    return 1.0 if t.is_floating_point() else 255.0


def _gray(t):
    if t.shape[0] == 1:
        return _float(t)
    r, g, b = _float(t)[0], _float(t)[1], _float(t)[2]
    return (0.299 * r + 0.587 * g + 0.114 * b)[None]


def adjust_brightness(img, brightness_factor):
    im = _Img(img)
    t = im.t
    return im.out(_blend(_float(t), torch.zeros_like(_float(t)), brightness_factor, _bound(t)))


def adjust_contrast(img, contrast_factor):
    im = _Img(img)
    t = im.t
    mean = _gray(t).mean()
    return im.out(_blend(_float(t), mean, contrast_factor, _bound(t)))


def adjust_saturation(img, saturation_factor):
    im = _Img(img)
    t = im.t
    return im.out(_blend(_float(t), _gray(t), saturation_factor, _bound(t)))


def _rgb2hsv(x):
    r, g, b = x.unbind(0)
    maxc, _ = x.max(0)
    minc, _ = x.min(0)
    v = maxc
    cr = maxc - minc
    s = cr / torch.where(maxc == 0, torch.ones_like(maxc), maxc)
    crd = torch.where(cr == 0, torch.ones_like(cr), cr)
    rc, gc, bc = (maxc - r) / crd, (maxc - g) / crd, (maxc - b) / crd
    h = torch.where(maxc == r, bc - gc, torch.where(maxc == g, 2.0 + rc - bc, 4.0 + gc - rc))
    h = torch.where(cr == 0, torch.zeros_like(h), h)
    h = (h / 6.0) % 1.0
    return torch.stack([h, s, v])


def _hsv2rgb(x):
    h, s, v = x.unbind(0)
    i = torch.floor(h * 6.0)
    f = h * 6.0 - i
    i = i.to(torch.int64) % 6
    p, q, t = v * (1 - s), v * (1 - s * f), v * (1 - s * (1 - f))
    sel = [torch.stack(c) for c in ((v, t, p), (q, v, p), (p, v, t), (p, q, v), (t, p, v), (v, p, q))]
    out = torch.zeros_like(x)
    for k in range(6):
        out = torch.where((i == k)[None], sel[k], out)
    return out


def adjust_hue(img, hue_factor):
    if not -0.5 <= hue_factor <= 0.5:
        raise ValueError("hue_factor must be in [-0.5, 0.5]")
    im = _Img(img)
    t = im.t
    scale = _bound(t)
    x = _float(t) / scale
    hsv = _rgb2hsv(x)
    hsv[0] = (hsv[0] + hue_factor) % 1.0
    return im.out(_hsv2rgb(hsv) * scale)


def to_grayscale(img, num_output_channels=1):
    if _is_pil_image(img):
        g = img.convert("L")
        return g if num_output_channels == 1 else Image.merge("RGB", [g, g, g])
    im = _Img(img)
    g = _gray(im.t)
    if num_output_channels == 3:
        g = g.expand(3, -1, -1)
    return im.out(g)


def normalize(img, mean, std, data_format="CHW", to_rgb=False):
    if _is_tensor_image(img):
        t = _float(img._t)
        m = torch.as_tensor(mean, dtype=t.dtype, device=t.device)
        s = torch.as_tensor(std, dtype=t.dtype, device=t.device)
        if data_format == "CHW":
            m, s = m.view(-1, 1, 1), s.view(-1, 1, 1)
        return _wrap((t - m) / s)
    a = np.asarray(img).astype("float32")
    if to_rgb:
        a = a[..., ::-1]
    m, s = np.asarray(mean, "float32"), np.asarray(std, "float32")
    if data_format == "CHW":
        m, s = m.reshape(-1, 1, 1), s.reshape(-1, 1, 1)
    return (a - m) / s


def _affine_grid(theta, h, w):
    return TF.affine_grid(theta[None], [1, 1, h, w], align_corners=False)


def _get_inverse_affine(center, angle, translate, scale, shear):
    rot = math.radians(angle)
    sx, sy = [math.radians(s) for s in shear]
    cx, cy = center
    tx, ty = translate
    a = math.cos(rot - sy) / math.cos(sy)
    b = -math.cos(rot - sy) * math.tan(sx) / math.cos(sy) - math.sin(rot)
    c = math.sin(rot - sy) / math.cos(sy)
    d = -math.sin(rot - sy) * math.tan(sx) / math.cos(sy) + math.cos(rot)
    M = np.array([[d, -b, 0.0], [-c, a, 0.0]]) / scale
    M[0, 2] = M[0, 0] * (-cx - tx) + M[0, 1] * (-cy - ty) + cx
    M[1, 2] = M[1, 0] * (-cx - tx) + M[1, 1] * (-cy - ty) + cy
    return M


def _warp(im, M_inv, interpolation, fill, out_hw=None):
    t = _float(im.t)
    h, w = t.shape[-2:]
    oh, ow = out_hw or (h, w)
    ys, xs = torch.meshgrid(torch.arange(oh, dtype=torch.float32) + 0.5, torch.arange(ow, dtype=torch.float32) + 0.5,
                            indexing="ij")
    M = torch.as_tensor(M_inv, dtype=torch.float32)
    sx = M[0, 0] * xs + M[0, 1] * ys + M[0, 2]
    sy = M[1, 0] * xs + M[1, 1] * ys + M[1, 2]
    grid = torch.stack([sx / w * 2 - 1, sy / h * 2 - 1], -1)[None].to(t.device)
    mode = "nearest" if interpolation == "nearest" else "bilinear"
    ones = torch.ones_like(t[:1])
    out = TF.grid_sample(torch.cat([t, ones])[None], grid, mode=mode, padding_mode="zeros", align_corners=False)[0]
    val, mask = out[:-1], out[-1:]
    fillv = torch.as_tensor(fill if isinstance(fill, (list, tuple)) else [fill] * val.shape[0],
                            dtype=val.dtype, device=val.device).view(-1, 1, 1)
    return im.out(torch.where(mask > 0.5, val, fillv))


def affine(img, angle, translate, scale, shear, interpolation="nearest", fill=0, center=None):
    w, h = _size(img)
    shear = shear if isinstance(shear, (list, tuple)) else (shear, 0.0)
    center = center or (w * 0.5, h * 0.5)
    M = _get_inverse_affine(center, angle, translate, scale, shear)
    return _warp(_Img(img), M, interpolation, fill)


def rotate(img, angle, interpolation="nearest", expand=False, center=None, fill=0):
    w, h = _size(img)
    center = center or (w * 0.5, h * 0.5)
    M = _get_inverse_affine(center, -angle, (0, 0), 1.0, (0.0, 0.0))
    out_hw = None
    if expand:
        corners = np.array([[0, 0, 1], [w, 0, 1], [w, h, 1], [0, h, 1]], dtype=np.float64)
        rot = math.radians(-angle)
        R = np.array([[math.cos(rot), -math.sin(rot)], [math.sin(rot), math.cos(rot)]])
        pts = (corners[:, :2] - center) @ R.T
        nw = int(math.ceil(pts[:, 0].max() - pts[:, 0].min()))
        nh = int(math.ceil(pts[:, 1].max() - pts[:, 1].min()))
        M[0, 2] += M[0, 0] * (-(nw - w) / 2) + M[0, 1] * (-(nh - h) / 2)
        M[1, 2] += M[1, 0] * (-(nw - w) / 2) + M[1, 1] * (-(nh - h) / 2)
        out_hw = (nh, nw)
    return _warp(_Img(img), M, interpolation, fill, out_hw)


def _perspective_coeffs(startpoints, endpoints):
    a = np.zeros((8, 8))
    for i, (p1, p2) in enumerate(zip(endpoints, startpoints)):
        a[2 * i] = [p1[0], p1[1], 1, 0, 0, 0, -p2[0] * p1[0], -p2[0] * p1[1]]
        a[2 * i + 1] = [0, 0, 0, p1[0], p1[1], 1, -p2[1] * p1[0], -p2[1] * p1[1]]
    b = np.array(startpoints, dtype=np.float64).reshape(8)
    return np.linalg.lstsq(a, b, rcond=None)[0]


def perspective(img, startpoints, endpoints, interpolation="nearest", fill=0):
    c = _perspective_coeffs(startpoints, endpoints)
    im = _Img(img)
    t = _float(im.t)
    h, w = t.shape[-2:]
    ys, xs = torch.meshgrid(torch.arange(h, dtype=torch.float64) + 0.5, torch.arange(w, dtype=torch.float64) + 0.5,
                            indexing="ij")
    den = c[6] * xs + c[7] * ys + 1.0
    sx = (c[0] * xs + c[1] * ys + c[2]) / den
    sy = (c[3] * xs + c[4] * ys + c[5]) / den
    grid = torch.stack([sx / w * 2 - 1, sy / h * 2 - 1], -1)[None].float().to(t.device)
    mode = "nearest" if interpolation == "nearest" else "bilinear"
    out = TF.grid_sample(t[None], grid, mode=mode, padding_mode="zeros", align_corners=False)[0]
    return im.out(out)


def erase(img, i, j, h, w, v, inplace=False):
    if _is_tensor_image(img):
        t = img._t if inplace else img._t.clone()
        t[..., i:i + h, j:j + w] = v._t if isinstance(v, Tensor) else torch.as_tensor(v, dtype=t.dtype)
        return _wrap(t) if not inplace else img
    a = np.array(img) if not inplace else img
    a[i:i + h, j:j + w] = np.asarray(v)
    return a
