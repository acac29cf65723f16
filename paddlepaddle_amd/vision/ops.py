"""paddle.vision.ops: detection / sampling operators.
Reference: python/paddle/vision/ops.py (nms:1934, roi_align:1705, roi_pool:1572, psroi_pool:1441,
box_coder:584, prior_box:438, yolo_box:277, yolo_loss:69, deform_conv2d:766, distribute_fpn_proposals,
generate_proposals, matrix_nms, read_file, decode_jpeg, ConvNormActivation).

Implemented as vectorised device-tensor programs (bilinear sampling via gather, IoU matrices on
the device) so they run where the feature maps live; greedy NMS suppression loops on the host only
over the kept boxes.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as TF

from .. import nn
from ..framework.tensor import Tensor, _wrap


def _t(x):
    return x._t if isinstance(x, Tensor) else (torch.as_tensor(x) if x is not None else None)


# ---------------------------------------------------------------------------- boxes / NMS
def _iou(a, b):
    area_a = (a[:, 2] - a[:, 0]).clamp(min=0) * (a[:, 3] - a[:, 1]).clamp(min=0)
    area_b = (b[:, 2] - b[:, 0]).clamp(min=0) * (b[:, 3] - b[:, 1]).clamp(min=0)
    lt = torch.max(a[:, None, :2], b[None, :, :2])
    rb = torch.min(a[:, None, 2:], b[None, :, 2:])
    wh = (rb - lt).clamp(min=0)
    inter = wh[..., 0] * wh[..., 1]
    return inter / (area_a[:, None] + area_b[None, :] - inter).clamp(min=1e-10)


def _nms_single(boxes, scores, thr):
    order = scores.argsort(descending=True) if scores is not None else torch.arange(boxes.shape[0],
                                                                                     device=boxes.device)
    b = boxes[order]
    iou = _iou(b, b).cpu()
    n = b.shape[0]
    keep = []
    suppressed = torch.zeros(n, dtype=torch.bool)
    for i in range(n):
        if suppressed[i]:
            continue
        keep.append(i)
        suppressed |= iou[i] > thr
    return order[torch.as_tensor(keep, dtype=torch.long, device=order.device)]


def nms(boxes, iou_threshold=0.3, scores=None, category_idxs=None, categories=None, top_k=None):
    b = _t(boxes).float()
    s = _t(scores)
    if category_idxs is None:
        keep = _nms_single(b, s.float() if s is not None else None, iou_threshold)
    else:
        ci = _t(category_idxs)
        keeps = []
        cats = categories if categories is not None else ci.unique().tolist()
        for c in cats:
            idx = (ci == c).nonzero().flatten()
            if idx.numel() == 0:
                continue
            k = _nms_single(b[idx], s[idx].float(), iou_threshold)
            keeps.append(idx[k])
        keep = torch.cat(keeps) if keeps else torch.zeros(0, dtype=torch.long, device=b.device)
        if s is not None:
            keep = keep[s[keep].argsort(descending=True)]
    if top_k is not None:
        keep = keep[:top_k]
    return _wrap(keep)


def matrix_nms(bboxes, scores, score_threshold, post_threshold, nms_top_k, keep_top_k, use_gaussian=False,
               gaussian_sigma=2.0, background_label=0, normalized=True, return_index=False, return_rois_num=True,
               name=None):
    """Matrix NMS (SOLOv2): decay scores by the max IoU with higher-scored boxes of the same class."""
    B = _t(bboxes).float()   # [N, M, 4]
    S = _t(scores).float()   # [N, C, M]
    outs, idxs, nums = [], [], []
    for n in range(B.shape[0]):
        dets = []
        for c in range(S.shape[1]):
            if c == background_label:
                continue
            sc = S[n, c]
            cand = (sc > score_threshold).nonzero().flatten()
            if cand.numel() == 0:
                continue
            cand = cand[sc[cand].argsort(descending=True)][:nms_top_k if nms_top_k > 0 else None]
            bx, s0 = B[n, cand], sc[cand]
            off = 0.0 if normalized else 1.0
            bxo = bx.clone()
            bxo[:, 2:] += off
            iou = _iou(bxo, bxo).triu(1)
            comp = iou.max(0).values
            if use_gaussian:
                decay = torch.exp((comp[:, None] ** 2 - iou ** 2) / gaussian_sigma).min(0).values
            else:
                decay = ((1 - iou) / (1 - comp[:, None]).clamp(min=1e-10)).min(0).values
            s1 = s0 * decay
            ok = s1 > post_threshold
            for j in ok.nonzero().flatten().tolist():
                dets.append((float(s1[j]), c, bx[j], n * B.shape[1] + int(cand[j])))
        dets.sort(key=lambda d: -d[0])
        if keep_top_k > 0:
            dets = dets[:keep_top_k]
        for sc_, c, bx, gi in dets:
            outs.append(torch.cat([torch.tensor([c, sc_], device=B.device), bx]))
            idxs.append(gi)
        nums.append(len(dets))
    out = torch.stack(outs) if outs else torch.zeros(0, 6, device=B.device)
    res = [_wrap(out)]
    if return_index:
        res.append(_wrap(torch.as_tensor(idxs, dtype=torch.int64).reshape(-1, 1)))
    if return_rois_num:
        res.append(_wrap(torch.as_tensor(nums, dtype=torch.int32)))
    return tuple(res) if len(res) > 1 else res[0]


def box_coder(prior_box, prior_box_var, target_box, code_type="encode_center_size", box_normalized=True, axis=0,
              name=None):
    pb = _t(prior_box).float()
    tb = _t(target_box).float()
    off = 0.0 if box_normalized else 1.0
    pw, ph = pb[:, 2] - pb[:, 0] + off, pb[:, 3] - pb[:, 1] + off
    pcx, pcy = pb[:, 0] + pw / 2, pb[:, 1] + ph / 2
    if prior_box_var is None:
        var = torch.ones(4, device=pb.device)
    elif isinstance(prior_box_var, (list, tuple)):
        var = torch.as_tensor(prior_box_var, dtype=torch.float32, device=pb.device)
    else:
        var = _t(prior_box_var).float()
    if code_type == "encode_center_size":
        tw, th = tb[:, 2] - tb[:, 0] + off, tb[:, 3] - tb[:, 1] + off
        tcx, tcy = tb[:, 0] + tw / 2, tb[:, 1] + th / 2
        out = torch.stack([(tcx[:, None] - pcx[None]) / pw[None], (tcy[:, None] - pcy[None]) / ph[None],
                           torch.log((tw[:, None] / pw[None]).abs()), torch.log((th[:, None] / ph[None]).abs())], -1)
        out = out / (var if var.dim() == 1 else var[None])
        return _wrap(out)
    # decode: target [N, M, 4]
    if tb.dim() == 2:
        tb = tb[:, None]
    if axis == 0:
        pw_, ph_, pcx_, pcy_ = pw[None], ph[None], pcx[None], pcy[None]
        v = var if var.dim() == 1 else var[None]
    else:
        pw_, ph_, pcx_, pcy_ = pw[:, None], ph[:, None], pcx[:, None], pcy[:, None]
        v = var if var.dim() == 1 else var[:, None]
    d = tb * v
    cx = d[..., 0] * pw_ + pcx_
    cy = d[..., 1] * ph_ + pcy_
    w = torch.exp(d[..., 2]) * pw_
    h = torch.exp(d[..., 3]) * ph_
    out = torch.stack([cx - w / 2, cy - h / 2, cx + w / 2 - off, cy + h / 2 - off], -1)
    return _wrap(out)


def prior_box(input, image, min_sizes, max_sizes=None, aspect_ratios=(1.0,), variance=(0.1, 0.1, 0.2, 0.2),
              flip=False, clip=False, steps=(0.0, 0.0), offset=0.5, min_max_aspect_ratios_order=False, name=None):
    H, W = input.shape[2], input.shape[3]
    IH, IW = image.shape[2], image.shape[3]
    sw = steps[0] if steps[0] > 0 else IW / W
    sh = steps[1] if steps[1] > 0 else IH / H
    ars = [1.0]
    for a in aspect_ratios:
        if all(abs(a - b) > 1e-6 for b in ars):
            ars.append(a)
            if flip:
                ars.append(1.0 / a)
    boxes = []
    for i, ms in enumerate(min_sizes):
        per = []
        if min_max_aspect_ratios_order:
            per.append((ms, ms))
            if max_sizes:
                s = math.sqrt(ms * max_sizes[i])
                per.append((s, s))
            for a in ars:
                if abs(a - 1.0) > 1e-6:
                    per.append((ms * math.sqrt(a), ms / math.sqrt(a)))
        else:
            for a in ars:
                per.append((ms * math.sqrt(a), ms / math.sqrt(a)))
            if max_sizes:
                s = math.sqrt(ms * max_sizes[i])
                per.append((s, s))
        boxes += per
    cy, cx = torch.meshgrid((torch.arange(H, dtype=torch.float32) + offset) * sh,
                            (torch.arange(W, dtype=torch.float32) + offset) * sw, indexing="ij")
    cx, cy = cx[..., None], cy[..., None]  # [H, W, 1]
    bw = torch.tensor([b[0] for b in boxes]) / 2
    bh = torch.tensor([b[1] for b in boxes]) / 2
    out = torch.stack([(cx - bw) / IW, (cy - bh) / IH, (cx + bw) / IW, (cy + bh) / IH], -1)  # [H, W, P, 4]
    if clip:
        out = out.clamp(0, 1)
    var = torch.tensor(variance, dtype=torch.float32).expand_as(out)
    dev = _t(input).device
    return _wrap(out.to(dev)), _wrap(var.contiguous().to(dev))


def yolo_box(x, img_size, anchors, class_num, conf_thresh, downsample_ratio, clip_bbox=True, name=None,
             scale_x_y=1.0, iou_aware=False, iou_aware_factor=0.5):
    X = _t(x).float()
    N, C, H, W = X.shape
    na = len(anchors) // 2
    an = torch.tensor(anchors, dtype=torch.float32, device=X.device).view(na, 2)
    if iou_aware:
        ioup = torch.sigmoid(X[:, :na])
        X = X[:, na:]
    X = X.view(N, na, 5 + class_num, H, W)
    gy, gx = torch.meshgrid(torch.arange(H, device=X.device), torch.arange(W, device=X.device), indexing="ij")
    bias = -0.5 * (scale_x_y - 1.0)
    cx = (gx + torch.sigmoid(X[:, :, 0]) * scale_x_y + bias) / W
    cy = (gy + torch.sigmoid(X[:, :, 1]) * scale_x_y + bias) / H
    in_w, in_h = downsample_ratio * W, downsample_ratio * H
    w = torch.exp(X[:, :, 2]) * an[:, 0, None, None] / in_w
    h = torch.exp(X[:, :, 3]) * an[:, 1, None, None] / in_h
    conf = torch.sigmoid(X[:, :, 4])
    if iou_aware:
        conf = conf ** (1 - iou_aware_factor) * ioup ** iou_aware_factor
    isz = _t(img_size).float().to(X.device)
    ih, iw = isz[:, 0].view(N, 1, 1, 1), isz[:, 1].view(N, 1, 1, 1)
    x0, y0 = (cx - w / 2) * iw, (cy - h / 2) * ih
    x1, y1 = (cx + w / 2) * iw, (cy + h / 2) * ih
    if clip_bbox:
        x0, y0 = x0.clamp(min=0), y0.clamp(min=0)
        x1, y1 = torch.min(x1, iw - 1), torch.min(y1, ih - 1)
    keep = (conf >= conf_thresh).float()
    boxes = torch.stack([x0, y0, x1, y1], -1) * keep[..., None]
    scores = torch.sigmoid(X[:, :, 5:]) * (conf * keep)[:, :, None]
    boxes = boxes.reshape(N, -1, 4)
    scores = scores.permute(0, 1, 3, 4, 2).reshape(N, -1, class_num)
    return _wrap(boxes), _wrap(scores)


def yolo_loss(x, gt_box, gt_label, anchors, anchor_mask, class_num, ignore_thresh, downsample_ratio,
              gt_score=None, use_label_smooth=True, name=None, scale_x_y=1.0):
    """YOLOv3 loss: per-image sum of xy/wh regression, objectness (with ignore mask) and class BCE."""
    X = _t(x).float()
    N, _, H, W = X.shape
    mask_an = [anchors[2 * i:2 * i + 2] for i in anchor_mask]
    na = len(mask_an)
    all_an = torch.tensor(anchors, dtype=torch.float32).view(-1, 2)
    X = X.view(N, na, 5 + class_num, H, W)
    gtb = _t(gt_box).float().to(X.device)
    gtl = _t(gt_label).long().to(X.device)
    gts = _t(gt_score).float().to(X.device) if gt_score is not None else torch.ones(gtl.shape, device=X.device)
    in_w, in_h = downsample_ratio * W, downsample_ratio * H
    pred_box, _ = yolo_box(_wrap(X.reshape(N, -1, H, W)), torch.tensor([[in_h, in_w]] * N), sum(mask_an, []),
                           class_num, 0.0, downsample_ratio, clip_bbox=False, scale_x_y=scale_x_y)
    pb = pred_box._t.view(N, na, H, W, 4) / torch.tensor([in_w, in_h, in_w, in_h], device=X.device)
    loss = torch.zeros(N, device=X.device)
    obj_target = torch.zeros(N, na, H, W, device=X.device)
    obj_mask = torch.ones(N, na, H, W, device=X.device)
    bce = TF.binary_cross_entropy_with_logits
    pos_smooth = 1.0 - 1.0 / class_num if use_label_smooth else 1.0
    neg_smooth = 1.0 / class_num if use_label_smooth else 0.0
    for n in range(N):
        g = gtb[n]
        valid = (g[:, 2] > 0) & (g[:, 3] > 0)
        gxyxy = torch.stack([g[:, 0] - g[:, 2] / 2, g[:, 1] - g[:, 3] / 2, g[:, 0] + g[:, 2] / 2,
                             g[:, 1] + g[:, 3] / 2], -1)
        if valid.any():
            iou = _iou(pb[n].reshape(-1, 4), gxyxy[valid]).max(1).values.view(na, H, W)
            obj_mask[n] = (iou <= ignore_thresh).float()
        for t in valid.nonzero().flatten().tolist():
            gw, gh = float(g[t, 2]) * in_w, float(g[t, 3]) * in_h
            inter = torch.min(all_an[:, 0], torch.tensor(gw)) * torch.min(all_an[:, 1], torch.tensor(gh))
            ious = inter / (all_an[:, 0] * all_an[:, 1] + gw * gh - inter)
            best = int(ious.argmax())
            if best not in anchor_mask:
                continue
            a = anchor_mask.index(best)
            gi, gj = int(g[t, 0] * W), int(g[t, 1] * H)
            gi, gj = min(max(gi, 0), W - 1), min(max(gj, 0), H - 1)
            sc = gts[n, t]
            tx, ty = float(g[t, 0]) * W - gi, float(g[t, 1]) * H - gj
            tw = math.log(max(gw / mask_an[a][0], 1e-9))
            th = math.log(max(gh / mask_an[a][1], 1e-9))
            wscale = (2.0 - float(g[t, 2]) * float(g[t, 3])) * sc
            p = X[n, a, :, gj, gi]
            loss[n] = loss[n] + wscale * (bce(p[0], torch.tensor(tx, device=X.device)) +
                                          bce(p[1], torch.tensor(ty, device=X.device)) +
                                          (p[2] - tw).abs() + (p[3] - th).abs())
            cls_t = torch.full((class_num,), neg_smooth, device=X.device)
            cls_t[gtl[n, t]] = pos_smooth
            loss[n] = loss[n] + sc * bce(p[5:], cls_t, reduction="sum")
            obj_target[n, a, gj, gi] = sc
            obj_mask[n, a, gj, gi] = 1.0
    obj = bce(X[:, :, 4], obj_target, reduction="none") * obj_mask
    loss = loss + obj.sum((1, 2, 3))
    return _wrap(loss)


# ---------------------------------------------------------------------------- RoI ops
def _rois_batch_idx(boxes_num, n_rois, device):
    bn = _t(boxes_num).long().to(device)
    return torch.repeat_interleave(torch.arange(bn.numel(), device=device), bn)


def _bilinear(feat, y, x):
    """feat [C,H,W]; y,x [...] float -> [C, ...] (zero outside, border-clamped inside)."""
    C, H, W = feat.shape
    valid = (y > -1.0) & (y < H) & (x > -1.0) & (x < W)
    y = y.clamp(min=0)
    x = x.clamp(min=0)
    y0 = y.floor().long().clamp(max=H - 1)
    x0 = x.floor().long().clamp(max=W - 1)
    y1 = (y0 + 1).clamp(max=H - 1)
    x1 = (x0 + 1).clamp(max=W - 1)
    y = torch.where(y0 >= H - 1, y0.float(), y)
    x = torch.where(x0 >= W - 1, x0.float(), x)
    ly, lx = y - y0, x - x0
    hy, hx = 1 - ly, 1 - lx
    f = feat.reshape(C, -1)

    def g(yy, xx):
        return f[:, (yy * W + xx).reshape(-1)].reshape((C,) + yy.shape)
    out = g(y0, x0) * (hy * hx) + g(y0, x1) * (hy * lx) + g(y1, x0) * (ly * hx) + g(y1, x1) * (ly * lx)
    return out * valid


def roi_align(x, boxes, boxes_num, output_size, spatial_scale=1.0, sampling_ratio=-1, aligned=True, name=None):
    X = _t(x)
    Bx = _t(boxes).float()
    oh, ow = (output_size, output_size) if isinstance(output_size, int) else output_size
    bidx = _rois_batch_idx(boxes_num, Bx.shape[0], X.device)
    off = 0.5 if aligned else 0.0
    outs = []
    for r in range(Bx.shape[0]):
        x0, y0, x1, y1 = (Bx[r] * spatial_scale - off).tolist()
        rw, rh = x1 - x0, y1 - y0
        if not aligned:
            rw, rh = max(rw, 1.0), max(rh, 1.0)
        bw, bh = rw / ow, rh / oh
        gh = sampling_ratio if sampling_ratio > 0 else int(math.ceil(rh / oh))
        gw = sampling_ratio if sampling_ratio > 0 else int(math.ceil(rw / ow))
        gh, gw = max(gh, 1), max(gw, 1)
        iy = (torch.arange(oh, device=X.device)[:, None] * bh + (torch.arange(gh, device=X.device)[None] + 0.5) * bh / gh
              + y0).reshape(-1)
        ix = (torch.arange(ow, device=X.device)[:, None] * bw + (torch.arange(gw, device=X.device)[None] + 0.5) * bw / gw
              + x0).reshape(-1)
        yy, xx = torch.meshgrid(iy, ix, indexing="ij")
        v = _bilinear(X[bidx[r]].float(), yy, xx)  # [C, oh*gh, ow*gw]
        v = v.reshape(v.shape[0], oh, gh, ow, gw).mean((2, 4))
        outs.append(v)
    out = torch.stack(outs) if outs else torch.zeros(0, X.shape[1], oh, ow, device=X.device)
    return _wrap(out.to(X.dtype))


def roi_pool(x, boxes, boxes_num, output_size, spatial_scale=1.0, name=None):
    X = _t(x)
    Bx = _t(boxes).float()
    oh, ow = (output_size, output_size) if isinstance(output_size, int) else output_size
    bidx = _rois_batch_idx(boxes_num, Bx.shape[0], X.device)
    H, W = X.shape[2], X.shape[3]
    outs = []
    for r in range(Bx.shape[0]):
        x0, y0, x1, y1 = [int(round(v * spatial_scale)) for v in Bx[r].tolist()]
        rh, rw = max(y1 - y0 + 1, 1), max(x1 - x0 + 1, 1)
        o = torch.zeros(X.shape[1], oh, ow, dtype=X.dtype, device=X.device)
        for i in range(oh):
            hs = min(max(y0 + int(math.floor(i * rh / oh)), 0), H)
            he = min(max(y0 + int(math.ceil((i + 1) * rh / oh)), 0), H)
            for j in range(ow):
                ws = min(max(x0 + int(math.floor(j * rw / ow)), 0), W)
                we = min(max(x0 + int(math.ceil((j + 1) * rw / ow)), 0), W)
                if he > hs and we > ws:
                    o[:, i, j] = X[bidx[r], :, hs:he, ws:we].amax((1, 2))
        outs.append(o)
    out = torch.stack(outs) if outs else torch.zeros(0, X.shape[1], oh, ow, device=X.device)
    return _wrap(out)


def psroi_pool(x, boxes, boxes_num, output_size, spatial_scale=1.0, name=None):
    X = _t(x)
    Bx = _t(boxes).float()
    oh, ow = (output_size, output_size) if isinstance(output_size, int) else output_size
    C = X.shape[1] // (oh * ow)
    bidx = _rois_batch_idx(boxes_num, Bx.shape[0], X.device)
    H, W = X.shape[2], X.shape[3]
    outs = []
    for r in range(Bx.shape[0]):
        x0, y0 = [round(v) * spatial_scale for v in Bx[r, :2].tolist()]
        x1, y1 = [(round(v) + 1.0) * spatial_scale for v in Bx[r, 2:].tolist()]
        rh, rw = max(y1 - y0, 0.1), max(x1 - x0, 0.1)
        o = torch.zeros(C, oh, ow, dtype=X.dtype, device=X.device)
        for i in range(oh):
            hs = min(max(int(math.floor(y0 + i * rh / oh)), 0), H)
            he = min(max(int(math.ceil(y0 + (i + 1) * rh / oh)), 0), H)
            for j in range(ow):
                ws = min(max(int(math.floor(x0 + j * rw / ow)), 0), W)
                we = min(max(int(math.ceil(x0 + (j + 1) * rw / ow)), 0), W)
                if he > hs and we > ws:
                    ch = torch.arange(C, device=X.device) * oh * ow + i * ow + j
                    o[:, i, j] = X[bidx[r], ch, hs:he, ws:we].mean((1, 2))
        outs.append(o)
    out = torch.stack(outs) if outs else torch.zeros(0, C, oh, ow, device=X.device)
    return _wrap(out)


class RoIAlign(nn.Layer):
    def __init__(self, output_size, spatial_scale=1.0):
        super().__init__()
        self.output_size, self.spatial_scale = output_size, spatial_scale

    def forward(self, x, boxes, boxes_num, aligned=True):
        return roi_align(x, boxes, boxes_num, self.output_size, self.spatial_scale, aligned=aligned)


class RoIPool(nn.Layer):
    def __init__(self, output_size, spatial_scale=1.0):
        super().__init__()
        self.output_size, self.spatial_scale = output_size, spatial_scale

    def forward(self, x, boxes, boxes_num):
        return roi_pool(x, boxes, boxes_num, self.output_size, self.spatial_scale)


class PSRoIPool(nn.Layer):
    def __init__(self, output_size, spatial_scale=1.0):
        super().__init__()
        self.output_size, self.spatial_scale = output_size, spatial_scale

    def forward(self, x, boxes, boxes_num):
        return psroi_pool(x, boxes, boxes_num, self.output_size, self.spatial_scale)


# ---------------------------------------------------------------------------- deformable conv
def deform_conv2d(x, offset, weight, bias=None, stride=1, padding=0, dilation=1, deformable_groups=1, groups=1,
                  mask=None, name=None):
    """DCN v1/v2: bilinear-sample the input at offset positions (im2col), then one GEMM per group."""
    X, O, Wt = _t(x), _t(offset), _t(weight)
    M = _t(mask) if mask is not None else None
    s = (stride, stride) if isinstance(stride, int) else stride
    p = (padding, padding) if isinstance(padding, int) else padding
    d = (dilation, dilation) if isinstance(dilation, int) else dilation
    N, C, H, W = X.shape
    Co, Cg, kh, kw = Wt.shape
    Ho = (H + 2 * p[0] - d[0] * (kh - 1) - 1) // s[0] + 1
    Wo = (W + 2 * p[1] - d[1] * (kw - 1) - 1) // s[1] + 1
    K = kh * kw
    dg = deformable_groups
    base_y = (torch.arange(Ho, device=X.device) * s[0] - p[0]).view(1, Ho, 1) + \
        (torch.arange(kh, device=X.device) * d[0]).repeat_interleave(kw).view(K, 1, 1)
    base_x = (torch.arange(Wo, device=X.device) * s[1] - p[1]).view(1, 1, Wo) + \
        (torch.arange(kw, device=X.device) * d[1]).repeat(kh).view(K, 1, 1)
    cols = []
    for n in range(N):
        off = O[n].view(dg, K, 2, Ho, Wo)
        per_g = []
        for g in range(dg):
            yy = base_y + off[g, :, 0]
            xx = base_x + off[g, :, 1]
            feat = X[n, g * (C // dg):(g + 1) * (C // dg)].float()
            v = _bilinear(feat, yy, xx)  # [C/dg, K, Ho, Wo]
            if M is not None:
                v = v * M[n].view(dg, K, Ho, Wo)[g][None]
            per_g.append(v)
        cols.append(torch.cat(per_g, 0))  # [C, K, Ho, Wo]
    col = torch.stack(cols)  # [N, C, K, Ho, Wo]
    col = col.view(N, groups, C // groups * K, Ho * Wo)
    w = Wt.float().view(groups, Co // groups, Cg * K)
    out = torch.einsum("gok,ngkl->ngol", w, col).reshape(N, Co, Ho, Wo)
    if bias is not None:
        out = out + _t(bias).float().view(1, -1, 1, 1)
    return _wrap(out.to(X.dtype))


class DeformConv2D(nn.Layer):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, deformable_groups=1,
                 groups=1, weight_attr=None, bias_attr=None):
        super().__init__()
        k = (kernel_size, kernel_size) if isinstance(kernel_size, int) else tuple(kernel_size)
        self.stride, self.padding, self.dilation = stride, padding, dilation
        self.deformable_groups, self.groups = deformable_groups, groups
        fan_in = in_channels // groups * k[0] * k[1]
        from ..nn import initializer as I
        self.weight = self.create_parameter([out_channels, in_channels // groups, k[0], k[1]], attr=weight_attr,
                                            default_initializer=I.Normal(0.0, math.sqrt(2.0 / fan_in)))
        self.bias = self.create_parameter([out_channels], attr=bias_attr, is_bias=True) if bias_attr is not False \
            else None

    def forward(self, x, offset, mask=None):
        return deform_conv2d(x, offset, self.weight, self.bias, self.stride, self.padding, self.dilation,
                             self.deformable_groups, self.groups, mask)


# ---------------------------------------------------------------------------- proposals
def distribute_fpn_proposals(fpn_rois, min_level, max_level, refer_level, refer_scale, pixel_offset=False,
                             rois_num=None, name=None):
    R = _t(fpn_rois).float()
    off = 1.0 if pixel_offset else 0.0
    area = ((R[:, 2] - R[:, 0] + off) * (R[:, 3] - R[:, 1] + off)).clamp(min=0)
    lvl = torch.floor(torch.log2(area.sqrt() / refer_scale + 1e-8) + refer_level).clamp(min_level, max_level).long()
    multi, idxs, nums = [], [], []
    bidx = _rois_batch_idx(rois_num, R.shape[0], R.device) if rois_num is not None else None
    for L in range(min_level, max_level + 1):
        i = (lvl == L).nonzero().flatten()
        multi.append(_wrap(R[i]))
        idxs.append(i)
        if bidx is not None:
            nb = _t(rois_num).numel()
            nums.append(_wrap(torch.bincount(bidx[i], minlength=nb).to(torch.int32)))
    order = torch.cat(idxs)
    restore = torch.empty_like(order)
    restore[order] = torch.arange(order.numel(), device=order.device)
    return multi, _wrap(restore.view(-1, 1)), (nums if rois_num is not None else None)


def generate_proposals(scores, bbox_deltas, img_size, anchors, variances, pre_nms_top_n=6000, post_nms_top_n=1000,
                       nms_thresh=0.5, min_size=0.1, eta=1.0, pixel_offset=False, return_rois_num=False, name=None):
    S, D = _t(scores).float(), _t(bbox_deltas).float()
    A, V = _t(anchors).float().reshape(-1, 4), _t(variances).float().reshape(-1, 4)
    isz = _t(img_size).float()
    N = S.shape[0]
    rois, probs, nums = [], [], []
    off = 1.0 if pixel_offset else 0.0
    for n in range(N):
        sc = S[n].permute(1, 2, 0).reshape(-1)
        dl = D[n].permute(1, 2, 0).reshape(-1, 4)
        k = min(pre_nms_top_n, sc.numel()) if pre_nms_top_n > 0 else sc.numel()
        top = sc.topk(k).indices
        sc, dl, an, va = sc[top], dl[top], A[top], V[top]
        aw, ah = an[:, 2] - an[:, 0] + off, an[:, 3] - an[:, 1] + off
        acx, acy = an[:, 0] + 0.5 * aw, an[:, 1] + 0.5 * ah
        cx = va[:, 0] * dl[:, 0] * aw + acx
        cy = va[:, 1] * dl[:, 1] * ah + acy
        w = torch.exp(torch.clamp(va[:, 2] * dl[:, 2], max=math.log(1000.0 / 16))) * aw
        h = torch.exp(torch.clamp(va[:, 3] * dl[:, 3], max=math.log(1000.0 / 16))) * ah
        bx = torch.stack([cx - w / 2, cy - h / 2, cx + w / 2 - off, cy + h / 2 - off], -1)
        ih, iw = float(isz[n, 0]), float(isz[n, 1])
        bx[:, 0::2] = bx[:, 0::2].clamp(0, iw - off)
        bx[:, 1::2] = bx[:, 1::2].clamp(0, ih - off)
        ws, hs = bx[:, 2] - bx[:, 0] + off, bx[:, 3] - bx[:, 1] + off
        ok = (ws >= max(min_size, 1.0 if pixel_offset else min_size)) & (hs >= max(min_size, 1.0 if pixel_offset
                                                                                      else min_size))
        bx, sc = bx[ok], sc[ok]
        keep = _nms_single(bx, sc, nms_thresh)[:post_nms_top_n]
        rois.append(bx[keep])
        probs.append(sc[keep][:, None])
        nums.append(keep.numel())
    out = (_wrap(torch.cat(rois)), _wrap(torch.cat(probs)))
    if return_rois_num:
        out = out + (_wrap(torch.as_tensor(nums, dtype=torch.int32)),)
    return out


# ---------------------------------------------------------------------------- io
def read_file(filename, name=None):
    with open(filename, "rb") as f:
        data = np.frombuffer(f.read(), dtype=np.uint8)
    return _wrap(torch.from_numpy(data.copy()))


def decode_jpeg(x, mode="unchanged", name=None):
    import io
    from PIL import Image
    img = Image.open(io.BytesIO(_t(x).cpu().numpy().tobytes()))
    if mode == "gray":
        img = img.convert("L")
    elif mode == "rgb":
        img = img.convert("RGB")
    a = np.asarray(img)
    a = a[None] if a.ndim == 2 else a.transpose(2, 0, 1)
    return _wrap(torch.from_numpy(np.ascontiguousarray(a)))


class ConvNormActivation(nn.Sequential):
    def __init__(self, in_channels, out_channels, kernel_size=3, stride=1, padding=None, groups=1,
                 norm_layer=nn.BatchNorm2D, activation_layer=nn.ReLU, dilation=1, bias=None):
        if padding is None:
            padding = (kernel_size - 1) // 2 * dilation
        if bias is None:
            bias = norm_layer is None
        layers = [nn.Conv2D(in_channels, out_channels, kernel_size, stride, padding, dilation=dilation, groups=groups,
                            bias_attr=None if bias else False)]
        if norm_layer is not None:
            layers.append(norm_layer(out_channels))
        if activation_layer is not None:
            layers.append(activation_layer())
        super().__init__(*layers)
