"""Sparse tensor algorithms on device index / value buffers (no sparse-library calls).

Reference behaviour: paddle/phi/kernels/sparse/ (coalesce_kernel, sparse_utils_kernel (coo<->csr<->dense),
elementwise_kernel, matmul_kernel (SpMM / SpGEMM / SDDMM), unary_kernel (sum / reshape / transpose / slice),
gpu/conv_kernel.cu + conv.cu.h (rulebook), gpu/pool_kernel.cu).

Representation: a COO tensor is (indices [sparse_ndim, nnz] int64, values [nnz, *dense_dims]) plus the full
shape; CSR is (crows [*batch, rows + 1], cols [nnz], values [nnz]) for 2-D / batched 3-D matrices. The
container is a PyTorch sparse-layout tensor (just index + value storage); every operation here works on
those buffers with sort / search / gather / scatter kernels:
  * coalesce: linearise the sparse coordinates, stable sort, merge equal keys with a segment sum;
  * union (add / subtract): concatenate and coalesce; intersection (multiply): sorted-key search;
  * SpMM: rows gather the dense operand and scatter-add (index_add) into the output rows;
  * SpGEMM: every nnz a[i, k] is paired with row k of b (CSR offsets) and the products coalesced;
  * convolution: a rulebook of (input site, output site) pairs per kernel offset, then one GEMM per
    offset on the gathered active rows with a scatter-add into the output sites (gather-GEMM-scatter).
"""
from __future__ import annotations

import math

import numpy as np
import torch


def linearize(idx, dims):
    """indices [k, nnz] -> int64 keys (row-major over ``dims``)."""
    key = torch.zeros(idx.shape[1], dtype=torch.int64, device=idx.device)
    for d, n in enumerate(dims):
        key = key * int(n) + idx[d]
    return key


def unravel(key, dims):
    out = []
    for n in reversed(dims):
        out.append(key % int(n))
        key = torch.div(key, int(n), rounding_mode="floor")
    return torch.stack(out[::-1], 0) if out else key.new_zeros((0, key.numel()))


def coalesce(idx, vals, dims):
    """Sort by coordinate and sum duplicates."""
    if idx.shape[1] == 0:
        return idx, vals
    key = linearize(idx, dims)
    skey, order = torch.sort(key, stable=True)
    uniq, inverse = torch.unique_consecutive(skey, return_inverse=True)
    out_v = torch.zeros((uniq.numel(),) + tuple(vals.shape[1:]), dtype=vals.dtype, device=vals.device)
    out_v.index_add_(0, inverse, vals[order])
    return unravel(uniq, dims), out_v


def make_coo(idx, vals, shape, coalesced=True):
    t = torch.sparse_coo_tensor(idx, vals, tuple(shape), is_coalesced=coalesced)
    return t


def coo_parts(t):
    """(indices, values, shape, sparse_dims) of a COO tensor, coalesced with our own kernel if needed."""
    idx, vals = t._indices(), t._values()
    sd = t.sparse_dim()
    dims = tuple(t.shape[:sd])
    if not t.is_coalesced():
        idx, vals = coalesce(idx, vals, dims)
    return idx, vals, tuple(t.shape), sd


def csr_parts(t):
    return t.crow_indices(), t.col_indices(), t.values(), tuple(t.shape)


def csr_rows(crows, nnz):
    """Row index of every stored value from the CSR offsets (2-D) / (batch, row) for 3-D."""
    if crows.dim() == 1:
        counts = crows[1:] - crows[:-1]
        return torch.repeat_interleave(torch.arange(counts.numel(), device=crows.device), counts)
    B, R1 = crows.shape
    counts = (crows[:, 1:] - crows[:, :-1]).reshape(-1)
    flat = torch.repeat_interleave(torch.arange(counts.numel(), device=crows.device), counts)
    return torch.stack([torch.div(flat, R1 - 1, rounding_mode="floor"), flat % (R1 - 1)], 0)


def csr_to_coo(t):
    crows, cols, vals, shape = csr_parts(t)
    rows = csr_rows(crows, cols.numel())
    idx = torch.stack([rows, cols], 0) if rows.dim() == 1 else torch.cat([rows, cols[None]], 0)
    return make_coo(idx, vals, shape)


def coo_to_csr(t):
    idx, vals, shape, sd = coo_parts(t)
    if sd == 2:
        R = shape[0]
        counts = torch.bincount(idx[0], minlength=R)
        crows = torch.zeros(R + 1, dtype=torch.int64, device=idx.device)
        crows[1:] = torch.cumsum(counts, 0)
        return torch.sparse_csr_tensor(crows, idx[1], vals, shape)
    if sd == 3:
        B, R = shape[0], shape[1]
        counts = torch.bincount(idx[0] * R + idx[1], minlength=B * R).reshape(B, R)
        crows = torch.zeros(B, R + 1, dtype=torch.int64, device=idx.device)
        crows[:, 1:] = torch.cumsum(counts, 1)
        return torch.sparse_csr_tensor(crows, idx[2], vals, shape)
    raise ValueError("CSR needs a 2-D or 3-D tensor")


def dense_to_coo(d, sparse_dim=None):
    sd = d.dim() if sparse_dim is None else int(sparse_dim)
    mask = d != 0
    if sd < d.dim():
        mask = mask.reshape(d.shape[:sd] + (-1,)).any(-1)
    idx = mask.nonzero().t().contiguous()
    vals = d[tuple(idx)]
    return make_coo(idx, vals, d.shape)


def coo_to_dense(t):
    idx, vals, shape, sd = coo_parts(t)
    out = torch.zeros(shape, dtype=vals.dtype, device=vals.device)
    out[tuple(idx)] = vals
    return out


def to_coo(t):
    if t.layout == torch.sparse_coo:
        return t
    if t.layout == torch.sparse_csr:
        return csr_to_coo(t)
    return dense_to_coo(t)


def same_layout(out_coo, like):
    return coo_to_csr(out_coo) if like.layout == torch.sparse_csr else out_coo


# ----------------------------------------------------------------------------------------- elementwise
def union(a, b, sign_b=1.0):
    ia, va, shape, sd = coo_parts(to_coo(a))
    ib, vb, _, _ = coo_parts(to_coo(b))
    idx = torch.cat([ia, ib], 1)
    vals = torch.cat([va, vb * sign_b if sign_b != 1.0 else vb.to(va.dtype)], 0)
    i, v = coalesce(idx, vals, shape[:sd])
    return make_coo(i, v, shape)


def intersect(a, b, fn):
    """fn(a_vals, b_vals) on the coordinates stored in both (others are zero for products)."""
    ia, va, shape, sd = coo_parts(to_coo(a))
    ib, vb, _, _ = coo_parts(to_coo(b))
    ka, kb = linearize(ia, shape[:sd]), linearize(ib, shape[:sd])
    pos = torch.searchsorted(kb, ka).clamp_max(max(kb.numel() - 1, 0))
    hit = (kb.numel() > 0) & (kb[pos] == ka) if kb.numel() else torch.zeros_like(ka, dtype=torch.bool)
    return make_coo(ia[:, hit], fn(va[hit], vb[pos[hit]]), shape)


def map_values(t, fn):
    if t.layout == torch.sparse_coo:
        i, v, shape, _ = coo_parts(t)
        return make_coo(i, fn(v), shape)
    crows, cols, v, shape = csr_parts(t)
    return torch.sparse_csr_tensor(crows, cols, fn(v), shape)


# ----------------------------------------------------------------------------------------- matmul
def spmm(a, dense):
    """sparse [.., M, K] @ dense [.., K, N] -> dense, by row gather + scatter-add."""
    ia, va, shape, sd = coo_parts(to_coo(a))
    if len(shape) == 2:
        out = torch.zeros(shape[0], dense.shape[-1], dtype=torch.result_type(va, dense), device=dense.device)
        out.index_add_(0, ia[0], va.unsqueeze(-1) * dense[ia[1]])
        return out
    B, M = shape[0], shape[1]
    out = torch.zeros(B * M, dense.shape[-1], dtype=torch.result_type(va, dense), device=dense.device)
    out.index_add_(0, ia[0] * M + ia[1], va.unsqueeze(-1) * dense[ia[0], ia[2]])
    return out.reshape(B, M, -1)


def spgemm(a, b):
    """sparse [M, K] @ sparse [K, N] -> sparse COO: pair each a[i, k] with row k of b, coalesce products."""
    ia, va, (M, K), _ = coo_parts(to_coo(a))
    bc = coo_to_csr(to_coo(b)) if b.layout != torch.sparse_csr else b
    crows, cols, vb, (_, N) = csr_parts(bc)
    start, count = crows[ia[1]], crows[ia[1] + 1] - crows[ia[1]]
    a_of = torch.repeat_interleave(torch.arange(ia.shape[1], device=ia.device), count)
    first = torch.repeat_interleave(start - torch.cumsum(count, 0) + count, count)
    pos = first + torch.arange(a_of.numel(), device=ia.device)
    idx = torch.stack([ia[0][a_of], cols[pos]], 0)
    i, v = coalesce(idx, va[a_of] * vb[pos], (M, N))
    return make_coo(i, v, (M, N))


def sddmm(x, y, mask):
    """(x @ y) evaluated at mask's stored coordinates."""
    im, _, shape, _ = coo_parts(to_coo(mask))
    if len(shape) == 2:
        vals = (x[im[0]] * y.transpose(-2, -1)[im[1]]).sum(-1)
    else:
        vals = (x[im[0], im[1]] * y.transpose(-2, -1)[im[0], im[2]]).sum(-1)
    return make_coo(im, vals, shape)


# ----------------------------------------------------------------------------------------- shape ops
def reduce_sum(t, axis=None, keepdim=False):
    i, v, shape, sd = coo_parts(to_coo(t))
    if axis is None:
        tot = v.sum()
        return make_coo(torch.zeros(1, 1, dtype=torch.int64, device=v.device), tot.reshape(1), (1,))
    axes = [a % len(shape) for a in (axis if isinstance(axis, (list, tuple)) else [axis])]
    dense_axes = [a - sd for a in axes if a >= sd]
    if dense_axes:
        v = v.sum([1 + a for a in dense_axes], keepdim=keepdim)
    sparse_axes = [a for a in axes if a < sd]
    keep = [d for d in range(sd) if d not in sparse_axes]
    if keepdim:
        i2 = i.clone()
        i2[sparse_axes] = 0
        new_sparse = tuple(1 if d in sparse_axes else shape[d] for d in range(sd))
    else:
        i2 = i[keep]
        new_sparse = tuple(shape[d] for d in keep)
    dense_shape = tuple(v.shape[1:])
    if len(new_sparse) == 0:
        return make_coo(torch.zeros(1, 1, dtype=torch.int64, device=v.device), v.sum(0, keepdim=True), (1,) + dense_shape)
    i3, v3 = coalesce(i2, v, new_sparse)
    return make_coo(i3, v3, new_sparse + dense_shape)


def permute(t, perm):
    i, v, shape, sd = coo_parts(to_coo(t))
    if any(p >= sd for p in perm[:sd]):
        raise NotImplementedError("transposing dense dims of a hybrid sparse tensor")
    i2 = i[list(perm)]
    new_shape = tuple(shape[p] for p in perm)
    i3, v3 = coalesce(i2, v, new_shape[:sd])
    return make_coo(i3, v3, new_shape)


def reshape(t, new_shape):
    i, v, shape, sd = coo_parts(to_coo(t))
    dense = tuple(shape[sd:])
    numel_s = int(np.prod(shape[:sd]))
    ns = list(new_shape)
    if -1 in ns:
        known = int(np.prod([s for s in ns if s != -1])) or 1
        ns[ns.index(-1)] = int(np.prod(shape)) // known
    ns_sparse = ns[:len(ns) - len(dense)] if dense else ns
    if int(np.prod(ns_sparse)) != numel_s:
        raise ValueError(f"cannot reshape sparse dims {shape[:sd]} to {ns}")
    key = linearize(i, shape[:sd])
    return make_coo(unravel(key, ns_sparse), v, tuple(ns_sparse) + dense)


def slice_(t, axes, starts, ends):
    i, v, shape, sd = coo_parts(to_coo(t))
    keep = torch.ones(i.shape[1], dtype=torch.bool, device=i.device)
    shift = torch.zeros(sd, 1, dtype=torch.int64, device=i.device)
    new_shape = list(shape)
    for a, s, e in zip(axes, starts, ends):
        a = a % len(shape)
        n = shape[a]
        s = max(0, s + n if s < 0 else s)
        e = min(n, e + n if e < 0 else e)
        new_shape[a] = max(e - s, 0)
        if a < sd:
            keep &= (i[a] >= s) & (i[a] < e)
            shift[a] = s
        else:
            v = v.narrow(1 + a - sd, s, max(e - s, 0))
    return make_coo(i[:, keep] - shift, v[keep], tuple(new_shape))


# ----------------------------------------------------------------------------------------- conv
def _out_size(n, k, s, p, d):
    return (n + 2 * p - d * (k - 1) - 1) // s + 1


def conv_rulebook(idx, spatial, ksize, stride, padding, dilation, subm):
    """-> (out_idx [1 + nd, n_out], [(in_rows, out_rows) per kernel offset]).
    idx: [1 + nd, nnz] (batch, *spatial) coordinates of the active input sites."""
    nd = len(spatial)
    dev = idx.device
    out_sp = [spatial[k] if subm else _out_size(spatial[k], ksize[k], stride[k], padding[k], dilation[k])
              for k in range(nd)]
    B = int(idx[0].max().item()) + 1 if idx.shape[1] else 1
    offsets = list(np.ndindex(*ksize))
    in_key = linearize(idx, [B] + list(spatial))
    pairs = []
    if subm:
        out_idx = idx
        skey, order = torch.sort(in_key)
        for off in offsets:
            # neighbour of output site o at offset k: i = o - pad + k * dil (stride 1)
            nb = [idx[0]] + [idx[1 + d] - padding[d] + off[d] * dilation[d] for d in range(nd)]
            ok = torch.ones(idx.shape[1], dtype=torch.bool, device=dev)
            for d in range(nd):
                ok &= (nb[1 + d] >= 0) & (nb[1 + d] < spatial[d])
            nbk = linearize(torch.stack(nb, 0).clamp_min(0), [B] + list(spatial))
            pos = torch.searchsorted(skey, nbk).clamp_max(max(skey.numel() - 1, 0))
            hit = ok & (skey[pos] == nbk)
            out_rows = torch.nonzero(hit).squeeze(1)
            pairs.append((order[pos[hit]], out_rows))
        return out_idx, pairs, out_sp
    cand = []
    for off in offsets:
        num = [idx[1 + d] + padding[d] - off[d] * dilation[d] for d in range(nd)]
        ok = torch.ones(idx.shape[1], dtype=torch.bool, device=dev)
        o = []
        for d in range(nd):
            ok &= (num[d] >= 0) & (num[d] % stride[d] == 0)
            od = torch.div(num[d], stride[d], rounding_mode="floor")
            ok &= od < out_sp[d]
            o.append(od)
        cand.append((ok, torch.stack([idx[0]] + o, 0)))
    all_keys = torch.cat([linearize(c[1][:, c[0]], [B] + out_sp) for c in cand])
    uniq = torch.unique(all_keys)
    out_idx = unravel(uniq, [B] + out_sp)
    for ok, oc in cand:
        rows_in = torch.nonzero(ok).squeeze(1)
        rows_out = torch.searchsorted(uniq, linearize(oc[:, ok], [B] + out_sp))
        pairs.append((rows_in, rows_out))
    return out_idx, pairs, out_sp


def sparse_conv(x, weight, bias, stride, padding, dilation, groups, subm):
    """x: COO [N, *spatial, C] (sparse dims N + spatial, dense channel dim); weight [*k, C / groups, Cout]."""
    i, v, shape, sd = coo_parts(to_coo(x))
    nd = len(shape) - 2
    ksize = list(weight.shape[:nd])
    out_idx, pairs, out_sp = conv_rulebook(i, list(shape[1:1 + nd]), ksize, stride, padding, dilation, subm)
    cout = weight.shape[-1]
    out = torch.zeros(out_idx.shape[1], cout, dtype=v.dtype, device=v.device)
    w = weight.reshape(-1, weight.shape[-2], cout)
    cin_g = weight.shape[-2]
    for k, (rin, rout) in enumerate(pairs):
        if rin.numel() == 0:
            continue
        feats = v[rin]
        if groups == 1:
            prod = feats @ w[k]
        else:
            cout_g = cout // groups
            prod = torch.cat([feats[:, g * cin_g:(g + 1) * cin_g] @ w[k][:, g * cout_g:(g + 1) * cout_g]
                              for g in range(groups)], 1)
        out.index_add_(0, rout, prod)
    if bias is not None:
        out = out + bias
    return make_coo(out_idx, out, (shape[0],) + tuple(out_sp) + (cout,))


def sparse_max_pool(x, ksize, stride, padding, dilation=None):
    i, v, shape, sd = coo_parts(to_coo(x))
    nd = len(shape) - 2
    dilation = dilation or [1] * nd
    out_idx, pairs, out_sp = conv_rulebook(i, list(shape[1:1 + nd]), ksize, stride, padding, dilation, False)
    C = v.shape[-1]
    out = torch.full((out_idx.shape[1], C), float("-inf"), dtype=v.dtype, device=v.device)
    for rin, rout in pairs:
        if rin.numel():
            out.scatter_reduce_(0, rout[:, None].expand(-1, C), v[rin], reduce="amax")
    return make_coo(out_idx, out, (shape[0],) + tuple(out_sp) + (C,))


def segment_softmax(vals, seg, nseg):
    """Softmax of ``vals`` within each segment id ``seg`` (scatter max / exp / scatter sum)."""
    mx = torch.full((nseg,) + tuple(vals.shape[1:]), float("-inf"), dtype=vals.dtype, device=vals.device)
    mx.scatter_reduce_(0, seg.reshape((-1,) + (1,) * (vals.dim() - 1)).expand_as(vals), vals, reduce="amax")
    e = torch.exp(vals - mx[seg])
    den = torch.zeros_like(mx).index_add_(0, seg, e)
    return e / den[seg]


def softmax(t, axis=-1):
    """Softmax over the stored entries along ``axis`` (missing entries are -inf, i.e. excluded)."""
    i, v, shape, sd = coo_parts(to_coo(t))
    axis = axis % len(shape)
    if axis >= sd:
        return make_coo(i, torch.softmax(v, axis - sd + 1), shape)
    keep = [d for d in range(sd) if d != axis]
    key = linearize(i[keep], [shape[d] for d in keep])
    uniq, seg = torch.unique(key, return_inverse=True)
    return make_coo(i, segment_softmax(v, seg, uniq.numel()), shape)


def sparse_attention(q, k, v, mask, key_padding_mask=None, attn_mask=None):
    """q, k, v [B, H, S, D]; mask CSR / COO [B * H, S, S]: scores only at the mask's coordinates (SDDMM),
    row softmax over them, then SpMM with v."""
    B, H, S, D = q.shape
    im, _, _, _ = coo_parts(to_coo(mask))
    bh, r, c = im[0], im[1], im[2]
    qf, kf, vf = q.reshape(B * H, S, D), k.reshape(B * H, S, D), v.reshape(B * H, S, D)
    s = (qf[bh, r] * kf[bh, c]).sum(-1) / math.sqrt(D)
    b = torch.div(bh, H, rounding_mode="floor")
    if key_padding_mask is not None:
        s = s + key_padding_mask[b, c]
    if attn_mask is not None:
        s = s + attn_mask[r, c]
    p = segment_softmax(s, bh * S + r, B * H * S)
    out = torch.zeros(B * H * S, D, dtype=q.dtype, device=q.device)
    out.index_add_(0, bh * S + r, p.unsqueeze(-1) * vf[bh, c])
    return out.reshape(B, H, S, D)
