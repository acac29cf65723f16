"""Layer wrappers for the less common ops + the beam-search decoding API.

References: python/paddle/nn/layer/pooling.py (FractionalMaxPool2D/3D), layer/loss.py (HSigmoidLoss,
RNNTLoss, AdaptiveLogSoftmaxWithLoss), python/paddle/nn/decode.py (Decoder, BeamSearchDecoder:161,
dynamic_decode:1238 — the imperative loop; our static programs are recorded from eager execution, so
the same loop serves both modes).
"""
from __future__ import annotations

import collections
import math

import torch

from .layers import Layer
from ..functional import extension as FX
from ..functional.common import gather_tree
from ...framework.tensor import Tensor, _wrap
from ...tensor._helpers import T

__all__ = ["FractionalMaxPool2D", "FractionalMaxPool3D", "HSigmoidLoss", "RNNTLoss", "AdaptiveLogSoftmaxWithLoss",
           "Decoder", "BeamSearchDecoder", "dynamic_decode"]


class FractionalMaxPool2D(Layer):
    def __init__(self, output_size, kernel_size=None, random_u=None, return_mask=False, name=None):
        super().__init__()
        self.output_size, self.kernel_size, self.random_u, self.return_mask = output_size, kernel_size, random_u, \
            return_mask

    def forward(self, x):
        return FX.fractional_max_pool2d(x, self.output_size, self.kernel_size, self.random_u, self.return_mask)


class FractionalMaxPool3D(FractionalMaxPool2D):
    def forward(self, x):
        return FX.fractional_max_pool3d(x, self.output_size, self.kernel_size, self.random_u, self.return_mask)


class HSigmoidLoss(Layer):
    """Hierarchical sigmoid; weight [num_classes - 1, feature_size] (default tree) or
    [num_classes, feature_size] (custom tree), bias [num_classes - 1 | num_classes, 1]."""

    def __init__(self, feature_size, num_classes, weight_attr=None, bias_attr=None, is_custom=False,
                 is_sparse=False, name=None):
        super().__init__()
        if num_classes < 2 and not is_custom:
            raise ValueError("num_classes must not be less than 2 with default tree")
        rows = num_classes if is_custom else num_classes - 1
        self.num_classes = num_classes
        self.weight = self.create_parameter([rows, feature_size], attr=weight_attr)
        self.bias = None if bias_attr is False else self.create_parameter([rows, 1], attr=bias_attr, is_bias=True)

    def forward(self, input, label, path_table=None, path_code=None):
        return FX.hsigmoid_loss(input, label, self.num_classes, self.weight, self.bias, path_table, path_code)


class RNNTLoss(Layer):
    def __init__(self, blank=0, fastemit_lambda=0.001, reduction="mean", name=None):
        super().__init__()
        self.blank, self.fastemit_lambda, self.reduction = blank, fastemit_lambda, reduction

    def forward(self, input, label, input_lengths, label_lengths):
        return FX.rnnt_loss(input, label, input_lengths, label_lengths, self.blank, self.fastemit_lambda,
                            self.reduction)


class AdaptiveLogSoftmaxWithLoss(Layer):
    """Efficient softmax approximation (Grave et al.): a head over the shortlist + one logit per tail cluster,
    each cluster a low-rank (in -> in / div_value^(i+1)) projection."""

    def __init__(self, in_features, n_classes, cutoffs, weight_attr=None, bias_attr=None, div_value=4.0,
                 head_bias=False, name=None):
        super().__init__()
        cutoffs = list(cutoffs)
        if sorted(cutoffs) != cutoffs or min(cutoffs) <= 0 or max(cutoffs) >= n_classes or \
                len(set(cutoffs)) != len(cutoffs):
            raise ValueError("cutoffs should be a sorted list of unique positive ints < n_classes")
        self.in_features, self.n_classes = in_features, n_classes
        self.cutoffs = cutoffs + [n_classes]
        self.shortlist_size = self.cutoffs[0]
        self.n_clusters = len(self.cutoffs) - 1
        self.head_size = self.shortlist_size + self.n_clusters
        self.head_weight = self.create_parameter([in_features, self.head_size], attr=weight_attr)
        self.head_bias = self.create_parameter([self.head_size], attr=bias_attr, is_bias=True) if head_bias else None
        self.tail_weights = []
        for i in range(self.n_clusters):
            hsz = int(in_features // (div_value ** (i + 1)))
            osz = self.cutoffs[i + 1] - self.cutoffs[i]
            proj = self.create_parameter([in_features, hsz], attr=weight_attr)
            out = self.create_parameter([hsz, osz], attr=weight_attr)
            self.add_parameter(f"tail_{i}_proj", proj)
            self.add_parameter(f"tail_{i}_out", out)
            self.tail_weights.append([proj, out])

    def forward(self, input, label):
        return FX.adaptive_log_softmax_with_loss(input, label, self.head_weight, self.tail_weights, self.cutoffs,
                                                 self.head_bias)

    def log_prob(self, input):
        x = T(input)
        head = x @ T(self.head_weight)
        if self.head_bias is not None:
            head = head + T(self.head_bias)
        head_lp = head.log_softmax(-1)
        out = [head_lp[:, :self.shortlist_size]]
        for i, (proj, o) in enumerate(self.tail_weights):
            tail_lp = ((x @ T(proj)) @ T(o)).log_softmax(-1)
            out.append(tail_lp + head_lp[:, self.shortlist_size + i:self.shortlist_size + i + 1])
        return _wrap(torch.cat(out, 1))

    def predict(self, input):
        return _wrap(T(self.log_prob(input)).argmax(1))


# ------------------------------------------------------------------------------------------ decoding
def _map(fn, *structs):
    s0 = structs[0]
    if isinstance(s0, (list, tuple)) and not hasattr(s0, "_fields"):
        return type(s0)(_map(fn, *xs) for xs in zip(*structs))
    if hasattr(s0, "_fields"):
        return type(s0)(*(_map(fn, *xs) for xs in zip(*structs)))
    if isinstance(s0, dict):
        return {k: _map(fn, *(s[k] for s in structs)) for k in s0}
    return fn(*structs)


def _flatten(s):
    if isinstance(s, (list, tuple)):
        return [y for x in s for y in _flatten(x)]
    if isinstance(s, dict):
        return [y for k in s for y in _flatten(s[k])]
    return [s]


class _Acc:
    """Per-leaf list of step outputs (a leaf, not a structure, for _map)."""

    def __init__(self, first):
        self.items = [first]


class Decoder:
    """Base decoder: initialize(inits) -> (inputs, states, finished); step(time, inputs, states) ->
    (outputs, next_states, next_inputs, finished); optional finalize."""

    def initialize(self, inits):
        raise NotImplementedError

    def step(self, time, inputs, states, **kwargs):
        raise NotImplementedError

    def finalize(self, outputs, final_states, sequence_lengths):
        raise NotImplementedError

    @property
    def tracks_own_finished(self):
        return False


class BeamSearchDecoder(Decoder):
    OutputWrapper = collections.namedtuple("OutputWrapper", ("scores", "predicted_ids", "parent_ids"))
    StateWrapper = collections.namedtuple("StateWrapper", ("cell_states", "log_probs", "finished", "lengths"))
    kinf = 1e9

    def __init__(self, cell, start_token, end_token, beam_size, embedding_fn=None, output_fn=None):
        self.cell, self.embedding_fn, self.output_fn = cell, embedding_fn, output_fn
        self.start_token, self.end_token, self.beam_size = start_token, end_token, beam_size

    @staticmethod
    def tile_beam_merge_with_batch(x, beam_size):
        t = T(x)
        t = t.unsqueeze(1).expand(t.shape[0], beam_size, *t.shape[1:])
        return _wrap(t.reshape(-1, *t.shape[2:]))

    def _split_batch_beams(self, x):
        t = T(x)
        return _wrap(t.reshape(-1, self.beam_size, *t.shape[1:]))

    def _merge_batch_beams(self, x):
        t = T(x)
        return _wrap(t.reshape(-1, *t.shape[2:]))

    def _expand_to_beam_size(self, x):
        t = T(x)
        return _wrap(t.unsqueeze(1).expand(t.shape[0], self.beam_size, *t.shape[1:]).contiguous())

    def _gather(self, x, indices):
        t, idx = T(x), T(indices)
        b = torch.arange(idx.shape[0], device=idx.device).view(-1, 1).expand_as(idx)
        return _wrap(t[b, idx])

    def initialize(self, initial_cell_states):
        state = T(_flatten(initial_cell_states)[0])
        self.batch_size = state.shape[0]
        dev = state.device
        cell_states = _map(self._expand_to_beam_size, initial_cell_states)
        inputs = torch.full((self.batch_size, self.beam_size), self.start_token, dtype=torch.int64, device=dev)
        lp = torch.tensor([[0.0] + [-self.kinf] * (self.beam_size - 1)], dtype=torch.float32, device=dev)
        log_probs = lp.repeat(self.batch_size, 1)
        finished = torch.zeros(self.batch_size, self.beam_size, dtype=torch.bool, device=dev)
        lengths = torch.zeros_like(inputs)
        init_inputs = self.embedding_fn(_wrap(inputs)) if self.embedding_fn else _wrap(inputs)
        return init_inputs, self.StateWrapper(cell_states, _wrap(log_probs), _wrap(finished), _wrap(lengths)), \
            _wrap(finished)

    def _mask_probs(self, probs, finished):
        noend = torch.full((self.vocab_size,), -self.kinf, dtype=probs.dtype, device=probs.device)
        noend[self.end_token] = 0.0
        f = finished.to(probs.dtype).unsqueeze(2)
        return f * noend - probs * (f - 1)

    def _beam_search_step(self, time, logits, next_cell_states, beam_state):
        lg = T(logits)
        self.vocab_size = lg.shape[-1]
        step_lp = torch.log(torch.softmax(lg, -1))
        step_lp = self._mask_probs(step_lp, T(beam_state.finished))
        log_probs = step_lp + T(beam_state.log_probs).unsqueeze(2)
        scores = log_probs.reshape(-1, self.beam_size * self.vocab_size)
        top_s, top_i = torch.topk(scores, self.beam_size)
        beam_idx = top_i // self.vocab_size
        tok_idx = top_i % self.vocab_size
        next_lp = self._gather(scores, top_i)
        next_cell = _map(lambda x: self._gather(x, beam_idx), next_cell_states)
        next_fin = T(self._gather(beam_state.finished, beam_idx))
        next_len = T(self._gather(beam_state.lengths, beam_idx))
        next_len = next_len + (~next_fin).to(next_len.dtype)
        next_fin = next_fin | (tok_idx == self.end_token)
        out = self.OutputWrapper(_wrap(top_s), _wrap(tok_idx), _wrap(beam_idx))
        st = self.StateWrapper(next_cell, next_lp, _wrap(next_fin), _wrap(next_len))
        return out, st

    def step(self, time, inputs, states, **kwargs):
        inputs = _map(self._merge_batch_beams, inputs)
        cell_states = _map(self._merge_batch_beams, states.cell_states)
        cell_outputs, next_cell_states = self.cell(inputs, cell_states, **kwargs)
        cell_outputs = _map(self._split_batch_beams, cell_outputs)
        next_cell_states = _map(self._split_batch_beams, next_cell_states)
        if self.output_fn is not None:
            cell_outputs = self.output_fn(cell_outputs)
        out, st = self._beam_search_step(time, cell_outputs, next_cell_states, states)
        ids = out.predicted_ids
        ids.stop_gradient = True
        next_inputs = self.embedding_fn(ids) if self.embedding_fn else ids
        return out, st, next_inputs, st.finished

    def finalize(self, outputs, final_states, sequence_lengths):
        pred = gather_tree(outputs.predicted_ids, outputs.parent_ids)
        return pred, final_states

    @property
    def tracks_own_finished(self):
        return True


def dynamic_decode(decoder, inits=None, max_step_num=None, output_time_major=False, impute_finished=False,
                   is_test=False, return_length=False, **kwargs):
    """Run ``decoder`` step by step until every sequence finished or ``max_step_num`` is exceeded."""
    inputs, states, finished = decoder.initialize(inits)
    seq_len = torch.zeros(T(finished).shape, dtype=torch.int64, device=T(finished).device)
    outs = None
    step = 0
    while not bool(T(finished).all()):
        t = _wrap(torch.full((1,), step, dtype=torch.int64))
        step_out, next_states, next_inputs, next_finished = decoder.step(t, inputs, states, **kwargs)
        if not decoder.tracks_own_finished:
            nf = T(next_finished) | T(finished)
            next_finished = _wrap(nf)
            next_len = seq_len + (~T(finished)).to(torch.int64)
            if impute_finished:
                fmask = T(finished)

                def keep(old, new):
                    o, n = T(old), T(new)
                    m = fmask.view(fmask.shape[0], *([1] * (o.dim() - 1)))
                    return _wrap(torch.where(m, o, n))
                next_states = _map(keep, states, next_states)
        else:
            next_len = T(getattr(next_states, "lengths", _wrap(seq_len)))
        if outs is None:
            outs = _map(lambda x: _Acc(T(x)), step_out)
        else:
            _map(lambda x, acc: acc.items.append(T(x)), step_out, outs)
        inputs, states, finished, seq_len = next_inputs, next_states, next_finished, next_len
        step += 1
        if max_step_num is not None and step > max_step_num:
            break
    final = _map(lambda acc: _wrap(torch.stack(acc.items, 0)), outs) if outs is not None else None
    final_states = states
    try:
        final, final_states = decoder.finalize(final, final_states, _wrap(seq_len))
    except NotImplementedError:
        pass
    if not output_time_major:
        final = _map(lambda x: _wrap(T(x).transpose(0, 1)), final)
    return (final, final_states, _wrap(seq_len)) if return_length else (final, final_states)
