"""Recurrent layers. Reference: python/paddle/nn/layer/rnn.py.
Multi-layer SimpleRNN/LSTM/GRU run on the fused MIOpen RNN kernels via ATen (_VF); cells are
plain GEMM + elementwise."""
from __future__ import annotations

import math

import torch

from ...framework.tensor import Tensor, _wrap
from ...tensor._helpers import T
from .. import initializer as I
from .layers import Layer


class RNNCellBase(Layer):
    def get_initial_states(self, batch_ref, shape=None, dtype=None, init_value=0.0, batch_dim_idx=0):
        b = T(batch_ref).shape[batch_dim_idx]
        h = torch.full((b, self.hidden_size), init_value, dtype=T(batch_ref).dtype, device=T(batch_ref).device)
        if isinstance(self, LSTMCell):
            return _wrap(h), _wrap(h.clone())
        return _wrap(h)

    def _init_params(self, input_size, hidden_size, gates, weight_ih_attr, weight_hh_attr, bias_ih_attr,
                     bias_hh_attr):
        std = 1.0 / math.sqrt(hidden_size)
        init = I.Uniform(-std, std)
        self.input_size, self.hidden_size = input_size, hidden_size
        self.weight_ih = self.create_parameter([gates * hidden_size, input_size], weight_ih_attr,
                                               default_initializer=init)
        self.weight_hh = self.create_parameter([gates * hidden_size, hidden_size], weight_hh_attr,
                                               default_initializer=init)
        self.bias_ih = self.create_parameter([gates * hidden_size], bias_ih_attr, is_bias=True,
                                             default_initializer=init)
        self.bias_hh = self.create_parameter([gates * hidden_size], bias_hh_attr, is_bias=True,
                                             default_initializer=init)


class SimpleRNNCell(RNNCellBase):
    def __init__(self, input_size, hidden_size, activation="tanh", weight_ih_attr=None, weight_hh_attr=None,
                 bias_ih_attr=None, bias_hh_attr=None, name=None):
        super().__init__()
        self._init_params(input_size, hidden_size, 1, weight_ih_attr, weight_hh_attr, bias_ih_attr, bias_hh_attr)
        self.activation = activation

    def forward(self, inputs, states=None):
        if states is None:
            states = self.get_initial_states(inputs)
        fn = torch.rnn_tanh_cell if self.activation == "tanh" else torch.rnn_relu_cell
        h = fn(T(inputs), T(states), self.weight_ih._t, self.weight_hh._t, T(self.bias_ih), T(self.bias_hh))
        return _wrap(h), _wrap(h)

    @property
    def state_shape(self):
        return (self.hidden_size,)


class LSTMCell(RNNCellBase):
    def __init__(self, input_size, hidden_size, weight_ih_attr=None, weight_hh_attr=None, bias_ih_attr=None,
                 bias_hh_attr=None, proj_size=0, name=None):
        super().__init__()
        self._init_params(input_size, hidden_size, 4, weight_ih_attr, weight_hh_attr, bias_ih_attr, bias_hh_attr)

    def forward(self, inputs, states=None):
        if states is None:
            states = self.get_initial_states(inputs)
        h, c = torch.lstm_cell(T(inputs), (T(states[0]), T(states[1])), self.weight_ih._t, self.weight_hh._t,
                               T(self.bias_ih), T(self.bias_hh))
        return _wrap(h), (_wrap(h), _wrap(c))

    @property
    def state_shape(self):
        return ((self.hidden_size,), (self.hidden_size,))


class GRUCell(RNNCellBase):
    def __init__(self, input_size, hidden_size, weight_ih_attr=None, weight_hh_attr=None, bias_ih_attr=None,
                 bias_hh_attr=None, name=None):
        super().__init__()
        self._init_params(input_size, hidden_size, 3, weight_ih_attr, weight_hh_attr, bias_ih_attr, bias_hh_attr)

    def forward(self, inputs, states=None):
        if states is None:
            states = self.get_initial_states(inputs)
        h = torch.gru_cell(T(inputs), T(states), self.weight_ih._t, self.weight_hh._t, T(self.bias_ih),
                           T(self.bias_hh))
        return _wrap(h), _wrap(h)

    @property
    def state_shape(self):
        return (self.hidden_size,)


class RNN(Layer):
    """Runs a cell over time. Reference: paddle.nn.RNN(cell, is_reverse, time_major)."""

    def __init__(self, cell, is_reverse=False, time_major=False):
        super().__init__()
        self.cell, self.is_reverse, self.time_major = cell, is_reverse, time_major

    def forward(self, inputs, initial_states=None, sequence_length=None, **kwargs):
        x = T(inputs)
        if not self.time_major:
            x = x.transpose(0, 1)
        steps = range(x.shape[0] - 1, -1, -1) if self.is_reverse else range(x.shape[0])
        states = initial_states
        outs = [None] * x.shape[0]
        for t in steps:
            o, states = self.cell(_wrap(x[t]), states)
            outs[t] = T(o)
        y = torch.stack(outs, 0)
        if not self.time_major:
            y = y.transpose(0, 1)
        return _wrap(y), states


class BiRNN(Layer):
    def __init__(self, cell_fw, cell_bw, time_major=False):
        super().__init__()
        self.rnn_fw = RNN(cell_fw, False, time_major)
        self.rnn_bw = RNN(cell_bw, True, time_major)

    def forward(self, inputs, initial_states=None, sequence_length=None, **kwargs):
        s_fw, s_bw = (None, None) if initial_states is None else initial_states
        o_fw, st_fw = self.rnn_fw(inputs, s_fw)
        o_bw, st_bw = self.rnn_bw(inputs, s_bw)
        return _wrap(torch.cat([T(o_fw), T(o_bw)], -1)), (st_fw, st_bw)


class _RNNBase(Layer):
    _mode = "LSTM"
    _gates = 4

    def __init__(self, input_size, hidden_size, num_layers=1, direction="forward", time_major=False, dropout=0.0,
                 weight_ih_attr=None, weight_hh_attr=None, bias_ih_attr=None, bias_hh_attr=None, name=None,
                 activation="tanh", proj_size=0):
        super().__init__()
        self.input_size, self.hidden_size, self.num_layers = input_size, hidden_size, num_layers
        self.bidirectional = direction in ("bidirect", "bidirectional")
        self.num_directions = 2 if self.bidirectional else 1
        self.time_major, self.dropout = time_major, dropout
        self.activation = activation
        std = 1.0 / math.sqrt(hidden_size)
        init = I.Uniform(-std, std)
        self._flat_names = []
        for layer in range(num_layers):
            for d in range(self.num_directions):
                sfx = f"_l{layer}" + ("_reverse" if d == 1 else "")
                in_sz = input_size if layer == 0 else hidden_size * self.num_directions
                g = self._gates * hidden_size
                for nm, shape, attr, is_bias in (("weight_ih", [g, in_sz], weight_ih_attr, False),
                                                 ("weight_hh", [g, hidden_size], weight_hh_attr, False),
                                                 ("bias_ih", [g], bias_ih_attr, True),
                                                 ("bias_hh", [g], bias_hh_attr, True)):
                    p = self.create_parameter(shape, attr, is_bias=is_bias, default_initializer=init)
                    self.add_parameter(nm + sfx, p)
                    self._flat_names.append(nm + sfx)

    def forward(self, inputs, initial_states=None, sequence_length=None):
        x = T(inputs)
        batch = x.shape[1] if self.time_major else x.shape[0]
        L = self.num_layers * self.num_directions
        weights = [self._parameters[n]._t for n in self._flat_names]
        if initial_states is None:
            h0 = torch.zeros(L, batch, self.hidden_size, dtype=x.dtype, device=x.device)
            c0 = torch.zeros_like(h0)
        else:
            if self._mode == "LSTM":
                h0, c0 = T(initial_states[0]), T(initial_states[1])
            else:
                h0 = T(initial_states)
        train = self.training
        bf = not self.time_major
        if self._mode == "LSTM":
            out, h, c = torch._VF.lstm(x, (h0, c0), weights, True, self.num_layers, self.dropout, train,
                                       self.bidirectional, bf)
            return _wrap(out), (_wrap(h), _wrap(c))
        if self._mode == "GRU":
            out, h = torch._VF.gru(x, h0, weights, True, self.num_layers, self.dropout, train, self.bidirectional,
                                   bf)
        else:
            fn = torch._VF.rnn_tanh if self.activation == "tanh" else torch._VF.rnn_relu
            out, h = fn(x, h0, weights, True, self.num_layers, self.dropout, train, self.bidirectional, bf)
        return _wrap(out), _wrap(h)


class LSTM(_RNNBase):
    _mode, _gates = "LSTM", 4

    def __init__(self, input_size, hidden_size, num_layers=1, direction="forward", time_major=False, dropout=0.0,
                 weight_ih_attr=None, weight_hh_attr=None, bias_ih_attr=None, bias_hh_attr=None, proj_size=0,
                 name=None):  # reference positional order (rnn.py LSTM)
        super().__init__(input_size, hidden_size, num_layers, direction, time_major, dropout, weight_ih_attr,
                         weight_hh_attr, bias_ih_attr, bias_hh_attr, name, proj_size=proj_size)


class GRU(_RNNBase):
    _mode, _gates = "GRU", 3

    def __init__(self, input_size, hidden_size, num_layers=1, direction="forward", time_major=False, dropout=0.0,
                 weight_ih_attr=None, weight_hh_attr=None, bias_ih_attr=None, bias_hh_attr=None, name=None):
        super().__init__(input_size, hidden_size, num_layers, direction, time_major, dropout, weight_ih_attr,
                         weight_hh_attr, bias_ih_attr, bias_hh_attr, name)


class SimpleRNN(_RNNBase):
    _mode, _gates = "RNN", 1

    def __init__(self, input_size, hidden_size, num_layers=1, direction="forward", time_major=False, dropout=0.0,
                 activation="tanh", weight_ih_attr=None, weight_hh_attr=None, bias_ih_attr=None, bias_hh_attr=None,
                 name=None):  # reference positional order: activation after dropout
        super().__init__(input_size, hidden_size, num_layers, direction, time_major, dropout, weight_ih_attr,
                         weight_hh_attr, bias_ih_attr, bias_hh_attr, name, activation=activation)
