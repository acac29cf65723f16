"""PipelineLayer stage boundaries (reference pp_layers.py:93 SegmentLayers): uniform with the remainder on the last
stages, ``layer:<regex>`` balancing the matching layers, explicit boundary lists, virtual stages."""
import pytest

import paddlepaddle_amd.nn as nn
from paddlepaddle_amd.distributed.fleet.meta_parallel import LayerDesc, SegmentLayers


class Embed(nn.Layer):
    pass


class DecoderLayer(nn.Layer):
    pass


class Head(nn.Layer):
    pass


def _descs(n_dec):
    return [LayerDesc(Embed)] + [LayerDesc(DecoderLayer) for _ in range(n_dec)] + [LayerDesc(Head)]


def test_uniform_puts_the_remainder_on_the_last_stages():
    assert SegmentLayers(_descs(8), 4).do_segment() == [0, 2, 4, 7, 10]
    assert SegmentLayers(list(range(35)), 4).do_segment() == [0, 8, 17, 26, 35]
    assert SegmentLayers(list(range(8)), 4).do_segment() == [0, 2, 4, 6, 8]


def test_layer_regex_balances_matching_layers():
    d = _descs(8)
    # embedding joins the first stage, head the last; 2 decoders per stage
    assert SegmentLayers(d, 4, "layer:DecoderLayer").do_segment() == [0, 3, 5, 7, 10]
    assert SegmentLayers(d, 4, "layer:decoderlayer").do_segment() == [0, 3, 5, 7, 10]  # case-insensitive
    assert SegmentLayers(d, 2, "layer:Decoder", num_virtual_pipeline_stage=2).do_segment() == [0, 3, 5, 7, 10]
    with pytest.raises(ValueError):
        SegmentLayers(_descs(6), 4, "layer:DecoderLayer").do_segment()  # 6 does not divide into 4
    with pytest.raises(ValueError):
        SegmentLayers(d, 2, "layer:NoSuchLayer").do_segment()


def test_boundary_lists():
    d = _descs(8)
    assert SegmentLayers(d, 2, [0, 4]).do_segment() == [0, 4, 10]
    assert SegmentLayers(d, 2, [0, 4, 10]).do_segment() == [0, 4, 10]
    with pytest.raises(ValueError):
        SegmentLayers(d, 3, [0, 4]).do_segment()
    with pytest.raises(ValueError):
        SegmentLayers(d, 2, [1, 4, 10]).do_segment()


def test_pipeline_layer_uses_it(monkeypatch):
    from paddlepaddle_amd.distributed.fleet.meta_parallel import PipelineLayer
    pl = PipelineLayer(_descs(8), num_stages=4, seg_method="layer:DecoderLayer")
    assert pl.segment_parts == [0, 3, 5, 7, 10]
    assert [type(l).__name__ for l in pl.run_function] == ["Embed", "DecoderLayer", "DecoderLayer"]


def test_recompute_interval_checkpoints_segments_of_k_layers(monkeypatch):
    import numpy as np
    import paddlepaddle_amd as paddle
    import importlib
    R = importlib.import_module("paddlepaddle_amd.distributed.fleet.recompute")
    from paddlepaddle_amd.distributed.fleet.meta_parallel import PipelineLayer

    def build(k):
        paddle.seed(3)
        return PipelineLayer([LayerDesc(nn.Linear, 6, 6) for _ in range(5)], num_stages=1, recompute_interval=k)

    x = paddle.randn([4, 6])
    x.stop_gradient = False
    ref = build(0)
    ref(x).sum().backward()
    calls = []
    orig = R.recompute
    monkeypatch.setattr(R, "recompute", lambda fn, *a, **kw: (calls.append(len(a)), orig(fn, *a, **kw))[1])
    pl = build(2)
    pl(x).sum().backward()
    assert len(calls) == 3  # segments [0, 2), [2, 4), [4, 5)
    for p, q in zip(ref.parameters(), pl.parameters()):
        np.testing.assert_allclose(p.grad.numpy(), q.grad.numpy(), rtol=1e-5, atol=1e-6)
    calls.clear()
    x2 = paddle.randn([4, 6])  # stop_gradient input: the first segment's output still needs grad (parameters)
    pl(x2).sum().backward()
    assert len(calls) == 2


def test_recompute_sequential_checkpoints_all_but_the_last_segment(monkeypatch):
    import importlib
    import numpy as np
    import paddlepaddle_amd as paddle
    R = importlib.import_module("paddlepaddle_amd.distributed.fleet.recompute")
    paddle.seed(4)
    seq = paddle.nn.Sequential(*[paddle.nn.Linear(5, 5) for _ in range(6)])
    x = paddle.randn([3, 5])
    x.stop_gradient = False
    seq(x).sum().backward()
    ref = [p.grad.numpy().copy() for p in seq.parameters()]
    seq.clear_gradients()
    calls = []
    orig = R.recompute
    monkeypatch.setattr(R, "recompute", lambda fn, *a, **kw: (calls.append(kw.get("preserve_rng_state")),
                                                              orig(fn, *a, **kw))[1])
    R.recompute_sequential({"segments": 3, "preserve_rng_state": False}, seq, x).sum().backward()
    assert calls == [False, False]  # segments [0, 2) and [2, 4) checkpointed, [4, 6) plain
    for r, p in zip(ref, seq.parameters()):
        np.testing.assert_allclose(r, p.grad.numpy(), rtol=1e-5, atol=1e-6)
    calls.clear()
    R.recompute_sequential({"segments": 1}, seq, x)
    assert calls == []
