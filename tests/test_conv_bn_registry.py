"""Producer / consumer bookkeeping of the conv -> BN fusion (ops/_conv_bn.py), on CPU tensors."""
import torch

from paddlepaddle_amd.ops import _conv_bn as CB


def test_take_records_the_producer_and_consumes_the_partials_once():
    CB._FEEDS_BN.clear()
    y = torch.zeros(2, 4, 4, 8)
    key = ((2, 4, 4, 8), (8, 8, 1, 1), 1, 0, 1)
    stats = torch.ones(2 * 3 * 8)
    CB.tag(y, key, (stats, 3))
    with torch.enable_grad():
        assert not CB.wanted(key)
        got = CB.take(y.view(-1, 8))          # a view of the conv output finds its producer
        assert got is not None and got[1] == 3 and got[0] is stats
        assert key in CB._FEEDS_BN and CB.wanted(key)
    assert CB.take(y) is None                 # consumed once
    with torch.no_grad():
        assert not CB.wanted(key)             # evaluation does not produce statistics


def test_modified_or_sliced_outputs_do_not_use_the_partials():
    CB._FEEDS_BN.clear()
    key = ((1, 2, 2, 8), (8, 8, 1, 1), 1, 0, 1)
    y = torch.zeros(1, 2, 2, 8)
    CB.tag(y, key, (torch.ones(16), 1))
    y.add_(1.0)                               # in-place change after the statistics were written
    assert CB.take(y) is None
    y2 = torch.zeros(1, 2, 2, 8)
    CB.tag(y2, key, (torch.ones(16), 1))
    assert CB.take(y2[:, :1]) is None         # a slice is not the whole output
    assert CB.take(torch.zeros(1, 2, 2, 8)) is None
