"""paddle.cost_model.CostModel (reference python/paddle/cost_model/cost_model.py): the op cost table in the
reference's record format (generated here on CPU with tiny shapes by tools/gen_op_cost_table.py; the shipped
table is measured on MI355X) and per-op profiling of a static program."""
import json
import os
import sys

import pytest

import paddlepaddle_amd as paddle
from paddlepaddle_amd import cost_model as cm

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


def test_table_lookup(tmp_path, monkeypatch):
    import gen_op_cost_table as gen
    rows = gen.measure(dtypes=("float32",), small=True, warmup=1, reps=1, device="cpu")
    p = tmp_path / "t.json"
    p.write_text(json.dumps(rows))
    monkeypatch.setattr(cm, "_TABLE", str(p))
    m = cm.CostModel()
    data = m.static_cost_data()
    assert {r["op"] for r in data} >= {"matmul", "softmax", "conv2d", "layer_norm", "flash_attention"}
    fwd = m.get_static_op_time("matmul")
    bwd = m.get_static_op_time("matmul", forward=False)
    assert fwd["op_time"] >= 0 and bwd["op_time"] >= 0 and "float32" in fwd["config"]
    assert m.get_static_op_time("matmul", dtype="bfloat16") == {}
    with pytest.raises(ValueError):
        m.get_static_op_time(None)


def test_shipped_table_is_well_formed():
    if not os.path.exists(cm._TABLE):
        pytest.skip("MI355X table not generated yet")
    data = cm.CostModel().static_cost_data()
    assert len(data) > 50 and all(r["gpu_time"] > 0 for r in data)
    assert all("MI355" in r["device"] or "AMD" in r["device"] or "gfx950" in r["device"] for r in data)


def test_profile_measure_program():
    m = cm.CostModel()
    try:
        startup, main = m.build_program()
        cost = m.profile_measure(startup, main, device="cpu")
    finally:
        paddle.disable_static()
    assert cost and all(v >= 0 for v in cost.values())
    assert any("linear" in k or "matmul" in k or "addmm" in k for k in cost), cost
