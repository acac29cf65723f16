"""paddle.save state-dict layout and the distributed checkpoint files (single process, CPU).
Reference: python/paddle/framework/io.py:163 (_build_saved_state_dict), python/paddle/distributed/checkpoint/
(save_state_dict.py, load_state_dict.py, metadata.py)."""
import os
import pickle

import numpy as np
import pytest

import paddlepaddle_amd as paddle
from paddlepaddle_amd.distributed.checkpoint import flatten_state_dict
from paddlepaddle_amd.distributed.checkpoint.metadata import LocalTensorIndex, LocalTensorMetadata, Metadata


class _Raw(pickle.Unpickler):
    """Reads the file as plain data: records which globals it names, builds dummies for them."""

    def __init__(self, f):
        super().__init__(f)
        self.globals = set()

    def find_class(self, module, name):
        self.globals.add((module, name))
        if module.startswith("numpy") or module in ("builtins", "collections", "_codecs"):
            return super().find_class(module, name)
        return type(name, (), {})


def test_state_dict_saved_as_ndarrays_with_name_table(tmp_path):
    lin = paddle.nn.Linear(3, 2)
    p = str(tmp_path / "m.pdparams")
    paddle.save(lin.state_dict(), p)
    with open(p, "rb") as f:
        raw = _Raw(f).load()
    assert isinstance(raw["weight"], np.ndarray) and raw["weight"].shape == (3, 2)
    assert raw["StructuredToParameterName@@"] == {"weight": lin.weight.name, "bias": lin.bias.name}
    loaded = paddle.load(p)
    assert set(loaded) == {"weight", "bias"}
    assert loaded["weight"].name == lin.weight.name
    np.testing.assert_array_equal(loaded["weight"].numpy(), lin.weight.numpy())
    kept = paddle.load(p, keep_name_table=True)
    assert "StructuredToParameterName@@" in kept


def test_bf16_state_dict_round_trip(tmp_path):
    t = paddle.to_tensor(np.linspace(-3, 3, 12).astype("float32")).astype("bfloat16")
    p = str(tmp_path / "b.pdparams")
    paddle.save({"x": t}, p)
    assert paddle.load(p, return_numpy=True)["x"].dtype == np.uint16
    back = paddle.load(p)["x"]
    assert back.dtype == paddle.bfloat16
    np.testing.assert_array_equal(back.astype("float32").numpy(), t.astype("float32").numpy())


def test_non_state_dict_objects_keep_tuple_form(tmp_path):
    obj = {"step": 3, "nested": [paddle.ones([2])]}
    p = str(tmp_path / "o.pd")
    paddle.save(obj, p)
    got = paddle.load(p)
    assert got["step"] == 3 and got["nested"][0].numpy().tolist() == [1.0, 1.0]


def test_flatten_state_dict_mapping():
    flat, mapping = flatten_state_dict({"model": {"w0": 1, "sub": {"b": 2}}, "step": 3})
    assert flat == {"model.w0": 1, "model.sub.b": 2, "step": 3}
    assert mapping["model.sub.b"] == ("model", "sub", "b")


def test_distributed_checkpoint_single_process_layout(tmp_path):
    ck = str(tmp_path / "ck")
    lin = paddle.nn.Linear(4, 3)
    sd = {"model": lin.state_dict(), "extra": paddle.arange(6, dtype="float32").reshape([2, 3])}
    paddle.distributed.save_state_dict(sd, ck)
    paddle.distributed.save_state_dict(sd, ck)  # a second save gets the next unique id
    assert sorted(os.listdir(ck)) == ["0.metadata", "0_0.distcp", "0_1.distcp", "1.metadata"]
    with open(os.path.join(ck, "1.metadata"), "rb") as f:
        r = _Raw(f)
        r.load()
    assert ("paddle.distributed.checkpoint.metadata", "Metadata") in r.globals
    assert ("paddle.distributed.checkpoint.metadata", "LocalTensorIndex") in r.globals
    md = paddle.load(os.path.join(ck, "1.metadata"))
    assert isinstance(md, Metadata)
    assert md.state_dict_metadata["model.weight"] == [LocalTensorMetadata((0, 0), (4, 3), "float32")]
    assert md.storage_metadata[LocalTensorIndex("extra", (0, 0))] == "0_1.distcp"
    assert md.flat_mapping["model.bias"] == ("model", "bias")
    target = {"model": paddle.nn.Linear(4, 3).state_dict(), "extra": paddle.zeros([2, 3])}
    paddle.distributed.load_state_dict(target, ck)
    np.testing.assert_array_equal(target["model"]["weight"].numpy(), lin.weight.numpy())
    np.testing.assert_array_equal(target["extra"].numpy(), np.arange(6).reshape(2, 3))


def test_checkpoint_loader_refuses_foreign_globals(tmp_path):
    class Evil:
        def __reduce__(self):
            return (os.system, ("echo pwned",))
    p = str(tmp_path / "bad.metadata")
    with open(p, "wb") as f:
        pickle.dump({"x": Evil()}, f)
    with pytest.raises(pickle.UnpicklingError):
        paddle.load(p)
