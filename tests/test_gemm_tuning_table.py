"""GEMM backend decisions persist as JSON (committed table + per-user overlay) — CPU test of the table logic."""
import json

import torch

from paddlepaddle_amd.ops import gemm as G


def test_canon_keys_are_json_stable():
    key = ("mm", 4096, 5120, 5120, torch.bfloat16, (True, False), None)
    c = G._canon(key)
    assert c == ("mm", 4096, 5120, 5120, "torch.bfloat16", (True, False), None)
    assert G._canon(json.loads(G._key_str(c))) == c


def test_persist_and_reload(tmp_path, monkeypatch):
    path = tmp_path / "tuning.json"
    monkeypatch.setenv("PADDLE_AMD_TUNING_FILE", str(path))
    key = G._canon(("mm", 8, 16, 32, torch.float16))
    G._persist(key, "hip")
    G._persist(G._canon(("mm", 1, 2, 3, torch.bfloat16)), "blas")
    d = json.loads(path.read_text())
    assert len(d["choices"]) == 2
    monkeypatch.setattr(G, "_CHOICE", {})
    monkeypatch.setattr(G, "_TABLE_LOADED", False)
    monkeypatch.setattr(G, "_TUNING_DIR", str(tmp_path / "none"))
    assert G.known(("mm", 8, 16, 32, torch.float16))
    assert G._CHOICE[key] == "hip"
    # a cached decision is reused without timing, unless it is not a candidate any more
    assert G.choose(("mm", 8, 16, 32, torch.float16), {"hip": None, "blas": None}) == "hip"
    out = tmp_path / "dump.json"
    G.dump_tuning_table(str(out))
    assert G._read_table(str(out))[key] == "hip"


def test_committed_table_parses():
    import glob
    import os
    for p in glob.glob(os.path.join(G._TUNING_DIR, "*.json")):
        t = G._read_table(p)
        assert t, p
