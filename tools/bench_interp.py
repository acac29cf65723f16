"""Per-call latency of a saved inference program: the C++ interpreter (_C_interp) vs the Python PIR replay.
A 24-layer MLP (fc + gelu + layer_norm, hidden 256, batch 8) saved with save_inference_model(program_format="pir");
small shapes so the per-op host cost, not the GPU, sets the time."""
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, ".")
import paddlepaddle_amd as paddle  # noqa: E402
from paddlepaddle_amd.framework import pir_json as pir  # noqa: E402


def main():
    dev = "gpu" if paddle.device.is_compiled_with_cuda() and os.environ.get("PADDLE_AMD_FORCE_CPU") != "1" else "cpu"
    paddle.set_device(dev)
    tmp = tempfile.mkdtemp()
    paddle.enable_static()
    main_p, start = paddle.static.Program(), paddle.static.Program()
    with paddle.static.program_guard(main_p, start):
        x = paddle.static.data("x", [8, 256], "float32")
        h = x
        for _ in range(24):
            h = paddle.static.nn.fc(h, 256)
            h = paddle.nn.functional.gelu(h)
            h = paddle.static.nn.layer_norm(h) if hasattr(paddle.static.nn, "layer_norm") else h
        out = paddle.mean(h, axis=-1)
    exe = paddle.static.Executor()
    exe.run(start)
    prefix = os.path.join(tmp, "mlp")
    paddle.static.save_inference_model(prefix, [x], [out], exe, program=main_p, program_format="pir")
    paddle.disable_static()
    feeds = {"x": paddle.to_tensor(np.random.randn(8, 256).astype("float32"))}
    res = {}
    for flag in (True, False):
        paddle.set_flags({"FLAGS_pir_native_interpreter": flag})
        r = pir.load(prefix)
        for _ in range(5):
            r.run(feeds)
        paddle.device.synchronize()
        n = 200
        t0 = time.perf_counter()
        for _ in range(n):
            o = r.run(feeds)
        paddle.device.synchronize()
        res[type(r).__name__] = (time.perf_counter() - t0) / n * 1e3
        res[type(r).__name__ + "_out"] = o[0].numpy()
    paddle.set_flags({"FLAGS_pir_native_interpreter": True})
    err = np.abs(res["NativeRunner_out"] - res["PirRunner_out"]).max()
    print(f"device={dev} ops={r.program.ops.__len__()} native {res['NativeRunner']:.3f} ms/call, "
          f"python replay {res['PirRunner']:.3f} ms/call, speed-up x{res['PirRunner'] / res['NativeRunner']:.2f}, "
          f"max |diff| {err:.1e}", flush=True)


if __name__ == "__main__":
    main()
