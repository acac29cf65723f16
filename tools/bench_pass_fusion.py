"""Static-program latency before / after the fuse_gemm_epilogue pass (distributed/passes/program_passes.py):
a bf16 transformer-FFN block written as matmul + bias-add + GELU, run through the static Executor."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import paddlepaddle_amd as paddle  # noqa: E402
from paddlepaddle_amd.distributed import passes as dp  # noqa: E402


def build(M, H, F):
    paddle.enable_static()
    main, st = paddle.static.Program(), paddle.static.Program()
    with paddle.static.program_guard(main, st):
        x = paddle.static.data("x", [M, H], "bfloat16")
        w1 = paddle.create_parameter([H, F], "bfloat16")
        b1 = paddle.create_parameter([F], "bfloat16", is_bias=True)
        w2 = paddle.create_parameter([F, H], "bfloat16")
        b2 = paddle.create_parameter([H], "bfloat16", is_bias=True)
        h = paddle.nn.functional.gelu(paddle.matmul(x, w1) + b1, approximate=True)
        y = paddle.matmul(h, w2) + b2
    return main, st, y


def timeit(exe, main, feed, y, reps=20):
    for _ in range(3):
        exe.run(main, feed=feed, fetch_list=[y], return_numpy=False)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        out = exe.run(main, feed=feed, fetch_list=[y], return_numpy=False)
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3, out[0]


def main():
    M, H, F = 8192, 5120, 20480
    paddle.set_device("gpu")
    main_p, st, y = build(M, H, F)
    exe = paddle.static.Executor(paddle.CUDAPlace(0))
    xv = paddle.to_tensor(torch.randn(M, H, device="cuda", dtype=torch.bfloat16))
    feed = {"x": xv}
    t0, r0 = timeit(exe, main_p, feed, y)
    ctx = dp.new_pass("fuse_gemm_epilogue", {"fetch_vars": [y]}).apply([main_p], [st])
    t1, r1 = timeit(exe, main_p, feed, y)
    err = (r0._t.float() - r1._t.float()).abs().max().item()
    flops = 2 * 2 * M * H * F
    print(f"FFN M{M} H{H} F{F} bf16: unfused {t0:.3f} ms ({flops / t0 / 1e9:.0f} TF/s), fused "
          f"{t1:.3f} ms ({flops / t1 / 1e9:.0f} TF/s), x{t0 / t1:.3f}, fused nodes "
          f"{ctx.get_attr('fuse_gemm_epilogue.fused')}, max|diff| {err:.3g}")


if __name__ == "__main__":
    main()
