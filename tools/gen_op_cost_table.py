"""Measure the per-op cost table that paddle.cost_model.CostModel.static_cost_data() serves (reference:
python/paddle/cost_model/static_op_benchmark.json, a table of op forward / backward GPU times per config).

Every entry runs the framework's public op (paddle.<name> / paddle.nn.functional.<name>) on the device,
times forward and forward+backward with device events (median of --reps after --warmup), and records
backward = (fwd+bwd) - fwd. Run on the MI355X:  python tools/gen_op_cost_table.py --out <json>
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import paddlepaddle_amd as paddle  # noqa: E402

F = paddle.nn.functional


def _cases(small):
    s = (lambda big, tiny: tiny if small else big)
    img = s([16, 128, 257, 257], [2, 3, 9, 9])
    act = s([8192, 8192], [64, 64])
    tok = s([16, 2048, 5120], [2, 8, 32])
    C = [
        ("abs", paddle.abs, [img], {}), ("exp", paddle.exp, [act], {}), ("log", paddle.log, [act], {}),
        ("sqrt", paddle.sqrt, [act], {}), ("rsqrt", paddle.rsqrt, [act], {}), ("tanh", paddle.tanh, [act], {}),
        ("sigmoid", F.sigmoid, [act], {}), ("relu", F.relu, [img], {}), ("gelu", F.gelu, [tok], {}),
        ("silu", F.silu, [tok], {}), ("leaky_relu", F.leaky_relu, [img], {}), ("square", paddle.square, [act], {}),
        ("scale", lambda x: paddle.scale(x, 2.0, 1.0), [act], {}),
        ("add", paddle.add, [act, act], {}), ("subtract", paddle.subtract, [act, act], {}),
        ("multiply", paddle.multiply, [act, act], {}), ("divide", paddle.divide, [act, act], {}),
        ("maximum", paddle.maximum, [act, act], {}), ("pow", lambda x: paddle.pow(x, 2.0), [act], {}),
        ("matmul", paddle.matmul, [s([4096, 5120], [16, 32]), s([5120, 5120], [32, 24])], {}),
        ("matmul", paddle.matmul, [s([4096, 5120], [16, 32]), s([5120, 20480], [32, 48])], {}),
        ("matmul", paddle.matmul, [s([32, 2048, 128], [2, 8, 16]), s([32, 128, 2048], [2, 16, 8])], {}),
        ("linear", lambda x, w, b: F.linear(x, w, b), [s([4096, 5120], [16, 32]), s([5120, 15360], [32, 24]),
                                                       s([15360], [24])], {}),
        ("softmax", F.softmax, [s([8, 40, 2048, 2048], [2, 2, 8, 8])], {}),
        ("log_softmax", F.log_softmax, [s([4096, 50304], [16, 40])], {}),
        ("layer_norm", lambda x: F.layer_norm(x, x.shape[-1:]), [tok], {}),
        ("rms_norm", lambda x, w: paddle.incubate.nn.functional.fused_rms_norm(x, w, None, 1e-6, 2)[0],
         [tok, tok[-1:]], {}),
        ("batch_norm", lambda x: F.batch_norm(x, paddle.zeros([x.shape[1]]), paddle.ones([x.shape[1]]),
                                              training=True), [s([256, 64, 56, 56], [2, 4, 5, 5])], {}),
        ("conv2d", lambda x, w: F.conv2d(x, w, padding=1), [s([256, 64, 56, 56], [2, 4, 6, 6]),
                                                            s([64, 64, 3, 3], [4, 4, 3, 3])], {}),
        ("conv2d", lambda x, w: F.conv2d(x, w, stride=2, padding=3), [s([256, 3, 224, 224], [2, 3, 12, 12]),
                                                                      s([64, 3, 7, 7], [4, 3, 7, 7])], {}),
        ("max_pool2d", lambda x: F.max_pool2d(x, 3, 2, 1), [s([256, 64, 112, 112], [2, 4, 8, 8])], {}),
        ("avg_pool2d", lambda x: F.avg_pool2d(x, 2, 2), [s([256, 64, 112, 112], [2, 4, 8, 8])], {}),
        ("mean", paddle.mean, [act], {}), ("sum", paddle.sum, [act], {}), ("max", paddle.max, [act], {}),
        ("logsumexp", lambda x: paddle.logsumexp(x, axis=-1), [act], {}),
        ("transpose", lambda x: paddle.transpose(x, [0, 2, 1, 3]), [s([16, 2048, 40, 128], [2, 8, 2, 4])], {}),
        ("concat", lambda x, y: paddle.concat([x, y], axis=-1), [tok, tok], {}),
        ("cast", lambda x: paddle.cast(x, "float16"), [act], {}),
        ("dropout", lambda x: F.dropout(x, 0.1), [tok], {}),
        ("cross_entropy", lambda x, y: F.cross_entropy(x, y), [s([4096, 50304], [16, 40]), ("int", s([4096, 1], [16, 1]),
                                                                                           s(50304, 40))], {}),
        ("embedding", lambda i, w: F.embedding(i, w), [("int", s([16, 2048], [2, 8]), s(50304, 40)),
                                                       s([50304, 5120], [40, 32])], {}),
        ("flash_attention", lambda q, k, v: F.scaled_dot_product_attention(q, k, v, is_causal=True),
         [s([4, 2048, 40, 128], [1, 16, 2, 32])] * 3, {}),
        ("topk", lambda x: paddle.topk(x, 8)[0], [s([4096, 50304], [16, 40])], {}),
        ("cumsum", lambda x: paddle.cumsum(x, axis=-1), [act], {}),
    ]
    return C


def _make(spec, dtype, dev):
    if isinstance(spec, tuple) and spec[0] == "int":
        return paddle.to_tensor(torch.randint(0, spec[2], spec[1], device=dev))
    t = torch.rand(spec, device=dev, dtype=torch.float32) + 0.5
    t = t.to(dtype)
    x = paddle.to_tensor(t)
    x.stop_gradient = False
    return x


def _timer(dev):
    if dev.type == "cuda":
        def run(fn):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            b.synchronize()
            return a.elapsed_time(b)
    else:
        def run(fn):
            t = time.perf_counter()
            fn()
            return (time.perf_counter() - t) * 1e3
    return run


def measure(dtypes=("float32", "bfloat16"), small=False, warmup=3, reps=10, device=None):
    dev = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
    paddle.set_device("gpu" if dev.type == "cuda" else "cpu")
    timed = _timer(dev)
    rows = []
    counts = {}
    for name, fn, specs, kw in _cases(small):
        for dt in dtypes:
            tdt = getattr(torch, dt)
            try:
                args = [_make(sp, tdt, dev) for sp in specs]
                def fwd():
                    return fn(*args, **kw)
                def fwdbwd():
                    y = fn(*args, **kw)
                    y.astype("float32").sum().backward()
                for _ in range(warmup):
                    fwdbwd()
                tf = statistics.median(timed(fwd) for _ in range(reps))
                tb = statistics.median(timed(fwdbwd) for _ in range(reps))
            except Exception as e:  # an op/dtype pair the framework does not support: recorded, not fatal
                print(f"skip {name} {dt}: {type(e).__name__}: {str(e)[:100]}", flush=True)
                continue
            k = counts.get(name, 0)
            counts[name] = k + 1
            cfg = "".join(f"{chr(ord('x') + i) if i < 3 else 'in' + str(i)} (Variable) - dtype: "
                          f"{'int64' if isinstance(sp, tuple) else dt}, shape: {sp[1] if isinstance(sp, tuple) else sp}\n"
                          for i, sp in enumerate(specs))
            rows.append({"name": f"{name}_{k}", "op": name, "config": cfg, "device": torch.cuda.get_device_name(dev)
                         if dev.type == "cuda" else "cpu", "gpu_time": round(tf, 5),
                         "gpu_time_backward": round(max(tb - tf, 0.0), 5)})
            print(f"{name:16s} {dt:9s} fwd {tf:9.4f} ms  bwd {max(tb - tf, 0):9.4f} ms", flush=True)
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/mi355x_op_benchmark.json",
                    help="copy the result to paddlepaddle_amd/cost_model/mi355x_op_benchmark.json to ship it")
    ap.add_argument("--small", action="store_true")
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    rows = measure(small=a.small, reps=a.reps)
    with open(a.out, "w") as f:
        json.dump(rows, f, indent=1)
    print(f"wrote {len(rows)} entries to {a.out}")


if __name__ == "__main__":
    main()
