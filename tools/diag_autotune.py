"""Stage-by-stage forward comparison of ResNet-50 NHWC vs NCHW + FLAGS_layout_autotune on the GPU (same weights,
same input): relative max difference after every top-level stage."""
import sys

import torch

sys.path.insert(0, ".")
import paddlepaddle_amd as paddle  # noqa: E402
from paddlepaddle_amd.vision.models import resnet50  # noqa: E402


def build(fmt):
    paddle.seed(5)
    m = resnet50(num_classes=10, data_format=fmt)
    opt = paddle.optimizer.Momentum(learning_rate=0.1, momentum=0.9, parameters=m.parameters(), multi_precision=True)
    m, opt = paddle.amp.decorate(m, opt, level="O2", dtype="bfloat16")
    return m


def run(m, x, autotune, nhwc):
    outs = []
    names = ["conv1", "bn1", "maxpool", "layer1", "layer2", "layer3", "layer4", "avgpool", "fc"]
    hooks = [getattr(m, n).register_forward_post_hook(lambda l, i, o, n=n: outs.append((n, o._t.detach().float())))
             for n in names]
    paddle.set_flags({"FLAGS_layout_autotune": autotune})
    with paddle.amp.auto_cast(level="O2", dtype="bfloat16"):
        y = m(paddle.Tensor(x))
    paddle.set_flags({"FLAGS_layout_autotune": False})
    for h in hooks:
        h.remove()
    res = {}
    for n, o in outs:
        if nhwc and o.dim() == 4:
            o = o.permute(0, 3, 1, 2)
        res[n] = o.reshape(o.shape[0], -1) if n == "fc" or o.dim() != 4 else o
    return res


def main():
    paddle.set_device("gpu:0")
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(8, 3, 64, 64, device="cuda", generator=g).bfloat16()
    a = build("NHWC")
    run(a, x.permute(0, 2, 3, 1).contiguous(), False, True)  # settle per-shape choices
    ra = run(a, x.permute(0, 2, 3, 1).contiguous(), False, True)
    rb_nhwc = run(build("NHWC"), x.permute(0, 2, 3, 1).contiguous(), False, True)
    rc = run(build("NCHW"), x, True, False)
    for n in ra:
        ref = ra[n]
        d1 = (rb_nhwc[n] - ref).abs().max().item() / max(ref.abs().max().item(), 1e-9)
        d2 = (rc[n].reshape(ref.shape) - ref).abs().max().item() / max(ref.abs().max().item(), 1e-9)
        print(f"{n:8s} shape {list(ref.shape)}: nhwc-vs-nhwc(fresh model) {d1:.3e}  nchw_autotune-vs-nhwc {d2:.3e}")


if __name__ == "__main__":
    main()
