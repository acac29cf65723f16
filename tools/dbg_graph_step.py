"""Debug: eager vs eager and eager vs captured ResNet training steps (max parameter differences)."""
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import paddlepaddle_amd as paddle  # noqa: E402
from paddlepaddle_amd.device.cuda.graphs import CUDAGraph  # noqa: E402
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from test_train_step_graph import _make  # noqa: E402

paddle.set_device("gpu")
g = torch.Generator(device="cuda").manual_seed(3)
x = paddle.Tensor(torch.randn(16, 64, 64, 3, device="cuda", dtype=torch.bfloat16, generator=g))
y = paddle.Tensor(torch.randint(0, 16, (16,), device="cuda", generator=g))
ms = [_make(paddle) for _ in range(3)]


def mk(model, opt):
    def step():
        with paddle.amp.auto_cast(level="O2", dtype="bfloat16"):
            out = model(x)
        loss = paddle.nn.functional.cross_entropy(out.astype("float32"), y)
        loss.backward()
        opt.step()
        opt.clear_grad(set_to_zero=False)
        return loss
    return step


steps = [mk(m, o) for m, o in ms]


def diff(a, b):
    return max((p._t.float() - q._t.float()).abs().max().item() for p, q in zip(a.parameters(), b.parameters()))


print("init", diff(ms[0][0], ms[1][0]), diff(ms[0][0], ms[2][0]), flush=True)
for i in range(3):
    la = [float(s()) for s in steps]
    print("warm", i, la, diff(ms[0][0], ms[1][0]), diff(ms[0][0], ms[2][0]), flush=True)
torch.cuda.synchronize()
cg = CUDAGraph()
cg.capture_begin()
lg = steps[2]()
cg.capture_end()
print("after capture (no exec)", diff(ms[0][0], ms[2][0]), flush=True)
for i in range(5):
    l0 = float(steps[0]())
    l1 = float(steps[1]())
    cg.replay()
    torch.cuda.synchronize()
    print("step", i, l0, l1, float(lg), "eager-eager", diff(ms[0][0], ms[1][0]), "eager-graph", diff(ms[0][0], ms[2][0]),
          flush=True)
