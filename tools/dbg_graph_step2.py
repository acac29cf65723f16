"""Debug: replay a captured ResNet step N times back to back; variant via argv: zero (set_to_zero=True)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import paddlepaddle_amd as paddle  # noqa: E402
from paddlepaddle_amd.device.cuda.graphs import CUDAGraph  # noqa: E402
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from test_train_step_graph import _make  # noqa: E402

zero = "zero" in sys.argv
paddle.set_device("gpu")
g = torch.Generator(device="cuda").manual_seed(3)
x = paddle.Tensor(torch.randn(16, 64, 64, 3, device="cuda", dtype=torch.bfloat16, generator=g))
y = paddle.Tensor(torch.randint(0, 16, (16,), device="cuda", generator=g))
model, opt = _make(paddle)


def step():
    with paddle.amp.auto_cast(level="O2", dtype="bfloat16"):
        out = model(x)
    loss = paddle.nn.functional.cross_entropy(out.astype("float32"), y)
    loss.backward()
    opt.step()
    opt.clear_grad(set_to_zero=zero)
    return loss


for i in range(3):
    print("warm", float(step()), flush=True)
torch.cuda.synchronize()
cg = CUDAGraph()
cg.capture_begin()
lg = step()
cg.capture_end()
for i in range(5):
    cg.replay()
    torch.cuda.synchronize()
    mx = max(p._t.float().abs().max().item() for p in model.parameters())
    print("replay", i, float(lg), "max|param|", mx, flush=True)
