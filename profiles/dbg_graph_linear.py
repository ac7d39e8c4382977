"""Debug: gradients of Linear / stem forward+backward replayed from a captured HIP graph vs eager."""
import os
import sys

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "maze-solving-agent-gymnasium_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

from test_stem import _bits  # noqa: E402

what, bs = sys.argv[1], int(sys.argv[2])
if len(sys.argv) > 3:
    torch.backends.cuda.preferred_blas_library(sys.argv[3])
torch.manual_seed(0)
if what == "linear":
    net = nn.Linear(1574, 1024).cuda()
elif what == "linear_nobias":
    net = nn.Linear(1574, 1024, bias=False).cuda()
elif what == "mlp":
    net = nn.Sequential(nn.Linear(1574, 1024), nn.LeakyReLU(), nn.Linear(1024, 512), nn.LeakyReLU(),
                        nn.Linear(512, 1)).cuda()
elif what in ("linear_mv", "mlp_mv"):
    class LinFn(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, w, b):
            ctx.save_for_backward(x, w)
            return torch.nn.functional.linear(x, w, b)

        @staticmethod
        def backward(ctx, gy):
            x, w = ctx.saved_tensors
            gx = gy @ w if ctx.needs_input_grad[0] else None
            gw = gy.t() @ x
            gb = torch.mv(gy.t(), torch.ones(gy.shape[0], device=gy.device, dtype=gy.dtype))
            return gx, gw, gb

    class Lin(nn.Linear):
        def forward(self, x):
            return LinFn.apply(x, self.weight, self.bias)
    if what == "linear_mv":
        net = Lin(1574, 1024).cuda()
    else:
        net = nn.Sequential(Lin(1574, 1024), nn.LeakyReLU(), Lin(1024, 512), nn.LeakyReLU(),
                            Lin(512, 1)).cuda()
elif what == "stem":
    from mazerl.agents.nets import QNet
    net = QNet(variant="dqn").cuda()
X = torch.zeros(bs, 1574, device="cuda")
Wb = torch.zeros(bs, 22, dtype=torch.int32, device="cuda")
S6 = torch.zeros(bs, 6, device="cuda")


def fwd():
    if what == "stem":
        return net((S6, Wb)).pow(2).sum()
    return net(X).pow(2).sum()


def fill(k):
    g = torch.Generator(device="cuda").manual_seed(k)
    X.copy_(torch.randn(bs, 1574, device="cuda", generator=g))
    Wb.copy_(_bits(bs, k).cuda())
    S6.copy_(torch.randn(bs, 6, device="cuda", generator=g))


s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for k in range(3):
        fill(k)
        net.zero_grad(set_to_none=True)
        fwd().backward()
torch.cuda.current_stream().wait_stream(s)
zero_in_graph = len(sys.argv) > 4 and sys.argv[4] == "zero"
if zero_in_graph:
    for p in net.parameters():
        p.grad = torch.zeros_like(p)
else:
    net.zero_grad(set_to_none=True)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    if zero_in_graph:
        for p in net.parameters():
            p.grad.zero_()
    L = fwd()
    L.backward()
gg = [p.grad for p in net.parameters()]
bad = 0
for k in range(3, 9):
    fill(k)
    g.replay()
    torch.cuda.synchronize()
    got = [x.clone() for x in gg]
    ref = torch.autograd.grad(fwd(), list(net.parameters()))
    with torch.no_grad():
        lref = float(fwd())
    names = [n for n, _ in net.named_parameters()]
    for nm, a, b in zip(names, got, ref):
        e = float((a - b).abs().max()) / (float(b.abs().max()) + 1e-30)
        bad += e > 1e-3
        if e > 1e-3 and k < 5:
            print(f"  replay {k}: {nm} rel err {e:.3g}; loss graph {float(L):.6g} eager {lref:.6g}")
print(f"{what:14s} zero_in_graph {zero_in_graph} bs {bs} blas {torch.backends.cuda.preferred_blas_library()}: wrong grads {bad}/{6 * len(gg)}")
