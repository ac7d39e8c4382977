"""Debug: torch reductions replayed from a captured HIP graph vs eager, on fresh data each replay."""
import torch

res = []
for shape, fn_name in [((2048, 1024), "sum0"), ((2048, 1024), "sum1"), ((2048, 1024), "sumall"),
                       ((256, 1024), "sum0"), ((2048, 1024), "mv"), ((2048, 512), "sum0"),
                       ((2048, 4), "sum0"), ((8192, 1024), "sum0"), ((1024, 1024), "sum0"),
                       ((512, 1024), "sum0")]:
    fns = {"sum0": lambda x: x.sum(0), "sum1": lambda x: x.sum(1), "sumall": lambda x: x.sum(),
           "mv": lambda x: torch.mv(x.t(), torch.ones(x.shape[0], device=x.device))}
    fn = fns[fn_name]
    X = torch.randn(*shape, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn(X)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        Y = fn(X)
    bad = 0
    for k in range(6):
        X.copy_(torch.randn(*shape, device="cuda"))
        g.replay()
        torch.cuda.synchronize()
        ref = fn(X)
        bad += float((Y - ref).abs().max()) > 1e-4 * float(ref.abs().max())
    res.append(f"{fn_name:6s} {str(shape):14s} wrong replays {bad}/6")
print("\n".join(res))
