import json, sys, torch
sys.path.insert(0, "maze-solving-agent-gymnasium_amd")
import mazerl
B = 65536
env = mazerl.VectorMazeEnv(B, 81, enrich=True, device="cuda:0")
idx = torch.arange(B, dtype=torch.int32, device="cuda")
for n in (1024, 65536):
    cnt = torch.tensor([n], dtype=torch.int32, device="cuda")
    env.reset_list(idx, cnt); torch.cuda.synchronize()
    assert int(cnt.item()) == 0
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        cnt.fill_(n)
        env.reset_list(idx, cnt)
    e.record(); torch.cuda.synchronize()
    print(json.dumps({"listed": n, "ms_per_call_incl_fill": s.elapsed_time(e) / 20, "count_after": int(cnt.item())}))
env.close()
