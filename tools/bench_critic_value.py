import sys, torch
sys.path.insert(0, "marl-maze_amd")
from marlmaze.networks import Critic
cr = Critic(2, hidden_sizes=[64, 64]).cuda()
for M in (4096, 33 * 4096, 17 * 65536):
    x = torch.randn(M, 130, device="cuda")
    v = torch.empty(M, device="cuda")
    for _ in range(3): cr.value_into(x, v)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20): cr.value_into(x, v)
    e1.record(); torch.cuda.synchronize()
    print(f"critic value M={M}: {e0.elapsed_time(e1) / 20 * 1e3:.1f} us", flush=True)
