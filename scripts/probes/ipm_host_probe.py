import os, sys, time, torch
sys.path.insert(0, '/root/repo')
from hfens.models import svc_lowrank as sl
dev = torch.device('cuda')
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
g = torch.Generator(device=dev).manual_seed(0)
Z = torch.randn(n, 17, generator=g, device=dev, dtype=torch.float64)
y = torch.where(torch.rand(n, generator=g, device=dev) < 0.2, -1.0, 1.0).to(torch.float64)
idx = torch.randperm(n, device=dev)[:512]
Phi, T = sl.nystrom_map(Z, idx, 1 / 17)
c = torch.where(y > 0, 0.625, 2.5).to(torch.float64)
# host-side cost of one iteration's op stream: time the python loop with CUDA launch blocking off,
# using torch.profiler to split host vs device
sl.ipm_svc_dual(Phi[:100000], y[:100000], c[:100000])
torch.cuda.synchronize()
from torch.profiler import profile, ProfilerActivity
with profile(activities=[ProfilerActivity.CPU]) as prof:
    t0 = time.perf_counter()
    a, rho, it = sl.ipm_svc_dual(Phi, y, c, max_iter=10)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
print(f"10 iters wall {dt*1e3:.1f} ms")
print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=25))
