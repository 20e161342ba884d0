"""Does work on the default stream wait for a pool stream (implicit null-stream sync)?"""
import time
import torch

dev = torch.device("cuda")
a = torch.randn(4096, 4096, device=dev)
torch.cuda.synchronize()
side = torch.cuda.Stream()
t0 = time.perf_counter()
with torch.cuda.stream(side):
    for _ in range(50):
        a = a @ a / 64.0
x = torch.ones(10, device=dev)
t1 = time.perf_counter()
v = float(x.sum())          # sync on the default stream only
t2 = time.perf_counter()
side.synchronize()
t3 = time.perf_counter()
print(f"enqueue {1e3*(t1-t0):.2f} ms, default-stream sync {1e3*(t2-t1):.2f} ms, side done {1e3*(t3-t1):.2f} ms")
s2 = torch.cuda.Stream()
with torch.cuda.stream(side):
    for _ in range(50):
        a = a @ a / 64.0
t1 = time.perf_counter()
with torch.cuda.stream(s2):
    v = float(torch.ones(10, device=dev).sum())
t2 = time.perf_counter()
side.synchronize()
t3 = time.perf_counter()
print(f"second pool stream sync {1e3*(t2-t1):.2f} ms, side done {1e3*(t3-t1):.2f} ms")
