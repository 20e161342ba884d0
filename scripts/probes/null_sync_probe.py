"""Does a host read on the default (null) stream wait for work queued on the fit's pool streams?
A ~8 ms spin kernel on a pool stream, then a tiny kernel + read on another stream; host wait times."""
import time

import torch

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
x = torch.zeros(4, device=dev)
pool = torch.cuda.Stream(dev)
other = torch.cuda.Stream(dev)
torch.cuda._sleep(1000)
torch.cuda.synchronize()
c = 1 << 22
for _ in range(6):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    torch.cuda._sleep(c)
    e1.record()
    torch.cuda.synchronize()
    c = int(c * 8.0 / max(e0.elapsed_time(e1), 1e-3))


def trial(name, read_stream, how):
    torch.cuda.synchronize()
    with torch.cuda.stream(pool):
        torch.cuda._sleep(c)
    time.sleep(0.0005)
    t0 = time.perf_counter()
    with torch.cuda.stream(read_stream):
        y = x + 1.0
        if how == "item":
            float(y.sum())
        elif how == "cpu":
            y.cpu()
        elif how == "event":
            ev = torch.cuda.Event()
            ev.record()
            ev.synchronize()
        elif how == "stream_sync":
            torch.cuda.current_stream().synchronize()
    dt = 1e3 * (time.perf_counter() - t0)
    torch.cuda.synchronize()
    print(f"{name:40s} host wait {dt:7.3f} ms (pool kernel ≈ 8 ms)", flush=True)


main = torch.cuda.current_stream(dev)
for rep in range(2):      # (the first round loads each kernel's code object: a device-wide wait)
    print(f"-- round {rep}", flush=True)
    for how in ("item", "cpu", "event", "stream_sync"):
        trial(f"read on the default stream ({how})", main, how)
        trial(f"read on another pool stream ({how})", other, how)
print("default stream id", main.cuda_stream, "pool", pool.cuda_stream)
