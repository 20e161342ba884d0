"""Host/device cost of a 512x512 f64 Cholesky on the GPU through torch.linalg (library choice)."""
import time

import torch

dev = torch.device("cuda")
r = 512
A = torch.randn(r, 2 * r, device=dev, dtype=torch.float64)
S = A @ A.T + torch.eye(r, device=dev, dtype=torch.float64)
for lib in ("default", "magma", "cusolver"):
    if lib != "default":
        torch.backends.cuda.preferred_linalg_library(lib)
    for fn_name, fn in (("cholesky_ex", lambda: torch.linalg.cholesky_ex(S)),
                        ("cholesky", lambda: torch.linalg.cholesky(S)),
                        ("cholesky_ex batched[1]", lambda: torch.linalg.cholesky_ex(S[None]))):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(10):
            fn()
        th = (time.perf_counter() - t) / 10
        torch.cuda.synchronize()
        tw = (time.perf_counter() - t) / 10
        print(f"{lib:9s} {fn_name:24s} host {th * 1e3:7.3f} ms  wall {tw * 1e3:7.3f} ms", flush=True)
