"""Batched / streaming inference engine for a fitted HF stack (SURVEY.md §2 "batched
inference" row, BASELINE config 4; reference ``predict_hf.py:5-40`` scores one patient with
``model.predict_proba``).

The whole stack runs as ONE fused HIP kernel per chunk (:func:`hfens.ops.stack_infer`):

* :meth:`BatchedPredictor.predict_device` — rows already resident in HBM (288 GB holds
  ~4·10⁹ rows of 17 f32 features).  The chunked launch sequence for a given
  (buffer, rows, dtype) is captured once into a HIP graph and replayed, so a 100M-row pass
  is a single ``hipGraphLaunch``.
* :meth:`BatchedPredictor.predict_host` — rows in (pinned) host memory.  Chunks are
  double-buffered over three streams: the H2D copy of chunk i+1 overlaps the kernel on chunk i,
  probabilities return D2H on a third stream; events order the buffer reuse.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Optional, Tuple

import torch

from . import ops


class BatchedPredictor:
    def __init__(self, model, device="cuda", chunk_rows: int = 1 << 23, use_graph: bool = True):
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("BatchedPredictor runs the fused HIP kernel: device must be cuda")
        ops.ext()
        self.model = model.to(self.device)
        self.pk = model._packed_stack(self.device)
        if self.pk is None:
            raise ValueError("model is not an HF-shaped stack (scaler+SVC, GBC, LR -> LR)")
        self.chunk = int(chunk_rows)
        self.use_graph = use_graph
        self._graphs: "OrderedDict[Tuple, Tuple[torch.cuda.CUDAGraph, torch.Tensor]]" = OrderedDict()

    MAX_GRAPHS = 4   # captured (input, size, dtype, output) combinations kept, least recently used evicted

    @property
    def n_features(self) -> int:
        return self.pk.F

    # ------------------------------------------------------------------ device-resident
    def _launch_all(self, X: torch.Tensor, out: torch.Tensor):
        n = X.shape[0]
        for s in range(0, n, self.chunk):
            e = min(n, s + self.chunk)
            ops.stack_infer(X[s:e], self.pk, out=out[s:e])

    def predict_device(self, X: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """P(class 1) for every row of device tensor ``X`` ([n, F] f32/f64, contiguous)."""
        if not X.is_cuda or X.dim() != 2 or X.shape[1] != self.pk.F:
            raise ValueError(f"predict_device: expected a cuda [n, {self.pk.F}] tensor")
        X = X.contiguous()
        n = X.shape[0]
        if not self.use_graph:
            out = out if out is not None else torch.empty(n, dtype=torch.float32, device=X.device)
            self._launch_all(X, out)
            return out[:n]
        # a captured graph replays on fixed pointers: keyed by (input, size, dtype, output); with no
        # ``out`` the graph writes a buffer of its own and the caller gets a COPY (a later call would
        # overwrite a returned view); pass ``out`` to skip the copy
        key = (X.data_ptr(), n, X.dtype, None if out is None else out.data_ptr())
        hit = self._graphs.get(key)
        if hit is None:
            buf = out if out is not None else torch.empty(n, dtype=torch.float32, device=X.device)
            from . import runtime
            side = runtime.stream(X.device, "infer_warmup")
            side.wait_stream(torch.cuda.current_stream(X.device))
            with torch.cuda.stream(side):      # warm-up launch outside capture
                self._launch_all(X, buf)
            torch.cuda.current_stream(X.device).wait_stream(side)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._launch_all(X, buf)
            hit = self._graphs[key] = (g, buf)
            while len(self._graphs) > self.MAX_GRAPHS:
                self._graphs.popitem(last=False)
        else:
            self._graphs.move_to_end(key)
        g, buf = hit
        g.replay()
        return buf[:n] if out is not None else buf[:n].clone()

    # ------------------------------------------------------------------ host streaming
    def predict_host(self, X_host: torch.Tensor, out_host: Optional[torch.Tensor] = None,
                     chunk_rows: Optional[int] = None) -> torch.Tensor:
        """Stream host rows through the GPU (double-buffered H2D / kernel / D2H overlap).
        ``X_host`` should be pinned for full PCIe bandwidth (``tensor.pin_memory()``)."""
        X_host = torch.as_tensor(X_host)
        if X_host.is_cuda or X_host.dim() != 2 or X_host.shape[1] != self.pk.F:
            raise ValueError(f"predict_host: expected a host [n, {self.pk.F}] tensor")
        if X_host.dtype not in (torch.float32, torch.float64):
            X_host = X_host.to(torch.float32)
        X_host = X_host.contiguous()
        n, F = X_host.shape
        ch = int(chunk_rows or self.chunk)
        if out_host is None:
            out_host = torch.empty(n, dtype=torch.float32, pin_memory=X_host.is_pinned())
        dev = self.device
        comp = torch.cuda.current_stream(dev)
        copy = torch.cuda.Stream(dev)     # H2D
        back = torch.cuda.Stream(dev)     # D2H (separate, so H2D i+1 never queues behind kernel i)
        bufs = [torch.empty(ch, F, dtype=X_host.dtype, device=dev) for _ in range(2)]
        outs = [torch.empty(ch, dtype=torch.float32, device=dev) for _ in range(2)]
        loaded = [torch.cuda.Event() for _ in range(2)]
        done = [torch.cuda.Event() for _ in range(2)]
        drained = [torch.cuda.Event() for _ in range(2)]
        nchunks = (n + ch - 1) // ch
        for i in range(nchunks):
            b = i & 1
            s, e = i * ch, min(n, (i + 1) * ch)
            with torch.cuda.stream(copy):
                if i >= 2:
                    copy.wait_event(done[b])        # kernel i-2 finished reading bufs[b]
                bufs[b][: e - s].copy_(X_host[s:e], non_blocking=True)
                loaded[b].record(copy)
            comp.wait_event(loaded[b])
            if i >= 2:
                comp.wait_event(drained[b])         # D2H of chunk i-2 finished reading outs[b]
            ops.stack_infer(bufs[b][: e - s], self.pk, out=outs[b])
            done[b].record(comp)
            with torch.cuda.stream(back):
                back.wait_event(done[b])
                out_host[s:e].copy_(outs[b][: e - s], non_blocking=True)
                drained[b].record(back)
        comp.wait_stream(copy)
        comp.wait_stream(back)
        torch.cuda.synchronize(dev)
        return out_host
