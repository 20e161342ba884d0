"""Peer-memory ("one-shot xGMI") all-reduce of int64 payloads between the ranks of one node
(the per-stage GBDT histograms are ~50 KB per model — latency-bound, where an
RCCL ring pays ≈130 µs per call even at world 1, profiles/r2_runs/stage_graph_overhead_125k.log).

Each rank allocates one uncached device buffer (``ops/csrc/xgmi.hip`` layout: recv[W][3][cap]
int64 + flags) and exchanges its IPC handle once over the process group; every rank maps every
other rank's buffer (``hipIpcOpenMemHandle``, lazy peer access over xGMI).  A reduction is then ONE
kernel on the caller's stream — push the local payload into every peer, flag it, wait for the
peers' flags, sum — so it can sit inside a captured HIP graph and costs no host round trip and no
RCCL call.  Integer sums make it bit-identical to ``torch.distributed.all_reduce``.

The same code serves ranks on different GPUs (peer access over xGMI) and several ranks sharing
one GPU (tests: IPC mappings of the same device).  Handles are exchanged with
``all_gather_object`` (gloo or nccl); ranks on different hosts cannot map each other, so
:func:`peer_comm` returns None there and callers keep RCCL.

Policy (``HFENS_XGMI``): ``auto`` (default) keeps RCCL — the peer kernel has only been validated
with ranks sharing one GPU, where every rank reads through the same L2, and cross-GPU visibility of
the remote stores and flags has not been checked bit for bit against RCCL on a multi-GPU node yet;
``try`` attempts the peer path and drops to RCCL on every rank together when any rank cannot map a
peer; ``1`` requires it; ``0`` never uses it.  Only uncached (fine-grained) buffers are mapped: if
the driver cannot share one, the group keeps RCCL (no coarse-grained fallback, whose L2 lines an
acquire would not invalidate).  A peer wait that times out sets an error flag that
:meth:`PeerComm.check` all-reduces over the group, so every rank raises together.

Self-validation: the first time a group's peer buffers exist, :func:`validate`
runs probe reductions through the peer kernel — an int64 sum spanning several chunks and f64
sum / max / min — and compares them bit for bit with the collective library's answer (int64:
``all_reduce``; f64: ``all_gather`` then the same rank-order fold).  Every rank then keeps the peer
path or drops to RCCL TOGETHER (one MIN agreement), and the outcome is logged and kept in
:data:`PROBES`.  ``HFENS_XGMI_PROBE_CORRUPT=<rank>`` perturbs that rank's peer result (tests of the
mismatch path).  Every user of a PeerComm takes slot = epoch mod 3, so consecutive reductions
never share a slot whichever caller issued them.
"""
from __future__ import annotations

import logging
import os
import socket
from typing import Dict, Optional

import numpy as np
import torch

CHUNK = 2048          # int64 per block of xgmi_allreduce_kernel (ops/csrc/xgmi.hip kXgChunk)
MAX_RANKS = 16
MODE = os.environ.get("HFENS_XGMI", "auto")    # "auto" (= RCCL) | "try" | "0" (RCCL only) | "1" (require)
TIMEOUT_S = float(os.environ.get("HFENS_XGMI_TIMEOUT", "60"))
UNCACHED = os.environ.get("HFENS_XGMI_UNCACHED", "1") != "0"   # "0": plain device memory (one-GPU tests only)


def buffer_bytes(W: int, cap: int) -> int:
    nchunk = -(-cap // CHUNK)
    return W * 3 * cap * 8 + (-(-(3 * W * nchunk * 4) // 256)) * 256


class PeerUnavailable(RuntimeError):
    """Some rank of the group could not map a peer's buffer (every rank raises it together)."""


class PeerComm:
    """IPC-mapped peer buffers of a process group; ``allreduce_`` sums int64 slots in place."""

    def __init__(self, group, device, cap: int):
        import torch.distributed as dist
        from .. import ops
        self.E = E = ops.ext()
        self.group = group
        self.W, self.me = dist.get_world_size(group), dist.get_rank(group)
        self.device = torch.device(device)
        self.cap = int(cap) + (int(cap) & 1)
        self.epoch = 0            # stage sequence number (identical on every rank)
        out = np.zeros(1, dtype=np.uint64)
        with torch.cuda.device(self.device):
            h = np.zeros(64, dtype=np.uint8)
            self.uncached = UNCACHED
            E.xgmi_alloc(buffer_bytes(self.W, self.cap), int(self.uncached), out.ctypes.data)
            self.own = int(out[0])
            err = ""
            try:
                E.xgmi_ipc_handle(self.own, h.ctypes.data)
            except RuntimeError as e:
                # no IPC handle for this (uncached) buffer: the whole group keeps RCCL — a plain
                # coarse-grained buffer is not a safe substitute across GPUs
                err = f"rank {self.me} cannot share its peer buffer: {e}"
            handles = [None] * self.W
            dist.all_gather_object(handles, (h.tobytes(), err), group=group)
            ptrs, self.opened = [], []
            if any(e for _, e in handles):
                err = err or "a peer rank cannot share its buffer"
            for r, (hb, _) in enumerate(handles):
                if err:
                    break
                if r == self.me:
                    ptrs.append(self.own)
                    continue
                hh = np.frombuffer(hb, dtype=np.uint8).copy()
                try:
                    E.xgmi_ipc_open(hh.ctypes.data, out.ctypes.data)
                except RuntimeError as e:   # this rank cannot map that peer's buffer
                    err = f"rank {self.me} cannot map rank {r}'s buffer: {e}"
                    break
                ptrs.append(int(out[0]))
                self.opened.append(int(out[0]))
            # every rank takes the same path: the peer kernel only if ALL mappings exist
            errs = [None] * self.W
            dist.all_gather_object(errs, err, group=group)
            bad = [e for e in errs if e]
            if bad:
                for p in self.opened:
                    E.xgmi_ipc_close(p)
                self.opened = []
                dist.barrier(group=group)   # every mapping of this buffer is closed before it is freed
                E.xgmi_free(self.own)
                self.own = 0
                raise PeerUnavailable("; ".join(bad))
        self.peers = torch.tensor(np.array(ptrs, dtype=np.uint64).view(np.int64), device=self.device)
        self.err = torch.zeros(1, dtype=torch.int32, device=self.device)
        dist.barrier(group=group)   # every mapping exists before anyone writes into it

    def allreduce_(self, t: torch.Tensor, k: int, t_host: int, t_dev: Optional[torch.Tensor] = None,
                   epoch_base: Optional[int] = None, stream: Optional[int] = None):
        """Sum the int64 tensor ``t`` (≤ cap elements) over the ranks, in place, on the current
        stream; ``k`` = stage % 3 (slot), epoch = base + stage + 1 (from ``t_dev`` when given)."""
        from .. import ops
        assert t.dtype == torch.int64 and t.is_contiguous() and t.numel() <= self.cap
        self.E.xgmi_allreduce_i64(t.data_ptr(), t.numel(), self.peers.data_ptr(), self.W, self.me, k, self.cap,
                                  self.epoch if epoch_base is None else epoch_base, int(t_host),
                                  t_dev.data_ptr() if t_dev is not None else 0, self.err.data_ptr(), TIMEOUT_S,
                                  stream if stream is not None else ops.stream_ptr(self.device))

    def reduce_f64_(self, t: torch.Tensor, op: str = "sum", stream: Optional[int] = None):
        """All-reduce the f64 tensor ``t`` in place (``op`` sum / max / min, folded in rank order
        0 … W−1: the same bits on every rank, deterministic for a fixed world) — ONE kernel on the
        current stream, no RCCL call.  Calls are collective and sequenced: every rank makes the same
        calls in the same order (epochs and slots follow the call count)."""
        from .. import ops
        assert t.dtype == torch.float64 and t.is_contiguous() and t.numel() <= self.cap
        k = (self.epoch + 1) % 3
        self.E.xgmi_allreduce(t.data_ptr(), t.numel(), 1, {"sum": 0, "max": 1, "min": 2}[op], self.peers.data_ptr(),
                              self.W, self.me, k, self.cap, self.epoch, 0, 0, self.err.data_ptr(), TIMEOUT_S,
                              stream if stream is not None else ops.stream_ptr(self.device))
        self.epoch += 1
        return t

    def advance(self, stages: int):
        """Reserve ``stages`` epochs after a loop that used epochs base+1 … base+stages."""
        self.epoch += int(stages)

    def check(self):
        """Collective: every rank of the group learns whether ANY rank's peer wait timed out (a
        late rank's own sums are fine, its peers' are not), and all raise together; the flag is
        reset so a later fit starts clean."""
        import torch.distributed as dist
        e = self.err.to(torch.int64)
        if dist.get_backend(self.group) == "gloo":
            e = e.cpu()
        dist.all_reduce(e, op=dist.ReduceOp.MAX, group=self.group)
        self.err.zero_()
        if int(e.item()) != 0:
            raise RuntimeError("xGMI peer all-reduce timed out waiting for a peer rank "
                               f"(HFENS_XGMI_TIMEOUT={TIMEOUT_S} s); set HFENS_XGMI=0 to use RCCL")


_CACHE: Dict[tuple, PeerComm] = {}
_OK: Dict[int, bool] = {}
PROBES: Dict[int, dict] = {}     # id(group) → outcome of the first-use validation
PROBE = os.environ.get("HFENS_XGMI_PROBE", "1") != "0"
_LOG = logging.getLogger("hfens.xgmi")


def _probe_payloads(rank: int, n: int):
    rng = np.random.default_rng(0x5EED + 7919 * rank)
    ints = rng.integers(-(1 << 40), 1 << 40, n, dtype=np.int64)
    # no zeros (−0.0 + 0.0 and 0.0 + −0.0 differ in sign): magnitudes over 12 decades
    f = rng.standard_normal(n) * np.exp(rng.uniform(-14.0, 14.0, n))
    f[f == 0.0] = 1.0
    return ints, f


def validate(pc: "PeerComm") -> bool:
    """Collective: probe the peer kernel against the collective library, bit for bit; returns the
    group's joint verdict (True on every rank or False on every rank)."""
    import torch.distributed as dist
    W, me, group = pc.W, pc.me, pc.group
    n = int(min(pc.cap, 2 * CHUNK + 37))
    gloo = dist.get_backend(group) == "gloo"
    lib_dev = torch.device("cpu") if gloo else pc.device
    mine_i, mine_f = _probe_payloads(me, n)
    corrupt = os.environ.get("HFENS_XGMI_PROBE_CORRUPT", "")
    fail_local = os.environ.get("HFENS_XGMI_PROBE_RAISE", "")
    detail = ""
    ok = True
    # (1) local phase: the peer kernels (which synchronise only through their own flags) and the
    # local reads; a failure here — an exception or a timed-out peer wait — is this rank's alone.
    # No collective-library call may sit inside it: a rank that jumped out of it early would issue
    # a different collective sequence from the others.
    try:
        if fail_local != "" and int(fail_local) == me:
            raise RuntimeError("HFENS_XGMI_PROBE_RAISE")
        ti = torch.from_numpy(mine_i.copy()).to(pc.device)
        pc.allreduce_(ti, (pc.epoch + 1) % 3, 0, epoch_base=pc.epoch)
        pc.epoch += 1
        tf = {op: pc.reduce_f64_(torch.from_numpy(mine_f.copy()).to(pc.device), op) for op in ("sum", "max", "min")}
        torch.cuda.synchronize(pc.device)
        got_i = ti.cpu()
        got_f = {op: t.cpu() for op, t in tf.items()}
        timed_out = int(pc.err.item()) != 0
        pc.err.zero_()
        if timed_out:
            raise RuntimeError("peer wait timed out")
        if corrupt != "" and int(corrupt) == me:
            got_i[n // 2] += 1
    except RuntimeError as e:
        ok, detail = False, f"rank {me}: {e}"
    # (2) every rank issues the same collectives from here on, whatever happened locally: the
    # library's answers, then one MIN agreement on the verdict
    ref_i = torch.from_numpy(mine_i.copy()).to(lib_dev)
    dist.all_reduce(ref_i, op=dist.ReduceOp.SUM, group=group)
    allf = [torch.empty(n, dtype=torch.float64, device=lib_dev) for _ in range(W)]
    dist.all_gather(allf, torch.from_numpy(mine_f.copy()).to(lib_dev), group=group)
    if ok:
        allf = [t.cpu() for t in allf]
        ref_f = {"sum": allf[0].clone(), "max": allf[0].clone(), "min": allf[0].clone()}
        for r in range(1, W):
            ref_f["sum"] = ref_f["sum"] + allf[r]
            ref_f["max"] = torch.maximum(ref_f["max"], allf[r])
            ref_f["min"] = torch.minimum(ref_f["min"], allf[r])
        bad = []
        if not torch.equal(got_i, ref_i.cpu()):
            bad.append(f"int64 sum ({int((got_i != ref_i.cpu()).sum())} of {n} differ)")
        for op in ("sum", "max", "min"):
            if not torch.equal(got_f[op].view(torch.int64), ref_f[op].view(torch.int64)):
                bad.append(f"f64 {op} ({int((got_f[op] != ref_f[op]).sum())} of {n} differ)")
        if bad:
            ok, detail = False, f"rank {me}: " + ", ".join(bad)
    flag = torch.tensor([1 if ok else 0], dtype=torch.int64, device=lib_dev)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
    joint = bool(int(flag.item()))
    notes = [None] * W
    dist.all_gather_object(notes, detail, group=group)
    rec = dict(ok=joint, world=W, elements=n, mismatches=[d for d in notes if d])
    PROBES[id(group)] = rec
    if joint:
        _LOG.info("xGMI peer path validated against the collective library (world %d, %d elements)", W, n)
    else:
        _LOG.warning("xGMI peer path disagrees with the collective library: %s — every rank uses RCCL",
                     "; ".join(rec["mismatches"]))
    return joint


def _same_host(group) -> bool:
    import torch.distributed as dist
    names = [None] * dist.get_world_size(group)
    dist.all_gather_object(names, socket.gethostname(), group=group)
    return len(set(names)) == 1


def peer_comm(group, device, cap: int, tag: str = "") -> Optional[PeerComm]:
    """The group's peer buffers (created once, grown when ``cap`` grows) or None when the ranks
    cannot map each other (different hosts, > 16 ranks, HFENS_XGMI=0, no GPU).  ``tag``: an
    independent set of buffers (its own epochs and slot rotation) for another user of the group,
    e.g. the interior point's reductions ("ipm") beside the GBDT stage sums ("")."""
    import torch.distributed as dist
    if group is None or MODE in ("0", "auto") or torch.device(device).type != "cuda":
        return None
    gid = id(group)
    if gid not in _OK:
        W = dist.get_world_size(group)
        _OK[gid] = W <= MAX_RANKS and _same_host(group)
        if not _OK[gid] and MODE == "1":
            raise RuntimeError("HFENS_XGMI=1 but the ranks cannot map each other's memory")
    if not _OK[gid]:
        return None
    key = (gid, str(torch.device(device)), tag)
    pc = _CACHE.get(key)
    if pc is None or pc.cap < cap:
        epoch = pc.epoch if pc is not None else 0
        if pc is not None:
            pc.close()
        try:
            pc = PeerComm(group, device, cap)
        except PeerUnavailable:
            if MODE == "1":
                raise
            _OK[gid] = False   # auto: the group keeps RCCL (all ranks decided together)
            _CACHE.pop(key, None)
            return None
        pc.epoch = epoch
        if PROBE and gid not in PROBES and not validate(pc):
            pc.close()
            _OK[gid] = False
            if MODE == "1":
                raise RuntimeError("HFENS_XGMI=1 but the peer path failed its validation: "
                                   + "; ".join(PROBES[gid]["mismatches"]))
            return None
        _CACHE[key] = pc
    return pc


def _close(self: PeerComm):
    import torch.distributed as dist
    torch.cuda.synchronize(self.device)
    if dist.is_initialized():
        dist.barrier(group=self.group)   # no peer still writes into a buffer being unmapped
    for p in self.opened:
        self.E.xgmi_ipc_close(p)
    self.opened = []
    if self.own:
        self.E.xgmi_free(self.own)
        self.own = 0


PeerComm.close = _close


def release_all():
    """Unmap and free every peer buffer (before destroying the process group)."""
    for pc in list(_CACHE.values()):
        pc.close()
    _CACHE.clear()
    _OK.clear()
    PROBES.clear()
