"""Fail-fast numeric guards: non-finite inputs or solver state raise at the
stage that produced them instead of surfacing as a silently wrong model.  Each check is one
fused reduction + one host read."""
from __future__ import annotations

import os

import torch

ENABLED = os.environ.get("HFENS_GUARDS", "1") != "0"


class NonFiniteError(FloatingPointError):
    pass


def check_finite(t: torch.Tensor, what: str) -> torch.Tensor:
    if ENABLED and t.numel() and t.is_floating_point() and not bool(torch.isfinite(t).all()):
        bad = int((~torch.isfinite(t)).sum())
        raise NonFiniteError(f"{what}: {bad} non-finite value(s)")
    return t


def check_binary(y: torch.Tensor, what: str) -> torch.Tensor:
    if ENABLED and y.numel() and not bool(((y == 0) | (y == 1)).all()):
        raise ValueError(f"{what}: labels must be 0/1")
    return y


def finite_flag(t: torch.Tensor) -> torch.Tensor:
    """Deferred form of ``check_finite``: a device bool (no host read) for a caller that reads it
    together with other device results in ONE transfer, then calls ``raise_flags``."""
    if not (ENABLED and t.numel() and t.is_floating_point()):
        return torch.ones((), dtype=torch.bool, device=t.device)
    return torch.isfinite(t).all()


def binary_flag(y: torch.Tensor) -> torch.Tensor:
    if not (ENABLED and y.numel()):
        return torch.ones((), dtype=torch.bool, device=y.device)
    return ((y == 0) | (y == 1)).all()


def raise_flags(vals, specs) -> None:
    """``vals``: host bools read from ``finite_flag``/``binary_flag``; ``specs``: (kind, what) per flag."""
    for ok, (kind, what) in zip(vals, specs):
        if not bool(ok):
            if kind == "finite":
                raise NonFiniteError(f"{what}: non-finite value(s)")
            raise ValueError(f"{what}: labels must be 0/1")


class Deferred:
    """Device-side checks of a chain of fits read back in ONE transfer at its end (the stacking
    trainer's base models: no host synchronisation between their launches and the meta model's).

    ``flag(t, kind, what)``: a device bool (``finite_flag`` / ``binary_flag``) that raises like the
    synchronous check if false; ``word(t, on_fail)``: a device integer whose non-zero value calls
    ``on_fail(value)`` (solver fallbacks).  ``resolve()`` reads everything, runs the fallbacks, then
    raises the first failed guard."""

    def __init__(self):
        self._flags, self._specs, self._words, self._hooks = [], [], [], []
        self._staged = None

    def stage(self) -> None:
        """Queue the read-back now, on the current stream, behind the kernels that produce the
        values (pinned copy + event): :meth:`resolve` then waits for those kernels only, not for
        whatever a later join queues in front of a plain read."""
        if not len(self) or not self._flags + self._words or not (self._words + self._flags)[0].is_cuda:
            return
        dev = torch.cat(self._words + self._flags)
        from .hostread import stage
        host, ev = stage(dev)
        self._staged = (host, ev, len(self._words), len(self._flags), dev)

    def flag(self, t: torch.Tensor, kind: str, what: str) -> None:
        self._flags.append(t.reshape(1).to(torch.int64))
        self._specs.append((kind, what))

    def word(self, t: torch.Tensor, on_fail) -> None:
        self._words.append(t.reshape(-1)[:1].to(torch.int64))
        self._hooks.append(on_fail)

    def __len__(self) -> int:
        return len(self._flags) + len(self._words)

    def ready(self) -> bool:
        """True when :meth:`resolve` would not wait: nothing to read, or the staged copy has landed."""
        if not len(self):
            return True
        st = self._staged
        if st is None or st[2] != len(self._words) or st[3] != len(self._flags):
            return False
        from .hostread import _pending
        return not _pending(st[0].numpy())

    def resolve(self) -> None:
        if not len(self):
            return
        st = self._staged
        self._staged = None
        if st is not None and st[2] == len(self._words) and st[3] == len(self._flags):
            from .hostread import landed
            host = landed(st[0], st[1]).tolist()
        else:
            host = torch.cat(self._words + self._flags).cpu().tolist()
        nw = len(self._words)
        words, flags = host[:nw], host[nw:]
        specs, hooks = self._specs, self._hooks
        self._flags, self._specs, self._words, self._hooks = [], [], [], []
        for v, h in zip(words, hooks):
            if v != 0:
                h(v)
        raise_flags(flags, specs)
