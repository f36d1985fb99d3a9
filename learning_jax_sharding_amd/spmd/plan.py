"""Printable partition plans.

Every collective and every local kernel the partitioner issues is reported to
the active :class:`PlanRecorder` (if any).  ``with record_plan() as plan:`` is
how the tests check that each case lowers to exactly the collective plan of
SURVEY §2.7, and how ``jit(...).lower(...).as_text()`` prints a plan.
"""
from __future__ import annotations

import threading
from contextlib import contextmanager
from typing import Any, Dict, List

__all__ = ["PlanRecorder", "record_plan", "record", "PlanStep", "suspend_recording"]

_TLS = threading.local()


class PlanStep:
    __slots__ = ("kind", "info")

    def __init__(self, kind: str, info: Dict[str, Any]):
        self.kind = kind
        self.info = info

    def __repr__(self):
        items = ", ".join(f"{k}={v}" for k, v in self.info.items() if k != "transfers")
        return f"{self.kind}({items})"


class PlanRecorder:
    def __init__(self):
        self.steps: List[PlanStep] = []

    def add(self, kind: str, **info):
        self.steps.append(PlanStep(kind, info))

    @property
    def collectives(self) -> List[PlanStep]:
        return [s for s in self.steps if s.kind in COLLECTIVE_KINDS]

    def collective_kinds(self) -> List[str]:
        return [s.kind for s in self.collectives]

    def as_text(self) -> str:
        return "\n".join(repr(s) for s in self.steps)

    def __repr__(self):
        return f"Plan({self.steps})"


COLLECTIVE_KINDS = ("all_gather", "reduce_scatter", "all_reduce", "all_to_all", "collective_permute",
                    "exchange")


def _stack():
    s = getattr(_TLS, "stack", None)
    if s is None:
        s = _TLS.stack = []
    return s


@contextmanager
def record_plan():
    rec = PlanRecorder()
    _stack().append(rec)
    try:
        yield rec
    finally:
        _stack().pop()


@contextmanager
def suspend_recording():
    s = _stack()
    saved = list(s)
    s.clear()
    try:
        yield
    finally:
        s.extend(saved)


def record(kind: str, **info) -> None:
    for rec in _stack():
        rec.add(kind, **info)
