"""Failure detection for one-process-per-GPU jobs (``ncclCommGetAsyncError`` and a
timeout on collectives).

The reference's collectives are XLA's in-process CPU ones and never fail
(``case6_attention.py:212-214`` relies on the implicit gradient all-reduce).  Over RCCL a lost
or wedged peer leaves every other rank blocked inside a collective - and, with the training
step captured into a HIP graph, blocked in ``torch.cuda.synchronize()`` with no Python running.
:class:`CommWatchdog` is a daemon thread that watches the job while the main thread blocks:

* every ``poll_s`` it asks each native RCCL communicator for its asynchronous error
  (``RankRccl.check``, i.e. ``ncclCommGetAsyncError``);
* the main thread names what it is doing with :meth:`phase` (``"warmup"``, ``"timed steps"``,
  ...); a phase that runs longer than ``timeout_s`` is a hang.

On an error or a hang the watchdog aborts every communicator (``ncclCommAbort`` makes RCCL
kernels spinning on a dead peer return), prints the phase, each communicator's partition and
the collectives issued on it, and ends the process with exit code :data:`EXIT_CODE` - so a
launcher (torchrun) sees a failed rank within the deadline instead of a job that hangs until
someone kills it.
"""
from __future__ import annotations

import os
import sys
import threading
import time
from typing import Callable, Optional

__all__ = ["CommWatchdog", "EXIT_CODE", "default_timeout"]

EXIT_CODE = 75


def default_timeout() -> float:
    """``LJS_COMM_TIMEOUT_S`` (default 300 s: the first capture of a step compiles nothing, but
    the first RCCL call of a fresh node can take tens of seconds to set up its rings)."""
    return float(os.environ.get("LJS_COMM_TIMEOUT_S", "300"))


class CommWatchdog:
    def __init__(self, comm=None, timeout_s: Optional[float] = None, poll_s: float = 0.1,
                 exit_fn: Optional[Callable[[int], None]] = None, grace_s: float = 2.0):
        """``comm``: the collective backend (``comm.backend.DistComm``) whose native communicators
        are polled; None polls nothing and enforces only the phase deadline."""
        self.comm = comm
        self.timeout_s = default_timeout() if timeout_s is None else float(timeout_s)
        self.poll_s = float(poll_s)
        self.grace_s = float(grace_s)
        self._exit = exit_fn or os._exit
        # (phase name, start, deadline) replaced as ONE object and read once per poll: the polling
        # thread never pairs a new, shorter deadline with the previous phase's start time
        self._state = ("startup", time.monotonic(), self.timeout_s)
        # called (reason) -> exit code, after the abort and before the exit: a caller that still has
        # a result to report (bench.py's headline, measured before a secondary layout hung) prints
        # it here and may choose the exit status
        self.on_fail: Optional[Callable[[str], Optional[int]]] = None
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.failed: Optional[str] = None

    # ------------------------------------------------------------------ main-thread API
    def start(self) -> "CommWatchdog":
        if self._thread is None:
            self._thread = threading.Thread(target=self._run, name="ljs-comm-watchdog", daemon=True)
            self._thread.start()
        return self

    def phase(self, name: str, timeout_s: Optional[float] = None) -> None:
        """Enter a new phase: its deadline (``timeout_s``, default the watchdog's) starts now."""
        self._state = (name, time.monotonic(), self.timeout_s if timeout_s is None else float(timeout_s))

    @property
    def _phase(self) -> str:
        return self._state[0]

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None and self._thread is not threading.current_thread():
            self._thread.join(timeout=5 * self.poll_s + 1.0)
        self._thread = None

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()
        return False

    # ------------------------------------------------------------------ watcher thread
    def _native(self):
        return getattr(self.comm, "_native", None) if self.comm is not None else None

    def _run(self) -> None:
        while not self._stop.wait(self.poll_s):
            reason = None
            nat = self._native()
            if nat is not None:
                try:
                    nat.check()
                except Exception as e:  # an asynchronous RCCL error on some communicator
                    reason = f"asynchronous RCCL error: {e}"
            _, t0, deadline = self._state
            if reason is None and time.monotonic() - t0 > deadline:
                reason = f"phase exceeded its {deadline:g} s deadline (hang: a peer rank lost or wedged)"
            if reason is not None:
                self._fail(reason)
                return

    def _fail(self, reason: str) -> None:
        self.failed = reason
        rank = os.environ.get("RANK", "?")
        phase, t0, _ = self._state
        lines = [f"[ljs watchdog] rank {rank}: {reason}",
                 f"[ljs watchdog] phase: {phase!r}, {time.monotonic() - t0:.1f} s in"]
        nat = self._native()
        if nat is not None:
            try:   # a diagnostic: whatever it raises, the abort and the exit below still run
                for desc in nat.describe():
                    lines.append(f"[ljs watchdog]   {desc}")
            except Exception as e:  # pragma: no cover - defensive
                lines.append(f"[ljs watchdog] describe failed: {e!r}")
            try:
                nat.abort()
                lines.append("[ljs watchdog] every RCCL communicator aborted (ncclCommAbort)")
            except Exception as e:  # pragma: no cover - abort itself failing
                lines.append(f"[ljs watchdog] abort failed: {e}")
        else:
            lines.append("[ljs watchdog] no native RCCL communicators (torch process groups only)")
        print("\n".join(lines), file=sys.stderr, flush=True)
        code = EXIT_CODE
        if self.on_fail is not None:
            try:
                rc = self.on_fail(f"{reason} (phase {phase!r})")
                if rc is not None:
                    code = int(rc)
            except Exception as e:  # pragma: no cover - defensive
                print(f"[ljs watchdog] on_fail hook raised {e!r}", file=sys.stderr, flush=True)
        # give a main thread released by the abort a moment to unwind, then end the process:
        # it may still be blocked in a device synchronize that never returns
        time.sleep(self.grace_s)
        self._exit(code)
