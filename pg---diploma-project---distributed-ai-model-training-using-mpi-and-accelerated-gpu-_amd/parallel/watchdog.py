"""Failure detection.

The reference has no timeouts, heartbeats or recovery: a dead rank leaves the
others blocked in an NCCL collective until the SLURM ``--time`` limit.  pgdist:

* collective timeout: ``init_process_group(timeout=...)`` (``parallel/bootstrap.py``);
* :class:`Watchdog` — a daemon thread per rank that expects a :meth:`kick` at
  least every ``timeout_s`` seconds (one per training step).  When a rank stops
  making progress it prints which rank / step / phase stalled and the Python
  stacks of all threads (``faulthandler``), optionally publishes that to the
  rendezvous store, and terminates the process with exit code 75 so the launcher
  (mpirun / srun / torchrun) tears the job down instead of hanging;
* heartbeats: with a ``torch.distributed`` store every rank writes
  ``pgdist/hb/<rank>`` = its step counter each kick; :meth:`stale_ranks` (rank 0)
  lists ranks whose heartbeat has not advanced for ``timeout_s``;
* recovery is resume-from-checkpoint (``--ckpt-dir`` / ``--resume``, §5.4).
"""
import faulthandler
import os
import sys
import threading
import time
from typing import Callable, Dict, List, Optional

EXIT_STALLED = 75


class Watchdog:
    def __init__(self, timeout_s: float, rank: int = 0, world: int = 1, store=None,
                 on_timeout: Optional[Callable[[str], None]] = None, poll_s: Optional[float] = None):
        self.timeout_s = float(timeout_s)
        self.rank, self.world, self.store = rank, world, store
        self.on_timeout = on_timeout
        self.poll_s = poll_s if poll_s is not None else max(0.05, min(5.0, self.timeout_s / 10))
        self.step = 0
        self.phase = "init"
        self._last = time.monotonic()
        self._stop = threading.Event()
        self._fired = False
        self._seen: Dict[int, tuple] = {}
        self._thread: Optional[threading.Thread] = None

    # ------------------------------------------------------------------ lifecycle
    def start(self) -> "Watchdog":
        if self.timeout_s > 0 and self._thread is None:
            self._last = time.monotonic()
            self._thread = threading.Thread(target=self._run, name=f"pgdist-watchdog-{self.rank}", daemon=True)
            self._thread.start()
        return self

    def stop(self):
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=2 * self.poll_s + 1)
            self._thread = None

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()

    # ------------------------------------------------------------------ progress
    def kick(self, step: Optional[int] = None, phase: Optional[str] = None):
        self.step = self.step + 1 if step is None else step
        if phase is not None:
            self.phase = phase
        self._last = time.monotonic()
        if self.store is not None:
            try:
                self.store.set(f"pgdist/hb/{self.rank}", str(self.step))
            except Exception:
                pass

    @property
    def fired(self) -> bool:
        return self._fired

    def stale_ranks(self) -> List[int]:
        """Ranks whose store heartbeat did not advance within ``timeout_s`` (call periodically)."""
        if self.store is None:
            return []
        now = time.monotonic()
        stale = []
        for r in range(self.world):
            try:
                v = self.store.get(f"pgdist/hb/{r}").decode()
            except Exception:
                v = None
            prev = self._seen.get(r)
            if prev is None or prev[0] != v:
                self._seen[r] = (v, now)
            elif now - prev[1] > self.timeout_s:
                stale.append(r)
        return stale

    # ------------------------------------------------------------------ internals
    def _run(self):
        while not self._stop.wait(self.poll_s):
            idle = time.monotonic() - self._last
            if idle > self.timeout_s:
                self._fire(idle)
                return

    def _fire(self, idle: float):
        self._fired = True
        msg = (f"[pgdist watchdog] rank {self.rank}/{self.world}: no progress for {idle:.1f}s "
               f"(step {self.step}, phase '{self.phase}', timeout {self.timeout_s:.0f}s)")
        print(msg, file=sys.stderr, flush=True)
        try:
            faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
        except Exception:
            pass
        if self.store is not None:
            try:
                self.store.set(f"pgdist/stalled/{self.rank}", msg)
            except Exception:
                pass
        if self.on_timeout is not None:
            self.on_timeout(msg)
        else:
            os._exit(EXIT_STALLED)
