"""Worker registry with liveness.

Parity: reference crates/coordinator/src/service.rs:11-51 — ClusterState is a
Mutex<HashMap<worker_id, WorkerState{last_seen}>>; RegisterWorker inserts and
answers "Registered"; SendHeartbeat updates last_seen or answers ok=false for
an unknown id; nothing ever evicts.

Here workers also report their GPU inventory, and a reaper evicts workers
whose last heartbeat is older than the timeout (default 3 intervals);
listeners are notified so in-flight queries on a dead worker group can be
retried elsewhere.
"""
from __future__ import annotations

import threading
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

from ..utils.log import get_logger
from .protocol import HeartbeatInfo, HeartbeatResponse, RegistrationAck, WorkerInfo

log = get_logger("registry")


@dataclass
class WorkerState:
    info: WorkerInfo
    last_seen: float = field(default_factory=time.time)
    alive: bool = True
    tasks_done: int = 0
    failures: int = 0
    quarantine_until: float = 0.0


class WorkerRegistry:
    def __init__(self, heartbeat_interval_s: float = 5.0, timeout_s: Optional[float] = None,
                 quarantine_s: Optional[float] = None):
        self.heartbeat_interval_s = heartbeat_interval_s
        self.timeout_s = timeout_s if timeout_s is not None else 3 * heartbeat_interval_s
        #: a group that failed a query stays out of routing this long even if
        #: it keeps heartbeating / re-registering (its process may be alive
        #: while its GPUs or communicator are not)
        self.quarantine_s = quarantine_s if quarantine_s is not None else 20 * heartbeat_interval_s
        self._lock = threading.RLock()
        self.workers: Dict[str, WorkerState] = {}
        self._listeners: List[Callable[[str], None]] = []
        self._stop = threading.Event()
        self._reaper: Optional[threading.Thread] = None

    def register(self, info: WorkerInfo) -> RegistrationAck:
        with self._lock:
            old = self.workers.get(info.id)
            if old is not None and old.quarantine_until > time.time():
                old.info = info
                return RegistrationAck("Quarantined", self.heartbeat_interval_s)
            st = WorkerState(info)
            if old is not None:
                st.failures, st.tasks_done = old.failures, old.tasks_done
            self.workers[info.id] = st
        log.info("registered worker %s at %s (%d GPUs)", info.id, info.address, info.world_size)
        return RegistrationAck("Registered", self.heartbeat_interval_s)

    def heartbeat(self, hb: HeartbeatInfo) -> HeartbeatResponse:
        with self._lock:
            st = self.workers.get(hb.worker_id)
            if st is None or not st.alive:
                return HeartbeatResponse(False)  # unknown (or evicted): the worker must re-register
            st.last_seen = time.time()
            return HeartbeatResponse(True)

    def alive(self) -> List[WorkerState]:
        with self._lock:
            return [w for w in self.workers.values() if w.alive]

    def mark_dead(self, worker_id: str, reason: str = "", quarantine: bool = False):
        with self._lock:
            st = self.workers.get(worker_id)
            if st is None or not st.alive:
                return
            st.alive = False
            if quarantine:
                st.quarantine_until = time.time() + self.quarantine_s
        log.warning("worker %s marked dead %s", worker_id, reason)
        for fn in self._listeners:
            fn(worker_id)

    def reap(self, now: Optional[float] = None) -> List[str]:
        now = now if now is not None else time.time()
        dead = []
        with self._lock:
            for wid, st in self.workers.items():
                if st.alive and now - st.last_seen > self.timeout_s:
                    dead.append(wid)
        for wid in dead:
            self.mark_dead(wid, f"(no heartbeat for > {self.timeout_s:.1f}s)")
        return dead

    def on_dead(self, fn: Callable[[str], None]):
        self._listeners.append(fn)

    def start(self):
        if self._reaper is not None:
            return

        def loop():
            while not self._stop.wait(max(self.heartbeat_interval_s / 2, 0.05)):
                self.reap()
        self._reaper = threading.Thread(target=loop, daemon=True, name="igloo-reaper")
        self._reaper.start()

    def stop(self):
        self._stop.set()

    def snapshot(self) -> List[dict]:
        with self._lock:
            return [{"id": w.info.id, "address": w.info.address, "alive": w.alive, "world_size": w.info.world_size,
                     "last_seen": w.last_seen, "devices": w.info.devices, "tasks_done": w.tasks_done}
                    for w in self.workers.values()]
