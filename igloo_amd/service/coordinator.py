"""``igloo-coordinator``: Flight SQL endpoint + worker registry + scheduler.

Parity: reference crates/coordinator/src/main.rs:19-80 builds an engine and a
MemoryCatalog, registers test_data.csv as ``test_table`` (col_a Int64, col_b
Utf8), runs a demo ``LIMIT 5`` query, then serves ONLY the Flight service on
127.0.0.1:50051 with Ctrl-C shutdown — its CoordinatorService (registration /
heartbeats) is never added to the server (:71-72), and its
DistributedExecutor is never wired (crates/coordinator/src/distributed_executor.rs).

Here the same endpoint also serves the control plane (DoAction), keeps a
liveness-checked registry of GPU worker groups, and routes each query to the
least-loaded live group (SPMD over that node's GPUs). A group that stops
answering is marked dead and the query is retried on another group, falling
back to local execution when no group is left (SQL queries are idempotent, so
retry is the recovery model — SURVEY §5.3/5.4).
"""
from __future__ import annotations

import argparse
import os
import signal
import sys
import threading
import time
from typing import Optional

import pyarrow as pa
import pyarrow.flight as fl

from ..utils.config import IglooConfig, load_config, register_config_tables
from ..utils.errors import IglooError
from ..utils.log import get_logger
from .flight_server import IglooFlightServer
from .registry import WorkerRegistry

log = get_logger("coordinator")

RETRYABLE = (fl.FlightUnavailableError, fl.FlightTimedOutError, fl.FlightCancelledError, ConnectionError,
             TimeoutError)


def _supervised(w) -> bool:
    return any(isinstance(d, dict) and d.get("supervisor") for d in (w.info.devices or []))


class DistributedExecutor:
    def __init__(self, registry: WorkerRegistry, engine, token: Optional[str] = None, max_attempts: int = 3,
                 timeout_s: float = 3600.0, recovery_wait_s: float = 30.0):
        self.registry = registry
        self.engine = engine
        self.token = token
        self.max_attempts = max_attempts
        self.timeout_s = timeout_s
        #: after a supervised group failed a query, how long to wait for its
        #: node supervisor's replacement group (the surviving GPUs) before
        #: falling back to local execution (service/supervisor.py)
        self.recovery_wait_s = recovery_wait_s
        self.log = []  # (sql, worker id | "local", ms, outcome)

    def _await_replacement(self, tried: set) -> list:
        deadline = time.time() + self.recovery_wait_s
        while time.time() < deadline:
            cands = [w for w in self.registry.alive() if w.info.id not in tried]
            if cands:
                return cands
            time.sleep(0.05)
        return []

    def run(self, sql: str) -> pa.Table:
        from .client import IglooClient
        tried = set()
        failed_supervised = False
        for _ in range(self.max_attempts):
            cands = [w for w in self.registry.alive() if w.info.id not in tried]
            if not cands and failed_supervised:
                cands = self._await_replacement(tried)
            if not cands:
                break
            w = min(cands, key=lambda s: s.tasks_done)
            tried.add(w.info.id)
            t0 = time.perf_counter()
            try:
                with IglooClient(w.info.address, self.token, timeout=self.timeout_s) as c:
                    t = c.query(sql)
                w.tasks_done += 1
                self.log.append((sql, w.info.id, (time.perf_counter() - t0) * 1e3, "ok"))
                return t
            except RETRYABLE as e:
                w.failures += 1
                failed_supervised = failed_supervised or _supervised(w)
                self.log.append((sql, w.info.id, (time.perf_counter() - t0) * 1e3, f"retry: {type(e).__name__}"))
                self.registry.mark_dead(w.info.id, f"(query failed: {type(e).__name__})", quarantine=True)
            except pa.ArrowKeyError:
                # NotFound = empty result from the worker
                return self.engine.logical_schema_table(sql) if hasattr(self.engine, "logical_schema_table") else \
                    self._empty(sql)
        t0 = time.perf_counter()
        t = self.engine.query(sql)
        self.log.append((sql, "local", (time.perf_counter() - t0) * 1e3, "ok"))
        return t

    def _empty(self, sql: str) -> pa.Table:
        plan, names = self.engine.logical_plan(sql)
        return pa.schema([pa.field(n, c.dtype.to_arrow()) for c, n in zip(plan.schema, names)]).empty_table()


class Coordinator:
    def __init__(self, cfg: Optional[IglooConfig] = None, engine=None, port: Optional[int] = None):
        import igloo_amd as ig
        self.cfg = cfg or IglooConfig()
        self.engine = engine or ig.QueryEngine(device=self.cfg.device)
        self.registry = WorkerRegistry(self.cfg.heartbeat_interval_s, self.cfg.heartbeat_timeout_s)
        self.executor = DistributedExecutor(self.registry, self.engine, self.cfg.auth_token,
                                            recovery_wait_s=getattr(self.cfg, "recovery_wait_s", 30.0))
        p = self.cfg.coordinator_port if port is None else port
        self.location = f"grpc://{self.cfg.coordinator_host}:{p}"
        self.server = IglooFlightServer(self.engine, self.location, self.registry, runner=self.executor.run,
                                        auth_token=self.cfg.auth_token)
        self.port = self.server.port
        self.address = f"grpc://{self.cfg.coordinator_host}:{self.port}"

    def start(self):
        self.registry.start()
        self.server.start_background(host=self.cfg.coordinator_host)
        return self

    def shutdown(self):
        self.registry.stop()
        self.server.shutdown()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="igloo-coordinator")
    ap.add_argument("-c", "--config")
    ap.add_argument("--host", default=None)
    ap.add_argument("--port", type=int, default=None)
    ap.add_argument("--device", default=None)
    ap.add_argument("--demo-csv", default=os.path.join(os.path.dirname(__file__), "..", "..", "tests", "data",
                                                       "test_data.csv"))
    ap.add_argument("--tpch", type=float, default=None)
    a = ap.parse_args(argv)
    cfg = load_config(a.config, {"coordinator_host": a.host, "coordinator_port": a.port, "device": a.device})
    import igloo_amd as ig
    from igloo_amd import types as T
    from igloo_amd.catalog import Field
    from igloo_amd.engine import print_batches
    engine = ig.QueryEngine(device=cfg.device)
    if a.demo_csv and os.path.exists(a.demo_csv):
        engine.register_csv("test_table", a.demo_csv, schema=[Field("col_a", T.INT64), Field("col_b", T.UTF8)])
        print("Demo query: SELECT col_a, col_b FROM test_table LIMIT 5;")
        print_batches(engine.sql("SELECT col_a, col_b FROM test_table LIMIT 5;"))
    register_config_tables(engine, cfg)
    if a.tpch:
        from ..models.tpch import datagen
        datagen.register(engine, a.tpch)
    co = Coordinator(cfg, engine).start()
    print(f"igloo coordinator (Flight SQL + control plane) listening on {co.address}", flush=True)
    stop = threading.Event()
    signal.signal(signal.SIGINT, lambda *_: stop.set())
    signal.signal(signal.SIGTERM, lambda *_: stop.set())
    stop.wait()
    print("shutting down coordinator")
    co.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
