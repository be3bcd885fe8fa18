"""``igloo-worker``: one process per GPU; a node's processes form one SPMD group.

Parity: reference crates/worker/src/main.rs:13-52 — random uuid id, fixed
address 127.0.0.1:50052, coordinator URL as positional argv[1], RegisterWorker
then a heartbeat every 5 s (errors printed, responses ignored), WorkerService
whose ExecuteTask only prints and answers "SUBMITTED"
(crates/worker/src/service.rs:10-33).

Here (launched by torchrun, one rank per GPU):
* every rank binds its GPU, joins the RCCL communicator and holds its hash
  partition of the tables (from --tpch / --config);
* rank 0 hosts the group's Flight endpoint, registers the group with the
  coordinator (GPU inventory of all ranks), heartbeats, re-registers when the
  coordinator forgets it, and for every query broadcasts the SQL to the other
  ranks over a gloo control group, so all ranks execute the same SPMD plan;
  exchanges between ranks go over RCCL/xGMI and rank 0 streams the result.
"""
from __future__ import annotations

import argparse
import os
import signal
import sys
import threading
import time
import uuid
from datetime import timedelta
from typing import Optional

import pyarrow as pa
import torch

from ..utils import faults
from ..utils.config import IglooConfig, load_config, register_config_tables
from ..utils.log import get_logger
from . import protocol as P

log = get_logger("worker")


class GroupBroken(Exception):
    """A rank of the SPMD group died or its communicator failed."""


class WorkerGroup:
    #: a follower whose in-group heartbeat is older than this is presumed dead
    RANK_TIMEOUT_S = 3.0
    RANK_HEARTBEAT_S = 0.5

    def __init__(self, engine, comm=None, coordinator: Optional[str] = None, host: str = "127.0.0.1",
                 port: int = 50052, token: Optional[str] = None, heartbeat_s: float = 5.0,
                 collective_timeout_s: float = 60.0):
        self.engine = engine
        self.comm = comm
        self.rank = comm.rank if comm else 0
        self.world = comm.world_size if comm else 1
        self.coordinator = coordinator
        self.token = token
        self.heartbeat_s = heartbeat_s
        self.id = str(uuid.uuid4())
        self.host, self.port = host, port
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self.server = None
        self.ctrl = None
        self.status = None
        self.broken: Optional[str] = None
        self.exit_code = 0
        if self.world > 1:
            import torch.distributed as dist
            # control messages may wait for hours between queries: a CPU (gloo)
            # group with a long timeout, separate from the RCCL data group
            self.ctrl = dist.new_group(backend="gloo", timeout=timedelta(days=7))
            # per-query status agreement: every rank reports success / its error
            # after each SPMD query, bounded by the collective timeout
            self.status = dist.new_group(backend="gloo", timeout=timedelta(seconds=collective_timeout_s))
            self.store = dist.distributed_c10d._get_default_store()
            threading.Thread(target=self._rank_heartbeat, daemon=True, name="igloo-rank-hb").start()
            if self.rank == 0:
                threading.Thread(target=self._watchdog, daemon=True, name="igloo-watchdog").start()

    # ------------------------------------------------------- group liveness
    def _rank_heartbeat(self):
        """Every rank stamps its liveness into the group's rendezvous store."""
        while not self._stop.is_set():
            try:
                self.store.set(f"igloo/hb/{self.rank}", repr(time.time()))
            except Exception:  # noqa: BLE001 - rank 0 (the store host) is gone
                if self.rank != 0:
                    log.warning("rank %d: group store unreachable, exiting", self.rank)
                    os._exit(3)
                return
            self._stop.wait(self.RANK_HEARTBEAT_S)

    def _watchdog(self):
        """Rank 0: a follower that stopped stamping is dead. The group is then
        marked broken: its communicator is aborted (a collective blocked on the
        dead rank errors out instead of hanging until the collective timeout),
        the coordinator is no longer heartbeated (it evicts the group and
        retries queries elsewhere) and the process exits non-zero once the
        in-flight query has been answered with a retryable error."""
        start = time.time()
        while not self._stop.wait(self.RANK_HEARTBEAT_S):
            now = time.time()
            for r in range(1, self.world):
                try:
                    ts = float(self.store.get(f"igloo/hb/{r}").decode())
                except Exception:  # noqa: BLE001 - not stamped yet
                    ts = start
                if now - ts > self.RANK_TIMEOUT_S:
                    self._break(f"rank {r} stopped heartbeating ({now - ts:.1f}s)")
                    return

    def _break(self, why: str):
        if self.broken:
            return
        self.broken = why
        self.exit_code = 3
        log.warning("worker group %s broken: %s", self.id, why)
        if self.comm is not None:
            self.comm.abort()
        # answer the in-flight query first, then leave (no re-exec: a fresh process restarts us)
        threading.Timer(2.0, self._stop.set).start()

    def _agree(self, ok: bool, err: str):
        """All ranks exchange (ok, error) after a query; returns the failures."""
        import torch.distributed as dist
        box = [None] * self.world
        dist.all_gather_object(box, (self.rank, ok, err), group=self.status)
        return [(r, e) for r, o, e in box if not o]

    # ---------------------------------------------------------------- SPMD
    def _bcast(self, obj=None):
        import torch.distributed as dist
        box = [obj]
        dist.broadcast_object_list(box, src=0, group=self.ctrl)
        return box[0]

    def run_spmd(self, sql: str) -> pa.Table:
        if faults.ACTIVE:
            faults.check("kill_worker")
            faults.check("fail_query", sql)
        return self._spmd(("query", sql), lambda: self.engine.query(sql))

    def run_spmd_fragment(self, payload: bytes) -> pa.Table:
        from ..parallel.fragments import run_encoded_fragment
        return self._spmd(("fragment", payload), lambda: run_encoded_fragment(self.engine, payload))

    def _spmd(self, cmd, fn) -> pa.Table:
        """Rank 0: broadcast the command, run it, then agree with every rank on
        the outcome. A rank-local failure (device fault on one GPU) or a broken
        group surfaces as a retryable CommError / DeviceError; an error every
        rank hit (bad SQL) is re-raised as is."""
        from ..utils.errors import CommError, DeviceError, IglooError
        with self._lock:
            if self.broken:
                raise CommError(f"worker group broken: {self.broken}")
            if self.world == 1:
                return fn()
            try:
                self._bcast(cmd)
            except Exception as e:  # noqa: BLE001
                self._break(f"control broadcast failed: {e}")
                raise CommError(f"worker group broken: {self.broken}") from None
            res, err, exc = None, "", None
            try:
                res = fn()
            except Exception as e:  # noqa: BLE001
                exc, err = e, f"{type(e).__name__}: {e}"
            if self.broken:
                raise CommError(f"worker group broken: {self.broken}")
            try:
                failed = self._agree(exc is None, err)
            except Exception as e:  # noqa: BLE001 - a rank died before reporting
                self._break(f"status exchange failed: {e}")
                raise CommError(f"worker group broken: {self.broken}") from None
            if not failed:
                return res
            if exc is not None and len(failed) == self.world and isinstance(exc, IglooError) \
                    and not isinstance(exc, (CommError, DeviceError)):
                raise exc   # the query itself is wrong on every rank
            raise DeviceError("query failed on rank(s) " + "; ".join(f"{r}: {e}" for r, e in failed))

    def follower_loop(self):
        """Ranks > 0: execute whatever rank 0 broadcasts, then report the outcome."""
        from ..parallel.fragments import run_encoded_fragment
        while True:
            try:
                cmd = self._bcast()
            except Exception as e:  # noqa: BLE001 - rank 0 is gone
                log.warning("rank %d: control channel lost (%s), exiting", self.rank, e)
                self.exit_code = 3
                return
            if cmd[0] == "shutdown":
                return
            if faults.ACTIVE:
                faults.check("kill_worker", f"rank{self.rank}")
            ok, err = True, ""
            try:
                if cmd[0] == "query":
                    if faults.ACTIVE:
                        faults.check("fail_query", f"rank{self.rank}:{cmd[1]}")
                    self.engine.query(cmd[1])
                elif cmd[0] == "fragment":
                    run_encoded_fragment(self.engine, cmd[1])
            except Exception as e:  # noqa: BLE001 - reported to rank 0 below
                ok, err = False, f"{type(e).__name__}: {e}"
                log.warning("rank %d: %s failed: %s", self.rank, cmd[0], err)
            try:
                self._agree(ok, err)
            except Exception as e:  # noqa: BLE001
                log.warning("rank %d: status exchange failed (%s), exiting", self.rank, e)
                self.exit_code = 3
                return

    # ------------------------------------------------------------- rank 0
    def devices(self) -> list:
        info = {"rank": self.rank, "device": str(self.engine.device)}
        if os.environ.get("IGLOO_SUPERVISOR_ID"):
            # started by a node supervisor (service/supervisor.py): a replacement
            # group follows if this one breaks, the coordinator waits for it
            info.update(supervisor=os.environ["IGLOO_SUPERVISOR_ID"],
                        generation=int(os.environ.get("IGLOO_GENERATION", "0")))
        if self.engine.device.type == "cuda":
            from ..ops._lib import native
            try:
                info.update(native().device_info(self.engine.device.index or 0))
            except Exception:  # noqa: BLE001
                pass
        if self.world > 1:
            return self.comm.allgather_object(info)
        return [info]

    def start_server(self):
        from .flight_server import IglooFlightServer
        self.server = IglooFlightServer(self.engine, f"grpc://{self.host}:{self.port}", runner=self.run_spmd,
                                        auth_token=self.token, fragment_runner=self.run_spmd_fragment)
        self.port = self.server.port
        self.address = f"grpc://{self.host}:{self.port}"
        self.server.start_background(host=self.host)

    def register(self) -> bool:
        if not self.coordinator:
            return False
        from .client import IglooClient
        try:
            with IglooClient(self.coordinator, self.token, timeout=10) as c:
                ack = c.register_worker(P.WorkerInfo(self.id, self.address, self._devices, self.world))
            log.info("registered with %s: %s", self.coordinator, ack.message)
            self.heartbeat_s = ack.heartbeat_interval_s or self.heartbeat_s
            return True
        except Exception as e:  # noqa: BLE001
            print(f"failed to register with coordinator {self.coordinator}: {e}", file=sys.stderr)
            return False

    def heartbeat_loop(self):
        from .client import IglooClient
        while not self._stop.wait(self.heartbeat_s):
            if self.broken or faults.fire("drop_heartbeat", self.id):
                continue
            try:
                with IglooClient(self.coordinator, self.token, timeout=5) as c:
                    r = c.heartbeat(P.HeartbeatInfo(self.id))
                if not r.ok:  # coordinator restarted or evicted us
                    self.register()
            except Exception as e:  # noqa: BLE001
                print(f"heartbeat failed: {e}", file=sys.stderr)

    def serve(self):
        """Blocking: rank 0 serves + heartbeats; other ranks follow."""
        # the startup heap (catalog, loaded tables, caches) moves to the
        # permanent GC generation: full collections during queries stay short
        import gc
        gc.collect()
        gc.freeze()
        devs = self.devices()  # collective: every rank
        if self.rank != 0:
            self.follower_loop()
            return
        self._devices = devs
        self.start_server()
        if self.register():
            threading.Thread(target=self.heartbeat_loop, daemon=True, name="igloo-heartbeat").start()
        print(f"igloo worker group {self.id} ({self.world} GPU rank(s)) serving on {self.address}", flush=True)
        signal.signal(signal.SIGINT, lambda *_: self._stop.set())
        signal.signal(signal.SIGTERM, lambda *_: self._stop.set())
        self._stop.wait()
        self.shutdown()

    def shutdown(self):
        self._stop.set()
        if self.world > 1 and self.rank == 0 and not self.broken:
            with self._lock:
                try:
                    self._bcast(("shutdown",))
                except Exception:  # noqa: BLE001
                    pass
        if self.server is not None:
            self.server.shutdown()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="igloo-worker")
    ap.add_argument("coordinator_pos", nargs="?", default=None, help="coordinator URL (reference: argv[1])")
    ap.add_argument("--coordinator", default=None)
    ap.add_argument("--host", default=None)
    ap.add_argument("--port", type=int, default=None)
    ap.add_argument("-c", "--config", default=None)
    ap.add_argument("--tpch", type=float, default=None, help="generate this rank's TPC-H partition at SF")
    ap.add_argument("--device", default=None)
    a = ap.parse_args(argv)
    cfg = load_config(a.config, {"worker_host": a.host, "worker_port": a.port, "device": a.device})
    if cfg.fault:
        faults.configure(cfg.fault)
    coord = a.coordinator or a.coordinator_pos or f"grpc://{cfg.coordinator_host}:{cfg.coordinator_port}"
    coord = coord.replace("http://", "grpc://")
    import igloo_amd as ig
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    device = cfg.device or (f"cuda:{local}" if torch.cuda.is_available() else "cpu")
    comm = None
    if world > 1:
        from ..parallel.comm import Communicator
        comm = Communicator.init(device=device, timeout_s=cfg.collective_timeout_s)
    engine = ig.QueryEngine(device=device, comm=comm)
    rank = comm.rank if comm else 0
    if a.tpch:
        from ..models.tpch import datagen
        for name, t in datagen.generate(a.tpch, device, rank, world).items():
            engine.register_table(name, t)
    register_config_tables(engine, cfg)
    wg = WorkerGroup(engine, comm, coord, cfg.worker_host, cfg.worker_port + (0 if rank == 0 else 0),
                     cfg.auth_token, cfg.heartbeat_interval_s, cfg.collective_timeout_s)
    wg.serve()
    if wg.exit_code:
        # broken group: leave without collective teardown (a peer is gone)
        sys.stdout.flush()
        os._exit(wg.exit_code)
    engine.close()      # release query graphs (RCCL teardown waits on graph-held collectives)
    if comm is not None:
        comm.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
