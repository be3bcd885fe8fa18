"""``igloo-node``: per-node supervisor of the SPMD worker group (one worker
process per GPU), with recovery on the surviving GPUs.

The reference's worker is a single process that heartbeats every 5 s and
whose fragment errors fail the whole query with no retry (reference
crates/worker/src/main.rs:29-41, crates/coordinator/src/distributed_executor.rs:79-83,
:143-161). SURVEY §5.3 asks for recovery by retrying the query re-planned on
the N-1 GPUs that are left. Inside one node that needs a new process group:
a communicator that lost a rank cannot be repaired, and a process that has
touched the GPU must never be re-exec'd. So recovery here is generational:

1. the supervisor (which never touches a GPU) starts generation 0: one fresh
   ``igloo_amd.service.worker`` process per device, forming one SPMD group of
   N ranks (own rendezvous port), each holding its partition of the tables;
2. when a rank dies, its group breaks: rank 0's watchdog aborts the
   communicator, answers the in-flight query with a retryable error and exits
   with status 3 ("healthy, group broken"), as do the other survivors. A
   worker that exits with any other status (a fault, a kill, a GPU error)
   marks its device dead;
3. the supervisor reaps the generation (stragglers are killed after a grace
   period) and starts generation g+1 as FRESH processes on the surviving
   devices: a new process group of N-1 ranks whose members re-derive their
   partitions for the new world size (row groups / hash partitions are
   reassigned by rank and world) and register with the coordinator as a new
   group;
4. the coordinator, which marked the broken group dead, waits up to
   ``recovery_wait_s`` for a replacement group of a supervised node before
   falling back to local execution, and retries the query there.

    python -m igloo_amd.service.supervisor --devices cuda:0,cuda:1,... \
        --coordinator grpc://host:50051 [worker options: --tpch SF | --config FILE]
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import threading
import time
import uuid
from typing import Dict, List, Optional, Sequence

from ..utils.log import get_logger

log = get_logger("supervisor")

#: worker exit status of a healthy rank whose group broke (service/worker.py)
EXIT_GROUP_BROKEN = 3


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class NodeSupervisor:
    def __init__(self, devices: Sequence[str], coordinator: str, worker_args: Sequence[str] = (),
                 env: Optional[Dict[str, str]] = None, min_world: int = 1, max_generations: int = 4,
                 grace_s: float = 3.0, first_generation_env: Optional[Dict[str, str]] = None):
        self.devices = list(devices)
        self.coordinator = coordinator
        self.worker_args = list(worker_args)
        self.env = dict(os.environ if env is None else env)
        # extra environment for generation 0 only (e.g. an injected fault)
        self.first_env = dict(first_generation_env or {})
        self.min_world = min_world
        self.max_generations = max_generations
        self.grace_s = grace_s
        self.id = f"node-{uuid.uuid4().hex[:8]}"
        self.generation = -1
        self.procs: List[subprocess.Popen] = []
        self.history: List[dict] = []      # per generation: devices, exit codes, dead devices
        self._stop = threading.Event()

    # ------------------------------------------------------------ lifecycle
    def start_generation(self) -> None:
        self.generation += 1
        world = len(self.devices)
        port = _free_port()
        self.procs = []
        for rank, dev in enumerate(self.devices):
            env = dict(self.env, RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                       MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), IGLOO_SUPERVISOR_ID=self.id,
                       IGLOO_GENERATION=str(self.generation))
            if self.generation == 0:
                env.update(self.first_env)
            else:
                env.pop("IGLOO_FAULT", None)
            cmd = [sys.executable, "-m", "igloo_amd.service.worker", "--coordinator", self.coordinator,
                   "--port", "0", "--device", dev] + self.worker_args
            self.procs.append(subprocess.Popen(cmd, env=env))
        log.info("%s generation %d: %d rank(s) on %s", self.id, self.generation, world, ",".join(self.devices))

    def _reap(self) -> Dict[int, int]:
        """After the first exit of a generation: give the others ``grace_s``
        to leave on their own (a broken group's survivors exit with status 3),
        then kill the rest (they count as survivors)."""
        deadline = time.time() + self.grace_s
        while time.time() < deadline and any(p.poll() is None for p in self.procs):
            time.sleep(0.05)
        codes = {}
        for r, p in enumerate(self.procs):
            if p.poll() is None:
                p.kill()
                p.wait()
                codes[r] = EXIT_GROUP_BROKEN
            else:
                codes[r] = p.returncode
        return codes

    def step(self) -> bool:
        """Wait for the current generation to end; start the next one on the
        surviving devices. False when the node is done (clean shutdown, too
        few devices left, or the generation budget is spent)."""
        while not self._stop.is_set():
            if any(p.poll() is not None for p in self.procs):
                break
            time.sleep(0.05)
        if self._stop.is_set():
            return False
        codes = self._reap()
        dead = [r for r, c in codes.items() if c not in (0, EXIT_GROUP_BROKEN)]
        rec = {"generation": self.generation, "devices": list(self.devices), "exit_codes": codes,
               "dead": [self.devices[r] for r in dead], "t": time.time()}
        self.history.append(rec)
        if all(c == 0 for c in codes.values()):
            return False
        survivors = [d for r, d in enumerate(self.devices) if r not in dead]
        log.warning("%s generation %d ended (exit codes %s); dead device(s): %s", self.id, self.generation,
                    codes, rec["dead"] or "none")
        if len(survivors) < self.min_world or self.generation + 1 >= self.max_generations:
            return False
        self.devices = survivors
        self.start_generation()
        return True

    def run(self) -> int:
        self.start_generation()
        while self.step():
            pass
        self.shutdown()
        return 0

    def shutdown(self) -> None:
        self._stop.set()
        for p in self.procs:
            if p.poll() is None:
                p.terminate()
        for p in self.procs:
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                p.kill()


def count_gpus(env=None, topology: str = "/sys/class/kfd/kfd/topology/nodes") -> int:
    """Visible GPUs, counted WITHOUT touching the HIP runtime (the supervisor
    forks and execs worker generations, which a GPU-initialised process must
    not do): an explicit ``*_VISIBLE_DEVICES`` list wins, else the KFD
    topology's nodes with SIMDs (CPU nodes report ``simd_count 0``)."""
    env = os.environ if env is None else env
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = env.get(var)
        if v is not None:
            return len([x for x in v.split(",") if x.strip() and x.strip() != "-1"])
    n = 0
    try:
        for node in sorted(os.listdir(topology)):
            try:
                with open(os.path.join(topology, node, "properties")) as f:
                    props = dict(line.split()[:2] for line in f if len(line.split()) >= 2)
            except OSError:
                continue
            if int(props.get("simd_count", "0")) > 0:
                n += 1
    except OSError:
        return 0
    return n


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="igloo-node", description=__doc__.split("\n\n")[0])
    ap.add_argument("--devices", default=None,
                    help="comma-separated devices, one worker rank each (default: every visible GPU)")
    ap.add_argument("--coordinator", required=True)
    ap.add_argument("--min-world", type=int, default=1)
    ap.add_argument("--max-generations", type=int, default=4)
    ap.add_argument("--grace-s", type=float, default=3.0)
    a, rest = ap.parse_known_args(argv)
    devs = a.devices.split(",") if a.devices else None
    if devs is None:
        n = count_gpus()
        devs = [f"cuda:{i}" for i in range(n)] or ["cpu"]
    sup = NodeSupervisor(devs, a.coordinator, rest, min_world=a.min_world, max_generations=a.max_generations,
                         grace_s=a.grace_s)
    signal.signal(signal.SIGTERM, lambda *_: sup.shutdown())
    signal.signal(signal.SIGINT, lambda *_: sup.shutdown())
    return sup.run()


if __name__ == "__main__":
    sys.exit(main())
