"""Flight endpoint, control plane, coordinator routing and worker failover."""
import os
import subprocess
import sys
import threading
import time

import pyarrow as pa
import pyarrow.flight as fl
import pytest

import igloo_amd as ig
from igloo_amd.service import protocol as P
from igloo_amd.service.client import IglooClient
from igloo_amd.service.coordinator import Coordinator
from igloo_amd.service.flight_server import IglooFlightServer
from igloo_amd.service.registry import WorkerRegistry
from igloo_amd.utils.config import IglooConfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def server():
    # one server per module: restarting servers on recycled ports trips gRPC's
    # shared subchannel backoff (connection refused for the new server)
    e = ig.QueryEngine(device="cpu")
    e.register_table("t", pa.table({"a": pa.array([1, 2, 3], pa.int64()), "b": ["x", "y", "z"]}))
    s = IglooFlightServer(e, "grpc://127.0.0.1:0", registry=WorkerRegistry(0.2))
    s.start_background()
    yield s, f"grpc://127.0.0.1:{s.port}"
    s.shutdown()


def test_query_raw_and_flight_sql(server):
    s, uri = server
    with IglooClient(uri) as c:
        t = c.query("SELECT a, b FROM t WHERE a >= 2 ORDER BY a")
        assert t.to_pylist() == [{"a": 2, "b": "y"}, {"a": 3, "b": "z"}]
        t2 = c.query("SELECT sum(a) s FROM t", flight_sql=True)
        assert t2.to_pylist() == [{"s": 6}]
        assert c.execute_raw("SELECT count(*) n FROM t").to_pylist() == [{"n": 3}]
        # schema comes from planning only: no query ran
        before = s.metrics["queries"]
        assert c.schema("SELECT a FROM t").names == ["a"]
        assert s.metrics["queries"] == before


def test_flight_status_codes(server):
    _, uri = server
    with IglooClient(uri) as c:
        with pytest.raises(pa.ArrowKeyError):  # NotFound on empty result (reference api/src/lib.rs:125-128)
            c.execute_raw("SELECT a FROM t WHERE a > 100")
        assert c.query("SELECT a FROM t WHERE a > 100", flight_sql=True).num_rows == 0
        with pytest.raises(pa.ArrowInvalid):  # bad UTF-8 ticket -> InvalidArgument
            c.client.do_get(fl.Ticket(b"\xff\xfe")).read_all()
        with pytest.raises(pa.ArrowInvalid):  # empty command
            c.client.get_flight_info(fl.FlightDescriptor.for_command(b""))
        with pytest.raises(pa.ArrowInvalid):  # SQL error -> InvalidArgument, not a crash
            c.query("SELECT nope FROM t")


def test_put_list_actions(server):
    _, uri = server
    with IglooClient(uri) as c:
        c.upload("up", pa.table({"k": [1, 2, 3, 4]}))
        assert "up" in c.tables()
        assert c.query("SELECT sum(k) s FROM up").to_pylist() == [{"s": 10}]
        assert "Scan" in c.explain("SELECT k FROM up")
        assert c.metrics()["queries"] >= 1
        ack = c.register_worker(P.WorkerInfo("w1", "grpc://127.0.0.1:1"))
        assert ack.message == "Registered"
        assert c.heartbeat(P.HeartbeatInfo("w1")).ok
        assert not c.heartbeat(P.HeartbeatInfo("unknown")).ok
        assert c.list_workers()[0]["id"] == "w1"
        st = c.execute_task(P.TaskDefinition("task-1", "SELECT a FROM t ORDER BY a"))
        assert st.status == "DONE" and st.rows == 3
        assert c.get_data_for_task("task-1").column("a").to_pylist() == [1, 2, 3]


def test_execute_query_streams_batches_and_completion(server, monkeypatch):
    """ExecuteQuery: QueryRequest{sql, session_config} -> record-batch stream +
    QueryComplete; the session setting applies to that query only."""
    from igloo_amd.parallel import fragments as F
    s, uri = server
    monkeypatch.setattr(F, "STREAM_BATCH_ROWS", 2)
    with IglooClient(uri) as c:
        bodies = list(c.action_stream("execute_query", P.QueryRequest("SELECT a, b FROM t ORDER BY a").to_json()))
        assert len(bodies) == 3 and bodies[-1][:2] == b"QC"      # 2 batches of <= 2 rows + completion
        t, done = c.execute_query("SELECT a, b FROM t ORDER BY a", {"probe_setting": 7})
        assert t.column("a").to_pylist() == [1, 2, 3]
        assert done["total_rows"] == 3 and done["execution_time_ms"] >= 0
        empty, done = c.execute_query("SELECT a FROM t WHERE a > 10")
        assert empty.num_rows == 0 and done["total_rows"] == 0
    assert "probe_setting" not in s.engine.session


def test_fragment_carries_session_config():
    import igloo_amd as ig
    from igloo_amd.parallel import fragments as F
    e = ig.QueryEngine(device="cpu")
    e.register_table("t", pa.table({"a": [1, 2, 3]}))
    plan, _ = e.logical_plan("SELECT sum(a) AS s FROM t")
    from igloo_amd.sql import logical as L
    frag = next(f for f in F.DistributedPlanner(["w0"]).plan(plan)
                if not any(isinstance(p, F.FragmentRef) for p in L.walk_plan(f.plan)))
    payload = F.encode_fragment(frag, {}, {"device_budget_gb": 0.5, "obj": object()})
    seen = {}
    orig = e.make_context

    def spy():
        seen.update(e.session)
        return orig()
    e.make_context = spy
    out = F.run_encoded_fragment(e, payload)
    assert out.num_rows >= 1 and seen.get("device_budget_gb") == 0.5   # leaf (scan) fragment
    assert "device_budget_gb" not in e.session


def test_registry_eviction():
    r = WorkerRegistry(heartbeat_interval_s=1.0, timeout_s=2.0)
    r.register(P.WorkerInfo("a", "x"))
    dead = []
    r.on_dead(dead.append)
    assert r.reap(now=time.time() + 1) == []
    assert r.reap(now=time.time() + 5) == ["a"] and dead == ["a"]
    assert not r.heartbeat(P.HeartbeatInfo("a")).ok  # evicted workers must re-register


def test_protocol_any_roundtrip():
    b = P.command_statement_query("SELECT 1")
    name, f = P.unpack_any(b)
    assert name == "CommandStatementQuery" and f[1][0].decode() == "SELECT 1"
    assert P.unpack_any(b"SELECT 1") is None


def _spawn_worker(coord, tag, fault=None):
    env = dict(os.environ, PYTHONPATH=ROOT, IGLOO_HEARTBEAT_INTERVAL_S="0.3")
    if fault:
        env["IGLOO_FAULT"] = fault
    return subprocess.Popen([sys.executable, "-m", "igloo_amd.service.worker", "--coordinator", coord, "--port", "0",
                             "--tpch", "0.01", "--device", "cpu"], env=env, cwd=ROOT,
                            stdout=subprocess.PIPE, stderr=subprocess.STDOUT)


def test_coordinator_routes_and_fails_over():
    co = Coordinator(IglooConfig(coordinator_port=0, heartbeat_interval_s=0.3, heartbeat_timeout_s=1.5,
                                 device="cpu")).start()
    from igloo_amd.models.tpch import datagen
    datagen.register(co.engine, 0.01)  # local fallback has the same data
    ws = [_spawn_worker(co.address, i) for i in range(2)]
    try:
        t0 = time.time()
        while len(co.registry.alive()) < 2 and time.time() - t0 < 120:
            time.sleep(0.2)
        assert len(co.registry.alive()) == 2, [w.stdout.read1(4096) for w in ws if w.poll() is not None]
        sql = "SELECT count(*) AS n FROM lineitem"
        with IglooClient(co.address) as c:
            n = c.query(sql).to_pylist()[0]["n"]
            assert n == 59875
            ran_on = co.executor.log[-1][1]
            assert ran_on != "local"
            # kill the group that answered; the next query is retried elsewhere
            victim = [w for w in co.registry.alive() if w.info.id == ran_on][0]
            for p in ws:
                p.terminate()
                break
            time.sleep(2.5)  # heartbeat timeout -> eviction
            assert c.query(sql).to_pylist()[0]["n"] == n
            assert len(co.registry.alive()) <= 1
    finally:
        for p in ws:
            p.kill()
        co.shutdown()


def test_fault_spec_and_local_hooks():
    from igloo_amd.ops import _lib
    from igloo_amd.parallel.comm import LocalComm
    from igloo_amd.utils import faults
    from igloo_amd.utils.errors import CommError, DeviceError
    fs = faults.parse("drop_heartbeat; kernel_error@join_probe:1, comm_timeout@all_to_all_v:2")
    assert [(f.kind, f.target, f.remaining) for f in fs] == [
        ("drop_heartbeat", None, None), ("kernel_error", "join_probe", 1), ("comm_timeout", "all_to_all_v", 2)]
    with pytest.raises(ValueError):
        faults.parse("explode@x")
    import torch
    with faults.inject("kernel_error@join_probe:1;comm_timeout@all_to_all_v:2"):
        with pytest.raises(DeviceError):
            _lib.launch("join_probe")
        assert faults.active()[0].remaining == 0   # count consumed: fires once
        c = LocalComm("cpu")
        t = torch.arange(4)
        for _ in range(2):
            with pytest.raises(CommError):
                c.all_to_all_v(t, [4])
        assert torch.equal(c.all_to_all_v(t, [4])[0], t)
        c.all_gather_v(t)   # other collectives unaffected
    assert not faults.ACTIVE


def test_injected_faults_drive_eviction_and_retry():
    """drop_heartbeat -> the reaper evicts a live worker; fail_query -> the
    coordinator marks the failing group dead and reruns the query elsewhere."""
    co = Coordinator(IglooConfig(coordinator_port=0, heartbeat_interval_s=0.3, heartbeat_timeout_s=1.5,
                                 device="cpu")).start()
    from igloo_amd.models.tpch import datagen
    datagen.register(co.engine, 0.01)  # the coordinator plans schemas locally
    ws = [_spawn_worker(co.address, 0, fault="fail_query@lineitem"), _spawn_worker(co.address, 1),
          _spawn_worker(co.address, 2, fault="drop_heartbeat")]
    try:
        t0 = time.time()
        while len(co.registry.snapshot()) < 3 and time.time() - t0 < 120:
            time.sleep(0.2)
        assert len(co.registry.snapshot()) == 3, [w.stdout.read1(4096) for w in ws if w.poll() is not None]
        time.sleep(2.5)   # the heartbeat-dropping worker is evicted although its process lives
        assert ws[2].poll() is None and len(co.registry.alive()) == 2
        sql = "SELECT count(*) AS n FROM lineitem"
        with IglooClient(co.address) as c:
            for _ in range(2):   # least-loaded routing reaches the faulty group by the second query
                assert c.query(sql).to_pylist()[0]["n"] == 59875
        outcomes = [o for (_, _, _, o) in co.executor.log]
        assert any(o.startswith("retry") for o in outcomes), co.executor.log
        assert co.executor.log[-1][1] != "local" and len(co.registry.alive()) == 1
    finally:
        for p in ws:
            p.kill()
        co.shutdown()


def _spawn_group_rank(coord, rank, world, port, fault=None):
    env = dict(os.environ, PYTHONPATH=ROOT, IGLOO_HEARTBEAT_INTERVAL_S="0.3", RANK=str(rank), LOCAL_RANK=str(rank),
               WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
               IGLOO_COLLECTIVE_TIMEOUT_S="20")
    if fault:
        env["IGLOO_FAULT"] = fault
    return subprocess.Popen([sys.executable, "-m", "igloo_amd.service.worker", "--coordinator", coord, "--port", "0",
                             "--tpch", "0.01", "--device", "cpu"], env=env, cwd=ROOT,
                            stdout=subprocess.PIPE, stderr=subprocess.STDOUT)


def test_rank_death_inside_group_fails_over_within_30s():
    """SPMD recovery: rank 1 of a 2-rank worker group dies
    mid-query (IGLOO_FAULT=kill_worker@rank1). Rank 0's collective fails
    promptly, the group agrees the query failed and marks itself broken, the
    coordinator quarantines it and reruns the query on the healthy group, and
    the broken group's rank 0 exits non-zero instead of hanging."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    co = Coordinator(IglooConfig(coordinator_port=0, heartbeat_interval_s=0.3, heartbeat_timeout_s=1.5,
                                 device="cpu")).start()
    from igloo_amd.models.tpch import datagen
    datagen.register(co.engine, 0.01)
    group = [_spawn_group_rank(co.address, r, 2, port, fault="kill_worker@rank1") for r in range(2)]
    healthy = None
    try:
        t0 = time.time()
        while len(co.registry.alive()) < 1 and time.time() - t0 < 120:
            time.sleep(0.2)
        assert len(co.registry.alive()) == 1, [p.stdout.read1(4096) for p in group if p.poll() is not None]
        healthy = _spawn_worker(co.address, 9)
        while len(co.registry.alive()) < 2 and time.time() - t0 < 180:
            time.sleep(0.2)
        assert len(co.registry.alive()) == 2
        sql = "SELECT count(*) AS n FROM lineitem"
        t1 = time.time()
        with IglooClient(co.address) as c:
            assert c.query(sql).to_pylist()[0]["n"] == 59875
        took = time.time() - t1
        assert took < 30, took
        outcomes = [o for (_, _, _, o) in co.executor.log]
        assert outcomes[0].startswith("retry") and outcomes[-1] == "ok", co.executor.log
        assert co.executor.log[-1][1] != "local"
        assert group[1].wait(timeout=10) == 17          # the injected death
        assert group[0].wait(timeout=20) == 3           # broken group left instead of hanging
    finally:
        for p in group + ([healthy] if healthy else []):
            p.kill()
        co.shutdown()


def test_rank_death_recovers_on_surviving_ranks_of_the_node():
    """SURVEY §5.3 retry on N-1: a node supervisor runs a 3-rank SPMD worker
    group (gloo, CPU). Rank 2 dies mid-query (kill_worker@rank2); there is NO
    other worker group. The supervisor starts a fresh 2-rank group on the
    surviving devices (new process group, partitions re-derived for world 2),
    the coordinator waits for it and retries, and the answer is correct —
    within 30 s of submitting the query."""
    from igloo_amd.models.tpch import datagen, queries
    from igloo_amd.service.supervisor import NodeSupervisor
    co = Coordinator(IglooConfig(coordinator_port=0, heartbeat_interval_s=0.3, heartbeat_timeout_s=1.5,
                                 device="cpu", recovery_wait_s=40.0)).start()
    datagen.register(co.engine, 0.01)
    want = co.engine.query(queries.QUERIES[5]).to_pylist()
    env = dict(os.environ, PYTHONPATH=ROOT, IGLOO_HEARTBEAT_INTERVAL_S="0.3", IGLOO_COLLECTIVE_TIMEOUT_S="20")
    sup = NodeSupervisor(["cpu", "cpu", "cpu"], co.address, ["--tpch", "0.01"], env=env,
                         first_generation_env={"IGLOO_FAULT": "kill_worker@rank2"}, grace_s=2.0)
    t = threading.Thread(target=sup.run, daemon=True)
    t.start()
    try:
        t0 = time.time()
        while len(co.registry.alive()) < 1 and time.time() - t0 < 120:
            time.sleep(0.2)
        assert len(co.registry.alive()) == 1
        first = co.registry.alive()[0]
        assert first.info.world_size == 3
        t1 = time.time()
        with IglooClient(co.address) as c:
            got = c.query(queries.QUERIES[5]).to_pylist()
        took = time.time() - t1
        assert got == want
        assert took < 30, took
        outcomes = [(w, o) for (_, w, _, o) in co.executor.log]
        assert outcomes[0][0] == first.info.id and outcomes[0][1].startswith("retry"), co.executor.log
        assert outcomes[-1][1] == "ok" and outcomes[-1][0] not in ("local", first.info.id), co.executor.log
        ran = [w for w in co.registry.snapshot() if w["id"] == outcomes[-1][0]][0]
        assert ran["world_size"] == 2
        h = sup.history[0]
        assert h["exit_codes"][2] == 17 and h["dead"] == ["cpu"] and sup.generation == 1
    finally:
        sup.shutdown()
        co.shutdown()


def test_supervisor_counts_gpus_without_hip(tmp_path):
    """The node supervisor counts devices from the environment or the KFD
    topology (never through the HIP runtime: it forks worker generations)."""
    from igloo_amd.service.supervisor import count_gpus
    assert count_gpus({"HIP_VISIBLE_DEVICES": "0,3,5"}) == 3
    assert count_gpus({"ROCR_VISIBLE_DEVICES": ""}) == 0
    topo = tmp_path / "nodes"
    for i, simds in enumerate([0, 256, 256]):
        (topo / str(i)).mkdir(parents=True)
        (topo / str(i) / "properties").write_text(f"cpu_cores_count {4 if not simds else 0}\nsimd_count {simds}\n")
    assert count_gpus({}, str(topo)) == 2
    assert count_gpus({}, str(tmp_path / "missing")) == 0
