"""Control-plane and data-plane messages.

Parity with the reference's protobuf services (reference
crates/api/proto/coordinator.proto:1-69, distributed.proto:1-70):

  CoordinatorService.RegisterWorker(WorkerInfo) -> RegistrationAck
  CoordinatorService.SendHeartbeat(HeartbeatInfo) -> HeartbeatResponse
  WorkerService.ExecuteTask(TaskDefinition) -> TaskStatus
  WorkerService.GetDataForTask(DataForTaskRequest) -> DataForTaskResponse
  DistributedQueryService.ExecuteQuery(QueryRequest) -> stream QueryResponse
  DistributedQueryService.ExecuteFragment(FragmentRequest) -> stream RecordBatchMessage

There is no protoc / grpc_tools in this environment, so every message is a
dataclass carried as JSON in an Arrow Flight ``DoAction`` body (control) and
record batches travel as Arrow IPC through ``DoGet`` (data). Flight SQL
commands arrive as protobuf ``google.protobuf.Any``; the few fields needed are
decoded by the tiny wire codec below.
"""
from __future__ import annotations

import json
import time
from dataclasses import asdict, dataclass, field
from typing import Any, Dict, List, Optional, Tuple, Type, TypeVar

T = TypeVar("T")


class Message:
    def to_json(self) -> bytes:
        return json.dumps(asdict(self)).encode()

    @classmethod
    def from_json(cls: Type[T], b: bytes) -> T:
        d = json.loads(b.decode() if isinstance(b, (bytes, bytearray)) else b)
        return cls(**d)  # type: ignore[call-arg]


@dataclass
class WorkerInfo(Message):
    id: str
    address: str
    devices: List[Dict[str, Any]] = field(default_factory=list)  # GPU inventory (name, arch, HBM, CUs)
    world_size: int = 1                                         # ranks (GPUs) behind this address


@dataclass
class RegistrationAck(Message):
    message: str
    heartbeat_interval_s: float = 5.0


@dataclass
class HeartbeatInfo(Message):
    worker_id: str
    timestamp: int = field(default_factory=lambda: int(time.time()))
    hbm_used: int = 0
    active_tasks: int = 0


@dataclass
class HeartbeatResponse(Message):
    ok: bool


@dataclass
class TaskDefinition(Message):
    task_id: str
    payload: str               # SQL text or serialized plan
    session: Dict[str, Any] = field(default_factory=dict)


@dataclass
class TaskStatus(Message):
    status: str                # SUBMITTED | RUNNING | DONE | FAILED
    task_id: str = ""
    rows: int = 0
    elapsed_ms: float = 0.0
    error: str = ""


@dataclass
class DataForTaskRequest(Message):
    task_id: str


@dataclass
class QueryRequest(Message):
    sql: str
    session_config: Dict[str, Any] = field(default_factory=dict)


@dataclass
class QueryComplete(Message):
    total_rows: int
    execution_time_ms: float


@dataclass
class QueryError(Message):
    error_type: str
    message: str
    details: str = ""


# ----------------------------------------------------------- protobuf (tiny)
def _varint(b: bytes, p: int) -> Tuple[int, int]:
    shift = acc = 0
    while True:
        c = b[p]
        p += 1
        acc |= (c & 0x7F) << shift
        if not c & 0x80:
            return acc, p
        shift += 7


def _enc_varint(n: int) -> bytes:
    out = bytearray()
    while True:
        x = n & 0x7F
        n >>= 7
        out.append(x | 0x80 if n else x)
        if not n:
            return bytes(out)


def pb_decode(b: bytes) -> Dict[int, List[Any]]:
    """field number -> list of values (varint ints or length-delimited bytes)."""
    out: Dict[int, List[Any]] = {}
    p = 0
    while p < len(b):
        key, p = _varint(b, p)
        fno, wt = key >> 3, key & 7
        if wt == 0:
            v, p = _varint(b, p)
        elif wt == 2:
            n, p = _varint(b, p)
            v = b[p:p + n]
            p += n
        elif wt == 1:
            v = b[p:p + 8]
            p += 8
        elif wt == 5:
            v = b[p:p + 4]
            p += 4
        else:
            raise ValueError(f"unsupported protobuf wire type {wt}")
        out.setdefault(fno, []).append(v)
    return out


def pb_field(fno: int, value) -> bytes:
    if isinstance(value, int):
        return _enc_varint(fno << 3) + _enc_varint(value)
    data = value.encode() if isinstance(value, str) else bytes(value)
    return _enc_varint((fno << 3) | 2) + _enc_varint(len(data)) + data


FLIGHT_SQL = "type.googleapis.com/arrow.flight.protocol.sql."


def pack_any(type_name: str, body: bytes) -> bytes:
    return pb_field(1, FLIGHT_SQL + type_name) + pb_field(2, body)


def unpack_any(b: bytes) -> Optional[Tuple[str, Dict[int, List[Any]]]]:
    """Decode ``google.protobuf.Any`` -> (short type name, fields); None if not an Any."""
    try:
        f = pb_decode(b)
        url = f.get(1, [b""])[0].decode()
        if not url.startswith("type.googleapis.com/"):
            return None
        return url.rsplit(".", 1)[-1], pb_decode(f.get(2, [b""])[0])
    except (ValueError, IndexError, UnicodeDecodeError):
        return None


def command_statement_query(sql: str) -> bytes:
    """Flight SQL CommandStatementQuery{query=1} wrapped in Any (client side)."""
    return pack_any("CommandStatementQuery", pb_field(1, sql))


def ticket_statement_query(handle: bytes) -> bytes:
    return pack_any("TicketStatementQuery", pb_field(1, handle))
