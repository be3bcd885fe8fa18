"""PostgreSQL source over the v3 frontend/backend wire protocol.

Parity: the reference's Postgres connector is empty (reference
crates/connectors/postgres/src/lib.rs:1-9). No libpq / psycopg exists in this
environment, so the protocol is spoken directly:

* startup + authentication (trust, cleartext, MD5, SCRAM-SHA-256);
* schema discovery from the RowDescription of ``SELECT ... LIMIT 0``;
* bulk reads through ``COPY (SELECT <projected cols> FROM t [WHERE ...]) TO
  STDOUT WITH (FORMAT csv)`` — the server streams CSV that Arrow's multithreaded
  CSV reader parses straight into columns, which are uploaded to HBM once
  (projection pushdown: only referenced columns cross the wire);
* a CDC version probe (``version_sql``, e.g. ``SELECT max(updated_at) FROM t``)
  for cache invalidation.
"""
from __future__ import annotations

import base64
import hashlib
import hmac
import io
import os
import socket
import struct
import threading
from typing import Any, Dict, List, Optional, Sequence, Tuple
from urllib.parse import unquote, urlparse

import pyarrow as pa
import pyarrow.csv as pacsv

from .. import types as T
from ..catalog import Field, TableSource
from ..columnar import Batch, Column
from ..utils.errors import CommError, ExecutionError, IoError

# type OID -> DataType
OIDS = {16: T.BOOL, 20: T.INT64, 21: T.INT16, 23: T.INT32, 26: T.INT64, 700: T.FLOAT32, 701: T.FLOAT64,
        1082: T.DATE32, 1114: T.TIMESTAMP, 1184: T.TIMESTAMP, 25: T.UTF8, 1043: T.UTF8, 1042: T.UTF8, 19: T.UTF8,
        18: T.UTF8}


def _oid_type(oid: int, typmod: int) -> T.DataType:
    if oid == 1700:
        if typmod >= 4:
            tm = typmod - 4
            return T.DECIMAL((tm >> 16) & 0xFFFF, tm & 0xFFFF)
        return T.DECIMAL(38, 6)
    return OIDS.get(oid, T.UTF8)


class PgError(ExecutionError):
    pass


class PgConnection:
    def __init__(self, dsn: str, timeout: float = 30.0):
        u = urlparse(dsn)
        if u.scheme not in ("postgres", "postgresql"):
            raise ValueError(f"not a postgres DSN: {dsn}")
        self.user = unquote(u.username or os.environ.get("PGUSER", "postgres"))
        self.password = unquote(u.password or os.environ.get("PGPASSWORD", ""))
        self.database = (u.path or "/").lstrip("/") or self.user
        try:
            self.sock = socket.create_connection((u.hostname or "127.0.0.1", u.port or 5432), timeout=timeout)
        except OSError as e:
            raise CommError(f"cannot connect to postgres {u.hostname}:{u.port}: {e}") from e
        self.buf = b""
        self.params: Dict[str, str] = {}
        self._lock = threading.Lock()
        self._startup()

    # ----------------------------------------------------------------- io
    def _send(self, tag: bytes, body: bytes):
        self.sock.sendall(tag + struct.pack("!I", len(body) + 4) + body)

    def _recv_exact(self, n: int) -> bytes:
        while len(self.buf) < n:
            chunk = self.sock.recv(max(65536, n - len(self.buf)))
            if not chunk:
                raise CommError("postgres connection closed")
            self.buf += chunk
        out, self.buf = self.buf[:n], self.buf[n:]
        return out

    def _msg(self) -> Tuple[bytes, bytes]:
        head = self._recv_exact(5)
        n = struct.unpack("!I", head[1:])[0]
        return head[:1], self._recv_exact(n - 4)

    @staticmethod
    def _error(body: bytes) -> str:
        fields = {}
        for part in body.split(b"\0"):
            if part:
                fields[chr(part[0])] = part[1:].decode(errors="replace")
        return f"{fields.get('S', 'ERROR')}: {fields.get('M', '')} ({fields.get('C', '')})"

    # ------------------------------------------------------------ startup
    def _startup(self):
        body = struct.pack("!I", 196608) + b"".join(k.encode() + b"\0" + v.encode() + b"\0" for k, v in
                                                    (("user", self.user), ("database", self.database),
                                                     ("client_encoding", "UTF8"))) + b"\0"
        self.sock.sendall(struct.pack("!I", len(body) + 4) + body)
        scram = None
        while True:
            tag, b = self._msg()
            if tag == b"R":
                code = struct.unpack("!I", b[:4])[0]
                if code == 0:
                    continue
                if code == 3:
                    self._send(b"p", self.password.encode() + b"\0")
                elif code == 5:
                    salt = b[4:8]
                    inner = hashlib.md5(self.password.encode() + self.user.encode()).hexdigest().encode()
                    self._send(b"p", b"md5" + hashlib.md5(inner + salt).hexdigest().encode() + b"\0")
                elif code == 10:
                    scram = _Scram(self.user, self.password)
                    first = scram.client_first()
                    self._send(b"p", b"SCRAM-SHA-256\0" + struct.pack("!I", len(first)) + first)
                elif code == 11:
                    self._send(b"p", scram.client_final(b[4:]))
                elif code == 12:
                    scram.verify(b[4:])
                else:
                    raise CommError(f"unsupported postgres auth method {code}")
            elif tag == b"S":
                k, v = b.rstrip(b"\0").split(b"\0", 1)
                self.params[k.decode()] = v.decode()
            elif tag == b"K":
                pass
            elif tag == b"E":
                raise PgError(self._error(b))
            elif tag == b"Z":
                return

    # -------------------------------------------------------------- queries
    def query(self, sql: str) -> Tuple[List[Tuple[str, int, int]], List[List[Optional[str]]]]:
        """Simple query -> (fields [(name, oid, typmod)], text rows)."""
        with self._lock:
            self._send(b"Q", sql.encode() + b"\0")
            fields, rows, err = [], [], None
            while True:
                tag, b = self._msg()
                if tag == b"T":
                    n = struct.unpack("!H", b[:2])[0]
                    p = 2
                    fields = []
                    for _ in range(n):
                        e = b.index(b"\0", p)
                        name = b[p:e].decode()
                        p = e + 1
                        _tbl, _att, oid, _len, typmod, _fmt = struct.unpack("!IhIhih", b[p:p + 18])
                        p += 18
                        fields.append((name, oid, typmod))
                elif tag == b"D":
                    n = struct.unpack("!H", b[:2])[0]
                    p = 2
                    row = []
                    for _ in range(n):
                        ln = struct.unpack("!i", b[p:p + 4])[0]
                        p += 4
                        if ln < 0:
                            row.append(None)
                        else:
                            row.append(b[p:p + ln].decode())
                            p += ln
                    rows.append(row)
                elif tag == b"E":
                    err = self._error(b)
                elif tag == b"Z":
                    if err:
                        raise PgError(err)
                    return fields, rows
                # C (CommandComplete), N (notice), I (empty), S: ignored

    def copy_out(self, sql: str) -> bytes:
        """``COPY (sql) TO STDOUT`` -> raw text payload."""
        with self._lock:
            self._send(b"Q", f"COPY ({sql}) TO STDOUT WITH (FORMAT csv)".encode() + b"\0")
            out = io.BytesIO()
            err = None
            while True:
                tag, b = self._msg()
                if tag == b"d":
                    out.write(b)
                elif tag == b"E":
                    err = self._error(b)
                elif tag == b"Z":
                    if err:
                        raise PgError(err)
                    return out.getvalue()

    def close(self):
        try:
            self._send(b"X", b"")
        except OSError:
            pass
        self.sock.close()


class _Scram:
    def __init__(self, user: str, password: str):
        self.password = password.encode()
        self.nonce = base64.b64encode(os.urandom(18)).decode()
        self.first_bare = f"n=,r={self.nonce}"

    def client_first(self) -> bytes:
        return ("n,," + self.first_bare).encode()

    def client_final(self, server_first: bytes) -> bytes:
        sf = server_first.decode()
        attrs = dict(kv.split("=", 1) for kv in sf.split(","))
        salt = base64.b64decode(attrs["s"])
        it = int(attrs["i"])
        salted = hashlib.pbkdf2_hmac("sha256", self.password, salt, it)
        ckey = hmac.new(salted, b"Client Key", "sha256").digest()
        skey = hashlib.sha256(ckey).digest()
        final_wo = f"c=biws,r={attrs['r']}"
        auth = f"{self.first_bare},{sf},{final_wo}".encode()
        sig = hmac.new(skey, auth, "sha256").digest()
        proof = bytes(a ^ b for a, b in zip(ckey, sig))
        self.server_sig = hmac.new(hmac.new(salted, b"Server Key", "sha256").digest(), auth, "sha256").digest()
        return f"{final_wo},p={base64.b64encode(proof).decode()}".encode()

    def verify(self, server_final: bytes):
        v = dict(kv.split("=", 1) for kv in server_final.decode().split(","))
        if base64.b64decode(v.get("v", "")) != self.server_sig:
            raise CommError("SCRAM server signature mismatch")


def _arrow_from_copy(payload: bytes, fields: List[Field]) -> pa.Table:
    if not payload:
        return pa.table({f.name: pa.array([], f.dtype.to_arrow()) for f in fields})
    ro = pacsv.ReadOptions(column_names=[f.name for f in fields])
    po = pacsv.ParseOptions(newlines_in_values=True)
    types = {}
    for f in fields:
        if f.dtype.kind == "bool":
            types[f.name] = pa.string()
        else:
            types[f.name] = f.dtype.to_arrow()
    # CSV COPY: NULL is an unquoted empty field, an empty string is ""
    co = pacsv.ConvertOptions(column_types=types, null_values=[""], strings_can_be_null=True,
                              quoted_strings_can_be_null=False)
    t = pacsv.read_csv(io.BytesIO(payload), read_options=ro, parse_options=po, convert_options=co)
    for i, f in enumerate(fields):
        if f.dtype.kind == "bool":
            col = t.column(i)
            t = t.set_column(i, f.name, pa.array([None if v is None else v in ("t", "true", "1")
                                                   for v in col.to_pylist()], pa.bool_()))
    return t


class PostgresTable(TableSource):
    # every SPMD rank reads the whole (small, dimension-like) table: the planner
    # treats it as replicated, so joins against partitioned facts need no shuffle
    replicated = True
    # resident copies live in the engine's cache tier (cache/cdc.py), keyed by ``version``
    cacheable = True
    cdc_poll_s = 0.0   # the version query runs before every scan

    def __init__(self, dsn: str, table: str, query: Optional[str] = None, version_sql: Optional[str] = None):
        self.dsn = dsn
        self.table = table
        self.base = query or f"SELECT * FROM {table}"
        self.version_sql = version_sql
        self._conn: Optional[PgConnection] = None
        self._fields: Optional[List[Field]] = None

    def conn(self) -> PgConnection:
        if self._conn is None:
            self._conn = PgConnection(self.dsn)
        return self._conn

    def schema(self) -> List[Field]:
        if self._fields is None:
            fields, _ = self.conn().query(f"SELECT * FROM ({self.base}) AS q LIMIT 0")
            self._fields = [Field(n, _oid_type(o, m), True) for n, o, m in fields]
        return self._fields

    def num_rows(self) -> Optional[int]:
        _, rows = self.conn().query(f"SELECT count(*) FROM ({self.base}) AS q")
        return int(rows[0][0])

    @property
    def version(self):
        if not self.version_sql:
            return None
        _, rows = self.conn().query(self.version_sql)
        return rows[0][0] if rows else None

    def read(self, columns: Sequence[str], where: Optional[str] = None) -> pa.Table:
        fmap = {f.name: f for f in self.schema()}
        cols = ", ".join(f'"{c}"' for c in columns) or "1"
        sql = f"SELECT {cols} FROM ({self.base}) AS q" + (f" WHERE {where}" if where else "")
        payload = self.conn().copy_out(sql)
        return _arrow_from_copy(payload, [fmap[c] for c in columns])

    def scan(self, columns: Sequence[str], ctx) -> Batch:
        import torch
        device = ctx.device if ctx is not None else torch.device("cpu")
        out = {}
        if columns:
            t = self.read(columns)
            types = {f.name: f.dtype for f in self.schema()}
            for c in columns:
                out[c] = Column.from_arrow(t.column(c), device=device, dtype=types[c])
        n = len(next(iter(out.values()))) if out else (self.num_rows() or 0)
        return Batch(out, n)
