"""MySQL source over the client/server protocol 4.1 (text resultsets).

Parity: the reference's MySQL connector is empty (reference
crates/connectors/mysql/src/lib.rs:1-9). No client library is available, so
the protocol is implemented directly: HandshakeV10 -> HandshakeResponse41
(mysql_native_password), COM_QUERY with text resultsets (column definitions,
length-encoded rows, EOF/OK), ERR packets as errors. Rows are converted into
Arrow columns on the host and uploaded to HBM once; only projected columns are
requested.
"""
from __future__ import annotations

import datetime
import hashlib
import socket
import struct
import threading
from decimal import Decimal
from typing import Dict, List, Optional, Sequence, Tuple
from urllib.parse import unquote, urlparse

import pyarrow as pa

from .. import types as T
from ..catalog import Field, TableSource
from ..columnar import Batch, Column
from ..utils.errors import CommError, ExecutionError

CLIENT_LONG_PASSWORD = 0x1
CLIENT_PROTOCOL_41 = 0x200
CLIENT_SECURE_CONNECTION = 0x8000
CLIENT_CONNECT_WITH_DB = 0x8
CLIENT_PLUGIN_AUTH = 0x80000

# column type -> DataType
TYPES = {1: T.INT8, 2: T.INT16, 3: T.INT32, 8: T.INT64, 9: T.INT32, 13: T.INT32, 4: T.FLOAT32, 5: T.FLOAT64,
         10: T.DATE32, 14: T.DATE32, 7: T.TIMESTAMP, 12: T.TIMESTAMP, 15: T.UTF8, 253: T.UTF8, 254: T.UTF8,
         252: T.UTF8, 249: T.UTF8, 250: T.UTF8, 251: T.UTF8, 16: T.INT64, 247: T.UTF8, 248: T.UTF8}


def native_password(password: str, salt: bytes) -> bytes:
    if not password:
        return b""
    s1 = hashlib.sha1(password.encode()).digest()
    s2 = hashlib.sha1(s1).digest()
    s3 = hashlib.sha1(salt + s2).digest()
    return bytes(a ^ b for a, b in zip(s1, s3))


def lenenc_int(b: bytes, p: int) -> Tuple[Optional[int], int]:
    c = b[p]
    if c < 0xFB:
        return c, p + 1
    if c == 0xFB:
        return None, p + 1
    if c == 0xFC:
        return struct.unpack("<H", b[p + 1:p + 3])[0], p + 3
    if c == 0xFD:
        return int.from_bytes(b[p + 1:p + 4], "little"), p + 4
    return struct.unpack("<Q", b[p + 1:p + 9])[0], p + 9


def lenenc_str(b: bytes, p: int) -> Tuple[Optional[bytes], int]:
    n, p = lenenc_int(b, p)
    if n is None:
        return None, p
    return b[p:p + n], p + n


def enc_lenenc_int(n: int) -> bytes:
    if n < 0xFB:
        return bytes([n])
    if n < 1 << 16:
        return b"\xfc" + struct.pack("<H", n)
    if n < 1 << 24:
        return b"\xfd" + n.to_bytes(3, "little")
    return b"\xfe" + struct.pack("<Q", n)


def enc_lenenc_str(s: bytes) -> bytes:
    return enc_lenenc_int(len(s)) + s


class MySqlError(ExecutionError):
    pass


class MySqlConnection:
    def __init__(self, dsn: str, timeout: float = 30.0):
        u = urlparse(dsn)
        if u.scheme != "mysql":
            raise ValueError(f"not a mysql DSN: {dsn}")
        self.user = unquote(u.username or "root")
        self.password = unquote(u.password or "")
        self.database = (u.path or "/").lstrip("/")
        try:
            self.sock = socket.create_connection((u.hostname or "127.0.0.1", u.port or 3306), timeout=timeout)
        except OSError as e:
            raise CommError(f"cannot connect to mysql {u.hostname}:{u.port}: {e}") from e
        self.buf = b""
        self.seq = 0
        self._lock = threading.Lock()
        self._handshake()

    def _recv_exact(self, n: int) -> bytes:
        while len(self.buf) < n:
            c = self.sock.recv(max(65536, n - len(self.buf)))
            if not c:
                raise CommError("mysql connection closed")
            self.buf += c
        out, self.buf = self.buf[:n], self.buf[n:]
        return out

    def _packet(self) -> bytes:
        out = b""
        while True:
            h = self._recv_exact(4)
            n = int.from_bytes(h[:3], "little")
            self.seq = (h[3] + 1) & 0xFF
            out += self._recv_exact(n)
            if n < 0xFFFFFF:
                return out

    def _send(self, payload: bytes):
        self.sock.sendall(len(payload).to_bytes(3, "little") + bytes([self.seq]) + payload)
        self.seq = (self.seq + 1) & 0xFF

    @staticmethod
    def _err(p: bytes) -> str:
        code = struct.unpack("<H", p[1:3])[0]
        msg = p[9:] if len(p) > 9 and p[3:4] == b"#" else p[3:]
        return f"MySQL error {code}: {msg.decode(errors='replace')}"

    def _handshake(self):
        g = self._packet()
        if g[0] == 0xFF:
            raise CommError(self._err(g))
        p = 1
        e = g.index(b"\0", p)
        self.server_version = g[p:e].decode()
        p = e + 1 + 4
        salt = g[p:p + 8]
        p += 9
        caps = struct.unpack("<H", g[p:p + 2])[0]
        p += 2 + 1 + 2
        caps |= struct.unpack("<H", g[p:p + 2])[0] << 16
        p += 2
        alen = g[p]
        p += 1 + 10
        salt += g[p:p + max(13, alen - 8) - 1]
        flags = CLIENT_LONG_PASSWORD | CLIENT_PROTOCOL_41 | CLIENT_SECURE_CONNECTION | CLIENT_PLUGIN_AUTH
        if self.database:
            flags |= CLIENT_CONNECT_WITH_DB
        auth = native_password(self.password, salt[:20])
        resp = struct.pack("<IIB", flags, 1 << 24, 33) + b"\0" * 23 + self.user.encode() + b"\0"
        resp += bytes([len(auth)]) + auth
        if self.database:
            resp += self.database.encode() + b"\0"
        resp += b"mysql_native_password\0"
        self._send(resp)
        r = self._packet()
        if r[0] == 0xFF:
            raise CommError(self._err(r))
        if r[0] == 0xFE:  # auth switch request
            plugin_end = r.index(b"\0", 1)
            salt2 = r[plugin_end + 1:].rstrip(b"\0")
            self._send(native_password(self.password, salt2[:20]))
            r = self._packet()
            if r[0] == 0xFF:
                raise CommError(self._err(r))

    def query(self, sql: str) -> Tuple[List[Tuple[str, int, int]], List[List[Optional[bytes]]]]:
        """COM_QUERY -> (columns [(name, type, decimals)], raw text rows)."""
        with self._lock:
            self.seq = 0
            self._send(b"\x03" + sql.encode())
            first = self._packet()
            if first[0] == 0xFF:
                raise MySqlError(self._err(first))
            if first[0] == 0x00:
                return [], []
            ncols, _ = lenenc_int(first, 0)
            cols = []
            for _ in range(ncols):
                c = self._packet()
                p = 0
                parts = []
                for _k in range(6):
                    s, p = lenenc_str(c, p)
                    parts.append(s)
                p += 1  # length of fixed fields (0x0c)
                _charset, _collen, ctype, _flags, dec = struct.unpack("<HIBHB", c[p:p + 10])
                cols.append((parts[4].decode(), ctype, dec))
            eof = self._packet()  # EOF after column definitions
            rows = []
            while True:
                r = self._packet()
                if r[0] == 0xFE and len(r) < 9:
                    break
                if r[0] == 0xFF:
                    raise MySqlError(self._err(r))
                p = 0
                row = []
                for _ in range(ncols):
                    if r[p] == 0xFB:
                        row.append(None)
                        p += 1
                    else:
                        s, p = lenenc_str(r, p)
                        row.append(s)
                rows.append(row)
            return cols, rows

    def close(self):
        try:
            self.seq = 0
            self._send(b"\x01")
        except OSError:
            pass
        self.sock.close()


def _col_type(ctype: int, dec: int) -> T.DataType:
    if ctype in (0, 246):
        return T.DECIMAL(38, dec)
    return TYPES.get(ctype, T.UTF8)


def _convert(vals: List[Optional[bytes]], t: T.DataType) -> pa.Array:
    s = [None if v is None else v.decode() for v in vals]
    if t.is_integer:
        return pa.array([None if v is None else int(v) for v in s], t.to_arrow())
    if t.is_float:
        return pa.array([None if v is None else float(v) for v in s], t.to_arrow())
    if t.is_decimal:
        return pa.array([None if v is None else Decimal(v) for v in s], pa.decimal128(38, t.scale))
    if t.kind == "date32":
        return pa.array([None if v is None else datetime.date.fromisoformat(v) for v in s], pa.date32())
    if t.kind == "timestamp":
        return pa.array([None if v is None else datetime.datetime.fromisoformat(v) for v in s], pa.timestamp("us"))
    return pa.array(s, pa.large_string())


class MySqlTable(TableSource):
    replicated = True  # see PostgresTable
    cacheable = True   # resident copies live in the engine's cache tier
    cdc_poll_s = 0.0   # the version query runs before every scan

    def __init__(self, dsn: str, table: str, query: Optional[str] = None, version_sql: Optional[str] = None):
        self.dsn = dsn
        self.table = table
        self.base = query or f"SELECT * FROM {table}"
        self.version_sql = version_sql
        self._conn = None
        self._fields = None

    @property
    def version(self):
        """CDC probe (e.g. ``SELECT max(updated_at) FROM t``); None = never changes."""
        if not self.version_sql:
            return None
        _, rows = self.conn().query(self.version_sql)
        return rows[0][0] if rows else None

    def conn(self) -> MySqlConnection:
        if self._conn is None:
            self._conn = MySqlConnection(self.dsn)
        return self._conn

    def schema(self) -> List[Field]:
        if self._fields is None:
            cols, _ = self.conn().query(f"SELECT * FROM ({self.base}) AS q LIMIT 0")
            self._fields = [Field(n, _col_type(t, d), True) for n, t, d in cols]
        return self._fields

    def num_rows(self):
        _, rows = self.conn().query(f"SELECT count(*) FROM ({self.base}) AS q")
        return int(rows[0][0])

    def read(self, columns: Sequence[str]) -> pa.Table:
        fmap = {f.name: f for f in self.schema()}
        cols = ", ".join(f"`{c}`" for c in columns) or "1"
        _, rows = self.conn().query(f"SELECT {cols} FROM ({self.base}) AS q")
        arrays = [_convert([r[i] for r in rows], fmap[c].dtype) for i, c in enumerate(columns)]
        return pa.Table.from_arrays(arrays, names=list(columns))

    def scan(self, columns: Sequence[str], ctx) -> Batch:
        import torch
        device = ctx.device if ctx is not None else torch.device("cpu")
        out = {}
        if columns:
            t = self.read(columns)
            types = {f.name: f.dtype for f in self.schema()}
            for c in columns:
                out[c] = Column.from_arrow(t.column(c), device=device, dtype=types[c])
        n = len(next(iter(out.values()))) if out else self.num_rows()
        return Batch(out, n)
