"""In-process fake PostgreSQL (v3 protocol) and MySQL (4.1 protocol) servers.

No database server exists in this environment, so the wire clients are tested
against these: each speaks the server half of the protocol (auth handshakes
included) and answers queries with an igloo CPU engine over Arrow tables.
"""
from __future__ import annotations

import base64
import datetime
import hashlib
import hmac
import os
import socket
import struct
import threading
from decimal import Decimal

import pyarrow as pa

import igloo_amd as ig
from igloo_amd.connectors.mysql import enc_lenenc_int, enc_lenenc_str


def _text(v) -> str:
    if isinstance(v, bool):
        return "t" if v else "f"
    if isinstance(v, (datetime.date, Decimal)):
        return str(v)
    return str(v)


class _Base:
    def __init__(self, tables):
        self.engine = ig.QueryEngine(device="cpu")
        self.tables = dict(tables)
        for k, t in self.tables.items():
            self.engine.register_table(k, t)
        self.sock = socket.socket()
        self.sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self.sock.bind(("127.0.0.1", 0))
        self.sock.listen(16)
        self.port = self.sock.getsockname()[1]
        self.queries = []
        self._stop = False
        threading.Thread(target=self._accept, daemon=True).start()

    def set_table(self, name, t):
        self.tables[name] = t
        self.engine.register_table(name, t)

    def _accept(self):
        while not self._stop:
            try:
                c, _ = self.sock.accept()
            except OSError:
                return
            threading.Thread(target=self._serve_safe, args=(c,), daemon=True).start()

    def _serve_safe(self, c):
        try:
            self._serve(c)
        except (ConnectionError, OSError, EOFError):
            pass
        finally:
            c.close()

    def close(self):
        self._stop = True
        self.sock.close()

    @staticmethod
    def _recv(c, n):
        b = b""
        while len(b) < n:
            x = c.recv(n - len(b))
            if not x:
                raise EOFError
            b += x
        return b

    def run(self, sql):
        self.queries.append(sql)
        return self.engine.query(sql)


class FakePostgres(_Base):
    """auth: "trust" | "md5" | "scram" | "password"."""

    def __init__(self, tables, user="igloo", password="secret", auth="md5"):
        self.user, self.password, self.auth = user, password, auth
        super().__init__(tables)

    @property
    def dsn(self):
        return f"postgres://{self.user}:{self.password}@127.0.0.1:{self.port}/db"

    def _msg(self, c):
        h = self._recv(c, 5)
        n = struct.unpack("!I", h[1:])[0]
        return h[:1], self._recv(c, n - 4)

    @staticmethod
    def _out(c, tag, body=b""):
        c.sendall(tag + struct.pack("!I", len(body) + 4) + body)

    def _fail(self, c, msg, code="28P01"):
        self._out(c, b"E", b"SFATAL\0C" + code.encode() + b"\0M" + msg.encode() + b"\0\0")

    def _serve(self, c):
        n = struct.unpack("!I", self._recv(c, 4))[0]
        body = self._recv(c, n - 4)
        parts = body[4:].split(b"\0")
        params = dict(zip(parts[::2], parts[1::2]))
        user = params.get(b"user", b"").decode()
        if self.auth == "md5":
            salt = os.urandom(4)
            self._out(c, b"R", struct.pack("!I", 5) + salt)
            _, pw = self._msg(c)
            inner = hashlib.md5(self.password.encode() + user.encode()).hexdigest().encode()
            if pw.rstrip(b"\0") != b"md5" + hashlib.md5(inner + salt).hexdigest().encode():
                return self._fail(c, f'password authentication failed for user "{user}"')
        elif self.auth == "password":
            self._out(c, b"R", struct.pack("!I", 3))
            _, pw = self._msg(c)
            if pw.rstrip(b"\0").decode() != self.password:
                return self._fail(c, "password authentication failed")
        elif self.auth == "scram":
            if not self._scram(c):
                return self._fail(c, "SCRAM authentication failed")
        self._out(c, b"R", struct.pack("!I", 0))
        self._out(c, b"S", b"server_version\x0016.0\0")
        self._out(c, b"Z", b"I")
        while True:
            tag, b = self._msg(c)
            if tag == b"X":
                return
            if tag != b"Q":
                continue
            sql = b.rstrip(b"\0").decode()
            try:
                if sql.upper().startswith("COPY ("):
                    assert sql.endswith("TO STDOUT WITH (FORMAT csv)")
                    inner = sql[sql.index("(") + 1:sql.rindex(") TO STDOUT")]
                    t = self.run(inner)
                    self._out(c, b"H", b"\0" + struct.pack("!H", t.num_columns) + b"\0\0" * t.num_columns)
                    cols = [col.to_pylist() for col in t.columns]

                    def csv_field(v):
                        if v is None:
                            return ""
                        s = _text(v)
                        if s == "" or any(ch in s for ch in ',"\n\r'):
                            return '"' + s.replace('"', '""') + '"'
                        return s
                    for i in range(t.num_rows):
                        self._out(c, b"d", (",".join(csv_field(col[i]) for col in cols) + "\n").encode())
                    self._out(c, b"c")
                    self._out(c, b"C", f"COPY {t.num_rows}\0".encode())
                else:
                    t = self.run(sql)
                    self._rowdesc(c, t.schema)
                    cols = [col.to_pylist() for col in t.columns]
                    for i in range(t.num_rows):
                        row = struct.pack("!H", len(cols))
                        for col in cols:
                            v = col[i]
                            if v is None:
                                row += struct.pack("!i", -1)
                            else:
                                e = _text(v).encode()
                                row += struct.pack("!i", len(e)) + e
                        self._out(c, b"D", row)
                    self._out(c, b"C", f"SELECT {t.num_rows}\0".encode())
            except Exception as e:  # noqa: BLE001
                self._out(c, b"E", b"SERROR\0C42P01\0M" + str(e).encode() + b"\0\0")
            self._out(c, b"Z", b"I")

    def _rowdesc(self, c, schema):
        body = struct.pack("!H", len(schema))
        for f in schema:
            t, mod = f.type, -1
            if pa.types.is_boolean(t):
                oid = 16
            elif pa.types.is_int64(t):
                oid = 20
            elif pa.types.is_integer(t):
                oid = 23
            elif pa.types.is_floating(t):
                oid = 701
            elif pa.types.is_decimal(t):
                oid, mod = 1700, ((t.precision << 16) | t.scale) + 4
            elif pa.types.is_date(t):
                oid = 1082
            else:
                oid = 25
            body += f.name.encode() + b"\0" + struct.pack("!IhIhih", 0, 0, oid, -1, mod, 0)
        self._out(c, b"T", body)

    def _scram(self, c) -> bool:
        self._out(c, b"R", struct.pack("!I", 10) + b"SCRAM-SHA-256\0\0")
        _, b = self._msg(c)
        mech_end = b.index(b"\0")
        first = b[mech_end + 5:].decode()
        bare = first[3:]
        cnonce = dict(kv.split("=", 1) for kv in bare.split(","))["r"]
        salt, it = os.urandom(16), 4096
        nonce = cnonce + base64.b64encode(os.urandom(12)).decode()
        sfirst = f"r={nonce},s={base64.b64encode(salt).decode()},i={it}"
        self._out(c, b"R", struct.pack("!I", 11) + sfirst.encode())
        _, fin = self._msg(c)
        fin = fin.decode()
        wo, proof = fin.rsplit(",p=", 1)
        salted = hashlib.pbkdf2_hmac("sha256", self.password.encode(), salt, it)
        ckey = hmac.new(salted, b"Client Key", "sha256").digest()
        stored = hashlib.sha256(ckey).digest()
        auth = f"{bare},{sfirst},{wo}".encode()
        sig = hmac.new(stored, auth, "sha256").digest()
        got = bytes(a ^ b for a, b in zip(base64.b64decode(proof), sig))
        if hashlib.sha256(got).digest() != stored:
            return False
        ssig = hmac.new(hmac.new(salted, b"Server Key", "sha256").digest(), auth, "sha256").digest()
        self._out(c, b"R", struct.pack("!I", 12) + f"v={base64.b64encode(ssig).decode()}".encode())
        return True


class FakeMySql(_Base):
    def __init__(self, tables, user="igloo", password="secret"):
        self.user, self.password = user, password
        super().__init__(tables)

    @property
    def dsn(self):
        return f"mysql://{self.user}:{self.password}@127.0.0.1:{self.port}/db"

    def _pkt(self, c):
        h = self._recv(c, 4)
        return h[3], self._recv(c, int.from_bytes(h[:3], "little"))

    @staticmethod
    def _out(c, seq, payload):
        c.sendall(len(payload).to_bytes(3, "little") + bytes([seq & 0xFF]) + payload)

    def _err(self, c, seq, code, msg):
        self._out(c, seq, b"\xff" + struct.pack("<H", code) + b"#28000" + msg.encode())

    def _serve(self, c):
        salt = bytes(x % 94 + 33 for x in os.urandom(20))
        caps = 0x200 | 0x8000 | 0x80000 | 0x8 | 0x1
        g = b"\x0a" + b"8.0.36-fake\0" + struct.pack("<I", 7) + salt[:8] + b"\0"
        g += struct.pack("<H", caps & 0xFFFF) + bytes([33]) + struct.pack("<H", 2) + struct.pack("<H", caps >> 16)
        g += bytes([21]) + b"\0" * 10 + salt[8:] + b"\0" + b"mysql_native_password\0"
        self._out(c, 0, g)
        seq, r = self._pkt(c)
        p = 4 + 4 + 1 + 23
        e = r.index(b"\0", p)
        user = r[p:e].decode()
        p = e + 1
        alen = r[p]
        token = r[p + 1:p + 1 + alen]
        s1 = hashlib.sha1(self.password.encode()).digest()
        stored = hashlib.sha1(s1).digest()
        ok = user == self.user
        if ok and self.password:
            x = hashlib.sha1(salt + stored).digest()
            cand = bytes(a ^ b for a, b in zip(token, x))
            ok = len(token) == 20 and hashlib.sha1(cand).digest() == stored
        if not ok:
            return self._err(c, seq + 1, 1045, f"Access denied for user '{user}'")
        self._out(c, seq + 1, b"\x00\x00\x00\x02\x00\x00\x00")
        while True:
            seq, r = self._pkt(c)
            if r[:1] == b"\x01":
                return
            if r[:1] != b"\x03":
                continue
            sql = r[1:].decode().replace("`", '"')
            try:
                t = self.run(sql)
            except Exception as e:  # noqa: BLE001
                self._err(c, 1, 1146, str(e))
                continue
            s = 1
            self._out(c, s, enc_lenenc_int(t.num_columns))
            for f in t.schema:
                s += 1
                ty, dec = 253, 0
                if pa.types.is_integer(f.type):
                    ty = 8
                elif pa.types.is_floating(f.type):
                    ty, dec = 5, 31
                elif pa.types.is_decimal(f.type):
                    ty, dec = 246, f.type.scale
                elif pa.types.is_date(f.type):
                    ty = 10
                cd = b"".join(enc_lenenc_str(x) for x in (b"def", b"db", b"q", b"q", f.name.encode(),
                                                           f.name.encode()))
                cd += b"\x0c" + struct.pack("<HIBHB", 33, 255, ty, 0, dec) + b"\0\0"
                self._out(c, s, cd)
            s += 1
            self._out(c, s, b"\xfe\0\0\x02\0")
            cols = [col.to_pylist() for col in t.columns]
            for i in range(t.num_rows):
                s += 1
                row = b"".join(b"\xfb" if col[i] is None else enc_lenenc_str(_text(col[i]).encode()) for col in cols)
                self._out(c, s, row)
            s += 1
            self._out(c, s, b"\xfe\0\0\x02\0")
