"""Flight SQL commands: metadata, prepared statements, updates.

The reference advertises a "Flight SQL endpoint ... faster than ODBC/JDBC"
(reference README.md:41, :60; roadmap.md:19-25) but its service only speaks
raw Flight with the SQL text in the command/ticket (crates/api/src/lib.rs:
81-149). JDBC/ODBC-class Flight SQL clients open a connection with
GetSqlInfo, browse metadata (GetCatalogs / GetDbSchemas / GetTables /
GetTableTypes / key commands) and run prepared statements; this module
implements those commands on the engine's catalog. No Flight SQL library
ships in this environment, so the protobuf messages (arrow/flight/sql/
FlightSql.proto) are decoded by hand (service/protocol.py) and every result
schema is built here following that proto's documentation.

Namespace: one catalog ``igloo`` with one schema ``public`` holding every
registered table (type ``TABLE``) and view (``VIEW``).
"""
from __future__ import annotations

import re
import threading
import time
import uuid
from typing import Dict, List, Optional, Sequence, Tuple

import pyarrow as pa

from . import protocol as P

CATALOG = "igloo"
SCHEMA = "public"

# ----------------------------------------------------------------- SqlInfo
#: SqlInfo ids (FlightSql.proto ``enum SqlInfo``) this server answers
SERVER_NAME, SERVER_VERSION, SERVER_ARROW_VERSION, SERVER_READ_ONLY = 0, 1, 2, 3
SERVER_SQL, SERVER_SUBSTRAIT, SERVER_TRANSACTION, SERVER_CANCEL = 4, 5, 8, 9
SERVER_BULK_INGESTION, SERVER_STATEMENT_TIMEOUT = 10, 100
SQL_DDL_CATALOG, SQL_DDL_SCHEMA, SQL_DDL_TABLE, SQL_IDENTIFIER_CASE = 500, 501, 502, 503
SQL_IDENTIFIER_QUOTE_CHAR, SQL_QUOTED_IDENTIFIER_CASE, SQL_ALL_TABLES_ARE_SELECTABLE = 504, 505, 506
SQL_NULL_ORDERING, SQL_KEYWORDS, SQL_NUMERIC_FUNCTIONS, SQL_STRING_FUNCTIONS = 507, 508, 509, 510
SQL_SYSTEM_FUNCTIONS, SQL_DATETIME_FUNCTIONS = 511, 512
SQL_SUPPORTS_COLUMN_ALIASING, SQL_NULL_PLUS_NULL_IS_NULL = 515, 516

#: dense union of an SqlInfo value (FlightSql.proto CommandGetSqlInfo)
SQL_INFO_VALUE = pa.dense_union([
    pa.field("string_value", pa.utf8()),
    pa.field("bool_value", pa.bool_()),
    pa.field("bigint_value", pa.int64()),
    pa.field("int32_bitmask", pa.int32()),
    pa.field("string_list", pa.list_(pa.utf8())),
    pa.field("int32_to_int32_list_map", pa.map_(pa.int32(), pa.list_(pa.int32()))),
])
SQL_INFO_SCHEMA = pa.schema([pa.field("info_name", pa.uint32(), False), pa.field("value", SQL_INFO_VALUE, False)])
CATALOGS_SCHEMA = pa.schema([pa.field("catalog_name", pa.utf8(), False)])
DB_SCHEMAS_SCHEMA = pa.schema([pa.field("catalog_name", pa.utf8()), pa.field("db_schema_name", pa.utf8(), False)])
TABLE_TYPES_SCHEMA = pa.schema([pa.field("table_type", pa.utf8(), False)])
_TABLES_FIELDS = [pa.field("catalog_name", pa.utf8()), pa.field("db_schema_name", pa.utf8()),
                  pa.field("table_name", pa.utf8(), False), pa.field("table_type", pa.utf8(), False)]
TABLES_SCHEMA = pa.schema(_TABLES_FIELDS)
TABLES_SCHEMA_WITH_SCHEMA = pa.schema(_TABLES_FIELDS + [pa.field("table_schema", pa.binary(), False)])
PRIMARY_KEYS_SCHEMA = pa.schema([pa.field("catalog_name", pa.utf8()), pa.field("db_schema_name", pa.utf8()),
                                 pa.field("table_name", pa.utf8(), False), pa.field("column_name", pa.utf8(), False),
                                 pa.field("key_name", pa.utf8()), pa.field("key_sequence", pa.int32(), False)])
KEYS_SCHEMA = pa.schema([pa.field("pk_catalog_name", pa.utf8()), pa.field("pk_db_schema_name", pa.utf8()),
                         pa.field("pk_table_name", pa.utf8(), False), pa.field("pk_column_name", pa.utf8(), False),
                         pa.field("fk_catalog_name", pa.utf8()), pa.field("fk_db_schema_name", pa.utf8()),
                         pa.field("fk_table_name", pa.utf8(), False), pa.field("fk_column_name", pa.utf8(), False),
                         pa.field("key_sequence", pa.int32(), False), pa.field("fk_key_name", pa.utf8()),
                         pa.field("pk_key_name", pa.utf8()), pa.field("update_rule", pa.uint8(), False),
                         pa.field("delete_rule", pa.uint8(), False)])

KEYWORDS = ["ANALYZE", "EXPLAIN", "EXTERNAL", "ILIKE", "INTERVAL", "LIMIT", "LOCATION", "NULLS", "OFFSET", "SHOW",
            "STORED"]
# generated from the binder's function registry (sql/functions.py), whose every
# entry tests/test_functions.py runs on the CPU and the GPU
from ..sql import functions as _F  # noqa: E402
NUMERIC_FUNCTIONS = sorted(n.upper() for n in list(_F.NUMERIC) + list(_F.AGGREGATE) + list(_F.WINDOW))
STRING_FUNCTIONS = sorted(n.upper() for n in _F.STRING)
SYSTEM_FUNCTIONS = sorted(n.upper() for n in _F.SYSTEM)
DATETIME_FUNCTIONS = sorted(n.upper() for n in _F.DATETIME)


def _sql_info_values(version: str) -> Dict[int, object]:
    return {
        SERVER_NAME: "igloo-amd", SERVER_VERSION: version, SERVER_ARROW_VERSION: pa.__version__,
        SERVER_READ_ONLY: False, SERVER_SQL: True, SERVER_SUBSTRAIT: False,
        SERVER_TRANSACTION: 0,            # SQL_SUPPORTED_TRANSACTION_NONE
        SERVER_CANCEL: False, SERVER_BULK_INGESTION: False, SERVER_STATEMENT_TIMEOUT: 0,
        SQL_DDL_CATALOG: False, SQL_DDL_SCHEMA: False, SQL_DDL_TABLE: True,
        SQL_IDENTIFIER_CASE: 3,           # SQL_CASE_SENSITIVITY_LOWERCASE (unquoted names fold to lower case)
        SQL_IDENTIFIER_QUOTE_CHAR: '"', SQL_QUOTED_IDENTIFIER_CASE: 0,   # UNKNOWN (quoted names keep their case)
        SQL_ALL_TABLES_ARE_SELECTABLE: True,
        SQL_NULL_ORDERING: 0,             # SQL_NULLS_SORTED_HIGH: ASC puts NULLs last (DataFusion's default)
        SQL_KEYWORDS: KEYWORDS, SQL_NUMERIC_FUNCTIONS: NUMERIC_FUNCTIONS, SQL_STRING_FUNCTIONS: STRING_FUNCTIONS,
        SQL_SYSTEM_FUNCTIONS: SYSTEM_FUNCTIONS, SQL_DATETIME_FUNCTIONS: DATETIME_FUNCTIONS,
        SQL_SUPPORTS_COLUMN_ALIASING: True, SQL_NULL_PLUS_NULL_IS_NULL: True,
    }


def sql_info_table(ids: Sequence[int], version: str) -> pa.Table:
    """CommandGetSqlInfo result: one row per requested (known) id, or every
    known id when none is requested."""
    vals = _sql_info_values(version)
    want = [i for i in ids if i in vals] if ids else sorted(vals)
    type_ids, offsets, kids = [], [], [[] for _ in range(6)]
    for i in want:
        v = vals[i]
        if isinstance(v, bool):
            t = 1
        elif isinstance(v, str):
            t = 0
        elif isinstance(v, list):
            t = 4
        elif i in (SERVER_TRANSACTION, SQL_IDENTIFIER_CASE, SQL_QUOTED_IDENTIFIER_CASE, SQL_NULL_ORDERING):
            t = 3
        else:
            t = 2
        type_ids.append(t)
        offsets.append(len(kids[t]))
        kids[t].append(v)
    children = [pa.array(kids[0], pa.utf8()), pa.array(kids[1], pa.bool_()), pa.array(kids[2], pa.int64()),
                pa.array(kids[3], pa.int32()), pa.array(kids[4], pa.list_(pa.utf8())),
                pa.array([], pa.map_(pa.int32(), pa.list_(pa.int32())))]
    value = pa.UnionArray.from_dense(pa.array(type_ids, pa.int8()), pa.array(offsets, pa.int32()), children,
                                     [f.name for f in SQL_INFO_VALUE], list(range(6)))
    return pa.Table.from_arrays([pa.array(want, pa.uint32()), value], schema=SQL_INFO_SCHEMA)


# ---------------------------------------------------------------- patterns
def like_regex(pattern: Optional[str]) -> Optional[re.Pattern]:
    """A Flight SQL filter pattern (SQL LIKE: % any run, _ one char, \\ escapes)."""
    if pattern is None:
        return None
    out, i = [], 0
    while i < len(pattern):
        ch = pattern[i]
        if ch == "\\" and i + 1 < len(pattern):
            out.append(re.escape(pattern[i + 1]))
            i += 2
            continue
        out.append(".*" if ch == "%" else "." if ch == "_" else re.escape(ch))
        i += 1
    return re.compile("^" + "".join(out) + "$", re.S)


def _opt_str(f: Dict[int, list], fno: int) -> Optional[str]:
    v = f.get(fno)
    return v[0].decode() if v else None


# ------------------------------------------------------- prepared statements
def _placeholders(sql: str):
    """The placeholders as ``(offset, length, parameter index)``: ``?`` takes
    the next index in order, ``$n`` (the DataFusion / PostgreSQL spelling)
    names parameter n-1. Only outside string literals, quoted
    identifiers, ``--`` line comments and ``/* */`` block comments -- with
    the SQL tokenizer's quoting rules (csrc/sql/parser.cpp tokenize): a
    '...' literal escapes a quote by doubling it; "..." and `...`
    identifiers end at their first closing quote."""
    i, n, seq = 0, len(sql), 0
    while i < n:
        ch = sql[i]
        if ch == "'":
            j = sql.find(ch, i + 1)
            while j != -1 and j + 1 < n and sql[j + 1] == ch:      # doubled quote inside the literal
                j = sql.find(ch, j + 2)
            i = n if j == -1 else j + 1
        elif ch in ('"', "`"):
            j = sql.find(ch, i + 1)
            i = n if j == -1 else j + 1
        elif ch == "-" and sql.startswith("--", i):
            j = sql.find("\n", i)
            i = n if j == -1 else j + 1
        elif ch == "/" and sql.startswith("/*", i):
            j = sql.find("*/", i + 2)
            i = n if j == -1 else j + 2
        elif ch == "?":
            yield i, 1, seq
            seq += 1
            i += 1
        elif ch == "$" and i + 1 < n and sql[i + 1].isdigit() and (i == 0 or not (sql[i - 1].isalnum() or sql[i - 1] == "_")):
            j = i + 1
            while j < n and sql[j].isdigit():
                j += 1
            yield i, j - i, int(sql[i + 1:j]) - 1
            i = j
        else:
            i += 1


def count_params(sql: str) -> int:
    return max((k + 1 for _, _, k in _placeholders(sql)), default=0)


def _literal(v) -> str:
    """A bound value as a self-delimiting SQL literal: numbers are
    parenthesised (``a-?`` with -5 must not become the comment ``a--5``),
    non-finite floats are spelled as casts."""
    import datetime
    import decimal
    import math
    if v is None:
        return "NULL"
    if isinstance(v, bool):
        return "TRUE" if v else "FALSE"
    if isinstance(v, float) and not math.isfinite(v):
        return "CAST('" + ("NaN" if math.isnan(v) else ("inf" if v > 0 else "-inf")) + "' AS DOUBLE)"
    if isinstance(v, decimal.Decimal) and not v.is_finite():
        raise ValueError(f"cannot bind decimal {v}")
    if isinstance(v, (int, float, decimal.Decimal)):
        return f"({v!r})" if isinstance(v, float) else f"({v})"
    if isinstance(v, datetime.datetime):
        return f"TIMESTAMP '{v.isoformat(sep=' ')}'"
    if isinstance(v, datetime.date):
        return f"DATE '{v.isoformat()}'"
    return "'" + str(v).replace("'", "''") + "'"


def bind_params(sql: str, values: Sequence) -> str:
    """Substitute ``?`` / ``$n`` placeholders with SQL literals of ``values``."""
    pos = list(_placeholders(sql))
    need = max((k + 1 for _, _, k in pos), default=0)
    if need > len(values):
        raise ValueError(f"prepared statement has more parameters than the {len(values)} bound")
    out, last = [], 0
    for p, ln, k in pos:
        if k < 0:
            raise ValueError("placeholder $0: parameters are numbered from $1")
        out.append(sql[last:p])
        out.append(_literal(values[k]))
        last = p + ln
    out.append(sql[last:])
    return "".join(out)


class PreparedStatements:
    """Server-side prepared statements: handle -> (SQL, result schema, bound
    parameter rows)."""

    def __init__(self, ttl_s: float = 3600.0):
        self._lock = threading.Lock()
        self._stmts: Dict[bytes, dict] = {}
        self.ttl_s = ttl_s

    def create(self, sql: str, schema: Optional[pa.Schema]) -> Tuple[bytes, dict]:
        h = uuid.uuid4().hex.encode()
        st = {"sql": sql, "schema": schema, "params": None, "n_params": count_params(sql), "t": time.time()}
        with self._lock:
            now = time.time()
            for k in [k for k, v in self._stmts.items() if now - v["t"] > self.ttl_s]:
                del self._stmts[k]
            self._stmts[h] = st
        return h, st

    def get(self, h: bytes) -> dict:
        with self._lock:
            st = self._stmts.get(bytes(h))
        if st is None:
            raise KeyError(f"unknown prepared statement handle {bytes(h)!r}")
        st["t"] = time.time()
        return st

    def close(self, h: bytes) -> None:
        with self._lock:
            self._stmts.pop(bytes(h), None)

    def bind(self, h: bytes, batch: pa.Table) -> None:
        st = self.get(h)
        st["params"] = batch.to_pylist() if batch.num_rows else []

    def sql_of(self, h: bytes) -> str:
        st = self.get(h)
        if st["n_params"] == 0:
            return st["sql"]
        rows = st["params"]
        if not rows:
            raise ValueError("prepared statement parameters are not bound (DoPut CommandPreparedStatementQuery)")
        return bind_params(st["sql"], list(rows[0].values()))

    def __len__(self):
        return len(self._stmts)


def parameter_schema(n: int) -> pa.Schema:
    return pa.schema([pa.field(f"${i + 1}", pa.null()) for i in range(n)])


def serialize_schema(schema: Optional[pa.Schema]) -> bytes:
    return schema.serialize().to_pybytes() if schema is not None else b""


# ---------------------------------------------------------------- metadata
class Metadata:
    """Catalog metadata commands over an engine's catalog."""

    def __init__(self, engine):
        self.engine = engine

    def _tables(self):
        cat = self.engine.catalog
        out = []
        for name in cat.table_names():
            out.append((name, "TABLE", cat.get_table(name)))
        for name in sorted(getattr(cat, "views", {}) or {}):
            out.append((name, "VIEW", None))
        return out

    def catalogs(self) -> pa.Table:
        return pa.Table.from_pylist([{"catalog_name": CATALOG}], schema=CATALOGS_SCHEMA)

    def db_schemas(self, catalog: Optional[str], pattern: Optional[str]) -> pa.Table:
        rx = like_regex(pattern)
        rows = []
        if catalog in (None, "", CATALOG) and (rx is None or rx.match(SCHEMA)):
            rows.append({"catalog_name": CATALOG, "db_schema_name": SCHEMA})
        return pa.Table.from_pylist(rows, schema=DB_SCHEMAS_SCHEMA)

    def table_types(self) -> pa.Table:
        return pa.Table.from_pylist([{"table_type": t} for t in ("TABLE", "VIEW")], schema=TABLE_TYPES_SCHEMA)

    def tables(self, catalog, schema_pattern, name_pattern, types: List[str], include_schema: bool) -> pa.Table:
        rows = []
        if catalog not in (None, "", CATALOG):
            return pa.Table.from_pylist([], schema=TABLES_SCHEMA_WITH_SCHEMA if include_schema else TABLES_SCHEMA)
        srx, nrx = like_regex(schema_pattern), like_regex(name_pattern)
        if srx is not None and not srx.match(SCHEMA):
            return pa.Table.from_pylist([], schema=TABLES_SCHEMA_WITH_SCHEMA if include_schema else TABLES_SCHEMA)
        for name, kind, src in self._tables():
            if (nrx is not None and not nrx.match(name)) or (types and kind not in types):
                continue
            row = {"catalog_name": CATALOG, "db_schema_name": SCHEMA, "table_name": name, "table_type": kind}
            if include_schema:
                if src is not None:
                    sch = src.arrow_schema()
                else:
                    plan, names = self.engine.logical_plan(f"SELECT * FROM {name}")
                    sch = pa.schema([pa.field(n, c.dtype.to_arrow(), c.nullable) for c, n in zip(plan.schema, names)])
                row["table_schema"] = serialize_schema(sch)
            rows.append(row)
        return pa.Table.from_pylist(rows, schema=TABLES_SCHEMA_WITH_SCHEMA if include_schema else TABLES_SCHEMA)

    @staticmethod
    def primary_keys() -> pa.Table:
        return PRIMARY_KEYS_SCHEMA.empty_table()

    @staticmethod
    def keys() -> pa.Table:
        return KEYS_SCHEMA.empty_table()


#: Flight SQL metadata command -> its result schema (GetSchema / GetFlightInfo)
METADATA_SCHEMAS = {
    "CommandGetSqlInfo": SQL_INFO_SCHEMA, "CommandGetCatalogs": CATALOGS_SCHEMA,
    "CommandGetDbSchemas": DB_SCHEMAS_SCHEMA, "CommandGetTableTypes": TABLE_TYPES_SCHEMA,
    "CommandGetPrimaryKeys": PRIMARY_KEYS_SCHEMA, "CommandGetExportedKeys": KEYS_SCHEMA,
    "CommandGetImportedKeys": KEYS_SCHEMA, "CommandGetCrossReference": KEYS_SCHEMA,
}


def metadata_schema(name: str, f: Dict[int, list]) -> Optional[pa.Schema]:
    if name == "CommandGetTables":
        return TABLES_SCHEMA_WITH_SCHEMA if (f.get(5) or [0])[0] else TABLES_SCHEMA
    return METADATA_SCHEMAS.get(name)


def metadata_result(meta: Metadata, name: str, f: Dict[int, list], version: str) -> pa.Table:
    """Result of a Flight SQL metadata command (its decoded protobuf fields)."""
    if name == "CommandGetSqlInfo":
        return sql_info_table([int(x) for x in _packed_uint32(f.get(1, []))], version)
    if name == "CommandGetCatalogs":
        return meta.catalogs()
    if name == "CommandGetDbSchemas":
        return meta.db_schemas(_opt_str(f, 1), _opt_str(f, 2))
    if name == "CommandGetTableTypes":
        return meta.table_types()
    if name == "CommandGetTables":
        types = [t.decode() for t in f.get(4, [])]
        return meta.tables(_opt_str(f, 1), _opt_str(f, 2), _opt_str(f, 3), types, bool((f.get(5) or [0])[0]))
    if name == "CommandGetPrimaryKeys":
        return meta.primary_keys()
    if name in ("CommandGetExportedKeys", "CommandGetImportedKeys", "CommandGetCrossReference"):
        return meta.keys()
    raise NotImplementedError(f"Flight SQL command {name} is not supported")


def _packed_uint32(vals: list) -> List[int]:
    """repeated uint32: unpacked varints (ints) or one packed run (bytes)."""
    out = []
    for v in vals:
        if isinstance(v, int):
            out.append(v)
        else:
            p = 0
            while p < len(v):
                x, p = P._varint(v, p)
                out.append(x)
    return out


# ------------------------------------------------------- message encoders
def encode_prepared_result(handle: bytes, dataset_schema: Optional[pa.Schema], param_schema: Optional[pa.Schema]
                           ) -> bytes:
    """ActionCreatePreparedStatementResult wrapped in Any."""
    body = P.pb_field(1, handle) + P.pb_field(2, serialize_schema(dataset_schema))
    if param_schema is not None and len(param_schema):
        body += P.pb_field(3, serialize_schema(param_schema))
    return P.pack_any("ActionCreatePreparedStatementResult", body)


def encode_update_result(count: int) -> bytes:
    """DoPutUpdateResult{record_count = 1} (not wrapped: sent as app_metadata)."""
    return P.pb_field(1, count & 0xFFFFFFFFFFFFFFFF)


def prepared_query_command(handle: bytes) -> bytes:
    return P.pack_any("CommandPreparedStatementQuery", P.pb_field(1, handle))
