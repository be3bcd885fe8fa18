"""Iceberg table source.

Parity: reference crates/connectors/iceberg/src/lib.rs — IcebergScanExec treats
a table as "every *.parquet under <table>/data/", erroring when data/ is
missing (:42-76), and ignores metadata/manifests/snapshots.

Here the metadata path is implemented: metadata/version-hint.text ->
vN.metadata.json -> current snapshot -> manifest list (Avro) -> manifests
(Avro) -> live data files (status != DELETED). The snapshot id is exposed for
cache invalidation (CDC / cache tier). When no usable metadata exists the
reference's data-directory listing is the fallback, with the same error for a
missing data/ directory. Data files are read by the Parquet source.
"""
from __future__ import annotations

import glob
import json
import os
from typing import List, Optional, Sequence

from ..catalog import Field, TableSource
from ..columnar import Batch
from ..utils.errors import IoError
from . import avro
from .parquet import ParquetTable


def _local(path: str, table_root: str) -> str:
    p = path[len("file://"):] if path.startswith("file://") else path
    p = p[len("file:"):] if p.startswith("file:") else p
    if os.path.exists(p):
        return p
    # tables copied elsewhere: re-root paths below the table directory
    for marker in ("/metadata/", "/data/"):
        if marker in p:
            cand = os.path.join(table_root, marker.strip("/"), p.split(marker, 1)[1])
            if os.path.exists(cand):
                return cand
    return p


def discover_data_files(table_path: str) -> List[str]:
    """Reference behaviour: recursive *.parquet under <table>/data (error if missing)."""
    data_dir = os.path.join(table_path, "data")
    if not os.path.isdir(data_dir):
        raise IoError(f"Iceberg data directory not found: {data_dir}")
    return sorted(os.path.join(d, f) for d, _, fs in os.walk(data_dir) for f in fs if f.endswith(".parquet"))


def read_metadata(table_path: str) -> Optional[dict]:
    mdir = os.path.join(table_path, "metadata")
    if not os.path.isdir(mdir):
        return None
    hint = os.path.join(mdir, "version-hint.text")
    cands = []
    if os.path.exists(hint):
        v = open(hint).read().strip()
        cands += [os.path.join(mdir, f"v{v}.metadata.json"), os.path.join(mdir, f"{v}.metadata.json")]
        cands += sorted(glob.glob(os.path.join(mdir, f"{int(v):05d}-*.metadata.json"))) if v.isdigit() else []
    cands += sorted(glob.glob(os.path.join(mdir, "*.metadata.json")), key=os.path.getmtime, reverse=True)
    for c in cands:
        if os.path.exists(c):
            with open(c) as f:
                return json.load(f)
    return None


def snapshot_files(table_path: str, meta: dict, snapshot_id: Optional[int] = None) -> Optional[List[str]]:
    sid = snapshot_id if snapshot_id is not None else meta.get("current-snapshot-id")
    if sid is None or sid == -1:
        return []
    snap = next((s for s in meta.get("snapshots", []) if s.get("snapshot-id") == sid), None)
    if snap is None:
        return None
    manifests = []
    if "manifest-list" in snap:
        _, entries = avro.read_ocf(_local(snap["manifest-list"], table_path))
        manifests = [e["manifest_path"] for e in entries]
    else:
        manifests = snap.get("manifests", [])
    files = []
    for m in manifests:
        _, entries = avro.read_ocf(_local(m, table_path))
        for e in entries:
            if e.get("status", 1) == 2:  # DELETED
                continue
            df = e["data_file"]
            if str(df.get("file_format", "PARQUET")).upper() != "PARQUET":
                continue
            files.append(_local(df["file_path"], table_path))
    return files


class IcebergTable(TableSource):
    cacheable = True   # resident copies live in the engine's cache tier, keyed by the snapshot id

    def __init__(self, path: str, snapshot_id: Optional[int] = None):
        self.path = path
        self._pinned = snapshot_id
        self._load(snapshot_id)

    def _load(self, snapshot_id: Optional[int]):
        path = self.path
        self.metadata = None
        files = None
        try:
            self.metadata = read_metadata(path)
        except (OSError, ValueError, json.JSONDecodeError):
            self.metadata = None
        if self.metadata is not None:
            try:
                files = snapshot_files(path, self.metadata, snapshot_id)
            except (OSError, ValueError, KeyError):
                files = None
        if files is None:
            files = discover_data_files(path)
        self.snapshot_id = (self.metadata or {}).get("current-snapshot-id") if snapshot_id is None else snapshot_id
        self.files = files
        self._inner = ParquetTable(path, files=files) if files else None

    def schema(self) -> List[Field]:
        if self._inner is None:
            raise IoError(f"Iceberg table {self.path} has no data files")
        return self._inner.schema()

    def num_rows(self) -> int:
        return self._inner.num_rows() if self._inner else 0

    prunes = True

    def scan(self, columns: Sequence[str], ctx, filters=None) -> Batch:
        if self._inner is None:
            raise IoError(f"Iceberg table {self.path} has no data files")
        return self._inner.scan(columns, ctx, filters=filters)

    @property
    def version(self):
        """CDC probe: the current snapshot id (re-read from the metadata, so a
        commit — new vN.metadata.json + version hint — is seen); without
        metadata the data files' mtimes."""
        if self._pinned is None:
            try:
                cur = read_metadata(self.path).get("current-snapshot-id")
            except (OSError, ValueError, json.JSONDecodeError):
                cur = None
            if cur is not None and cur != self.snapshot_id:
                self._load(None)
        if self.snapshot_id is not None:
            return self.snapshot_id
        return self._inner.version if self._inner is not None else None


# ----------------------------------------------------------------- writing
_MANIFEST_LIST_SCHEMA = {
    "type": "record", "name": "manifest_file", "fields": [
        {"name": "manifest_path", "type": "string"}, {"name": "manifest_length", "type": "long"},
        {"name": "partition_spec_id", "type": "int"}, {"name": "added_snapshot_id", "type": ["null", "long"]}]}
_MANIFEST_SCHEMA = {
    "type": "record", "name": "manifest_entry", "fields": [
        {"name": "status", "type": "int"}, {"name": "snapshot_id", "type": ["null", "long"]},
        {"name": "data_file", "type": {"type": "record", "name": "r2", "fields": [
            {"name": "file_path", "type": "string"}, {"name": "file_format", "type": "string"},
            {"name": "record_count", "type": "long"}, {"name": "file_size_in_bytes", "type": "long"}]}}]}


def write_table(path: str, table, snapshot_id: int = 1, append: bool = False, rows_per_file: int = 1 << 20,
                compression: str = "zstd", **parquet_options):
    """Write an Arrow table as a (v2-style) Iceberg table: parquet data files +
    Avro manifest/manifest list + vN.metadata.json + version-hint.text. Data
    files are ZSTD-compressed by default, like Iceberg's own writer
    (write.parquet.compression-codec)."""
    import pyarrow.parquet as pq
    import uuid
    os.makedirs(os.path.join(path, "data"), exist_ok=True)
    os.makedirs(os.path.join(path, "metadata"), exist_ok=True)
    meta = read_metadata(path) if append else None
    prev = snapshot_files(path, meta) if meta else []
    entries = [{"status": 0, "snapshot_id": snapshot_id,
                "data_file": {"file_path": f, "file_format": "PARQUET", "record_count": 0,
                              "file_size_in_bytes": os.path.getsize(f)}} for f in (prev or [])]
    for i in range(0, max(table.num_rows, 1), rows_per_file):
        f = os.path.join(path, "data", f"{uuid.uuid4().hex}.parquet")
        part = table.slice(i, rows_per_file)
        pq.write_table(part, f, compression=compression, **parquet_options)
        entries.append({"status": 1, "snapshot_id": snapshot_id,
                        "data_file": {"file_path": f, "file_format": "PARQUET", "record_count": part.num_rows,
                                      "file_size_in_bytes": os.path.getsize(f)}})
    mpath = os.path.join(path, "metadata", f"manifest-{snapshot_id}.avro")
    avro.write_ocf(mpath, _MANIFEST_SCHEMA, entries)
    lpath = os.path.join(path, "metadata", f"snap-{snapshot_id}.avro")
    avro.write_ocf(lpath, _MANIFEST_LIST_SCHEMA, [{"manifest_path": mpath, "manifest_length": os.path.getsize(mpath),
                                                  "partition_spec_id": 0, "added_snapshot_id": snapshot_id}])
    snaps = (meta or {}).get("snapshots", []) + [{"snapshot-id": snapshot_id, "manifest-list": lpath,
                                                 "timestamp-ms": 0}]
    version = len(snaps)
    md = {"format-version": 2, "location": path, "current-snapshot-id": snapshot_id, "snapshots": snaps}
    with open(os.path.join(path, "metadata", f"v{version}.metadata.json"), "w") as f:
        json.dump(md, f)
    with open(os.path.join(path, "metadata", "version-hint.text"), "w") as f:
        f.write(str(version))
    return md
