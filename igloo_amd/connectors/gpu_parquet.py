"""GPU Parquet reader: native footer/page planning + gfx950 page decode.

Parity: reference crates/engine/src/operators/parquet_scan.rs (ParquetScanExec:
parquet-rs decode of the whole file in 1024-row batches on a blocking thread,
projection by column index) and the DataFusion ListingTable+ParquetFormat path
(crates/engine/tests/integration_test.rs:46-56).

Pipeline per scan:
  1. footer: ``_native.pq_file_meta`` (C++ Thrift compact decoder,
     csrc/io/parquet_meta.cpp) — schema leaves, row groups, chunk offsets;
  2. staging: the projected column chunks of this rank's row groups are read
     with multithreaded ``pread`` straight into one pinned host buffer per
     column, then copied to HBM in one non-blocking H2D transfer (the next
     column's reads overlap the previous column's copy and decode);
  3. planning: the C++ planner walks the page headers in the pinned buffer and
     emits device page descriptors + snappy jobs;
  4. device: ``pq_snappy`` (one wave per compressed page, LDS history ring),
     ``pq_dict_strings`` (dictionary entry positions), ``pq_decode`` (levels ->
     validity, PLAIN / RLE_DICTIONARY values -> typed columns with the type
     conversion fused), ``pq_str_copy`` (string bytes after an offset scan).
     BYTE_ARRAY columns whose pages are all dictionary-encoded stay dictionary
     columns (codes over the concatenated chunk dictionaries, de-duplicated on
     the device).

The host only reads bytes and parses metadata; pages are decoded on the GPU.
Columns this decoder does not handle (nested, INT96, GZIP/ZSTD/LZ4 codecs,
DELTA encodings) are reported back, and the caller reads them with the host
decoder.
"""
from __future__ import annotations

import os
import time
from typing import Dict, Optional, Sequence, Tuple

import torch

from .. import types as T
from ..columnar import Column
from ..ops._lib import launch, native, ptr, stream
from ..ops.select import offsets_from_lengths
from ..utils.errors import ExecutionError, IoError

PHYS = {"BOOLEAN": 0, "INT32": 1, "INT64": 2, "INT96": 3, "FLOAT": 4, "DOUBLE": 5, "BYTE_ARRAY": 6, "FLBA": 7}
CONV = {"copy": 0, "narrow": 1, "sext": 2, "zext": 3, "f2d": 4, "flba": 5, "mul": 6, "div": 7, "bool": 8}
ERRORS = {1: "malformed RLE/bit-packed stream", 2: "dictionary index out of range", 3: "malformed BYTE_ARRAY values",
          4: "malformed snappy stream", 5: "snappy size mismatch", 6: "decimal value exceeds 64-bit fixed point",
          7: "unsupported page encoding", 8: "NULL in a column whose statistics say it has none",
          9: "truncated page"}
READ_THREADS = int(os.environ.get("IGLOO_PARQUET_READ_THREADS", "8"))


class FileMeta:
    """Native footer of one Parquet file."""

    def __init__(self, path: str):
        self.path = path
        if not os.path.exists(path):
            raise IoError(f"path does not exist: {path}")
        try:
            m = native().pq_file_meta(path)
        except RuntimeError as e:
            raise IoError(f"cannot read parquet footer of {path}: {e}") from e
        self.num_rows = m["num_rows"]
        self.leaves = m["leaves"]
        self.row_groups = m["row_groups"]
        self.leaf_index = {l["name"]: i for i, l in enumerate(self.leaves)}


def conversion(leaf: dict, dt: T.DataType) -> Optional[Tuple[str, int, int]]:
    """(conversion, output bytes, factor) turning the leaf's physical values into
    the engine's representation of ``dt``; None = not handled on the device."""
    phys, logical = leaf["type"], leaf["logical"]
    k = dt.kind
    if leaf["max_rep"] > 0 or leaf["max_def"] > 1 or phys == PHYS["INT96"]:
        return None
    if k == "bool":
        return ("bool", 1, 1) if phys == PHYS["BOOLEAN"] else None
    if k in ("int8", "int16"):
        return ("narrow", 1 if k == "int8" else 2, 1) if phys == PHYS["INT32"] else None
    if k in ("int32", "date32"):
        return ("copy", 4, 1) if phys == PHYS["INT32"] and not logical.startswith("uint32") else None
    if k == "int64":
        if phys == PHYS["INT64"]:
            return ("copy", 8, 1) if not logical.startswith("uint64") else None
        if phys == PHYS["INT32"]:
            return ("zext" if logical.startswith("uint") else "sext", 8, 1)
        return None
    if k == "float32":
        return ("copy", 4, 1) if phys == PHYS["FLOAT"] else None
    if k == "float64":
        if phys == PHYS["DOUBLE"]:
            return ("copy", 8, 1)
        if phys == PHYS["FLOAT"]:
            return ("f2d", 8, 1)
        return None
    if k == "timestamp":
        if phys != PHYS["INT64"]:
            return None
        unit = logical.rsplit("_", 1)[-1] if logical.startswith("timestamp") else "us"
        return {"ms": ("mul", 8, 1000), "us": ("copy", 8, 1), "ns": ("div", 8, 1000)}.get(unit)
    if k == "decimal":
        if logical != "decimal" or leaf["scale"] != dt.scale:
            return None
        if phys == PHYS["INT32"]:
            return ("sext", 8, 1)
        if phys == PHYS["INT64"]:
            return ("copy", 8, 1)
        if phys == PHYS["FLBA"] and 1 <= leaf["type_length"] <= 16:
            return ("flba", 8, 1)
        return None
    if k == "utf8":
        return ("copy", 0, 1) if phys == PHYS["BYTE_ARRAY"] else None
    return None


class GpuParquetReader:
    """Decodes projected columns of a set of Parquet files on one GPU."""

    def __init__(self, files: Sequence[str], metas: Optional[Sequence[FileMeta]] = None):
        self.files = list(files)
        self.metas = list(metas) if metas is not None else [FileMeta(f) for f in self.files]
        self.last_stats: Dict[str, float] = {}

    def supports(self, name: str, dt: T.DataType) -> Optional[str]:
        """None when ``name`` decodes on the GPU, else the reason it does not."""
        for m in self.metas:
            li = m.leaf_index.get(name)
            if li is None:
                return f"column {name} missing in {m.path}"
            leaf = m.leaves[li]
            if conversion(leaf, dt) is None:
                return f"type {dt} from physical type {leaf['type']} ({leaf['logical'] or 'plain'})"
            for g in m.row_groups:
                c = g["chunks"][li]
                if c["codec"] not in (0, 1):
                    return f"codec {c['codec']}"
                if c["external"]:
                    return "column chunk in an external file"
        return None

    def read(self, columns: Sequence[Tuple[str, T.DataType]], groups: Sequence[Tuple[int, int]],
             device) -> Tuple[Dict[str, Column], Dict[str, str]]:
        """Decode ``columns`` over row groups ``groups`` ([(file index, rg)]).
        Returns (decoded columns, {column: reason} for those left to the host)."""
        device = torch.device(device)
        N = native()
        out: Dict[str, Column] = {}
        rejected: Dict[str, str] = {}
        err = torch.zeros(1, dtype=torch.int32, device=device)
        keep = []  # pinned staging buffers must outlive their async H2D copies
        st = {"read_s": 0.0, "plan_s": 0.0, "bytes": 0, "pages": 0}
        t0 = time.perf_counter()
        nrows = sum(self.metas[fi].row_groups[rg]["num_rows"] for fi, rg in groups)
        for name, dt in columns:
            why = self.supports(name, dt)
            if why is not None:
                rejected[name] = why
                continue
            col = self._read_column(N, name, dt, groups, nrows, device, err, keep, st)
            if isinstance(col, str):
                rejected[name] = col
            else:
                out[name] = col
        if out:
            code = int(err.item())  # one sync for every column of the scan
            if code:
                raise ExecutionError(f"parquet decode failed: {ERRORS.get(code, code)}")
        st["total_s"] = time.perf_counter() - t0
        self.last_stats = st
        return out, rejected

    # --------------------------------------------------------------- internals
    def _read_column(self, N, name, dt, groups, nrows, device, err, keep, st):
        if not groups:
            return _empty_column(dt, device)
        m0 = self.metas[groups[0][0]]
        leaf0 = m0.leaves[m0.leaf_index[name]]
        conv, out_w, factor = conversion(leaf0, dt)
        chunks, per_file, total, first_row, may_null = [], {}, 0, 0, False
        for fi, rg in groups:
            m = self.metas[fi]
            li = m.leaf_index[name]
            leaf = m.leaves[li]
            if leaf["type"] != leaf0["type"] or conversion(leaf, dt) != (conv, out_w, factor) \
                    or leaf["max_def"] != leaf0["max_def"]:
                return "files disagree on the column's physical layout"
            g = m.row_groups[rg]
            c = g["chunks"][li]
            per_file.setdefault(fi, []).append((c["start"], c["length"], total))
            chunks.append((total, c["length"], c["codec"], first_row, g["num_rows"]))
            if leaf["max_def"] > 0 and (c["null_count"] is None or c["null_count"] > 0):
                may_null = True
            first_row += g["num_rows"]
            total += (c["length"] + 63) // 64 * 64
        t0 = time.perf_counter()
        host = torch.empty(total + 64, dtype=torch.uint8, pin_memory=True)
        hp = host.data_ptr()
        for fi, rs in per_file.items():
            N.pq_pread(self.files[fi], [(s, n, hp + off) for s, n, off in rs], READ_THREADS)
        st["read_s"] += time.perf_counter() - t0
        st["bytes"] += total
        raw = torch.empty(total + 64, dtype=torch.uint8, device=device)
        raw.copy_(host, non_blocking=True)
        keep.append(host)
        t1 = time.perf_counter()
        try:
            plan = N.pq_plan(hp, chunks, leaf0["type"], leaf0["max_def"], leaf0["max_rep"])
        except RuntimeError as e:
            raise IoError(f"corrupt parquet column {name}: {e}") from e
        st["plan_s"] += time.perf_counter() - t1
        if plan["unsupported"]:
            return plan["unsupported"]
        st["pages"] += plan["num_pages"]
        pages = _upload(plan["pages"], device)
        dec = torch.empty(plan["dec_bytes"] + 64, dtype=torch.uint8, device=device) if plan["dec_bytes"] else None
        s = stream(raw)
        if plan["num_jobs"]:
            jobs = _upload(plan["jobs"], device)
            launch("pq_snappy").pq_snappy(ptr(jobs), plan["num_jobs"], ptr(raw), ptr(dec), ptr(err), s)
        n = nrows
        valid = torch.empty(n, dtype=torch.bool, device=device) if (leaf0["max_def"] > 0 and may_null) else None
        scratch = torch.empty(max(n, 1), dtype=torch.int32, device=device)
        spec = dict(phys=leaf0["type"], type_len=leaf0["type_length"], out_width=out_w, conv=CONV[conv],
                    conv_k=factor, max_def=leaf0["max_def"], out=0, valid=ptr(valid), scratch=ptr(scratch),
                    str_len=0, str_pos=0, codes=0, dict_len=0, dict_pos=0, raw=ptr(raw), dec=ptr(dec),
                    error=ptr(err))
        if dt.kind != "utf8":
            tdt = torch.bool if dt.kind == "bool" else dt.torch_dtype
            data = torch.empty(n, dtype=tdt, device=device)
            spec["out"] = ptr(data)
            launch("pq_decode").pq_decode(ptr(pages), plan["num_pages"], spec, s)
            return Column(dt, data, valid)
        # ---- strings
        E = plan["dict_entries"]
        dlen = dpos = None
        if E:
            dlen = torch.empty(E, dtype=torch.int64, device=device)
            dpos = torch.empty(E, dtype=torch.int64, device=device)
            spec.update(dict_len=ptr(dlen), dict_pos=ptr(dpos))
            launch("pq_dict_strings").pq_dict_strings(ptr(pages), plan["num_pages"], spec, s)
        if E and plan["plain_pages"] == 0:
            codes = torch.empty(max(n, 1), dtype=torch.int32, device=device)
            spec["codes"] = ptr(codes)
            launch("pq_decode").pq_decode(ptr(pages), plan["num_pages"], spec, s)
            dictionary = _gather_strings(dpos, dlen, device, s)
            from ..ops.strings import dict_encode
            enc = dict_encode(dictionary)  # entries repeated across chunk dictionaries -> one code
            codes = enc.data.index_select(0, codes[:n].long()).to(torch.int32)
            return Column(T.UTF8, codes, valid, dictionary=enc.dictionary)
        slen = torch.empty(max(n, 1), dtype=torch.int64, device=device)
        spos = torch.empty(max(n, 1), dtype=torch.int64, device=device)
        spec.update(str_len=ptr(slen), str_pos=ptr(spos))
        launch("pq_decode").pq_decode(ptr(pages), plan["num_pages"], spec, s)
        return _gather_strings(spos[:n], slen[:n], device, s, valid)


def _upload(b: bytes, device) -> torch.Tensor:
    if not b:
        return torch.empty(0, dtype=torch.uint8, device=device)
    return torch.frombuffer(bytearray(b), dtype=torch.uint8).to(device)


def _gather_strings(pos: torch.Tensor, lens: torch.Tensor, device, s, valid=None) -> Column:
    off, total = offsets_from_lengths(lens)
    chars = torch.empty(total, dtype=torch.uint8, device=device)
    if total:
        launch("pq_str_copy").pq_str_copy(ptr(pos), ptr(off), lens.numel(), ptr(chars), s)
    return Column(T.UTF8, chars, valid, offsets=off)


def _empty_column(dt: T.DataType, device) -> Column:
    if dt.is_string:
        return Column(dt, torch.zeros(0, dtype=torch.uint8, device=device), None,
                      offsets=torch.zeros(1, dtype=torch.int64, device=device))
    return Column(dt, torch.zeros(0, dtype=torch.bool if dt.kind == "bool" else dt.torch_dtype, device=device))
