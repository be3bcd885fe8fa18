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
     batch of columns (<= 4 GiB), then copied to HBM in one non-blocking H2D
     transfer (the next batch's reads overlap the previous batch's decode);
  3. planning: the C++ planner walks the page headers in the pinned buffer and
     emits device page descriptors + snappy jobs; the pages of every column
     of a batch go to ONE launch of each kernel (page -> column spec table),
     so small columns do not leave the GPU idle;
  4. device: ``pq_snappy`` / ``pq_zstd`` (one wave per compressed page, LDS
     history ring; csrc/kernels/zstd.hip decodes ZSTD frames on the GPU),
     ``pq_dict_strings`` (dictionary entry positions), ``pq_decode`` (levels ->
     validity, PLAIN / RLE_DICTIONARY values -> typed columns with the type
     conversion fused), ``pq_str_copy`` (string bytes after an offset scan).
     BYTE_ARRAY columns whose pages are all dictionary-encoded stay dictionary
     columns (codes over the concatenated chunk dictionaries, de-duplicated on
     the device).

The host only reads bytes and parses metadata; pages are decoded on the GPU.
Columns this decoder does not handle (nested, INT96, GZIP/LZ4/BROTLI codecs,
DELTA_BYTE_ARRAY) are reported back, and the caller reads them with the host
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
          9: "truncated page", 20: "not a zstd frame", 21: "zstd frame needs a dictionary",
          22: "malformed zstd stream", 23: "zstd size mismatch", 24: "malformed zstd entropy table"}
#: batches whose positional reads run ahead of the batch being decoded
READ_AHEAD = 2
READ_THREADS = int(os.environ.get("IGLOO_PARQUET_READ_THREADS", str(min(16, os.cpu_count() or 8))))
#: staged bytes per decode batch (pinned host buffer + one set of launches):
#: small enough that the host reads batch i+1 while the GPU copies and
#: decodes batch i, large enough that every launch fills the chip
BATCH_BYTES = int(os.environ.get("IGLOO_PARQUET_BATCH_BYTES", str(256 << 20)))
#: process-wide decode totals (bench.py reports parquet_decode_gbps from them):
#: file bytes staged, decoded column bytes, seconds inside GpuParquetReader.read
#: (positional reads + H2D + planning + device decode, up to the error-flag sync)
#: cold-scan totals: file / output bytes, wall seconds of read(); read_s = positional-read
#: time (read-ahead thread), read_wait_s = time the decode thread waited for a batch's
#: reads, plan_s = host page planning
TOTALS = {"file_bytes": 0, "out_bytes": 0, "seconds": 0.0, "pages": 0, "zstd_pages": 0, "columns": 0,
          "read_s": 0.0, "read_wait_s": 0.0, "plan_s": 0.0}


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
                if c["codec"] not in (0, 1, 6):   # uncompressed, snappy, zstd
                    return f"codec {c['codec']}"
                if c["external"]:
                    return "column chunk in an external file"
        return None

    def read(self, columns: Sequence[Tuple[str, T.DataType]], groups: Sequence[Tuple[int, int]],
             device) -> Tuple[Dict[str, Column], Dict[str, str]]:
        """Decode ``columns`` over row groups ``groups`` ([(file index, rg)]).
        Returns (decoded columns, {column: reason} for those left to the host).

        Columns are staged in batches of at most BATCH_BYTES; every batch is one
        pinned buffer, one H2D copy, one snappy launch and one decode launch
        over the pages of all its columns (the next batch's reads overlap the
        previous batch's device work)."""
        device = torch.device(device)
        N = native()
        out: Dict[str, Column] = {}
        rejected: Dict[str, str] = {}
        err = torch.zeros(1, dtype=torch.int32, device=device)
        # pinned staging buffers are recycled by torch's caching host allocator,
        # which holds a block until the async H2D copy that read it completed
        keep = None
        st = {"read_s": 0.0, "plan_s": 0.0, "bytes": 0, "pages": 0, "batches": 0}
        t0 = time.perf_counter()
        nrows = sum(self.metas[fi].row_groups[rg]["num_rows"] for fi, rg in groups)
        todo = []
        for name, dt in columns:
            why = self.supports(name, dt)
            if why is not None:
                rejected[name] = why
            elif not groups:
                out[name] = _empty_column(dt, device)
            else:
                lay = self._layout(name, dt, groups)
                if isinstance(lay, str):
                    rejected[name] = lay
                else:
                    todo.append(lay)
        batches, batch, size = [], [], 0
        for lay in todo:
            if batch and size + lay["bytes"] > BATCH_BYTES:
                batches.append(batch)
                batch, size = [], 0
            batch.append(lay)
            size += lay["bytes"]
        if batch:
            batches.append(batch)
        # pipeline: the positional reads of the next READ_AHEAD batches run on
        # a host thread into their own pinned buffers while this thread plans,
        # copies and launches the decode of the current one (the device work is
        # asynchronous, so read k+1, H2D + decode k overlap)
        if len(batches) > 1:
            import concurrent.futures as cf
            with cf.ThreadPoolExecutor(max_workers=1, thread_name_prefix="igloo-pq-read") as pool:
                futs = [pool.submit(self._stage, N, b) for b in batches[:READ_AHEAD]]
                for k, b in enumerate(batches):
                    staged = futs[k].result()
                    if k + READ_AHEAD < len(batches):
                        futs.append(pool.submit(self._stage, N, batches[k + READ_AHEAD]))
                    self._read_batch(N, b, nrows, device, err, keep, st, out, rejected, staged)
        elif batches:
            self._read_batch(N, batches[0], nrows, device, err, keep, st, out, rejected)
        if out:
            code = int(err.item())  # one sync for every column of the scan
            if code:
                raise ExecutionError(f"parquet decode failed: {ERRORS.get(code, code)}")
        st["total_s"] = time.perf_counter() - t0
        self.last_stats = st
        TOTALS["file_bytes"] += st["bytes"]
        TOTALS["seconds"] += st["total_s"]
        TOTALS["pages"] += st["pages"]
        TOTALS["zstd_pages"] += st.get("zstd_pages", 0)
        TOTALS["read_s"] += st["read_s"]
        TOTALS["read_wait_s"] += st.get("read_wait_s", 0.0)
        TOTALS["plan_s"] += st["plan_s"]
        TOTALS["columns"] += len(out)
        for c in out.values():
            TOTALS["out_bytes"] += c.data.numel() * c.data.element_size() + (
                c.offsets.numel() * 8 if c.offsets is not None else 0)
        return out, rejected

    # --------------------------------------------------------------- internals
    def _layout(self, name, dt, groups):
        """Chunk byte ranges of one column over ``groups`` (or a reason string)."""
        m0 = self.metas[groups[0][0]]
        leaf0 = m0.leaves[m0.leaf_index[name]]
        conv = conversion(leaf0, dt)
        ranges, total, first_row, may_null = [], 0, 0, False
        for fi, rg in groups:
            m = self.metas[fi]
            leaf = m.leaves[m.leaf_index[name]]
            if leaf["type"] != leaf0["type"] or conversion(leaf, dt) != conv or leaf["max_def"] != leaf0["max_def"]:
                return "files disagree on the column's physical layout"
            g = m.row_groups[rg]
            c = g["chunks"][m.leaf_index[name]]
            ranges.append((fi, c["start"], c["length"], total, c["codec"], first_row, g["num_rows"]))
            if leaf["max_def"] > 0 and (c["null_count"] is None or c["null_count"] > 0):
                may_null = True
            first_row += g["num_rows"]
            total += (c["length"] + 63) // 64 * 64
        return {"name": name, "dt": dt, "leaf": leaf0, "conv": conv, "ranges": ranges, "bytes": total,
                "may_null": may_null}

    def _stage(self, N, batch):
        """Every column chunk of ``batch`` read into one pinned buffer
        (thread-safe: called ahead of the batch on the read thread)."""
        base = 0
        for lay in batch:
            lay["base"] = base
            base += lay["bytes"]
        t0 = time.perf_counter()
        host = torch.empty(base + 64, dtype=torch.uint8, pin_memory=True)
        hp = host.data_ptr()
        per_file: Dict[int, list] = {}
        for lay in batch:
            for fi, start, length, off, *_ in lay["ranges"]:
                per_file.setdefault(fi, []).append((start, length, hp + lay["base"] + off))
        for fi, rs in per_file.items():
            N.pq_pread(self.files[fi], rs, READ_THREADS)
        return host, base, time.perf_counter() - t0

    def _read_batch(self, N, batch, n, device, err, keep, st, out, rejected, staged=None):
        # ---- every column of the batch in one pinned buffer (read ahead on the pipeline thread)
        tw = time.perf_counter()
        host, base, read_s = staged if staged is not None else self._stage(N, batch)
        hp = host.data_ptr()
        st["read_s"] += read_s
        st["read_wait_s"] = st.get("read_wait_s", 0.0) + (time.perf_counter() - tw)
        st["bytes"] += base
        st["batches"] += 1
        raw = torch.empty(base + 64, dtype=torch.uint8, device=device)
        raw.copy_(host, non_blocking=True)
        # ---- plan pages of every column (shared raw / dec buffers)
        t1 = time.perf_counter()
        plans, dec_end = [], 0
        for lay in batch:
            chunks = [(lay["base"] + off, length, codec, first, rows)
                      for _fi, _s, length, off, codec, first, rows in lay["ranges"]]
            leaf = lay["leaf"]
            try:
                plan = N.pq_plan(hp, chunks, leaf["type"], leaf["max_def"], leaf["max_rep"], dec_end,
                                 leaf["type_length"])
            except RuntimeError as e:
                raise IoError(f"corrupt parquet column {lay['name']}: {e}") from e
            if plan["unsupported"]:
                rejected[lay["name"]] = plan["unsupported"]
                continue
            dec_end = plan["dec_bytes"]
            plans.append((lay, plan))
        st["plan_s"] += time.perf_counter() - t1
        if not plans:
            return
        s = stream(raw)
        dec = torch.empty(dec_end + 64, dtype=torch.uint8, device=device) if dec_end else None
        jobs = b"".join(p["jobs"] for _, p in plans)
        njobs = sum(p["num_jobs"] for _, p in plans)
        nzstd = sum(p["num_zstd_jobs"] for _, p in plans)
        if njobs:
            jt = _upload(jobs, device)
            if njobs > nzstd:
                launch("pq_snappy").pq_snappy(ptr(jt), njobs, ptr(raw), ptr(dec), ptr(err), s)
            if nzstd:
                slots = N.pq_zstd_slots(nzstd)
                lit = torch.empty(slots << 17, dtype=torch.uint8, device=device)   # 128 KiB literals per workgroup
                launch("pq_zstd").pq_zstd(ptr(jt), njobs, ptr(raw), ptr(dec), ptr(lit), slots, ptr(err), s)
                st["zstd_pages"] = st.get("zstd_pages", 0) + nzstd
        # ---- outputs + one spec per column
        specs, page_col, pages, posts = [], [], [], []
        scratch = torch.empty(max(n, 1) * len(plans), dtype=torch.int32, device=device)
        for ci, (lay, plan) in enumerate(plans):
            leaf, dt = lay["leaf"], lay["dt"]
            conv, out_w, factor = lay["conv"]
            valid = torch.empty(n, dtype=torch.bool, device=device) if (leaf["max_def"] > 0 and lay["may_null"]) else None
            spec = dict(phys=leaf["type"], type_len=leaf["type_length"], out_width=out_w, conv=CONV[conv],
                        conv_k=factor, max_def=leaf["max_def"], out=0, valid=ptr(valid),
                        scratch=ptr(scratch) + 4 * ci * max(n, 1), str_len=0, str_pos=0, codes=0, dict_len=0,
                        dict_pos=0, raw=ptr(raw), dec=ptr(dec), error=ptr(err))
            post = {"lay": lay, "valid": valid}
            if dt.kind != "utf8":
                data = torch.empty(n, dtype=torch.bool if dt.kind == "bool" else dt.torch_dtype, device=device)
                spec["out"] = ptr(data)
                post["data"] = data
            else:
                E = plan["dict_entries"]
                if E:
                    post["dlen"] = torch.empty(E, dtype=torch.int64, device=device)
                    post["dpos"] = torch.empty(E, dtype=torch.int64, device=device)
                    spec.update(dict_len=ptr(post["dlen"]), dict_pos=ptr(post["dpos"]))
                if E and plan["plain_pages"] == 0:
                    post["codes"] = torch.empty(max(n, 1), dtype=torch.int32, device=device)
                    spec["codes"] = ptr(post["codes"])
                else:
                    post["slen"] = torch.empty(max(n, 1), dtype=torch.int64, device=device)
                    post["spos"] = torch.empty(max(n, 1), dtype=torch.int64, device=device)
                    spec.update(str_len=ptr(post["slen"]), str_pos=ptr(post["spos"]))
            specs.append(N.pq_pack_spec(spec, True))
            pages.append(plan["pages"])
            page_col += [ci] * plan["num_pages"]
            posts.append(post)
            st["pages"] += plan["num_pages"]
        npages = len(page_col)
        pt = _upload(b"".join(pages), device)
        pc = torch.tensor(page_col, dtype=torch.int32).to(device)
        sp = _upload(b"".join(specs), device)
        if any("dlen" in p for p in posts):
            launch("pq_dict_strings").pq_dict_strings(ptr(pt), npages, ptr(pc), ptr(sp), s)
        launch("pq_decode").pq_decode(ptr(pt), npages, ptr(pc), ptr(sp), s)
        # ---- strings: dictionaries / offsets + bytes
        for post in posts:
            lay = post["lay"]
            name, dt, valid = lay["name"], lay["dt"], post["valid"]
            if "data" in post:
                out[name] = Column(dt, post["data"], valid)
            elif "codes" in post:
                dictionary = _gather_strings(post["dpos"], post["dlen"], device, s)
                from ..ops.strings import dict_encode
                enc = dict_encode(dictionary)  # entries repeated across chunk dictionaries -> one code
                codes = enc.data.index_select(0, post["codes"][:n].long()).to(torch.int32)
                out[name] = Column(T.UTF8, codes, valid, dictionary=enc.dictionary)
            else:
                out[name] = _gather_strings(post["spos"][:n], post["slen"][:n], device, s, valid)


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
