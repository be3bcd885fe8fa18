"""DataFusion SQL surface added in round 6 (VERDICT r5 "What's missing" 1-4),
each case on the CPU engine and (gpu marker) on the device:

* nested types: Arrow List / Struct columns, make_array / ``[..]`` literals,
  array_length / cardinality, ``l[i]``, unnest (SELECT and FROM), array_agg
  (ordered, DISTINCT, FILTER), struct / named_struct / get_field,
  array_has, array_to_string, regexp_match -- oracle: Python over the input;
* regex: regexp_like / ``~ ~* !~ !~*`` / SIMILAR TO -- oracle: Python ``re``
  (``$`` as ``\\Z``: Rust regex has no trailing-newline rule);
* md5 / sha224..sha512 / digest -- hashlib; to_char -- datetime.strftime;
  uuid -- ``uuid.UUID`` parses it, version 4;
* bit_and / bit_or / bit_xor, percentile_cont / percentile_disc WITHIN GROUP
  -- Python / numpy;
* DISTINCT ON -- sqlite with row_number(); generate_series / range -- range();
* COPY ... TO (Parquet / CSV / JSON / Arrow) read back with pyarrow, PREPARE /
  EXECUTE with $n, STORED AS JSON (NDJSON; GPU kernels json.hip) -- json module.

DataFusion's exact output types / formatting (e.g. Binary digests, UInt64
lengths) are parity unpinned: values are compared, not Arrow types."""
import hashlib
import json
import os
import random
import re
import sqlite3
import uuid

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import pytest

import igloo_amd as ig
from igloo_amd.ops._lib import KERNEL_CALLS

random.seed(11)
N = 400
WORDS = ["apple", "banana", "cherry", "Date", "elder-berry", "fig9", "grape_12", "Hello World", "", "naïve café"]
ROWS = [dict(id=i, g=random.choice([1, 2, 3, None]), x=random.choice([None] + list(range(-40, 200))),
             s=random.choice(WORDS + [None]), f=round(random.uniform(-5, 5), 3),
             d=random.randint(-400, 20000), ts=random.randint(-10**12, 2 * 10**15)) for i in range(N)]
LISTS = [None if i % 9 == 0 else [random.choice([None, random.randint(0, 50)]) for _ in range(random.randint(0, 5))]
         for i in range(N)]


def _table():
    return pa.table({
        "id": pa.array([r["id"] for r in ROWS], pa.int64()),
        "g": pa.array([r["g"] for r in ROWS], pa.int64()),
        "x": pa.array([r["x"] for r in ROWS], pa.int64()),
        "s": pa.array([r["s"] for r in ROWS], pa.string()),
        "f": pa.array([r["f"] for r in ROWS], pa.float64()),
        "d": pa.array([r["d"] for r in ROWS], pa.int32()).cast(pa.date32()),
        "ts": pa.array([r["ts"] for r in ROWS], pa.timestamp("us")),
        "l": pa.array(LISTS, pa.list_(pa.int64())),
    })


_ENG = {}


def eng(dev):
    if dev not in _ENG:
        e = ig.QueryEngine(device=dev)
        e.register_table("t", _table())
        _ENG[dev] = e
    return _ENG[dev]


def q(dev, sql):
    return eng(dev).sql(sql).table.to_pylist()


def _devices():
    return ["cpu", pytest.param("cuda:0", marks=pytest.mark.gpu)]


@pytest.fixture(params=_devices())
def dev(request):
    if request.param != "cpu":
        import torch
        if not torch.cuda.is_available():
            pytest.skip("no GPU")
    return request.param


# ------------------------------------------------------------------ nested
def test_list_literals_and_functions(dev):
    r = q(dev, "select [1, 2, 3] a, make_array(1, null, 3) b, array_length([1, 2]) c, [1, 2, 3][2] e, "
               "[1, 2, 3][-1] f, [[1, 2], [3]] n, cardinality(make_array()) z")
    assert r == [{"a": [1, 2, 3], "b": [1, None, 3], "c": 2, "e": 2, "f": 3, "n": [[1, 2], [3]], "z": 0}]
    before = KERNEL_CALLS["list_element_idx"] + KERNEL_CALLS["interleave_idx"]
    r = q(dev, "select id, make_array(id, x) m, array_length(l) n, l[1] a, l[-1] b, l[id % 3 + 1] c, "
               "array_has(l, 7) h from t order by id")
    for row, src, lst in zip(r, ROWS, LISTS):
        assert row["m"] == [src["id"], src["x"]]
        assert row["n"] == (None if lst is None else len(lst))
        assert row["a"] == (lst[0] if lst else None)
        assert row["b"] == (lst[-1] if lst else None)
        k = src["id"] % 3
        assert row["c"] == (lst[k] if lst and k < len(lst) else None)
        assert row["h"] == (None if lst is None else 7 in lst)
    if dev != "cpu":
        assert KERNEL_CALLS["list_element_idx"] + KERNEL_CALLS["interleave_idx"] > before


def test_list_columns_through_operators(dev):
    r = q(dev, "select id, l from t where x > 100 order by id desc limit 20")
    want = sorted([(s["id"], lst) for s, lst in zip(ROWS, LISTS) if s["x"] is not None and s["x"] > 100],
                  reverse=True)[:20]
    assert [(a["id"], a["l"]) for a in r] == want
    r = q(dev, "select a.id, b.l from t a join t b on a.id = b.id + 1 where a.g = 2 order by a.id")
    want = [(s["id"], LISTS[s["id"] - 1]) for s in ROWS if s["g"] == 2 and s["id"] >= 1]
    assert [(a["id"], a["l"]) for a in r] == want
    r = q(dev, "select l from t where id < 3 union all select [100, 200]")
    assert sorted(map(repr, (a["l"] for a in r))) == sorted(map(repr, LISTS[:3] + [[100, 200]]))


def test_unnest(dev):
    r = q(dev, "select id, unnest(l) as u from t order by id, u nulls last")
    want = []
    for s, lst in zip(ROWS, LISTS):
        for v in sorted(lst or [], key=lambda v: (v is None, v or 0)):
            want.append((s["id"], v))
    assert [(a["id"], a["u"]) for a in r] == want
    assert q(dev, "select * from unnest([4, 5, 6]) as u(v) where v > 4") == [{"v": 5}, {"v": 6}]
    assert [a["u"] for a in q(dev, "select unnest(make_array(3, 1, 2)) u")] == [3, 1, 2]


def test_array_agg(dev):
    r = q(dev, "select g, array_agg(x order by id) a, array_agg(distinct g) dg, array_agg(id) filter (where x > 150) f "
               "from t group by g order by g nulls last")
    groups = {}
    for s in ROWS:
        groups.setdefault(s["g"], []).append(s)
    for row in r:
        rs = groups[row["g"]]
        assert row["a"] == [s["x"] for s in sorted(rs, key=lambda s: s["id"])]
        assert row["dg"] == [row["g"]]
        fv = sorted(s["id"] for s in rs if s["x"] is not None and s["x"] > 150)
        assert (sorted(row["f"]) if row["f"] is not None else None) == (fv or None)
    r = q(dev, "select array_length(array_agg(s order by s desc)) n, array_agg(s order by s desc)[1] top from t")
    ss = [s["s"] for s in ROWS]
    assert r[0]["n"] == len(ss)
    assert r[0]["top"] is None      # DESC puts NULLs first


def test_struct(dev):
    r = q(dev, "select id, struct(id, s) st, named_struct('a', x, 'b', s)['b'] nb, get_field(named_struct('k', id), 'k') k "
               "from t order by id limit 30")
    for row, src in zip(r, ROWS):
        assert row["st"] == {"c0": src["id"], "c1": src["s"]}
        assert row["nb"] == src["s"] and row["k"] == src["id"]


def test_array_to_string_and_regexp_match(dev):
    r = q(dev, "select id, array_to_string(l, '-') j, regexp_match(s, '([a-z]+)([0-9]*)') m from t order by id")
    rx = re.compile("([a-z]+)([0-9]*)")
    for row, src, lst in zip(r, ROWS, LISTS):
        assert row["j"] == (None if lst is None else "-".join(str(v) for v in lst if v is not None))
        m = rx.search(src["s"]) if src["s"] is not None else None
        assert row["m"] == (None if m is None else list(m.groups()))


def test_arrow_typeof_nested(dev):
    r = q(dev, "select arrow_typeof(make_array(1, 2)) a, arrow_typeof(struct(1, 'x')) b")[0]
    assert r["a"].startswith("List(Field") and "Int64" in r["a"]
    assert r["b"] == "Struct(c0 Int64, c1 Utf8)"


# ------------------------------------------------------------------ regex
REGEX = [("^[a-c]", ""), ("an+a", ""), ("\\d+$", ""), ("^[A-Z]", "i"), ("e.*r", ""), ("(ap|ch)", ""),
         ("^.{5}$", ""), ("[^a-z]", ""), ("l{2}", ""), ("café", "")]


@pytest.mark.parametrize("pi", range(len(REGEX)))
def test_regex_match(dev, pi):
    pat, fl = REGEX[pi]
    rx = re.compile(pat.replace("$", "\\Z"), re.I if fl else 0)
    before = KERNEL_CALLS["regex_dfa"]
    op = "~*" if fl else "~"
    r = q(dev, f"select id, s {op} '{pat}' m, s !{op} '{pat}' nm, regexp_like(s, '{pat}', '{fl}') f from t order by id")
    for row, src in zip(r, ROWS):
        want = None if src["s"] is None else rx.search(src["s"]) is not None
        assert row["m"] == want and row["f"] == want, (pat, src["s"])
        assert row["nm"] == (None if want is None else not want)
    if dev != "cpu":
        assert KERNEL_CALLS["regex_dfa"] > before, "the GPU regex kernel did not run"


def test_similar_to(dev):
    r = q(dev, "select id, s similar to '(a|b)%' a, s similar to '%[0-9]' b, s not similar to '_____' c from t order by id")
    for row, src in zip(r, ROWS):
        v = src["s"]
        if v is None:
            assert row == {"id": src["id"], "a": None, "b": None, "c": None}
            continue
        assert row["a"] == bool(re.fullmatch("(a|b).*", v, re.S))
        assert row["b"] == bool(re.fullmatch(".*[0-9]", v, re.S))
        assert row["c"] == (not re.fullmatch(".....", v, re.S))


def test_dfa_compiler_matches_python_re():
    from igloo_amd.ops.regex_dfa import Unsupported, compile_dfa
    pats = ["abc", "^abc", "abc$", "^a.*c$", "a|b", "(ab)+c", "x{2,3}y", "[a-c]+\\d", "[^abc]z", "\\w+@\\w+\\.com",
            "colou?r", "(?:ab|cd){2}", "a.b", "\\s+", "^[A-Z][a-z]*$", "é+", "[\\d.]+", "\\D\\D", "^(a|b)*$"]
    rnd = random.Random(3)
    for p in pats:
        for icase in (False, True):
            d = compile_dfa(p, icase)
            rx = re.compile(p.replace("$", "\\Z"), re.I if icase else 0)
            for _ in range(300):
                s = "".join(rnd.choice("abcxyzABC019-.@ é_") for _ in range(rnd.randint(0, 10)))
                assert d.match(s.encode()) == (rx.search(s) is not None), (p, icase, s)
    for p in ["(?=a)", "\\1", "\\bword", "a^b"]:
        with pytest.raises(Unsupported):
            compile_dfa(p)


# ------------------------------------------------------------------ digests / formatting
def test_digests(dev):
    before = KERNEL_CALLS["digest_hex"]
    r = q(dev, "select id, md5(s) a, sha224(s) b, sha256(s) c, sha384(s) d, sha512(s) e, digest(s, 'sha256') f "
               "from t order by id")
    for row, src in zip(r, ROWS):
        v = src["s"]
        for k, algo in zip("abcde", ("md5", "sha224", "sha256", "sha384", "sha512")):
            assert row[k] == (None if v is None else hashlib.new(algo, v.encode()).hexdigest()), (algo, v)
        assert row["f"] == row["c"]
    long = "x" * 1000
    assert q(dev, f"select sha512(s || '{long}') h from t where id = 1")[0]["h"] == (
        None if ROWS[1]["s"] is None else hashlib.sha512((ROWS[1]["s"] + long).encode()).hexdigest())
    if dev != "cpu":
        assert KERNEL_CALLS["digest_hex"] > before


def test_to_char(dev):
    import datetime
    r = q(dev, "select id, to_char(d, '%Y-%m-%d %a %j') a, to_char(ts, '%F %T%.3f %p %A %B %e') b from t order by id")
    for row, src in zip(r, ROWS):
        day = datetime.date(1970, 1, 1) + datetime.timedelta(days=src["d"])
        assert row["a"] == f"{day:%Y-%m-%d} {day:%a} {day.timetuple().tm_yday:03d}"
        t = datetime.datetime(1970, 1, 1) + datetime.timedelta(microseconds=src["ts"])
        want = f"{t:%Y-%m-%d %H:%M:%S}.{t.microsecond // 1000:03d} {'AM' if t.hour < 12 else 'PM'} {t:%A %B} {t.day:2d}"
        assert row["b"] == want


def test_uuid(dev):
    r = q(dev, "select uuid() u from t limit 50")
    us = [uuid.UUID(x["u"]) for x in r]
    assert all(u.version == 4 for u in us) and len(set(us)) == len(us)


# ------------------------------------------------------------------ aggregates
def test_bit_aggregates(dev):
    r = q(dev, "select g, bit_and(x) a, bit_or(x) o, bit_xor(x) x from t group by g order by g nulls last")
    for row in r:
        vals = [s["x"] for s in ROWS if s["g"] == row["g"] and s["x"] is not None]
        a, o, x = -1, 0, 0
        for v in vals:
            a &= v
            o |= v
            x ^= v
        assert (row["a"], row["o"], row["x"]) == ((a, o, x) if vals else (None, None, None))


def test_percentiles(dev):
    r = q(dev, "select g, percentile_cont(0.3) within group (order by f) p, percentile_cont(0.3) within group "
               "(order by f desc) pd, percentile_disc(0.5) within group (order by x) m from t group by g order by g nulls last")
    for row in r:
        fs = np.array(sorted(s["f"] for s in ROWS if s["g"] == row["g"]))
        assert abs(row["p"] - np.quantile(fs, 0.3)) < 1e-9
        assert abs(row["pd"] - np.quantile(fs, 0.7)) < 1e-9
        xs = sorted(s["x"] for s in ROWS if s["g"] == row["g"] and s["x"] is not None)
        assert row["m"] == xs[int(np.ceil(len(xs) * 0.5)) - 1]


# ------------------------------------------------------------------ statements
def test_distinct_on(dev):
    con = sqlite3.connect(":memory:")
    con.execute("create table t(id int, g int, x int)")
    con.executemany("insert into t values (?,?,?)", [(s["id"], s["g"], s["x"]) for s in ROWS])
    want = con.execute("select g, x, id from (select *, row_number() over (partition by g order by x desc nulls last, id) "
                       "rn from t) where rn = 1 order by g nulls last").fetchall()
    r = q(dev, "select distinct on (g) g, x, id from t order by g nulls last, x desc nulls last, id")
    assert [(a["g"], a["x"], a["id"]) for a in r] == want


def test_table_functions(dev):
    assert [a["value"] for a in q(dev, "select * from generate_series(1, 5)")] == [1, 2, 3, 4, 5]
    assert [a["value"] for a in q(dev, "select * from generate_series(10, 1, -3)")] == [10, 7, 4, 1]
    assert [a["v"] for a in q(dev, "select value * 2 as v from range(0, 10, 3)")] == [0, 6, 12, 18]
    assert q(dev, "select count(*) c, sum(value) s from range(1000000)") == [{"c": 1000000, "s": 499999500000}]
    r = q(dev, "select t.id from t join generate_series(1, 3) g(k) on t.id = g.k order by 1")
    assert [a["id"] for a in r] == [1, 2, 3]


def test_prepare_execute(dev):
    e = eng(dev)
    e.sql("prepare p1(int, varchar) as select count(*) c from t where g = $1 or s = $2")
    for gv, sv in ((1, "apple"), (3, "fig9")):
        want = sum(1 for s in ROWS if s["g"] == gv or s["s"] == sv)
        assert e.sql(f"execute p1({gv}, '{sv}')").table.to_pylist() == [{"c": want}]
    e.sql("deallocate p1")
    with pytest.raises(Exception):
        e.sql("execute p1(1, 'x')")


def test_copy_to_and_json_source(dev, tmp_path):
    e = eng(dev)
    for fmt in ("parquet", "csv", "json", "arrow"):
        path = str(tmp_path / f"out.{fmt}")
        assert e.sql(f"copy (select id, g, s from t where id < 50) to '{path}'").table.to_pylist() == [{"count": 50}]
        if fmt == "parquet":
            back = pq.read_table(path)
        elif fmt == "csv":
            import pyarrow.csv as pc
            back = pc.read_csv(path)
        elif fmt == "arrow":
            back = pa.ipc.open_file(path).read_all()
        else:
            back = pa.Table.from_pylist([json.loads(ln) for ln in open(path)])
        assert back.column("id").to_pylist() == list(range(50))
    assert e.sql(f"copy t to '{tmp_path}/dir/' stored as parquet").table.to_pylist() == [{"count": N}]
    assert pq.read_table(str(tmp_path / "dir" / "part-0.parquet")).num_rows == N
    # NDJSON source (GPU: json.hip parse + string copy)
    p = str(tmp_path / "recs.json")
    recs = [{"a": i, "b": (None if i % 7 == 0 else f"v\\\"{i}\né"), "c": i / 4, "d": i % 2 == 0}
            for i in range(300)]
    with open(p, "w") as f:
        for r in recs:
            rr = {k: v for k, v in r.items() if not (k == "c" and r["a"] % 11 == 0)}
            f.write(json.dumps(rr) + "\n")
    before = KERNEL_CALLS["json_parse"]
    e.sql(f"create external table js{dev.replace(':', '')} stored as json location '{p}'")
    r = e.sql(f"select a, b, c, d from js{dev.replace(':', '')} order by a").table.to_pylist()
    for got, want in zip(r, recs):
        assert got["a"] == want["a"] and got["b"] == want["b"] and got["d"] == want["d"]
        assert got["c"] == (None if want["a"] % 11 == 0 else want["c"])
    if dev != "cpu":
        assert KERNEL_CALLS["json_parse"] > before
