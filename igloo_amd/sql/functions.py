"""Registry of the SQL functions the binder accepts, by category.

Each entry maps a function name to an example call over the columns of the
registry test table (``s`` string, ``n`` integer, ``f`` double, ``d`` date,
``ts`` timestamp). Flight SQL's SqlInfo function lists are generated from
this registry (service/flight_sql.py) and ``tests/test_functions.py`` runs
every example on the CPU engine and on the GPU, so nothing is advertised
that the engine rejects. Parity: the DataFusion function library behind
``SessionContext::sql`` (reference crates/engine/src/lib.rs:54-57;
Cargo.lock:1062 datafusion-functions, :1091 -aggregate, :1162 -window).
"""
from __future__ import annotations

from typing import Dict

STRING: Dict[str, str] = {
    "upper": "upper(s)", "lower": "lower(s)", "capitalize": "capitalize(s)", "length": "length(s)",
    "char_length": "char_length(s)", "character_length": "character_length(s)", "substr": "substr(s, 2, 3)",
    "substring": "substring(s from 2 for 2)", "concat": "concat(s, '-', n)", "concat_ws": "concat_ws('/', s, n)",
    "trim": "trim(s)", "btrim": "btrim(s, 'x')", "ltrim": "ltrim(s)", "rtrim": "rtrim(s)",
    "replace": "replace(s, 'a', 'AA')", "lpad": "lpad(s, 8, '*')", "rpad": "rpad(s, 6)", "reverse": "reverse(s)",
    "repeat": "repeat(s, 2)", "left": "left(s, 2)", "right": "right(s, 3)", "initcap": "initcap(s)",
    "translate": "translate(s, 'ab', 'xy')", "split_part": "split_part(s, ' ', 2)", "strpos": "strpos(s, 'a')",
    "instr": "instr(s, 'b')", "position": "position('a' in s)", "ascii": "ascii(s)",
    "octet_length": "octet_length(s)", "bit_length": "bit_length(s)", "starts_with": "starts_with(s, 'ab')",
    "ends_with": "ends_with(s, 'c')", "regexp_like": "regexp_like(s, '^a.*c$')",
    "regexp_replace": "regexp_replace(s, '[aeiou]', '_', 'g')", "regexp_count": "regexp_count(s, '[a-c]')",
    "chr": "chr(65)", "to_hex": "to_hex(255)",
}
NUMERIC: Dict[str, str] = {
    "abs": "abs(n - 3)", "round": "round(f, 1)", "ceil": "ceil(f)", "ceiling": "ceiling(f)", "floor": "floor(f)",
    "sqrt": "sqrt(abs(f))", "ln": "ln(abs(f) + 1)", "log": "log(abs(f) + 1)", "log10": "log10(abs(f) + 1)",
    "log2": "log2(abs(f) + 1)", "exp": "exp(f / 10)", "power": "power(f, 2)", "pow": "pow(n, 2)",
    "mod": "mod(n, 3)", "sign": "sign(f)", "signum": "signum(n - 2)", "trunc": "trunc(f, 1)", "cbrt": "cbrt(f)",
    "degrees": "degrees(f)", "radians": "radians(f)", "sin": "sin(f)", "cos": "cos(f)", "tan": "tan(f)",
    "asin": "asin(f / 100)", "acos": "acos(f / 100)", "atan": "atan(f)", "atan2": "atan2(f, n + 1)",
    "sinh": "sinh(f / 10)", "cosh": "cosh(f / 10)", "tanh": "tanh(f)", "pi": "pi()", "greatest": "greatest(n, 3)",
    "least": "least(n, 3, f)", "gcd": "gcd(n, 6)", "lcm": "lcm(n, 4)", "isnan": "isnan(f)", "iszero": "iszero(f)",
    "nanvl": "nanvl(f, 0)", "factorial": "factorial(n)", "random": "random() < 2",
}
DATETIME: Dict[str, str] = {
    "date_part": "date_part('month', d)", "extract": "extract(year from d)", "year": "year(d)",
    "month": "month(d)", "day": "day(d)", "hour": "hour(ts)", "minute": "minute(ts)", "second": "second(ts)",
    "quarter": "quarter(d)", "week": "week(d)", "date_trunc": "date_trunc('month', ts)", "now": "now() > ts",
    "current_timestamp": "current_timestamp > ts", "current_date": "current_date > d", "today": "today() > d",
    "to_timestamp": "to_timestamp(n)", "to_timestamp_seconds": "to_timestamp_seconds(n)",
    "to_timestamp_millis": "to_timestamp_millis(n)", "to_timestamp_micros": "to_timestamp_micros(n)",
    "from_unixtime": "from_unixtime(n)", "to_unixtime": "to_unixtime(ts)", "to_date": "to_date('2024-01-02')",
    "make_date": "make_date(2020, n, 1)",
}
SYSTEM: Dict[str, str] = {
    "coalesce": "coalesce(s, 'none')", "ifnull": "ifnull(n, 0)", "nvl": "nvl(n, -1)", "nullif": "nullif(n, 2)",
    "nvl2": "nvl2(s, 1, 0)", "grouping": "grouping(s)",
}
AGGREGATE: Dict[str, str] = {
    "count": "count(n)", "sum": "sum(n)", "avg": "avg(f)", "mean": "mean(f)", "min": "min(s)", "max": "max(d)",
    "median": "median(n)", "approx_median": "approx_median(f)", "approx_percentile_cont":
    "approx_percentile_cont(f, 0.25)", "approx_distinct": "approx_distinct(s)", "stddev": "stddev(f)",
    "stddev_samp": "stddev_samp(f)", "stddev_pop": "stddev_pop(f)", "var": "var(f)", "variance": "variance(f)",
    "var_samp": "var_samp(f)", "var_pop": "var_pop(f)", "covar": "covar(f, n)", "covar_samp": "covar_samp(f, n)",
    "covar_pop": "covar_pop(f, n)", "corr": "corr(f, n)", "bool_and": "bool_and(n > 0)",
    "bool_or": "bool_or(n > 2)", "every": "every(n > 0)", "string_agg": "string_agg(s, ',')",
}
WINDOW: Dict[str, str] = {
    "row_number": "row_number() over (order by n nulls last, s nulls last)", "rank": "rank() over (order by n nulls last)",
    "dense_rank": "dense_rank() over (order by n nulls last)", "percent_rank": "percent_rank() over (order by n nulls last)",
    "cume_dist": "cume_dist() over (order by n nulls last)", "ntile": "ntile(2) over (order by n nulls last, s nulls last)",
    "lag": "lag(n) over (order by n nulls last, s nulls last)", "lead": "lead(s, 1, '-') over (order by n nulls last, s nulls last)",
    "first_value": "first_value(s) over (order by n nulls last, s nulls last)", "last_value": "last_value(n) over (order by n nulls last, s nulls last)",
    "nth_value": "nth_value(s, 2) over (order by n nulls last, s nulls last)",
}

CATEGORIES = {"string": STRING, "numeric": NUMERIC, "datetime": DATETIME, "system": SYSTEM,
              "aggregate": AGGREGATE, "window": WINDOW}


def names(category: str):
    return sorted(CATEGORIES[category])
