"""Physical operators.

Each operator materialises its output as a device ``Batch`` keyed by column
id (operator-at-a-time over HBM-resident columns: with 288 GB per GPU an SF100
working set fits, and every operator is a handful of full-width kernels
instead of per-1024-row batches). Operators map one-to-one onto the
reference's ExecutionPlan implementations and DataFusion's inherited ones
(SURVEY §2.2 E5-E13):

  ScanExec        ParquetScanExec / DataSourceExec (+ fused filter)
  FilterExec      FilterExec           (reference operators/filter.rs)
  ProjectExec     ProjectionExec       (reference operators/projection.rs)
  HashJoinExec    HashJoinExec         (reference operators/hash_join.rs) — inner/left/right/full/semi/anti
  MultiJoinExec   DataFusion join reordering + HashJoinExec chain, ordered at run time
  HashAggExec     AggregateExec (partial/final)
  SortExec        SortExec / top-k
  LimitExec       GlobalLimitExec
  UnionExec, ValuesExec

The operators live in five modules -- ``context`` (ExecContext, ExecNode),
``scan`` (scan / values / filter / projection), ``joins`` (binary and
multi-way joins), ``aggregate`` (hash aggregation) and ``sorting`` (sort /
limit / union); this module re-exports all of their names. Tunables are
module constants of the module that reads them (e.g.
``joins.SORTED_JOIN_MIN_ROWS``): patch them there.
"""
from __future__ import annotations

from .context import (  # noqa: F401
    ExecContext, _NO_SCALAR, _device_scalar, _Span, _NoSpan, _NOSPAN, _sync, ExecNode,
)
from .scan import (  # noqa: F401
    _CID, LATE_SCAN, NDV_DERIVED, _tag_base, ScanExec, predicate_mask, LazyBatch, FragmentInputExec, ValuesExec,
    _column_from_values, FilterExec, filter_batch, ProjectExec, _ScanColumns, _LazyScanBatch,
)
from .joins import (  # noqa: F401
    key_tensors, _pair_key, _num_key, group_key_tensor, HashJoinExec, RUNTIME_FILTER_MAX_ROWS, _agg_group_source,
    push_key_filter, _index_key_filter, _index_then_filter, _semi_index_scan, _semi_index_then_filter,
    _rank_local_semi, apply_key_filters, _batch_bytes, JOIN_MEM_FACTOR, _to_host, _to_device, grace_join, hash_join,
    SORTED_JOIN_MIN_ROWS, _sorted_join, FLIP_OP, _CMP_KINDS, _col_compare, _nested_loop, _take_batch, _combine,
    _empty_like, concat_batches, concat_columns, _resident_ndv, _dense_lookup_ok, DENSE_JOIN, SEMI_INDEX,
    DENSE_JOIN_SMALL, inner_pairs, PERM_INDEX, PERM_INDEX_RATIO, PERM_INDEX_MAX_FRAC, PERM_INDEX_SORT_FRAC,
    _INT_KEYS, TWO_KEY_SORTED, _two_key_sorted_pairs, _LazyColumns, LateBatch, PRUNE_PARTS, LAZY_JOIN_OUTPUT,
    MultiJoinExec, _derived_ndv, _scan_info, _replicated, _global_rows, _global_rows_many, _edges,
)
from .aggregate import (  # noqa: F401
    EAGER_COUNT_DIRECT_SPAN, EAGER_COUNT_MASKED, SORTED_HAVING, SORTED_HAVING_MIN_ROWS, INDEX_THEN_FILTER,
    having_constant, HashAggExec, aggregate, _diff_bounds, _late_group_keys, _lead_key, _encode_groups, _empty_col,
    _plan_agg, _avg,
)
from .sorting import (  # noqa: F401
    SortExec, sort_batch, LimitExec, UnionExec,
)
