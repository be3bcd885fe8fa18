"""Physical execution.

Each operator materialises its output as a device ``Batch`` keyed by column
id (operator-at-a-time over HBM-resident columns: with 288 GB per GPU an SF100
working set fits, and every operator is a handful of full-width kernels
instead of per-1024-row batches). Operators map onto the reference's
ExecutionPlan implementations and DataFusion's inherited ones (SURVEY §2.2
E5-E13), one module per family:

  context    ExecContext, ExecNode
  scan       ScanExec (ParquetScanExec / DataSourceExec + fused filter), FilterExec, ProjectExec, ValuesExec
  joins      HashJoinExec (inner/left/right/full/semi/anti), MultiJoinExec (join reordering at run time)
  aggregate  HashAggExec (AggregateExec partial/final, fused sorted HAVING, eager COUNT)
  sorting    SortExec / top-k, LimitExec, UnionExec
  window     WindowExec, RecursiveCTEExec, WorkTableExec

Tunables are module constants of the module that reads them (e.g.
``joins.SORTED_JOIN_MIN_ROWS``): patch them there.
"""
