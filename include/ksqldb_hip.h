/*
 * ksqldb_hip.h — C ABI of the MI355X-native ksqlDB hot path (libksqldb_hip.so).
 *
 * This is the drop-in boundary between ksqlDB's Java operator surface and the
 * gfx950 HIP kernels.  Every entry point replaces one reference interface; the
 * reference file:line is cited above each declaration (paths relative to the
 * ksqlDB source root; S/ = ksqldb-streams/src/main/java/io/confluent/ksql/
 * execution/streams/, X/ = ksqldb-execution/src/main/java/io/confluent/ksql/
 * execution/, C/ = ksqldb-common/src/main/java/io/confluent/ksql/).
 *
 * Conventions:
 *   - extern "C", plain pointers and sizes, no exceptions cross the ABI.  Every
 *     call returns a khip_status; on failure khip_last_error() (thread-local)
 *     holds a message.
 *   - The caller owns every host buffer for the duration of a call.  The library
 *     owns all device memory it allocates and its HIP stream; it never retains a
 *     caller pointer after the call returns.  KHIP_MEM_DEVICE batches are read on
 *     the handle's stream and must stay valid until the call returns (aggregate
 *     push) or until the handle's *_sync() returns (asynchronous probes).
 *     The handle's stream is a BLOCKING HIP stream: its work is ordered after work
 *     the caller queued on the legacy default stream (torch's default stream), so
 *     a device batch produced there needs no extra synchronisation.  A producer on
 *     any other stream must be synchronised (or waited on) before the call.
 *   - Handles are independent; a single handle is not re-entrant (Kafka Streams
 *     task confinement, C/util/KsqlConstants.java:42 — one task per thread).
 *   - Validity bitmaps are Arrow-style: bit (i & 7) of byte (i >> 3), 1 = valid.
 *     A NULL bitmap pointer means "all valid".
 */
#ifndef KSQLDB_HIP_H
#define KSQLDB_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KHIP_ABI_VERSION 8

typedef int32_t khip_status;
#define KHIP_OK 0
#define KHIP_E_INVALID (-1)     /* bad argument / descriptor (plan-time KsqlException)      */
#define KHIP_E_NOMEM (-2)       /* device or host allocation failed                         */
#define KHIP_E_DEVICE (-3)      /* HIP runtime error                                         */
#define KHIP_E_UNSUPPORTED (-4) /* descriptor valid for ksqlDB but not for this path: the
                                   caller keeps the reference CPU builder for this query    */
#define KHIP_E_BUFFER (-5)      /* caller-provided output buffer too small                  */
#define KHIP_E_COMM (-6)        /* RCCL error                                                */
#define KHIP_E_STATE (-7)       /* call not valid in the handle's current state             */

/* Window kinds: X/windows/TumblingWindowExpression.java:32, HoppingWindowExpression.java:32.
 * NONE is the unwindowed StreamAggregate (X/plan/StreamAggregate.java:35). */
#define KHIP_WINDOW_NONE 0
#define KHIP_WINDOW_TUMBLING 1
#define KHIP_WINDOW_HOPPING 2
/* SESSION (gap = size_ms): X/windows/SessionWindowExpression.java, built by
 * S/StreamAggregateBuilder.java:296-323 (SessionWindows + KudafAggregator.getMerger, X/function/
 * udaf/KudafAggregator.java:87-111).  A record at ts joins (merges) every session of its key
 * with end >= ts - gap and start <= ts + gap; it is late when the merged session ends before
 * streamTime - grace - gap.  Rows are [key, aggs..., WINDOWSTART = session start, WINDOWEND =
 * session end]; a merge emits tombstones for the sessions it replaced. */
#define KHIP_WINDOW_SESSION 3

/* Key types.  Group identity is equality of the serialized KAFKA key
 * (BIGINT = 8-byte value, STRING = UTF-8 bytes), SURVEY.md §8.0. */
#define KHIP_KEY_INT64 0
#define KHIP_KEY_UTF8 1

/* Column (SQL) types carried on this path. */
#define KHIP_TYPE_INT32 0  /* INTEGER */
#define KHIP_TYPE_INT64 1  /* BIGINT  */
#define KHIP_TYPE_DOUBLE 2 /* DOUBLE  */

/* Built-in aggregate functions routed to the GPU (ksqldb-engine function/udaf):
 * CountKudaf.java:37, {Integer,Long,Double}SumKudaf.java:25, MinKudaf/MaxKudaf via
 * BaseComparableKudaf.java:55, AverageUdaf.java:104.  COUNT(*) is the analyzer's
 * COUNT(ROWTIME) rewrite (ksqldb-engine/.../analyzer/AggregateAnalyzer.java:339). */
#define KHIP_AGG_COUNT_STAR 0
#define KHIP_AGG_COUNT 1
#define KHIP_AGG_SUM 2
#define KHIP_AGG_MIN 3
#define KHIP_AGG_MAX 4
#define KHIP_AGG_AVG 5

/* Where a batch's column pointers live. */
#define KHIP_MEM_HOST 0
#define KHIP_MEM_DEVICE 1

/* grace_ms value meaning "no GRACE PERIOD clause": TimeWindows.of(size) without
 * grace (S/StreamAggregateBuilder.java:272,331) → Kafka 3.4 default
 * max(86_400_000 - size, 0) ms. */
#define KHIP_GRACE_DEFAULT (-1)

/* Comparison operators for the native HAVING / WHERE predicates. */
#define KHIP_OP_GT 0
#define KHIP_OP_GE 1
#define KHIP_OP_LT 2
#define KHIP_OP_LE 3
#define KHIP_OP_EQ 4
#define KHIP_OP_NE 5

/* Join types: S/StreamTableJoinBuilder.java:78-82. */
#define KHIP_JOIN_LEFT 0
#define KHIP_JOIN_INNER 1

/* ------------------------------------------------------------------ batches */

/* One columnar micro-batch of stream records, in arrival order.
 * Replaces the per-record GenericKey/GenericRow pair (C/GenericKey.java:30,
 * C/GenericRow.java:28) that Kafka Streams hands to the aggregate/join processor. */
typedef struct khip_batch {
  int64_t n_rows;
  int32_t mem;            /* KHIP_MEM_HOST or KHIP_MEM_DEVICE (all pointers below)   */
  int32_t n_cols;         /* number of value columns in col_data/col_valid           */
  const int64_t* key_i64; /* KHIP_KEY_INT64 keys (INT keys are widened by the caller) */
  const int64_t* key_offsets; /* KHIP_KEY_UTF8: n_rows+1 byte offsets into key_bytes */
  const uint8_t* key_bytes;
  const uint8_t* key_valid;   /* bitmap; null key → record dropped                   */
  const uint8_t* row_valid;   /* bitmap; 0 = null value (tombstone) → dropped
                                 (S/StreamGroupByBuilderBase.java:102) or, for a table
                                 upsert, a delete                                      */
  const int64_t* ts;          /* ROWTIME in ms; < 0 → dropped
                                 (S/timestamp/LoggingTimestampExtractor.java:72-84)    */
  const void* const* col_data;      /* n_cols column pointers (element type per desc) */
  const uint8_t* const* col_valid;  /* n_cols bitmaps (entries may be NULL)           */
  /* ABI 5: stream-time domains (khip_agg_desc.time_domain; both NULL for KHIP_TIME_TASK) */
  const int32_t* partition;   /* KHIP_TIME_PARTITION: the row's Kafka partition, 0..n_partitions-1.
                                 Rows of one partition form one contiguous run (a consumer poll's
                                 records per TopicPartition, concatenated)                       */
  const int64_t* stream_time; /* KHIP_TIME_SUPPLIED: the stream time observed at the row over the
                                 global arrival order (khip_stream_time_scan upstream, before the
                                 rows were routed to this handle); >= ts for accepted rows       */
} khip_batch;

/* Per-batch counters (the Kafka Streams dropped-records / late sensors). */
typedef struct khip_batch_stats {
  int64_t rows_in;
  int64_t rows_accepted;    /* reached the aggregate processor                        */
  int64_t dropped_null_key;
  int64_t dropped_null_row;
  int64_t dropped_bad_ts;
  int64_t windows_applied;  /* (record, window) updates applied                       */
  int64_t windows_late;     /* (record, window) pairs dropped: windowEnd <= streamTime-grace */
  int64_t stream_time;      /* observed stream time after the batch (-1 before any)  */
} khip_batch_stats;

/* --------------------------------------------------------- windowed aggregate */

/* Stream-time domains (late drop compares a window's end with streamTime - grace).
 * TASK: one stream time per handle — one Kafka Streams task (KStreamWindowAggregate's
 *   observedStreamTime, S/StreamAggregateBuilder.java:287-294), the reference's behaviour when the
 *   handle serves one input partition, and TopologyTestDriver's when it sees every record
 *   (F/tools/TestExecutorUtil.java:123-126).
 * PARTITION: the handle serves n_partitions Kafka partitions, one task each (one task per input
 *   partition, C/util/KsqlConstants.java:42): each partition has its own stream time, set by the
 *   batch's `partition` column.  The GROUP BY key must determine the partition (co-partitioned
 *   input, as groupByKey requires), so the tasks' stores are disjoint and one table holds them.
 *   Retention and EMIT FINAL are per task (ABI 7): the library records every key's partition
 *   (KHIP_E_INVALID when a key arrives on two partitions) and a row expires from snapshots, pull
 *   queries and row counts, or closes for EMIT FINAL, by its own partition's stream time.  Closed
 *   windows leave the live table by the smallest partition stream time, so every declared
 *   partition should receive records: an idle one holds that eviction back (memory and step
 *   time grow; results do not change).  The key → partition map keeps every key ever accepted
 *   until khip_agg_reset (it does not shrink with retention: memory grows with the distinct
 *   keys).  A batch rejected because a key arrived on a second partition leaves the partitions'
 *   stream times as they were before it; its new keys stay recorded with the partitions it named.
 * SUPPLIED: one GLOBAL stream time over several handles (ranks): each row carries the stream
 *   time observed at it over the global arrival order (`stream_time` column), computed where the
 *   rows were read, before routing: rank r scans its contiguous arrival chunk with
 *   khip_stream_time_scan seeded with max(global stream time before the batch, the maxima of the
 *   chunks of ranks < r) — an all-gather of one int64 per rank (or scans once unseeded and lets
 *   the pack apply the seed: khip_shuffle_stream_time_seed, ABI 8).  The rows that raise it are
 *   those the GROUP BY keeps (non-null value, non-null GROUP BY columns, ts >= 0).  The union of
 *   the ranks' tables then equals one task over the whole stream; EMIT FINAL closes windows by the
 *   GLOBAL stream time through khip_agg_supplied_close (ABI 8).
 *   SESSION windows take SUPPLIED with EMIT CHANGES (round 6: a non-key GROUP BY with a SESSION
 *   window through the repartition); PARTITION, and EMIT FINAL under SUPPLIED, return
 *   KHIP_E_UNSUPPORTED for SESSION windows (the reference CPU builder keeps them). */
#define KHIP_TIME_TASK 0
#define KHIP_TIME_PARTITION 1
#define KHIP_TIME_SUPPLIED 2

/* Window store retention (WINDOW ... RETENTION, X/windows/KsqlWindowExpression.java:26-54, passed to
 * the store by S/StreamAggregateBuilder.java:293,322,350 → X/runtime/MaterializedFactory.java:47).
 * Without the clause Kafka Streams keeps windows for size + grace. */
#define KHIP_RETENTION_DEFAULT (-1)

/* Output refinement (S/StreamAggregateBuilder.java:282-285): EMIT CHANGES emits every update,
 * EMIT FINAL (EmitStrategy.onWindowClose) emits a window once, when it closes. */
#define KHIP_EMIT_CHANGES 0
#define KHIP_EMIT_FINAL 1

/* HAVING predicate on one aggregate's result (S/TableFilterBuilder.java:46-74).
 * Rows failing it are absent from the materialized table (tombstoned). */
typedef struct khip_having {
  int32_t agg_index;
  int32_t op;        /* KHIP_OP_*                                                     */
  int64_t i64;       /* constant for integer-valued results                          */
  double f64;        /* constant for DOUBLE-valued results (AVG, SUM/MIN/MAX DOUBLE) */
} khip_having;

typedef struct khip_agg_spec {
  int32_t kind;    /* KHIP_AGG_*                                                      */
  int32_t arg_col; /* value column index (ignored for COUNT_STAR)                     */
} khip_agg_spec;

/* Plan-time descriptor: the content of StreamWindowedAggregate / StreamAggregate
 * (X/plan/StreamWindowedAggregate.java:47-70, X/plan/StreamAggregate.java:35-111)
 * after AggregateParamsFactory.create resolved the functions
 * (S/AggregateParamsFactory.java:70-121). */
typedef struct khip_agg_desc {
  int32_t window_kind;      /* KHIP_WINDOW_*                                          */
  int32_t key_type;         /* KHIP_KEY_*                                             */
  int64_t size_ms;          /* TUMBLING/HOPPING SIZE                                  */
  int64_t advance_ms;       /* HOPPING ADVANCE BY (= size for TUMBLING)              */
  int64_t grace_ms;         /* GRACE PERIOD, or KHIP_GRACE_DEFAULT                   */
  int32_t n_cols;
  const int32_t* col_types; /* KHIP_TYPE_* per value column                          */
  int32_t n_aggs;
  const khip_agg_spec* aggs;
  int32_t device;           /* HIP device ordinal                                    */
  int32_t flags;            /* KHIP_FLAG_* below, 0 by default                        */
  int64_t capacity_hint;    /* expected live (key, window) groups; 0 = default       */
  /* ABI 2 */
  int64_t retention_ms;     /* window retention, or KHIP_RETENTION_DEFAULT; must be >= size +
                               grace (Kafka Streams rejects a shorter one)               */
  int32_t emit;             /* KHIP_EMIT_CHANGES or KHIP_EMIT_FINAL                      */
  int32_t has_having;       /* 1: `having` is the query's HAVING (the TableFilter step after
                               the aggregate); the library then keeps its row count and
                               changelog tombstones up to date as records arrive          */
  khip_having having;
  /* ABI 5 */
  int32_t time_domain;      /* KHIP_TIME_TASK (0), KHIP_TIME_PARTITION, KHIP_TIME_SUPPLIED      */
  int32_t n_partitions;     /* KHIP_TIME_PARTITION: partitions the handle serves (<= 65536)     */
} khip_agg_desc;

typedef struct khip_agg khip_agg;

/* Final materialized table, sorted by (key, window_start).  Caller-allocated.
 * Row = [key, agg results..., WINDOWSTART, WINDOWEND]
 * (S/AggregateParamsFactory.java:156-190, S/StreamAggregateBuilder.java:355-373)
 * plus the row timestamp (max ROWTIME applied to the entry). */
typedef struct khip_snapshot {
  int64_t capacity;            /* rows the buffers below can hold                     */
  int64_t n_rows;              /* out                                                 */
  int64_t key_bytes_capacity;  /* UTF8                                                */
  int64_t key_bytes_len;       /* out                                                 */
  int64_t* key_i64;            /* INT64 keys                                          */
  int64_t* key_offsets;        /* UTF8: capacity+1                                    */
  uint8_t* key_bytes;
  int64_t* window_start;       /* 0 for KHIP_WINDOW_NONE                              */
  int64_t* window_end;
  int64_t* rowtime;
  void** agg_values;           /* per agg; element type from khip_agg_result_type()   */
  uint8_t** agg_null;          /* per agg; 1 byte per row, 1 = SQL NULL               */
} khip_snapshot;

/* KSPlanBuilder.visitStreamWindowedAggregate / visitStreamAggregate
 * (S/KSPlanBuilder.java:293-304, :144-155; interface X/plan/PlanBuilder.java:37,67):
 * builds the HBM-resident (key, windowStart) state for one query task. */
khip_status khip_agg_create(const khip_agg_desc* desc, khip_agg** out);

/* Result element type of aggregate i (KsqlAggregateFunction.getReturnType,
 * C/function/KsqlAggregateFunction.java:25-55): COUNT → INT64, SUM(T) → T,
 * MIN/MAX(T) → T, AVG → DOUBLE. */
khip_status khip_agg_result_type(const khip_agg_desc* desc, int32_t agg_index,
                                 int32_t* out_type);

/* Per-record KStreamWindowAggregate.process + KudafAggregator.apply
 * (X/function/udaf/KudafAggregator.java:56-80) over a whole micro-batch:
 * rows are applied as if one at a time in arrival order (stream time, late drop,
 * window fan-out).  stats may be NULL (then the call may return
 * before the device work completes). */
khip_status khip_agg_push(khip_agg* agg, const khip_batch* batch,
                          khip_batch_stats* stats);

/* ABI 5.  The stream time observed at each row of `batch` in arrival order, starting from `seed`
 * (-1: none): out[i] = max(seed, ts of the accepted rows 0..i) — rows with a null key, a null
 * value or ts < 0 never reach the aggregate and do not advance it.  *out_max = the value after the
 * last row.  `out` is in the batch's memory (host or device).  The upstream half of
 * KHIP_TIME_SUPPLIED (see above); the handle only provides the device and stream. */
khip_status khip_stream_time_scan(khip_agg* agg, const khip_batch* batch, int64_t seed, int64_t* out,
                                  int64_t* out_max);

/* ABI 8.  EMIT FINAL in the GLOBAL domain (KHIP_TIME_SUPPLIED: StreamAggregateBuilder.java:282-285
 * applies onWindowClose however the stream was repartitioned).  A window that the stream time's
 * jump at one record both closes and expires (retention) is never emitted (R9/R10); which windows
 * those are is a property of the global stream time alone, known where the rows are read:
 *   khip_agg_lost_windows: the window-start ranges [lo, hi] (n_ranges pairs into `ranges`,
 *     KHIP_E_BUFFER past `capacity`) that the jumps of `batch` — one rank's contiguous arrival
 *     chunk, its stream time starting at `seed` — close after they expired.  `agg` is an EMIT FINAL
 *     TUMBLING / HOPPING handle with the query's windows (its scratch only is used).
 *   khip_agg_supplied_close: before each push of a KHIP_TIME_SUPPLIED EMIT FINAL handle (required),
 *     or of any SUPPLIED handle that should keep the GLOBAL stream time: the global stream time
 *     before and after the whole global batch, and the union of every rank's lost ranges.  The
 *     push then closes the windows whose end lies in (before - grace, after - grace], except the
 *     lost ones — also when no row of the batch was routed to this handle (n_rows = 0) — and the
 *     handle's stream time becomes `st_after`. */
khip_status khip_agg_lost_windows(khip_agg* agg, const khip_batch* batch, int64_t seed, int64_t* ranges,
                                  int64_t capacity, int64_t* n_ranges);
khip_status khip_agg_supplied_close(khip_agg* agg, int64_t st_before, int64_t st_after, const int64_t* ranges,
                                    int64_t n_ranges);

/* Number of rows and key bytes the next snapshot will produce (no HAVING).  Snapshots, pull
 * queries and row counts read the window store: windows with start < obs - retention (obs =
 * the largest window start put, i.e. floor(streamTime / advance) * advance) have expired. */
khip_status khip_agg_snapshot_size(khip_agg* agg, int64_t* n_rows,
                                   int64_t* key_bytes);

/* Materialize the table (ResultTransformer map(): KudafAggregator.java:129-158).
 * having may be NULL. */
khip_status khip_agg_snapshot(khip_agg* agg, const khip_having* having,
                              khip_snapshot* out);

/* Pull query against the materialized table (KsMaterializedWindowTable.get(key, partition,
 * windowStartBounds, windowEndBounds), S/materialization/ks/KsMaterializedWindowTable.java:70-120,
 * and the all-keys scan get(partition, ...) :122-165; unwindowed KsMaterializedTable.get).
 * Bounds are closed ranges in epoch ms (an open Guava Range end becomes lo+1 / hi-1; unbounded =
 * INT64_MIN / INT64_MAX); they are ignored for KHIP_WINDOW_NONE tables.  UTF8 keys are mapped
 * to their dictionary ids by a read-only device probe; keys never pushed match no row. */
typedef struct khip_pull {
  int64_t n_keys;        /* 0 = every key (scan); else the n_keys keys below                   */
  const int64_t* keys;   /* INT64 key tables: host memory, any order, duplicates allowed       */
  int64_t ws_lo, ws_hi;  /* WINDOWSTART bounds, inclusive                                      */
  int64_t we_lo, we_hi;  /* WINDOWEND bounds, inclusive                                        */
  const int64_t* key_offsets;  /* UTF8 key tables: n_keys+1 offsets (from 0) into key_bytes    */
  const uint8_t* key_bytes;    /* serialized KAFKA STRING keys (byte equality, like the push)  */
} khip_pull;

/* Rows matching `q` (and `having`, may be NULL: HAVING-tombstoned rows are absent from the
 * table) in snapshot layout, sorted by (key, window start).  The filter runs on the device
 * over the HBM-resident state; only matching rows cross PCIe. */
khip_status khip_agg_get(khip_agg* agg, const khip_pull* q, const khip_having* having,
                         khip_snapshot* out);

/* ---- Emission (the aggregate's output topic: the table's changelog).
 * One push = one commit of Kafka Streams' record cache (C/util/KsqlConstants.java:40-41): the
 * rows a push emits are deduplicated per (key, window), carry their value after the push, and
 * are sorted by (key, window start).  SESSION windows are the exception: a record that lands in an
 * existing session [s, e] replaces it, and the push emits the tombstone of the old session and the
 * rewritten session as two rows — even when the rewritten one has the same (s, e) — delete first
 * (Kafka Streams' session store removes the merged sessions and puts the new one; the reference's
 * cache-off output has the same two records).  Pushing one record at a time reproduces the reference's
 * cache-off output sequence exactly (QTT, tests/test_gpu_emit.py).
 *   EMIT CHANGES (needs KHIP_FLAG_CHANGELOG): every (key, window) the push updated; with the
 *     descriptor's HAVING (S/TableFilterBuilder.java:63-75) a row that no longer passes but did
 *     before the push is a tombstone, one that passed neither before nor after is not emitted.
 *   EMIT FINAL (S/StreamAggregateBuilder.java:282-285, EmitStrategy.onWindowClose): every window
 *     the push closed (window end <= stream time - grace), emitted once with its final value
 *     unless it had already expired from the window store (retention) at the record that closed
 *     it, then filtered by the descriptor's HAVING.  SESSION windows (ABI 8; S/StreamAggregateBuilder
 *     .java:310-312, Kafka 3.4 KStreamSessionWindowAggregate.maybeForwardFinalResult): a session is
 *     emitted once, when streamTime - grace - gap passes its END — the sessions of the store after
 *     the push whose end the push's close time passed, and those a record of the push merged away
 *     after the close before that record had passed their end (a RETENTION beyond gap + grace) —
 *     row time = session end, HAVING applied.
 * khip_agg_changes_size returns the row count and (UTF8) key bytes of the last push's rows;
 * khip_agg_changes writes them in snapshot layout plus tombstone[n_rows] (1 = delete; may be
 * NULL).  Valid until the next push or reset. */
#define KHIP_FLAG_CHANGELOG 8
khip_status khip_agg_changes_size(khip_agg* agg, int64_t* n_rows, int64_t* key_bytes);
khip_status khip_agg_changes(khip_agg* agg, khip_snapshot* out, uint8_t* tombstone);

/* ---- Table aggregation: CREATE TABLE .. AS SELECT .. FROM <TABLE> GROUP BY .. (KSPlanBuilder
 * visitTableGroupBy + visitTableAggregate → S/TableGroupByBuilderBase.java:62-111,
 * S/TableAggregateBuilder.java:54-108; Kafka Streams KTable.groupBy().aggregate(init, adder,
 * subtractor), KTableAggregate).  Each source-table change (key k: old row → new row) undoes the
 * old row from its group (KudafUndoAggregator, X/function/udaf/KudafUndoAggregator.java:29-55,
 * TableUdaf.undo) and applies the new row to its group (KudafAggregator).  A group whose rows all
 * left keeps its row (COUNT 0, Q/count.json "should count back to zero"); HAVING removes it.
 * Only undoable aggregates are accepted: COUNT(*), COUNT, SUM, AVG (MIN/MAX on a table source is a
 * KsqlException in the reference, E/structured/SchemaKGroupedTable.java:82-95 → KHIP_E_UNSUPPORTED).
 * The handle is created with window_kind NONE and this flag; snapshots, pull queries and row counts
 * work as for a stream aggregate. */
#define KHIP_FLAG_TABLE_SOURCE 16

/* The source table's PRIMARY KEY of each batch row (same memory kind as the batch). */
typedef struct khip_table_src {
  int32_t key_type;            /* KHIP_KEY_INT64 or KHIP_KEY_UTF8 (fixed by the first push)     */
  int32_t reserved;
  const int64_t* key_i64;
  const int64_t* key_offsets;  /* UTF8: n_rows + 1 offsets into key_bytes                       */
  const uint8_t* key_bytes;
  const uint8_t* key_valid;    /* bitmap; a null PRIMARY KEY drops the record                   */
} khip_table_src;

/* Apply source-table changelog records in arrival order.  Batch rows: key = the row's GROUP BY
 * value (key_valid 0 = NULL: the row joins no group, S/GroupByParamsFactory.java:92-100), row_valid
 * 0 = tombstone (the key is deleted), ts = ROWTIME (< 0: dropped), value columns = the aggregate
 * arguments.  Group row time = the largest ts of the records that added to or undid from it.
 * stats: rows_accepted = source records applied, dropped_null_key = null PRIMARY KEY,
 * windows_applied = aggregate updates (adds + undos). */
khip_status khip_agg_push_table(khip_agg* agg, const khip_batch* batch, const khip_table_src* src,
                                khip_batch_stats* stats);

/* Count the rows that pass `having` entirely on the device (no copy-out).
 * having may be NULL (= total group count).  When `having` is the descriptor's own HAVING,
 * the count is the one the aggregate kernels maintain (returned without device work). */
khip_status khip_agg_count_rows(khip_agg* agg, const khip_having* having,
                                int64_t* n_rows);

/* Drop all state (a fresh query instance); keeps the device allocation.  Asynchronous:
 * queued on the handle's stream, ahead of every later call on the handle. */
khip_status khip_agg_reset(khip_agg* agg);

/* Block until all work queued on the handle has finished. */
khip_status khip_agg_sync(khip_agg* agg);

/* desc.flags bit: record HIP events around each kernel phase of khip_agg_push (the
 * Kafka Streams per-processor latency sensors' analogue; off by default). */
#define KHIP_FLAG_PROFILE 1
/* desc.flags bit: use the global-atomic engine (one HBM hash table updated with
 * agent-scope atomics) instead of the default partitioned LDS engine. */
#define KHIP_FLAG_ENGINE_ATOMIC 2
/* desc.flags bit (diagnostic): partitioned engine always uses the claim/ready slot protocol
 * instead of the packed-identity CAS it picks when a push's window range fits. */
#define KHIP_FLAG_PART_CLAIM 4

/* Cumulative device time per phase since creation or the last reset of the counters,
 * measured with HIP events on the handle's stream (valid with KHIP_FLAG_PROFILE). */
typedef struct khip_kernel_times {
  double stream_time_ms; /* stream-time maxima/scans (+ partition histogram, offsets)  */
  double dict_ms;        /* UTF8 key dictionary                                       */
  double partition_ms;   /* partitioned engine: k_part_scatter                        */
  double apply_ms;       /* k_part_agg (LDS aggregation) or k_apply (global atomics)  */
  double finalize_ms;    /* atomic engine: k_finalize + counter reduction             */
  int64_t apply_launches;
  int64_t records;       /* records covered by those apply launches (first passes)    */
  int64_t c1_pushes;     /* ABI 5: pushes the windowed COUNT(*) pipeline took           */
  int64_t c1_declined;   /* ABI 5: pushes it declined (late records possible, wide
                            ts span or key range): the general path ran instead        */
} khip_kernel_times;

khip_status khip_agg_kernel_times(khip_agg* agg, khip_kernel_times* out, int32_t reset);

/* The handle's hipStream_t (as void*), so callers can order their own work. */
khip_status khip_agg_stream(khip_agg* agg, void** hip_stream);

khip_status khip_agg_destroy(khip_agg* agg);

/* --------------------------------------------------------- stream-table join */

/* Table side: SourceBuilder.buildKTable (S/SourceBuilder.java:87-137) materializes
 * the latest non-null value per key; a null value deletes the key. */
typedef struct khip_table_desc {
  int32_t key_type;          /* KHIP_KEY_INT64, or KHIP_KEY_UTF8 (STRING keys: the batch's
                                key_offsets/key_bytes, identity = byte equality; the
                                stream batch probing it carries STRING keys too)      */
  int32_t n_cols;
  const int32_t* col_types;  /* KHIP_TYPE_* per table value column (VARCHAR columns are
                                dictionary codes, KHIP_TYPE_INT32)                    */
  int32_t device;
  int32_t flags;
  int64_t capacity_hint;     /* expected live keys                                    */
} khip_table_desc;

typedef struct khip_table khip_table;

/* WHERE predicate on one right-side column (S/StreamFilterBuilder.java:44-69);
 * a NULL right column never satisfies it (SQL three-valued logic). */
typedef struct khip_where {
  int32_t right_col;
  int32_t op;
  int64_t i64;
  double f64;
} khip_where;

/* Join output: one entry per emitted row, in stream arrival order.
 * Row = left values ++ right values|nulls (S/KsqlValueJoiner.java:41-63); the caller
 * gathers the left side by stream_row. */
typedef struct khip_join_out {
  int64_t capacity;
  int64_t n_rows;       /* out                                                       */
  int64_t* stream_row;  /* index of the stream record in the probe batch             */
  uint8_t* matched;     /* 1 = table hit, 0 = LEFT miss (right side null)            */
  void** col_data;      /* per right column (NULL entries are skipped)               */
  uint8_t** col_null;   /* per right column; 1 byte per row                          */
} khip_join_out;

khip_status khip_table_create(const khip_table_desc* desc, khip_table** out);

/* Apply table-topic records in arrival order: the last row per key wins, a row with
 * row_valid = 0 deletes the key, null keys are skipped. */
khip_status khip_table_upsert(khip_table* t, const khip_batch* rows);

khip_status khip_table_size(khip_table* t, int64_t* n_keys);

/* KStreamKTableJoin per stream record + KsqlValueJoiner.apply
 * (S/StreamTableJoinBuilder.java:38-88): null-key / null-value / negative-ts stream
 * records are dropped; INNER emits on hit only; LEFT always emits.  `where` may be
 * NULL.  Output is written to host buffers (out). */
khip_status khip_table_probe(khip_table* t, const khip_batch* stream, int32_t join_type,
                             const khip_where* where, khip_join_out* out);

/* Device-resident variant (selection-vector output, no compaction): all buffers are
 * caller-allocated DEVICE memory, row-aligned with the probe batch (n_rows entries /
 * bits).  emit bit i = stream row i produced an output row (INNER hit or LEFT, and
 * WHERE passed); matched bit i = table hit; col_data[c][i] / col_null bit i = right
 * column c (undefined / 1 where not matched).  Any pointer may be NULL to skip that
 * output.  *n_emitted (may be NULL: then the call does not synchronise) receives the
 * number of emitted rows.  The batch must be KHIP_MEM_DEVICE and stay valid until
 * khip_table_sync() returns. */
typedef struct khip_join_dev_out {
  uint8_t* emit;
  uint8_t* matched;
  void** col_data;
  uint8_t** col_null;
} khip_join_dev_out;

khip_status khip_table_probe_device(khip_table* t, const khip_batch* stream,
                                    int32_t join_type, const khip_where* where,
                                    const khip_join_dev_out* out, int64_t* n_emitted);

khip_status khip_table_sync(khip_table* t);
khip_status khip_table_destroy(khip_table* t);

/* ------------------------------------------------ repartition (non-key GROUP BY) */

/* The repartition topic that StreamGroupByBuilderBase.build inserts for a non-key GROUP BY or
 * PARTITION BY (S/StreamGroupByBuilderBase.java:101-103, S/StreamSelectKeyBuilder.java:73-74):
 * every record is re-keyed by a value column and routed to the partition Kafka's default
 * partitioner gives it: toPositive(murmur2(KAFKA-format key bytes)) % n_parts, the key bytes
 * being big-endian 4 (INT) / 8 (BIGINT) bytes (ksqldb-serde/.../kafka/KafkaSerdeFactory.java:42-43;
 * kafka-clients Utils.murmur2).  Null-value records and records whose new key is null are dropped
 * (S/GroupByParamsFactory.java:92-100).  Packed row (u64 words, 2 + n_cols of them):
 *   [new key][ts][value columns except key_col (raw, INT32 sign-extended)...]
 *   [validity bits: column c = bit c; the key column's bit is always set]
 * Order is stable: a destination receives each source's rows in arrival order.
 * ABI 7, KHIP_SHUFFLE_STREAM_TIME in `flags`: the rows also carry the batch's `stream_time` column
 * (the GLOBAL stream time observed at the row, khip_stream_time_scan before routing) as one more
 * word before the validity word:
 *   [new key][ts][value columns except key_col...][stream_time][validity bits]
 * so the owner's KHIP_TIME_SUPPLIED aggregation (khip_agg_push_shuffled) late-drops against the
 * stream time one task over the whole stream would have had (TopologyTestDriver: one task per
 * query, F/tools/TestExecutorUtil.java:123-126). */
#define KHIP_SHUFFLE_STREAM_TIME 1
typedef struct khip_shuffle_desc {
  int32_t n_parts;          /* destinations (tasks / GPUs)                                */
  int32_t key_col;          /* value column that becomes the new key (INT32/INT64)        */
  int32_t n_cols;           /* value columns carried (all of the batch's columns)         */
  const int32_t* col_types;
  int32_t device;
  int32_t flags;            /* KHIP_SHUFFLE_*                                             */
} khip_shuffle_desc;

typedef struct khip_shuffle khip_shuffle;

khip_status khip_shuffle_create(const khip_shuffle_desc* desc, khip_shuffle** out);

/* Words per packed row (2 + n_cols, + 1 with KHIP_SHUFFLE_STREAM_TIME). */
int32_t khip_shuffle_row_words(const khip_shuffle* s);

/* Partition a DEVICE batch into the caller's device buffer `send` (capacity rows x row
 * words), grouped by destination; counts[n_parts] (host) receives the rows per destination
 * (destination d's rows start at the sum of counts[0..d)). */
khip_status khip_shuffle_pack(khip_shuffle* s, const khip_batch* in, uint64_t* send,
                              int64_t capacity, int64_t* counts);

/* ABI 7.  The one-pass pack for n_parts > 1: every row is read once (no counting pass over the
 * source).  Destination d's rows are written contiguously, in arrival order, at row offsets[d] of
 * `send` (counts[d] of them): the library lays the destinations out in regions of a stride sized
 * from the batch's even share n_rows / n_parts plus slack, finds each tile's place in every region
 * by decoupled look-back over the earlier tiles' per-destination counts, and packs a batch whose
 * largest destination overflows its region again with the exact stride (or, when that does not
 * fit `capacity`, contiguously as khip_shuffle_pack does).  `capacity` (rows) must be at least
 * khip_shuffle_pack_capacity(s, n_rows).  The send side of khip_comm_alltoall_v. */
int64_t khip_shuffle_pack_capacity(const khip_shuffle* s, int64_t n_rows);
khip_status khip_shuffle_pack_v(khip_shuffle* s, const khip_batch* in, uint64_t* send,
                                int64_t capacity, int64_t* counts, int64_t* offsets);

/* Packed rows (device) → columnar device arrays owned by the caller: key[n], ts[n],
 * col_data[c][n] (8-byte raw for every column type except INT32 = 4 bytes) and
 * col_valid[c] bitmaps ((n+7)/8 bytes; may be NULL).  A NULL col_data[c] / col_valid[c]
 * entry skips that column / bitmap (e.g. the GROUP BY column, which is the key and valid by
 * construction).  The result is a khip_batch whose records are the received rows in
 * (source, arrival) order.
 * Capacity: khip_shuffle_pack's `send` may be sized for every batch row (n_rows x row words):
 * then one call computes the counts and scatters (a smaller buffer returns KHIP_E_BUFFER with
 * the counts, and the caller calls again). */
khip_status khip_shuffle_unpack(khip_shuffle* s, const uint64_t* rows, int64_t n, int64_t* key,
                                int64_t* ts, void* const* col_data, uint8_t* const* col_valid);

/* ABI 7.  KHIP_SHUFFLE_STREAM_TIME rows → their stream_time column (device, n entries): with
 * khip_shuffle_unpack, a KHIP_TIME_SUPPLIED batch. */
khip_status khip_shuffle_unpack_stream_time(khip_shuffle* s, const uint64_t* rows, int64_t n,
                                            int64_t* stream_time);

/* ABI 8.  KHIP_SHUFFLE_STREAM_TIME: the packs that follow write max(seed, stream_time[i]) as a
 * row's stream-time word (the default seed, -1, leaves the column as it is).  A rank scans its
 * arrival chunk ONCE, unseeded (khip_stream_time_scan with seed -1), learns the chunk maxima of
 * the ranks before it, and hands their max here: a seeded prefix max is the unseeded one raised
 * to the seed, so the column needs no second scan. */
khip_status khip_shuffle_stream_time_seed(khip_shuffle* s, int64_t seed);

/* ABI 6.  Received rows straight into the aggregation that reads the repartition topic (the
 * non-key GROUP BY's aggregate, S/StreamGroupByBuilderBase.java:101-103 → StreamAggregateBuilder),
 * without materialising them as columns first: the same effect and statistics as khip_agg_push of
 * khip_shuffle_unpack's batch (key = the shuffle's key column, every row valid).  `agg`'s columns
 * must be the shuffle's columns (count and types) and its GROUP BY key an integer (the new key).
 * `rows` (device, n rows of khip_shuffle_row_words words) stays the caller's.  Pushes the value
 * pipeline takes read the rows where they lie; every other push unpacks them into the handle's
 * staging columns and runs as a device batch.  Replaces khip_shuffle_unpack + khip_agg_push at the
 * reference's repartition source (S/StreamGroupByBuilderBase.java:101-103).
 * Time domains: TASK, and SUPPLIED when the shuffle carries KHIP_SHUFFLE_STREAM_TIME (the rows'
 * stream-time word is the batch's `stream_time` column; KHIP_E_INVALID without it).  PARTITION is
 * KHIP_E_UNSUPPORTED: received rows carry no source partition. */
khip_status khip_agg_push_shuffled(khip_agg* agg, const khip_shuffle* s, const uint64_t* rows, int64_t n,
                                   khip_batch_stats* stats);

khip_status khip_shuffle_sync(khip_shuffle* s);
khip_status khip_shuffle_destroy(khip_shuffle* s);

/* RCCL communicator, one rank per GPU (one process per GPU).  The 128-byte unique id is
 * created on rank 0 and distributed by the caller (the Kafka/ksqlDB control plane, or
 * torch.distributed in bench.py). */
typedef struct khip_comm khip_comm;
#define KHIP_COMM_ID_BYTES 128
khip_status khip_comm_unique_id(uint8_t id[KHIP_COMM_ID_BYTES]);
khip_status khip_comm_init(int32_t nranks, int32_t rank, const uint8_t id[KHIP_COMM_ID_BYTES],
                           int32_t device, khip_comm** out);

/* Collective, step 1: exchange the per-peer row counts (send_counts[nranks] host →
 * recv_counts[nranks] host), so every rank can size its receive buffer. */
khip_status khip_comm_exchange_counts(khip_comm* c, const int64_t* send_counts, int64_t* recv_counts);

/* Collective, step 2: all-to-all of packed rows over xGMI (grouped ncclSend/ncclRecv, one pair
 * per peer, no ring): send rows grouped by destination with send_counts[nranks]; recv_counts
 * are the ones step 1 returned and recv must hold their sum; the received rows are laid out by
 * source rank.  A capacity error here is a caller bug that leaves the peers blocked, so size
 * recv from step 1. */
khip_status khip_comm_alltoall(khip_comm* c, const uint64_t* send, const int64_t* send_counts,
                               uint64_t* recv, int64_t recv_capacity, const int64_t* recv_counts,
                               int32_t row_words);
/* ABI 7.  The same all-to-all with the send side laid out by khip_shuffle_pack_v: peer p's rows
 * are send_counts[p] rows at row send_offsets[p] of `send` (regions need not be adjacent).  The
 * received rows are laid out by source rank, as khip_comm_alltoall lays them out. */
khip_status khip_comm_alltoall_v(khip_comm* c, const uint64_t* send, const int64_t* send_counts,
                                 const int64_t* send_offsets, uint64_t* recv, int64_t recv_capacity,
                                 const int64_t* recv_counts, int32_t row_words);
khip_status khip_comm_destroy(khip_comm* c);

/* ------------------------------------------ deserialization (ksqldb-serde → device columns) */

/* Formats (ksqldb-serde/src/main/java/io/confluent/ksql/serde/):
 *   KAFKA      kafka/KafkaSerdeFactory.java:42-46 — Kafka's primitive serdes: INT = 4-byte and
 *              BIGINT = 8-byte big-endian, DOUBLE = 8-byte big-endian IEEE 754, STRING = UTF-8;
 *              one field per key / value (a wrong length is a SerializationException)
 *   DELIMITED  delimited/KsqlDelimitedDeserializer.java — CSVFormat.DEFAULT with the configured
 *              delimiter (RFC 4180 quoting), one field per column, empty field = NULL, numbers
 *              by Integer.parseInt / Long.parseLong / Double.parseDouble
 *   JSON       json/KsqlJsonDeserializer.java — one object per record; a column reads the field of
 *              the same name, else the field whose upper-cased name matches (:273-300); JSON null
 *              or a missing field = NULL; numbers coerced as JsonSerdeUtils.toInteger / toLong /
 *              toDouble (Jackson intValue / asLong / doubleValue, or the Java parsers on strings)
 *   AVRO       avro/KsqlAvroSerdeFactory.java:130-144 (Confluent's KafkaAvroDeserializer through
 *              connect/KsqlConnectDeserializer) — Confluent wire format: magic byte 0, 4-byte
 *              big-endian schema id, then the Avro binary encoding of the WRITER schema's record
 *              (zig-zag varint int / long, little-endian float / double, long-length-prefixed
 *              string / bytes, a varint branch index for a union [null, T] or [T, null]).  Writer
 *              fields land in the column of the same name, else of the upper-cased name
 *              (connect/ConnectDataTranslator.java:290-318); a writer type the column's type does
 *              not accept (validateSchema :123-146: BIGINT ← int / long, INT ← int, DOUBLE ← float /
 *              double, STRING ← any primitive) fails every record; missing columns are NULL.
 * A record that fails to deserialize is dropped by the reference (processing log): here it gets a
 * null key and a null value (every consumer drops it; a table upsert skips it) and is counted. */
#define KHIP_FMT_NONE 0
#define KHIP_FMT_KAFKA 1
#define KHIP_FMT_DELIMITED 2
#define KHIP_FMT_JSON 3
#define KHIP_FMT_AVRO 4
/* Avro writer-schema field types (primitive; unions of null and one of them via avro_field_union) */
#define KHIP_AVRO_BOOLEAN 1
#define KHIP_AVRO_INT 2
#define KHIP_AVRO_LONG 3
#define KHIP_AVRO_FLOAT 4
#define KHIP_AVRO_DOUBLE 5
#define KHIP_AVRO_STRING 6
#define KHIP_AVRO_BYTES 7
#define KHIP_TYPE_STRING 3  /* VARCHAR: keys → UTF-8 key columns; value fields are only checked for
                               NULL (an INT64 column of zeros + validity: what COUNT(col) reads)  */

typedef struct khip_serde_desc {
  int32_t key_format;              /* KHIP_FMT_NONE or KHIP_FMT_KAFKA                          */
  int32_t key_type;                /* KHIP_TYPE_INT32 / INT64 (→ int64 keys) / STRING (→ UTF-8) */
  int32_t value_format;            /* KHIP_FMT_KAFKA / DELIMITED / JSON / AVRO                 */
  int32_t n_fields;                /* value schema columns, in order                            */
  const int32_t* field_types;      /* KHIP_TYPE_INT32 / INT64 / DOUBLE / STRING                 */
  const char* const* field_names;  /* JSON / AVRO: column names as ksqlDB stores them           */
  const int32_t* field_out;        /* output column of each field, or -1 (not read)            */
  int32_t delimiter;               /* DELIMITED: the VALUE_DELIMITER byte (',')                 */
  int32_t device;
  /* AVRO: the writer schema (a record of avro_n_fields fields, in writer order) registered under
   * avro_schema_id (-1: accept any id; a different id is a deserialization error) */
  int32_t avro_schema_id;
  int32_t avro_n_fields;
  const char* const* avro_field_names;
  const int32_t* avro_field_types;  /* KHIP_AVRO_*                                               */
  const int32_t* avro_field_union;  /* 0: plain; 1: ["null", T]; 2: [T, "null"]                  */
} khip_serde_desc;

/* One batch of Kafka records as the consumer returns them (arrival order). */
typedef struct khip_raw_batch {
  int64_t n_rows;
  int32_t mem;                   /* KHIP_MEM_HOST or KHIP_MEM_DEVICE                           */
  const int64_t* ts;             /* record timestamps (ROWTIME)                                */
  const int64_t* key_offsets;    /* n_rows + 1 offsets into key_bytes                          */
  const uint8_t* key_bytes;
  const uint8_t* key_valid;      /* bitmap, 0 = null key; NULL = all present                  */
  const int64_t* value_offsets;  /* n_rows + 1 offsets into value_bytes                        */
  const uint8_t* value_bytes;
  const uint8_t* value_valid;    /* bitmap, 0 = null value (tombstone); NULL = all present     */
} khip_raw_batch;

typedef struct khip_serde khip_serde;

/* GenericKeySerDe / GenericRowSerDe deserializers (ksqldb-serde/.../GenericKeySerDe.java,
 * GenericRowSerDe.java) for one source topic's schema. */
khip_status khip_serde_create(const khip_serde_desc* desc, khip_serde** out);

/* Decode into device columns owned by the handle (valid until its next decode): *out becomes a
 * KHIP_MEM_DEVICE batch (value columns = the fields with field_out >= 0) for khip_agg_push /
 * khip_table_upsert / khip_table_probe_device.  UTF-8 keys of a device input point into the
 * input's key bytes (keep the input alive while using *out).  *n_errors (may be NULL) receives
 * the records that failed to deserialize. */
khip_status khip_serde_decode(khip_serde* s, const khip_raw_batch* in, khip_batch* out, int64_t* n_errors);
khip_status khip_serde_destroy(khip_serde* s);

/* ---------------------------------------------- serialization (device columns → record bytes) */

/* The output side of GenericKeySerDe / GenericRowSerDe for a sink topic (ksqldb-serde/src/main/
 * java/io/confluent/ksql/serde/GenericKeySerDe.java:95-117, GenericRowSerDe.java), run on the
 * device over columnar rows:
 *   key    the inner key in key_format — KAFKA (kafka/KafkaSerdeFactory.java:42-46: INT 4-byte /
 *          BIGINT 8-byte big-endian, DOUBLE 8-byte IEEE big-endian, STRING UTF-8; one column),
 *          JSON (one column unwrapped = the bare JSON value; several = an object in column order),
 *          DELIMITED (the CSV record of the columns) — then, for a windowed table, Kafka Streams'
 *          TimeWindowedSerializer (inner ++ 8-byte big-endian window start) or
 *          SessionWindowedSerializer (inner ++ 8-byte big-endian window end ++ window start).
 *   value  JSON: Kafka Connect JsonConverter with schemas off (json/KsqlJsonSerdeFactory.java:
 *          158-161) → compact object in column order; DELIMITED: KsqlDelimitedSerializer
 *          (delimited/KsqlDelimitedSerializer.java:59-71; commons-csv 1.4 MINIMAL quoting, null =
 *          empty field); KAFKA: the single column's primitive bytes (a NULL column = a null value).
 *          A tombstone row (the row left the table / a HAVING delete) has a null value.
 * Numbers print as Long.toString / Double.toString (JDK 19+ shortest-decimal specification;
 * non-finite doubles as the JSON strings "NaN" / "Infinity" / "-Infinity", Jackson's default).
 * Group identity in the reference is equality of the serialized key, so the bytes
 * khip_sink_key builds from several GROUP BY columns are also the composite key the aggregate
 * groups by (a KHIP_KEY_UTF8 handle). */
#define KHIP_SINK_MAX_COLS 32
#define KHIP_SINK_SRC_WS (-2)   /* value column source: WINDOWSTART                            */
#define KHIP_SINK_SRC_WE (-3)   /* value column source: WINDOWEND                              */

typedef struct khip_sink_desc {
  int32_t key_format;              /* KHIP_FMT_KAFKA / JSON / DELIMITED                          */
  int32_t n_key_cols;              /* 1..KHIP_SINK_MAX_COLS (KAFKA: 1)                            */
  const int32_t* key_types;        /* KHIP_TYPE_INT32 / INT64 / DOUBLE / STRING                   */
  const char* const* key_names;    /* JSON object field names (several key columns)              */
  int32_t window_kind;             /* KHIP_WINDOW_*: the table's window (NONE: plain key)        */
  int32_t value_format;            /* KHIP_FMT_KAFKA / JSON / DELIMITED                          */
  int32_t n_value_cols;            /* 0..KHIP_SINK_MAX_COLS (KAFKA: 1)                            */
  const int32_t* value_types;      /* KHIP_TYPE_INT32 / INT64 / DOUBLE                            */
  const char* const* value_names;  /* JSON field names, in output column order                   */
  const int32_t* value_src;        /* rows column index, or KHIP_SINK_SRC_WS / KHIP_SINK_SRC_WE   */
  int32_t delimiter;               /* DELIMITED: the delimiter byte (0 = ',')                     */
  int32_t device;
} khip_sink_desc;

typedef struct khip_sink khip_sink;

khip_status khip_sink_create(const khip_sink_desc* desc, khip_sink** out);

/* One GROUP BY column of a batch (same memory kind as the batch). */
typedef struct khip_key_col {
  const void* data;         /* INT32 / INT64 / DOUBLE: n_rows elements                            */
  const int64_t* offsets;   /* STRING: n_rows + 1 offsets into bytes                              */
  const uint8_t* bytes;
  const uint8_t* valid;     /* bitmap, NULL = all valid                                          */
} khip_key_col;

/* GROUP BY columns → the serialized inner key of every row (GroupByParamsFactory.ExpressionGrouper,
 * S/GroupByParamsFactory.java:137-150): key column i is cols[i], of type desc.key_types[i].  A row
 * with any NULL key column gets a null key (the reference drops it, :92-100).  *out = the input
 * batch with its key replaced by these bytes (KHIP_KEY_UTF8 layout, in the batch's memory kind,
 * owned by the handle and valid until its next call); ts, validity and value columns are the
 * input's. */
khip_status khip_sink_key(khip_sink* s, const khip_batch* in, const khip_key_col* cols, khip_batch* out);

/* Rows in khip_snapshot layout (what khip_agg_changes / khip_agg_snapshot write). */
typedef struct khip_sink_rows {
  int64_t n_rows;
  int32_t mem;                     /* KHIP_MEM_HOST or KHIP_MEM_DEVICE (every pointer below)     */
  int32_t key_serialized;          /* 1: key_offsets/key_bytes hold the serialized inner key      */
  const int64_t* key_i64;          /* one INT32 / INT64 key column                                */
  const int64_t* key_offsets;      /* STRING key column or serialized keys: n_rows + 1 offsets    */
  const uint8_t* key_bytes;
  const int64_t* window_start;
  const int64_t* window_end;
  const void* const* col_data;     /* the value sources (agg results); element type from desc     */
  const uint8_t* const* col_null;  /* 1 byte per row, 1 = NULL (entries may be NULL)             */
  const uint8_t* tombstone;        /* 1 byte per row, 1 = delete → null value (may be NULL)      */
} khip_sink_rows;

typedef struct khip_sink_out {
  int32_t mem;                     /* where the buffers below live                                */
  int32_t reserved;
  int64_t key_capacity;            /* bytes                                                       */
  int64_t value_capacity;          /* bytes                                                       */
  int64_t* key_offsets;            /* n_rows + 1 (from 0)                                         */
  uint8_t* key_bytes;
  int64_t* value_offsets;          /* n_rows + 1 (from 0)                                         */
  uint8_t* value_bytes;
  uint8_t* value_null;             /* 1 byte per row: 1 = null value (tombstone)                  */
  int64_t key_len;                 /* out: key bytes written (needed, on KHIP_E_BUFFER)           */
  int64_t value_len;               /* out: value bytes written (needed, on KHIP_E_BUFFER)         */
} khip_sink_out;

/* Serialize rows into sink records (key bytes, value bytes or null).  The encoding runs on the
 * device; host rows are staged in and host outputs copied back.  On KHIP_E_BUFFER key_len /
 * value_len hold the sizes needed and no bytes are written (device offset arrays, the lengths'
 * workspace, are overwritten). */
khip_status khip_sink_encode(khip_sink* s, const khip_sink_rows* rows, khip_sink_out* out);
khip_status khip_sink_sync(khip_sink* s);
khip_status khip_sink_destroy(khip_sink* s);

/* ------------------------------------------------------------ diagnostics */

/* Thread-local message of the last failing call on this thread ("" if none). */
const char* khip_last_error(void);

/* ABI version (KHIP_ABI_VERSION) and the gfx target the kernels were built for. */
int32_t khip_abi_version(void);
const char* khip_build_target(void);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* KSQLDB_HIP_H */
