/*
 * oracle.c — sequential CPU restatement of the ksqlDB hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Parity status: pinned by the
 * reference's QTT golden vectors (tests/golden/, extracted from
 * ksqldb-functional-tests/src/test/resources/query-validation-tests/ JSON files);
 * the 24 h default grace and NaN payload bits are unpinned.
 *
 * Every record is applied one at a time in arrival order, exactly as the Kafka
 * Streams processors do.  Rules and where they come from (paths relative to the
 * ksqlDB root; S/ X/ E/ as in include/ksqldb_hip.h, E/ = ksqldb-engine/src/main/
 * java/io/confluent/ksql/):
 *
 *  R1 drop before the aggregate: null key (Kafka KStreamWindowAggregate /
 *     KStreamAggregate key==null skip; S/GroupByParamsFactory.java:92-100 for
 *     computed keys), null value (S/StreamGroupByBuilderBase.java:102), negative
 *     timestamp (S/timestamp/LoggingTimestampExtractor.java:72-84).  Dropped
 *     records do not advance stream time.
 *  R2 stream time: observedStreamTime = max(observedStreamTime, ts), updated
 *     before the late check; initial -1 (Kafka 3.4 KStreamWindowAggregate).
 *  R3 windows: TimeWindows.windowsFor(ts): ws0 = (max(0, ts - size + adv) / adv)
 *     * adv; ws = ws0, ws0+adv, ... while ws <= ts (call sites
 *     S/StreamAggregateBuilder.java:269-295,328-352).
 *  R4 late drop: window updated iff ws + size > streamTime - grace
 *     (grace: GRACE PERIOD or max(86400000 - size, 0), S/StreamAggregateBuilder.java
 *     :275-277,332-334); with EMIT FINAL and no GRACE PERIOD the analyzer sets 0
 *     (E/analyzer/RewrittenAnalysis.java:65,149-154).  Unwindowed aggregation (StreamAggregateBuilder.java:81-138)
 *     has no windows and no late drop.
 *  R5 entry: created by the first applied record (KudafInitializer.apply,
 *     X/function/udaf/KudafInitializer.java:39-47), even if every aggregate input is
 *     null.  Row time = max(ts) over applied records.
 *  R6 aggregate math (KudafAggregator.apply, X/function/udaf/KudafAggregator.java:56-80):
 *     COUNT: +1 if arg non-null (E/function/udaf/count/CountKudaf.java:37-42);
 *     COUNT(*) = COUNT(ROWTIME), never null (E/analyzer/AggregateAnalyzer.java:339);
 *     SUM INT/BIGINT: wrapping add, null skipped (E/function/udaf/sum/IntegerSumKudaf
 *     .java:25-31, LongSumKudaf.java:25-31); SUM DOUBLE sequential + (DoubleSumKudaf
 *     .java:25-31); MIN/MAX: null identity, compareTo, ties keep the aggregate
 *     (E/function/udaf/BaseComparableKudaf.java:55-66, max/MaxKudaf.java:82,
 *     min/MinKudaf.java:81; Double.compareTo: -0.0 < 0.0, NaN largest);
 *     AVG: {sum (wrapping for INT/BIGINT), count} and map = count==0 ? 0.0 :
 *     (double)sum / (double)count (E/function/udaf/average/AverageUdaf.java:104-128).
 *  R9 retention (window store): a window is visible while ws >= obs - R, obs = the largest
 *     window start put into the store (the store's observedStreamTime, Kafka 3.4 segmented
 *     window stores), R = RETENTION or size + grace (X/runtime/MaterializedFactory.java:47 via
 *     S/StreamAggregateBuilder.java:293,322,350).  Pinned by the EMIT FINAL QTT cases
 *     (Q/suppress.json: expired windows are never emitted); snapshots and pull queries read
 *     the store, so they apply it too.
 *  R10 emission (one commit per push = the record cache flushed at commit,
 *     C/util/KsqlConstants.java:40-41): EMIT CHANGES emits every (key, window) the push
 *     updated with its new value; with HAVING (S/TableFilterBuilder.java:63-75) a row that
 *     fails now but passed before the push is a tombstone, one that failed before and after
 *     is not emitted (Q/having.json:7,25).  EMIT FINAL (S/StreamAggregateBuilder.java:282-285,
 *     EmitStrategy.onWindowClose; Q/suppress.json) emits, once per push whose close time
 *     (streamTime - grace) passed the last emitted one, the windows with start in
 *     [max(0, lastClose - size), close - size] that are still visible (R9) and pass HAVING.
 *  R11 SESSION windows (gap = size_ms; S/StreamAggregateBuilder.java:296-323, Kafka 3.4
 *     KStreamSessionWindowAggregate): per record, the key's visible sessions (end >= streamTime
 *     - retention, retention = gap + grace by default) with end >= ts - gap and start <= ts +
 *     gap merge with [ts, ts] (aggregates combined by KudafAggregator.getMerger, X/function/
 *     udaf/KudafAggregator.java:87-111: COUNT/SUM add, MIN/MAX compare, AVG adds both); the
 *     record is late when the merged session ends before streamTime - grace - gap; otherwise the
 *     merged-away sessions are deleted (tombstones) and the merged one is written with the
 *     record applied.  Row time = session end.  Pinned by Q/session-windows.json:4,45 (late
 *     drop and expiry with GRACE PERIOD); the default grace max(24h - gap, 0) is unpinned.
 *     EMIT FINAL on sessions (S/StreamAggregateBuilder.java:310-312, sessionWindowedKStream
 *     .emitStrategy(onWindowClose()); Kafka 3.4 KStreamSessionWindowAggregate.maybeForwardFinalResult):
 *     after every record that reaches the processor, with windowCloseTime = streamTime - grace -
 *     gap: when it passed the last emitted close time (or none was emitted yet) and close - 1 >= 0,
 *     every session in the store whose END lies in [max(0, lastClose), close - 1] is emitted once
 *     (row time = its end; HAVING applied as for time windows) and lastClose = close.  The time-
 *     ordered session store keeps sessions until their segment expires, so the emission does not
 *     apply R9's exact expiry; merges do (as EMIT CHANGES).  Pinned by Q/suppress.json "should
 *     support final results for session windows" (emit interval 0: a check after every record).
 *  R12 table aggregation (S/TableAggregateBuilder.java:54-108 over S/TableGroupByBuilderBase.java
 *     :62-111; Kafka 3.4 KTableRepartitionMap + KTableAggregate): the source table keeps the latest
 *     row per PRIMARY KEY (a tombstone deletes it); each accepted record first undoes the key's
 *     previous row from its group (TableUdaf.undo via KudafUndoAggregator, X/function/udaf/
 *     KudafUndoAggregator.java:29-55: COUNT -1 if non-null, SUM subtracts (wrapping), AVG
 *     {sum - x, count - 1}; E/function/udaf/count/CountKudaf.java:60-65, sum/(Integer,Long,Double)SumKudaf.java:44,
 *     average/AverageUdaf.java:140-150) when that row had a non-null GROUP BY value, then applies
 *     the new row to its group (created if absent).  Groups are never deleted (count back to zero,
 *     Q/count.json); group row time = max ts of the records touching it.
 *  R7 join: table keeps the latest non-null value per key, a null value deletes;
 *     stream records with null key / null value / negative ts are dropped; lookup
 *     against the table as of that point; INNER emits on hit, LEFT always
 *     (S/StreamTableJoinBuilder.java:77-86, S/KsqlValueJoiner.java:41-63).
 */
#define _GNU_SOURCE
#include "oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define ORACLE_DAY_MS 86400000LL

static int bit_get(const uint8_t* bm, int64_t i) {
  return bm == NULL ? 1 : (bm[i >> 3] >> (i & 7)) & 1;
}

#define KHIP_MAX_COLS_ORACLE 16

static int64_t read_col_raw(const khip_batch* b, int c, int type, int64_t r) {
  int64_t v = 0;
  if (type == KHIP_TYPE_INT32) v = ((const int32_t*)b->col_data[c])[r];
  else memcpy(&v, (const char*)b->col_data[c] + 8 * r, 8);
  return v;
}

uint64_t oracle_splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

int32_t oracle_murmur2(const uint8_t* data, int32_t len) {
  const uint32_t m = 0x5bd1e995u;
  uint32_t h = 0x9747b28cu ^ (uint32_t)len;
  int32_t i;
  for (i = 0; i + 4 <= len; i += 4) {
    uint32_t k = (uint32_t)data[i] | ((uint32_t)data[i + 1] << 8) | ((uint32_t)data[i + 2] << 16) |
                 ((uint32_t)data[i + 3] << 24);
    k *= m;
    k ^= k >> 24;
    k *= m;
    h *= m;
    h ^= k;
  }
  switch (len & 3) {
    case 3: h ^= (uint32_t)data[(len & ~3) + 2] << 16; /* fall through */
    case 2: h ^= (uint32_t)data[(len & ~3) + 1] << 8;  /* fall through */
    case 1:
      h ^= (uint32_t)data[len & ~3];
      h *= m;
  }
  h ^= h >> 13;
  h *= m;
  h ^= h >> 15;
  return (int32_t)h;
}

void oracle_kafka_partition(const int64_t* keys, int64_t n, int32_t key_bytes, int32_t n_parts, int32_t* out) {
  int64_t i;
  for (i = 0; i < n; i++) {
    uint8_t b[8];
    uint64_t v = (uint64_t)keys[i];
    int32_t j;
    for (j = 0; j < key_bytes; j++) b[j] = (uint8_t)(v >> (8 * (key_bytes - 1 - j)));
    out[i] = (int32_t)(((uint32_t)oracle_murmur2(b, key_bytes) & 0x7fffffffu) % (uint32_t)n_parts);
  }
}

static uint64_t mix64(uint64_t h) {
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdULL;
  h ^= h >> 33;
  h *= 0xc4ceb9fe1a85ec53ULL;
  h ^= h >> 33;
  return h;
}

static uint64_t hash_bytes(const uint8_t* p, int64_t n) {
  uint64_t h = 1469598103934665603ULL;
  for (int64_t i = 0; i < n; i++) h = (h ^ p[i]) * 1099511628211ULL;
  return mix64(h ^ (uint64_t)n);
}

/* Java Double.compare(a, b) (doubleToLongBits canonicalizes NaN). */
static int64_t java_double_bits(double d) {
  int64_t b;
  if (isnan(d)) return 0x7ff8000000000000LL;
  memcpy(&b, &d, 8);
  return b;
}
static int java_double_compare(double a, double b) {
  if (a < b) return -1;
  if (a > b) return 1;
  int64_t x = java_double_bits(a), y = java_double_bits(b);
  return x == y ? 0 : (x < y ? -1 : 1);
}

/* ------------------------------------------------------------- key dictionary */

typedef struct {
  int64_t* off;  /* per key id: arena offset */
  int64_t* len;
  uint8_t* arena;
  int64_t arena_len, arena_cap;
  int64_t n, cap;
  int64_t* slots; /* open addressing: key id or -1 */
  uint64_t* slot_hash;
  int64_t nslots;
} strdict;

static void strdict_init(strdict* d) {
  memset(d, 0, sizeof(*d));
  d->nslots = 1024;
  d->slots = (int64_t*)malloc(sizeof(int64_t) * d->nslots);
  d->slot_hash = (uint64_t*)malloc(sizeof(uint64_t) * d->nslots);
  for (int64_t i = 0; i < d->nslots; i++) d->slots[i] = -1;
}

static void strdict_free(strdict* d) {
  free(d->off); free(d->len); free(d->arena); free(d->slots); free(d->slot_hash);
}

static void strdict_grow(strdict* d) {
  int64_t ns = d->nslots * 2;
  int64_t* s = (int64_t*)malloc(sizeof(int64_t) * ns);
  uint64_t* sh = (uint64_t*)malloc(sizeof(uint64_t) * ns);
  for (int64_t i = 0; i < ns; i++) s[i] = -1;
  for (int64_t i = 0; i < d->nslots; i++) {
    if (d->slots[i] < 0) continue;
    uint64_t h = d->slot_hash[i];
    int64_t j = (int64_t)(h & (uint64_t)(ns - 1));
    while (s[j] >= 0) j = (j + 1) & (ns - 1);
    s[j] = d->slots[i];
    sh[j] = h;
  }
  free(d->slots); free(d->slot_hash);
  d->slots = s; d->slot_hash = sh; d->nslots = ns;
}

static int64_t strdict_intern(strdict* d, const uint8_t* p, int64_t n) {
  if (2 * (d->n + 1) > d->nslots) strdict_grow(d);
  uint64_t h = hash_bytes(p, n);
  int64_t j = (int64_t)(h & (uint64_t)(d->nslots - 1));
  while (d->slots[j] >= 0) {
    int64_t id = d->slots[j];
    if (d->slot_hash[j] == h && d->len[id] == n &&
        (n == 0 || memcmp(d->arena + d->off[id], p, (size_t)n) == 0))
      return id;
    j = (j + 1) & (d->nslots - 1);
  }
  if (d->n == d->cap) {
    d->cap = d->cap ? d->cap * 2 : 1024;
    d->off = (int64_t*)realloc(d->off, sizeof(int64_t) * d->cap);
    d->len = (int64_t*)realloc(d->len, sizeof(int64_t) * d->cap);
  }
  while (d->arena_len + n > d->arena_cap) {
    d->arena_cap = d->arena_cap ? d->arena_cap * 2 : 4096;
    d->arena = (uint8_t*)realloc(d->arena, (size_t)d->arena_cap);
  }
  int64_t id = d->n++;
  d->off[id] = d->arena_len;
  d->len[id] = n;
  if (n) memcpy(d->arena + d->arena_len, p, (size_t)n);
  d->arena_len += n;
  d->slots[j] = id;
  d->slot_hash[j] = h;
  return id;
}

/* ------------------------------------------------------------ aggregate state */

typedef struct {
  int64_t i;   /* COUNT, SUM INT/BIGINT (wrapping), MIN/MAX integer, AVG int sum */
  double d;    /* SUM DOUBLE, MIN/MAX DOUBLE, AVG double sum */
  int64_t cnt; /* AVG count */
  int has;     /* MIN/MAX: non-null */
} agg_state;

typedef struct {
  int64_t key; /* INT64 key, or dictionary id for UTF8 */
  int64_t ws;
  int64_t rowtime;
  agg_state* st; /* n_aggs */
  int64_t we;          /* SESSION: session end (time windows: ws + size)       */
  int dead;            /* SESSION: merged away (kept for the push's tombstones) */
  int64_t born_epoch;  /* push that created the entry                          */
  int64_t touch_epoch; /* last push that updated it                            */
  int old_pass;        /* HAVING before the push's first update (R10)          */
} entry;

struct oracle_agg {
  khip_agg_desc d;
  int32_t* col_types;
  khip_agg_spec* aggs;
  int64_t grace;
  int64_t stream_time;
  strdict dict;
  entry* e;
  int64_t n, cap;
  int64_t* slots;
  int64_t nslots;
  int64_t retention;  /* R9 (windowed)                                            */
  int64_t obs_ws;     /* largest window start put (-1: none)                      */
  int64_t epoch;      /* pushes so far                                            */
  int64_t* touched;   /* entries the current push updated                         */
  int64_t n_touched, cap_touched;
  int64_t* chg;       /* the last push's emitted rows (entry index), sorted       */
  uint8_t* chg_tomb;
  int64_t n_chg, cap_chg;
  int64_t st_before;  /* stream time before the current push                      */
  /* SESSION: per key, the indices of its live sessions (open addressing on the key) */
  int64_t* sk_key;
  int64_t** sk_list;
  int64_t* sk_n;
  int64_t* sk_cap;
  int64_t sk_slots, sk_used;
  /* SESSION + EMIT FINAL: live sessions by end (a min-heap of (end, entry)), the last emitted
   * close time, and the sessions the current push emitted */
  int64_t* fh_end;
  int64_t* fh_idx;
  int64_t fh_n, fh_cap;
  int64_t last_close;
  int64_t* fin_emit;
  int64_t n_fin, cap_fin;
  int64_t* stmax;     /* the push's stream-time maxima, in arrival order           */
  int64_t n_stmax, cap_stmax;
  int own_stmax;      /* stmax is this handle's (0: borrowed from the sharded push)  */
  /* R12 table source: the source table's current rows by PRIMARY KEY (id) */
  int src_key_type;   /* -1 until the first push_table                            */
  strdict src_dict;
  int64_t* src_key;   /* per source row */
  uint8_t* src_live;
  uint8_t* src_gvalid;
  int64_t* src_gkey;
  int64_t* src_vals;  /* n_cols raw words per source row */
  uint8_t* src_vvalid;
  int64_t src_n, src_cap;
  int64_t* src_slots;
  int64_t src_nslots;
};

static uint64_t entry_hash(int64_t key, int64_t ws) {
  return mix64((uint64_t)key ^ mix64((uint64_t)ws + 0x9E3779B97F4A7C15ULL));
}

static void slots_rebuild(oracle_agg* a, int64_t ns) {
  free(a->slots);
  a->nslots = ns;
  a->slots = (int64_t*)malloc(sizeof(int64_t) * ns);
  for (int64_t i = 0; i < ns; i++) a->slots[i] = -1;
  for (int64_t k = 0; k < a->n; k++) {
    int64_t j = (int64_t)(entry_hash(a->e[k].key, a->e[k].ws) & (uint64_t)(ns - 1));
    while (a->slots[j] >= 0) j = (j + 1) & (ns - 1);
    a->slots[j] = k;
  }
}

static entry* find_or_create(oracle_agg* a, int64_t key, int64_t ws) {
  if (2 * (a->n + 1) > a->nslots) slots_rebuild(a, a->nslots * 2);
  int64_t j = (int64_t)(entry_hash(key, ws) & (uint64_t)(a->nslots - 1));
  while (a->slots[j] >= 0) {
    entry* x = &a->e[a->slots[j]];
    if (x->key == key && x->ws == ws) return x;
    j = (j + 1) & (a->nslots - 1);
  }
  if (a->n == a->cap) {
    a->cap = a->cap ? a->cap * 2 : 1024;
    a->e = (entry*)realloc(a->e, sizeof(entry) * a->cap);
  }
  entry* x = &a->e[a->n];
  a->slots[j] = a->n++;
  x->key = key;
  x->ws = ws;
  x->rowtime = INT64_MIN;
  x->st = (agg_state*)calloc((size_t)(a->d.n_aggs > 0 ? a->d.n_aggs : 1), sizeof(agg_state));
  x->born_epoch = a->epoch;
  x->touch_epoch = -1;
  x->old_pass = 0;
  x->we = ws + a->d.size_ms;
  x->dead = 0;
  return x;
}

static int having_pass(const oracle_agg* a, const khip_having* h, const entry* x);

static const khip_having* query_having(const oracle_agg* a) {
  return a->d.has_having ? &a->d.having : NULL;
}

/* R10: remember the entry's HAVING result before this push's first update to it. */
static void touch(oracle_agg* a, entry* x) {
  if (x->touch_epoch == a->epoch) return;
  x->touch_epoch = a->epoch;
  x->old_pass = x->born_epoch == a->epoch ? 0 : having_pass(a, query_having(a), x);
  if (a->n_touched == a->cap_touched) {
    a->cap_touched = a->cap_touched ? a->cap_touched * 2 : 1024;
    a->touched = (int64_t*)realloc(a->touched, sizeof(int64_t) * a->cap_touched);
  }
  a->touched[a->n_touched++] = x - a->e;
}

/* R9: first visible window start (INT64_MIN: everything visible). */
static int64_t visible_from(const oracle_agg* a) {
  if (a->d.window_kind == KHIP_WINDOW_NONE || a->obs_ws < 0) return INT64_MIN;
  return a->obs_ws - a->retention;
}

/* R9 for one entry: time windows by start, sessions by end (the session store's segment time). */
static int entry_visible(const oracle_agg* a, const entry* x) {
  if (x->dead) return 0;
  const int64_t vis = visible_from(a);
  return (a->d.window_kind == KHIP_WINDOW_SESSION ? x->we : x->ws) >= vis;
}

static int valid_desc(const khip_agg_desc* d) {
  if (d->window_kind != KHIP_WINDOW_NONE && d->window_kind != KHIP_WINDOW_TUMBLING &&
      d->window_kind != KHIP_WINDOW_HOPPING && d->window_kind != KHIP_WINDOW_SESSION)
    return 0;
  if (d->window_kind != KHIP_WINDOW_NONE) {
    if (d->size_ms <= 0) return 0;
    if (d->window_kind == KHIP_WINDOW_HOPPING &&
        (d->advance_ms <= 0 || d->advance_ms > d->size_ms))
      return 0;
  }
  if (d->key_type != KHIP_KEY_INT64 && d->key_type != KHIP_KEY_UTF8) return 0;
  if (d->n_aggs < 0 || d->n_cols < 0) return 0;
  for (int i = 0; i < d->n_aggs; i++) {
    const khip_agg_spec* s = &d->aggs[i];
    if (s->kind < KHIP_AGG_COUNT_STAR || s->kind > KHIP_AGG_AVG) return 0;
    if (s->kind != KHIP_AGG_COUNT_STAR && (s->arg_col < 0 || s->arg_col >= d->n_cols))
      return 0;
  }
  for (int c = 0; c < d->n_cols; c++)
    if (d->col_types[c] < KHIP_TYPE_INT32 || d->col_types[c] > KHIP_TYPE_DOUBLE) return 0;
  if (d->emit != KHIP_EMIT_CHANGES && d->emit != KHIP_EMIT_FINAL) return 0;
  if (d->emit == KHIP_EMIT_FINAL && d->window_kind == KHIP_WINDOW_NONE) return 0;
  if (d->has_having && (d->having.agg_index < 0 || d->having.agg_index >= d->n_aggs)) return 0;
  if (d->flags & KHIP_FLAG_TABLE_SOURCE) { /* R12: unwindowed, undoable aggregates only */
    if (d->window_kind != KHIP_WINDOW_NONE) return 0;
    for (int i = 0; i < d->n_aggs; i++)
      if (d->aggs[i].kind == KHIP_AGG_MIN || d->aggs[i].kind == KHIP_AGG_MAX) return 0;
  }
  return 1;
}

khip_status oracle_agg_create(const khip_agg_desc* desc, oracle_agg** out) {
  if (!desc || !out || !valid_desc(desc)) return KHIP_E_INVALID;
  oracle_agg* a = (oracle_agg*)calloc(1, sizeof(oracle_agg));
  a->d = *desc;
  a->col_types = (int32_t*)malloc(sizeof(int32_t) * (desc->n_cols + 1));
  memcpy(a->col_types, desc->col_types, sizeof(int32_t) * desc->n_cols);
  a->aggs = (khip_agg_spec*)malloc(sizeof(khip_agg_spec) * (desc->n_aggs + 1));
  memcpy(a->aggs, desc->aggs, sizeof(khip_agg_spec) * desc->n_aggs);
  a->d.col_types = a->col_types;
  a->d.aggs = a->aggs;
  if (desc->window_kind == KHIP_WINDOW_TUMBLING) a->d.advance_ms = desc->size_ms;
  if (desc->window_kind == KHIP_WINDOW_NONE) {
    a->grace = 0;
  } else if (desc->grace_ms < 0 && desc->emit == KHIP_EMIT_FINAL) {
    a->grace = 0; /* EMIT FINAL without GRACE PERIOD: the analyzer's zero grace (R4) */
  } else if (desc->grace_ms < 0) {
    int64_t g = ORACLE_DAY_MS - desc->size_ms;
    a->grace = g > 0 ? g : 0;
  } else {
    a->grace = desc->grace_ms;
  }
  if (desc->window_kind == KHIP_WINDOW_SESSION) a->d.advance_ms = 1;  /* obs = stream time itself */
  if (desc->window_kind != KHIP_WINDOW_NONE) {
    const int64_t min_r = desc->size_ms + a->grace;
    if (desc->retention_ms == KHIP_RETENTION_DEFAULT) a->retention = min_r;
    else if (desc->retention_ms < min_r) { free(a->col_types); free(a->aggs); free(a); return KHIP_E_INVALID; }
    else a->retention = desc->retention_ms;
  }
  a->obs_ws = -1;
  a->last_close = -1;
  a->own_stmax = 1;
  a->src_key_type = -1;
  a->stream_time = -1;
  strdict_init(&a->dict);
  a->nslots = 1024;
  a->slots = NULL;
  slots_rebuild(a, 1024);
  *out = a;
  return KHIP_OK;
}

static void apply_aggs(oracle_agg* a, entry* x, const khip_batch* b, int64_t r) {
  for (int i = 0; i < a->d.n_aggs; i++) {
    const khip_agg_spec* s = &a->aggs[i];
    agg_state* st = &x->st[i];
    if (s->kind == KHIP_AGG_COUNT_STAR) {
      st->i += 1;
      continue;
    }
    int c = s->arg_col;
    int t = a->col_types[c];
    if (!bit_get(b->col_valid ? b->col_valid[c] : NULL, r)) continue; /* null input */
    int64_t iv = 0;
    double dv = 0.0;
    if (t == KHIP_TYPE_INT32) iv = ((const int32_t*)b->col_data[c])[r];
    else if (t == KHIP_TYPE_INT64) iv = ((const int64_t*)b->col_data[c])[r];
    else dv = ((const double*)b->col_data[c])[r];
    switch (s->kind) {
      case KHIP_AGG_COUNT:
        st->i += 1;
        break;
      case KHIP_AGG_SUM:
      case KHIP_AGG_AVG:
        if (t == KHIP_TYPE_INT32)
          st->i = (int64_t)(int32_t)((uint32_t)(int32_t)st->i + (uint32_t)(int32_t)iv);
        else if (t == KHIP_TYPE_INT64)
          st->i = (int64_t)((uint64_t)st->i + (uint64_t)iv);
        else
          st->d = st->d + dv;
        if (s->kind == KHIP_AGG_AVG) st->cnt += 1;
        break;
      case KHIP_AGG_MIN:
      case KHIP_AGG_MAX: {
        int take;
        if (!st->has) {
          take = 1;
        } else if (t == KHIP_TYPE_DOUBLE) {
          int c2 = java_double_compare(dv, st->d);
          take = s->kind == KHIP_AGG_MAX ? c2 > 0 : c2 < 0;
        } else {
          take = s->kind == KHIP_AGG_MAX ? iv > st->i : iv < st->i;
        }
        if (take) {
          st->has = 1;
          st->i = iv;
          st->d = dv;
        }
        break;
      }
      default:
        break;
    }
  }
}

static void finish_push(oracle_agg* a);
static void stmax_add(oracle_agg* a, int64_t st);

/* ------------------------------------------------------------- SESSION windows (R11) */

static int64_t* sk_lookup(oracle_agg* a, int64_t key) { /* the key's list slot (created) */
  if (2 * (a->sk_used + 1) > a->sk_slots) {
    const int64_t ns = a->sk_slots ? a->sk_slots * 2 : 1024;
    int64_t* nk = (int64_t*)malloc(sizeof(int64_t) * ns);
    int64_t** nl = (int64_t**)calloc((size_t)ns, sizeof(int64_t*));
    int64_t* nn = (int64_t*)calloc((size_t)ns, sizeof(int64_t));
    int64_t* nc = (int64_t*)calloc((size_t)ns, sizeof(int64_t));
    char* used = (char*)calloc((size_t)ns, 1);
    for (int64_t i = 0; i < a->sk_slots; i++) {
      if (!a->sk_cap[i]) continue;
      int64_t j = (int64_t)(mix64((uint64_t)a->sk_key[i]) & (uint64_t)(ns - 1));
      while (used[j]) j = (j + 1) & (ns - 1);
      used[j] = 1;
      nk[j] = a->sk_key[i];
      nl[j] = a->sk_list[i];
      nn[j] = a->sk_n[i];
      nc[j] = a->sk_cap[i];
    }
    free(used);
    free(a->sk_key); free(a->sk_list); free(a->sk_n); free(a->sk_cap);
    a->sk_key = nk; a->sk_list = nl; a->sk_n = nn; a->sk_cap = nc; a->sk_slots = ns;
  }
  int64_t j = (int64_t)(mix64((uint64_t)key) & (uint64_t)(a->sk_slots - 1));
  while (a->sk_cap[j] && a->sk_key[j] != key) j = (j + 1) & (a->sk_slots - 1);
  if (!a->sk_cap[j]) {
    a->sk_key[j] = key;
    a->sk_cap[j] = 4;
    a->sk_n[j] = 0;
    a->sk_list[j] = (int64_t*)malloc(sizeof(int64_t) * 4);
    a->sk_used++;
  }
  return &a->sk_n[j];
}

static entry* new_entry(oracle_agg* a, int64_t key, int64_t ws, int64_t we) {
  if (a->n == a->cap) {
    a->cap = a->cap ? a->cap * 2 : 1024;
    a->e = (entry*)realloc(a->e, sizeof(entry) * a->cap);
  }
  entry* x = &a->e[a->n++];
  memset(x, 0, sizeof(*x));
  x->key = key;
  x->ws = ws;
  x->we = we;
  x->rowtime = INT64_MIN;
  x->st = (agg_state*)calloc((size_t)(a->d.n_aggs > 0 ? a->d.n_aggs : 1), sizeof(agg_state));
  x->born_epoch = a->epoch;
  x->touch_epoch = -1;
  return x;
}

/* KudafAggregator.getMerger (X/function/udaf/KudafAggregator.java:87-111): dst = merge(dst, src). */
static void merge_state(oracle_agg* a, agg_state* dst, const agg_state* src) {
  for (int i = 0; i < a->d.n_aggs; i++) {
    const khip_agg_spec* sp = &a->aggs[i];
    const int t = sp->kind == KHIP_AGG_COUNT_STAR ? KHIP_TYPE_INT64 : a->col_types[sp->arg_col];
    agg_state* d = &dst[i];
    const agg_state* x = &src[i];
    switch (sp->kind) {
      case KHIP_AGG_COUNT_STAR:
      case KHIP_AGG_COUNT: d->i += x->i; break;
      case KHIP_AGG_SUM:
      case KHIP_AGG_AVG:
        if (t == KHIP_TYPE_INT32) d->i = (int64_t)(int32_t)((uint32_t)(int32_t)d->i + (uint32_t)(int32_t)x->i);
        else if (t == KHIP_TYPE_INT64) d->i = (int64_t)((uint64_t)d->i + (uint64_t)x->i);
        else d->d = d->d + x->d;
        d->cnt += x->cnt;
        break;
      case KHIP_AGG_MIN:
      case KHIP_AGG_MAX: { /* BaseComparableKudaf.merge = aggregate(aggOne, aggTwo): ties keep aggTwo */
        if (!x->has) break;
        int take = !d->has;
        if (!take) {
          if (t == KHIP_TYPE_DOUBLE) {
            const int c = java_double_compare(d->d, x->d);
            take = sp->kind == KHIP_AGG_MAX ? !(c > 0) : !(c < 0);
          } else {
            take = sp->kind == KHIP_AGG_MAX ? !(d->i > x->i) : !(d->i < x->i);
          }
        }
        if (take) *d = *x;
        break;
      }
    }
  }
}

/* SESSION + EMIT FINAL: a binary min-heap of the sessions by end. */
static void fh_push(oracle_agg* a, int64_t end, int64_t idx) {
  if (a->fh_n == a->fh_cap) {
    a->fh_cap = a->fh_cap ? a->fh_cap * 2 : 1024;
    a->fh_end = (int64_t*)realloc(a->fh_end, sizeof(int64_t) * a->fh_cap);
    a->fh_idx = (int64_t*)realloc(a->fh_idx, sizeof(int64_t) * a->fh_cap);
  }
  int64_t i = a->fh_n++;
  while (i > 0) {
    const int64_t p = (i - 1) / 2;
    if (a->fh_end[p] <= end) break;
    a->fh_end[i] = a->fh_end[p];
    a->fh_idx[i] = a->fh_idx[p];
    i = p;
  }
  a->fh_end[i] = end;
  a->fh_idx[i] = idx;
}

static int64_t fh_pop(oracle_agg* a) { /* the entry of the smallest end */
  const int64_t top = a->fh_idx[0];
  const int64_t e = a->fh_end[--a->fh_n], x = a->fh_idx[a->fh_n];
  int64_t i = 0;
  for (;;) {
    int64_t c = 2 * i + 1;
    if (c >= a->fh_n) break;
    if (c + 1 < a->fh_n && a->fh_end[c + 1] < a->fh_end[c]) c++;
    if (a->fh_end[c] >= e) break;
    a->fh_end[i] = a->fh_end[c];
    a->fh_idx[i] = a->fh_idx[c];
    i = c;
  }
  if (a->fh_n) {
    a->fh_end[i] = e;
    a->fh_idx[i] = x;
  }
  return top;
}

/* KStreamSessionWindowAggregate.maybeForwardFinalResult after one record (emit interval 0):
 * sessions of the store with end in [max(0, lastClose), close - 1], once.  A session merged away
 * before its close passed is no longer in the store (dead): never emitted. */
static void session_emit_final(oracle_agg* a, int64_t st) {
  const int64_t close = st - a->grace - a->d.size_ms;
  if (!(a->last_close == -1 || a->last_close < close)) return;
  if (close - 1 < 0) return;
  while (a->fh_n > 0 && a->fh_end[0] <= close - 1) {
    const int64_t k = fh_pop(a);
    const entry* x = &a->e[k];
    if (x->dead || x->we < (a->last_close > 0 ? a->last_close : 0)) continue;
    if (a->n_fin == a->cap_fin) {
      a->cap_fin = a->cap_fin ? a->cap_fin * 2 : 1024;
      a->fin_emit = (int64_t*)realloc(a->fin_emit, sizeof(int64_t) * a->cap_fin);
    }
    a->fin_emit[a->n_fin++] = k;
  }
  a->last_close = close;
}

/* One record of a SESSION aggregation (R11); st = the task's stream time after the record. */
static void session_apply(oracle_agg* a, int64_t key, int64_t ts, int64_t st, const khip_batch* b, int64_t r,
                          int64_t* applied, int64_t* late) {
  const int64_t gap = a->d.size_ms;
  const int64_t close = st - a->grace - gap, vis = st - a->retention;
  const int64_t j = sk_lookup(a, key) - a->sk_n;
  int64_t* L = a->sk_list[j];
  int64_t n = a->sk_n[j];
  int64_t mstart = ts, mend = ts, nover = 0, same = -1;
  for (int64_t k = 0; k < n; k++) {
    const entry* x = &a->e[L[k]];
    if (x->we < vis) continue; /* expired from the session store: invisible */
    if (x->we >= ts - gap && x->ws <= ts + gap) {
      nover++;
      if (x->ws < mstart) mstart = x->ws;
      if (x->we > mend) mend = x->we;
      if (x->ws == ts && x->we == ts) same = L[k];
    }
  }
  if (mend < close) {
    (*late)++;
    return;
  }
  (*applied)++;
  if (mstart == ts && mend == ts && same >= 0) { /* the session [ts, ts] itself: update in place */
    entry* x = &a->e[same];
    touch(a, x);
    apply_aggs(a, x, b, r);
    x->rowtime = x->we;
    return;
  }
  entry* nx = new_entry(a, key, mstart, mend);
  const int64_t ni = nx - a->e;
  if (a->d.emit == KHIP_EMIT_FINAL) fh_push(a, mend, ni);
  /* merge the overlapping sessions in store order (by end), delete them */
  int64_t m = 0;
  for (int64_t k = 0; k < n; k++) {
    entry* x = &a->e[L[k]];
    if (x->we >= vis && x->we >= ts - gap && x->ws <= ts + gap) {
      touch(a, x);
      merge_state(a, a->e[ni].st, x->st);
      x->dead = 1;
    } else {
      L[m++] = L[k];
    }
  }
  nx = &a->e[ni];
  apply_aggs(a, nx, b, r);
  nx->rowtime = mend;
  touch(a, nx);
  if (m == a->sk_cap[j]) {
    a->sk_cap[j] *= 2;
    a->sk_list[j] = (int64_t*)realloc(a->sk_list[j], sizeof(int64_t) * a->sk_cap[j]);
  }
  a->sk_list[j][m++] = ni;
  a->sk_n[j] = m;
}

khip_status oracle_agg_push(oracle_agg* a, const khip_batch* b, khip_batch_stats* stats) {
  if (!a || !b || b->mem != KHIP_MEM_HOST || b->n_rows < 0) return KHIP_E_INVALID;
  if (b->n_cols < a->d.n_cols || (a->d.flags & KHIP_FLAG_TABLE_SOURCE)) return KHIP_E_INVALID;
  khip_batch_stats s;
  memset(&s, 0, sizeof(s));
  s.rows_in = b->n_rows;
  const int windowed = a->d.window_kind != KHIP_WINDOW_NONE;
  const int64_t size = a->d.size_ms, adv = a->d.advance_ms;
  a->epoch++;
  a->n_touched = 0;
  a->st_before = a->stream_time;
  a->n_stmax = 0;
  a->n_fin = 0;
  for (int64_t r = 0; r < b->n_rows; r++) {
    if (!bit_get(b->key_valid, r)) { s.dropped_null_key++; continue; }
    if (!bit_get(b->row_valid, r)) { s.dropped_null_row++; continue; }
    int64_t ts = b->ts[r];
    if (ts < 0) { s.dropped_bad_ts++; continue; }
    s.rows_accepted++;
    int64_t key;
    if (a->d.key_type == KHIP_KEY_INT64) {
      key = b->key_i64[r];
    } else {
      int64_t o0 = b->key_offsets[r], o1 = b->key_offsets[r + 1];
      key = strdict_intern(&a->dict, b->key_bytes + o0, o1 - o0);
    }
    if (!windowed) {
      entry* x = find_or_create(a, key, 0);
      touch(a, x);
      if (ts > x->rowtime) x->rowtime = ts;
      apply_aggs(a, x, b, r);
      s.windows_applied++;
      if (ts > a->stream_time) a->stream_time = ts;
      continue;
    }
    if (a->d.window_kind == KHIP_WINDOW_SESSION) {
      if (ts > a->stream_time) {
        a->stream_time = ts;
        stmax_add(a, ts);
      }
      session_apply(a, key, ts, a->stream_time, b, r, &s.windows_applied, &s.windows_late);
      a->obs_ws = a->stream_time; /* every stream-time maximum is put into the session store */
      if (a->d.emit == KHIP_EMIT_FINAL) session_emit_final(a, a->stream_time);
      continue;
    }
    if (ts > a->stream_time) { /* R2: before the check */
      a->stream_time = ts;
      stmax_add(a, ts);
    }
    const int64_t close_time = a->stream_time - a->grace;
    int64_t lo = ts - size + adv;
    if (lo < 0) lo = 0;
    for (int64_t ws = (lo / adv) * adv; ws <= ts; ws += adv) {
      if (ws + size > close_time) {
        entry* x = find_or_create(a, key, ws);
        touch(a, x);
        if (ts > x->rowtime) x->rowtime = ts;
        apply_aggs(a, x, b, r);
        s.windows_applied++;
        if (ws > a->obs_ws) a->obs_ws = ws;
      } else {
        s.windows_late++;
      }
    }
  }
  s.stream_time = a->stream_time;
  finish_push(a);
  if (stats) *stats = s;
  return KHIP_OK;
}

/* ------------------------------------------------------------- table aggregation (R12) */

/* Apply (sign +1: KudafAggregator.apply) or undo (sign -1: KudafUndoAggregator.apply) one row given
 * as raw column words + validity. */
static void table_row_aggs(oracle_agg* a, entry* x, const int64_t* raw, const uint8_t* valid, int sign) {
  for (int i = 0; i < a->d.n_aggs; i++) {
    const khip_agg_spec* sp = &a->aggs[i];
    agg_state* st = &x->st[i];
    if (sp->kind == KHIP_AGG_COUNT_STAR) { /* COUNT(ROWTIME): never null */
      st->i = (int64_t)((uint64_t)st->i + (uint64_t)(int64_t)sign);
      continue;
    }
    const int c = sp->arg_col, t = a->col_types[c];
    if (!valid[c]) continue; /* null argument: aggregate unchanged (undo too) */
    switch (sp->kind) {
      case KHIP_AGG_COUNT: st->i += sign; break;
      case KHIP_AGG_SUM:
      case KHIP_AGG_AVG:
        if (t == KHIP_TYPE_INT32) {
          const uint32_t v = (uint32_t)(int32_t)raw[c];
          st->i = (int64_t)(int32_t)(sign > 0 ? (uint32_t)(int32_t)st->i + v : (uint32_t)(int32_t)st->i - v);
        } else if (t == KHIP_TYPE_INT64) {
          st->i = (int64_t)(sign > 0 ? (uint64_t)st->i + (uint64_t)raw[c] : (uint64_t)st->i - (uint64_t)raw[c]);
        } else {
          double v;
          memcpy(&v, &raw[c], 8);
          st->d = sign > 0 ? st->d + v : st->d - v;
        }
        if (sp->kind == KHIP_AGG_AVG) st->cnt += sign;
        break;
      default:
        break;
    }
  }
}

static int64_t src_find_or_add(oracle_agg* a, int64_t key) {
  if (2 * (a->src_n + 1) > a->src_nslots) {
    const int64_t ns = a->src_nslots ? a->src_nslots * 2 : 1024;
    free(a->src_slots);
    a->src_slots = (int64_t*)malloc(sizeof(int64_t) * ns);
    for (int64_t i = 0; i < ns; i++) a->src_slots[i] = -1;
    a->src_nslots = ns;
    for (int64_t r = 0; r < a->src_n; r++) {
      int64_t j = (int64_t)(mix64((uint64_t)a->src_key[r]) & (uint64_t)(ns - 1));
      while (a->src_slots[j] >= 0) j = (j + 1) & (ns - 1);
      a->src_slots[j] = r;
    }
  }
  int64_t j = (int64_t)(mix64((uint64_t)key) & (uint64_t)(a->src_nslots - 1));
  while (a->src_slots[j] >= 0) {
    if (a->src_key[a->src_slots[j]] == key) return a->src_slots[j];
    j = (j + 1) & (a->src_nslots - 1);
  }
  if (a->src_n == a->src_cap) {
    const int nc = a->d.n_cols > 0 ? a->d.n_cols : 1;
    a->src_cap = a->src_cap ? a->src_cap * 2 : 1024;
    a->src_key = (int64_t*)realloc(a->src_key, sizeof(int64_t) * a->src_cap);
    a->src_live = (uint8_t*)realloc(a->src_live, (size_t)a->src_cap);
    a->src_gvalid = (uint8_t*)realloc(a->src_gvalid, (size_t)a->src_cap);
    a->src_gkey = (int64_t*)realloc(a->src_gkey, sizeof(int64_t) * a->src_cap);
    a->src_vals = (int64_t*)realloc(a->src_vals, sizeof(int64_t) * a->src_cap * nc);
    a->src_vvalid = (uint8_t*)realloc(a->src_vvalid, (size_t)(a->src_cap * nc));
  }
  const int64_t r = a->src_n++;
  a->src_key[r] = key;
  a->src_live[r] = 0;
  a->src_slots[j] = r;
  return r;
}

khip_status oracle_agg_push_table(oracle_agg* a, const khip_batch* b, const khip_table_src* src,
                                  khip_batch_stats* stats) {
  if (!a || !b || !src || b->mem != KHIP_MEM_HOST || b->n_rows < 0) return KHIP_E_INVALID;
  if (!(a->d.flags & KHIP_FLAG_TABLE_SOURCE) || b->n_cols < a->d.n_cols) return KHIP_E_INVALID;
  if (src->key_type != KHIP_KEY_INT64 && src->key_type != KHIP_KEY_UTF8) return KHIP_E_INVALID;
  if (a->src_key_type < 0) {
    a->src_key_type = src->key_type;
    strdict_init(&a->src_dict);
  } else if (a->src_key_type != src->key_type) {
    return KHIP_E_INVALID;
  }
  khip_batch_stats s;
  memset(&s, 0, sizeof(s));
  s.rows_in = b->n_rows;
  a->epoch++;
  a->n_touched = 0;
  const int nc = a->d.n_cols > 0 ? a->d.n_cols : 1;
  int64_t raw[KHIP_MAX_COLS_ORACLE];
  uint8_t valid[KHIP_MAX_COLS_ORACLE];
  for (int64_t r = 0; r < b->n_rows; r++) {
    if (!bit_get(src->key_valid, r)) { s.dropped_null_key++; continue; }
    const int64_t ts = b->ts[r];
    if (ts < 0) { s.dropped_bad_ts++; continue; }
    s.rows_accepted++;
    const int64_t pk = src->key_type == KHIP_KEY_INT64
                           ? src->key_i64[r]
                           : strdict_intern(&a->src_dict, src->key_bytes + src->key_offsets[r],
                                            src->key_offsets[r + 1] - src->key_offsets[r]);
    const int64_t row = src_find_or_add(a, pk);
    /* undo the key's previous row from its group */
    if (a->src_live[row] && a->src_gvalid[row]) {
      entry* x = find_or_create(a, a->src_gkey[row], 0);
      touch(a, x);
      if (ts > x->rowtime) x->rowtime = ts;
      table_row_aggs(a, x, a->src_vals + row * nc, a->src_vvalid + row * nc, -1);
      s.windows_applied++;
    }
    if (!bit_get(b->row_valid, r)) { /* tombstone: the key leaves the table */
      a->src_live[row] = 0;
      continue;
    }
    for (int c = 0; c < a->d.n_cols; c++) {
      valid[c] = (uint8_t)bit_get(b->col_valid ? b->col_valid[c] : NULL, r);
      raw[c] = valid[c] ? read_col_raw(b, c, a->col_types[c], r) : 0;
    }
    const int gvalid = bit_get(b->key_valid, r);
    int64_t gkey = 0;
    if (gvalid)
      gkey = a->d.key_type == KHIP_KEY_INT64
                 ? b->key_i64[r]
                 : strdict_intern(&a->dict, b->key_bytes + b->key_offsets[r], b->key_offsets[r + 1] - b->key_offsets[r]);
    a->src_live[row] = 1;
    a->src_gvalid[row] = (uint8_t)gvalid;
    a->src_gkey[row] = gkey;
    memcpy(a->src_vals + row * nc, raw, sizeof(int64_t) * (size_t)a->d.n_cols);
    memcpy(a->src_vvalid + row * nc, valid, (size_t)a->d.n_cols);
    if (gvalid) {
      entry* x = find_or_create(a, gkey, 0);
      touch(a, x);
      if (ts > x->rowtime) x->rowtime = ts;
      table_row_aggs(a, x, raw, valid, +1);
      s.windows_applied++;
    }
    if (ts > a->stream_time) a->stream_time = ts;
  }
  s.stream_time = a->stream_time;
  finish_push(a);
  if (stats) *stats = s;
  return KHIP_OK;
}

/* Result type, mirrors khip_agg_result_type. */
static int result_type(const oracle_agg* a, int i) {
  const khip_agg_spec* s = &a->aggs[i];
  if (s->kind == KHIP_AGG_COUNT_STAR || s->kind == KHIP_AGG_COUNT) return KHIP_TYPE_INT64;
  if (s->kind == KHIP_AGG_AVG) return KHIP_TYPE_DOUBLE;
  return a->col_types[s->arg_col];
}

static void result_value(const oracle_agg* a, int i, const agg_state* st, int64_t* iv,
                         double* dv, int* is_null) {
  const khip_agg_spec* s = &a->aggs[i];
  int t = s->kind == KHIP_AGG_COUNT_STAR ? KHIP_TYPE_INT64 : a->col_types[s->arg_col];
  *is_null = 0;
  *iv = 0;
  *dv = 0.0;
  switch (s->kind) {
    case KHIP_AGG_COUNT_STAR:
    case KHIP_AGG_COUNT:
      *iv = st->i;
      break;
    case KHIP_AGG_SUM:
      if (t == KHIP_TYPE_DOUBLE) *dv = st->d; else *iv = st->i;
      break;
    case KHIP_AGG_MIN:
    case KHIP_AGG_MAX:
      if (!st->has) *is_null = 1;
      else if (t == KHIP_TYPE_DOUBLE) *dv = st->d;
      else *iv = st->i;
      break;
    case KHIP_AGG_AVG:
      if (st->cnt == 0) *dv = 0.0;
      else if (t == KHIP_TYPE_DOUBLE) *dv = st->d / (double)st->cnt;
      else if (t == KHIP_TYPE_INT32) *dv = (double)(int32_t)st->i / (double)st->cnt;
      else *dv = (double)st->i / (double)st->cnt;
      break;
  }
}

static int having_pass(const oracle_agg* a, const khip_having* h, const entry* x) {
  if (!h) return 1;
  int64_t iv;
  double dv;
  int is_null;
  result_value(a, h->agg_index, &x->st[h->agg_index], &iv, &dv, &is_null);
  if (is_null) return 0;
  int rt = result_type(a, h->agg_index);
  int c;
  if (rt == KHIP_TYPE_DOUBLE) c = dv < h->f64 ? -1 : (dv > h->f64 ? 1 : 0);
  else c = iv < h->i64 ? -1 : (iv > h->i64 ? 1 : 0);
  if (rt == KHIP_TYPE_DOUBLE && isnan(dv)) return h->op == KHIP_OP_NE;
  switch (h->op) {
    case KHIP_OP_GT: return c > 0;
    case KHIP_OP_GE: return c >= 0;
    case KHIP_OP_LT: return c < 0;
    case KHIP_OP_LE: return c <= 0;
    case KHIP_OP_EQ: return c == 0;
    case KHIP_OP_NE: return c != 0;
  }
  return 0;
}

/* Order of the snapshot: (key bytes, ws).  x and y may come from different shards
 * (oracle_agg_snapshot_sharded), each with its own key dictionary. */
static int cmp_entry2(const oracle_agg* ax, const entry* x, const oracle_agg* ay, const entry* y) {
  if (ax->d.key_type == KHIP_KEY_INT64) {
    if (x->key != y->key) return x->key < y->key ? -1 : 1;
  } else if (ax != ay || x->key != y->key) {
    int64_t lx = ax->dict.len[x->key], ly = ay->dict.len[y->key];
    int64_t m = lx < ly ? lx : ly;
    int c = m ? memcmp(ax->dict.arena + ax->dict.off[x->key], ay->dict.arena + ay->dict.off[y->key], (size_t)m) : 0;
    if (c) return c;
    if (lx != ly) return lx < ly ? -1 : 1;
  }
  if (x->ws != y->ws) return x->ws < y->ws ? -1 : 1;
  return 0;
}
/* Order of a push's emitted rows: key, then (sessions) tombstones before rows, then window start
 * and end — with one record per push this is the reference's own emission order. */
static int cmp_row(const oracle_agg* ax, const entry* x, int tx, const oracle_agg* ay, const entry* y, int ty) {
  if (ax->d.key_type == KHIP_KEY_INT64) {
    if (x->key != y->key) return x->key < y->key ? -1 : 1;
  } else if (ax != ay || x->key != y->key) {
    int64_t lx = ax->dict.len[x->key], ly = ay->dict.len[y->key];
    int64_t m = lx < ly ? lx : ly;
    int c = m ? memcmp(ax->dict.arena + ax->dict.off[x->key], ay->dict.arena + ay->dict.off[y->key], (size_t)m) : 0;
    if (c) return c;
    if (lx != ly) return lx < ly ? -1 : 1;
  }
  if (ax->d.window_kind == KHIP_WINDOW_SESSION && tx != ty) return tx ? -1 : 1;
  if (x->ws != y->ws) return x->ws < y->ws ? -1 : 1;
  if (x->we != y->we) return x->we < y->we ? -1 : 1;
  return 0;
}

static int cmp_entry(const void* pa, const void* pb, void* ctx) {
  const oracle_agg* a = (const oracle_agg*)ctx;
  return cmp_entry2(a, *(const entry* const*)pa, a, *(const entry* const*)pb);
}

static void stmax_add(oracle_agg* a, int64_t st) {
  if (a->n_stmax == a->cap_stmax) {
    a->cap_stmax = a->cap_stmax ? a->cap_stmax * 2 : 256;
    a->stmax = (int64_t*)realloc(a->stmax, sizeof(int64_t) * a->cap_stmax);
  }
  a->stmax[a->n_stmax++] = st;
}

static void chg_add(oracle_agg* a, int64_t idx, uint8_t tomb) {
  if (a->n_chg == a->cap_chg) {
    a->cap_chg = a->cap_chg ? a->cap_chg * 2 : 1024;
    a->chg = (int64_t*)realloc(a->chg, sizeof(int64_t) * a->cap_chg);
    a->chg_tomb = (uint8_t*)realloc(a->chg_tomb, (size_t)a->cap_chg);
  }
  a->chg[a->n_chg] = idx;
  a->chg_tomb[a->n_chg++] = tomb;
}

static int cmp_chg(const void* pa, const void* pb, void* ctx) { /* (entry << 1 | tombstone) */
  const oracle_agg* a = (const oracle_agg*)ctx;
  const int64_t u = *(const int64_t*)pa, v = *(const int64_t*)pb;
  return cmp_row(a, &a->e[u >> 1], (int)(u & 1), a, &a->e[v >> 1], (int)(v & 1));
}

/* R10: the rows this push emits (after the stream time of the push is known). */
static void finish_push(oracle_agg* a) {
  const khip_having* hv = query_having(a);
  a->n_chg = 0;
  if (a->d.emit == KHIP_EMIT_FINAL && a->d.window_kind == KHIP_WINDOW_SESSION) {
    for (int64_t k = 0; k < a->n_fin; k++)
      if (having_pass(a, hv, &a->e[a->fin_emit[k]])) chg_add(a, a->fin_emit[k], 0);
  } else if (a->d.emit == KHIP_EMIT_FINAL) {
    /* Every window that closed during this push (streamTime - grace passed its end), emitted iff it
     * was still visible (R9) at the record that closed it: with the emission check after every
     * record (Q/suppress.json's emit interval 0), that record's stream time st* is the first
     * maximum >= ws + size + grace, and the store's obs then is floor(st* / adv) * adv. */
    const int64_t size = a->d.size_ms, adv = a->d.advance_ms;
    const int64_t close0 = a->st_before - a->grace, close1 = a->stream_time - a->grace;
    for (int64_t k = 0; close1 > close0 && k < a->n; k++) {
      const entry* x = &a->e[k];
      const int64_t end = x->ws + size;
      if (end <= close0 || end > close1 || !having_pass(a, hv, x)) continue;
      const int64_t T = end + a->grace;
      int64_t lo = 0, hi = a->n_stmax - 1; /* first maximum >= T (the last one is >= T) */
      while (lo < hi) {
        const int64_t mid = (lo + hi) / 2;
        if (a->stmax[mid] >= T) hi = mid; else lo = mid + 1;
      }
      if (x->ws >= (a->stmax[lo] / adv) * adv - a->retention) chg_add(a, k, 0);
    }
  } else {
    for (int64_t t = 0; t < a->n_touched; t++) {
      const entry* x = &a->e[a->touched[t]];
      if (x->dead) { /* a session merged away: deleted if it existed before the push */
        if (x->born_epoch != a->epoch && x->old_pass) chg_add(a, a->touched[t], 1);
      } else if (having_pass(a, hv, x)) {
        chg_add(a, a->touched[t], 0);
      } else if (x->old_pass) {
        chg_add(a, a->touched[t], 1);
      }
    }
  }
  if (a->n_chg > 1) {
    for (int64_t k = 0; k < a->n_chg; k++) a->chg[k] = a->chg[k] << 1 | a->chg_tomb[k];
    qsort_r(a->chg, (size_t)a->n_chg, sizeof(int64_t), cmp_chg, a);
    for (int64_t k = 0; k < a->n_chg; k++) {
      a->chg_tomb[k] = (uint8_t)(a->chg[k] & 1);
      a->chg[k] >>= 1;
    }
  }
}

khip_status oracle_agg_snapshot_size(oracle_agg* a, int64_t* n_rows, int64_t* key_bytes) {
  if (!a) return KHIP_E_INVALID;
  int64_t n = 0, kb = 0;
  for (int64_t k = 0; k < a->n; k++) {
    if (!entry_visible(a, &a->e[k])) continue;
    n++;
    if (a->d.key_type == KHIP_KEY_UTF8) kb += a->dict.len[a->e[k].key];
  }
  if (n_rows) *n_rows = n;
  if (key_bytes) *key_bytes = kb;
  return KHIP_OK;
}

khip_status oracle_agg_changes_size(oracle_agg* a, int64_t* n_rows, int64_t* key_bytes) {
  if (!a) return KHIP_E_INVALID;
  int64_t kb = 0;
  if (a->d.key_type == KHIP_KEY_UTF8)
    for (int64_t k = 0; k < a->n_chg; k++) kb += a->dict.len[a->e[a->chg[k]].key];
  if (n_rows) *n_rows = a->n_chg;
  if (key_bytes) *key_bytes = kb;
  return KHIP_OK;
}

typedef struct {
  const oracle_agg* a; /* owner (shard) of the entry: its dictionary holds the key bytes */
  const entry* x;
} owned_entry;

/* Rows [0, m) of the snapshot (ResultTransformer map + WindowBoundsPopulator). */
static khip_status write_rows(const owned_entry* rows, int64_t m, khip_snapshot* out) {
  if (m > out->capacity) {
    out->n_rows = m;
    return KHIP_E_BUFFER;
  }
  int64_t kb = 0;
  if (m > 0 && rows[0].a->d.key_type == KHIP_KEY_UTF8 && out->key_offsets) out->key_offsets[0] = 0;
  for (int64_t r = 0; r < m; r++) {
    const oracle_agg* a = rows[r].a;
    const entry* x = rows[r].x;
    const int windowed = a->d.window_kind != KHIP_WINDOW_NONE;
    if (a->d.key_type == KHIP_KEY_INT64) {
      if (out->key_i64) out->key_i64[r] = x->key;
    } else {
      int64_t len = a->dict.len[x->key];
      if (kb + len > out->key_bytes_capacity) return KHIP_E_BUFFER;
      if (out->key_bytes && len) memcpy(out->key_bytes + kb, a->dict.arena + a->dict.off[x->key], (size_t)len);
      kb += len;
      if (out->key_offsets) out->key_offsets[r + 1] = kb;
    }
    if (out->window_start) out->window_start[r] = windowed ? x->ws : 0;
    if (out->window_end) out->window_end[r] = windowed ? x->we : 0;
    if (out->rowtime) out->rowtime[r] = x->rowtime;
    for (int i = 0; i < a->d.n_aggs; i++) {
      int64_t iv;
      double dv;
      int is_null;
      result_value(a, i, &x->st[i], &iv, &dv, &is_null);
      int rt = result_type(a, i);
      if (out->agg_values && out->agg_values[i]) {
        if (rt == KHIP_TYPE_INT32) ((int32_t*)out->agg_values[i])[r] = (int32_t)iv;
        else if (rt == KHIP_TYPE_INT64) ((int64_t*)out->agg_values[i])[r] = iv;
        else ((double*)out->agg_values[i])[r] = dv;
      }
      if (out->agg_null && out->agg_null[i]) out->agg_null[i][r] = (uint8_t)is_null;
    }
  }
  out->n_rows = m;
  out->key_bytes_len = kb;
  return KHIP_OK;
}

khip_status oracle_agg_snapshot(oracle_agg* a, const khip_having* h, khip_snapshot* out) {
  if (!a || !out) return KHIP_E_INVALID;
  if (h && (h->agg_index < 0 || h->agg_index >= a->d.n_aggs)) return KHIP_E_INVALID;
  entry** order = (entry**)malloc(sizeof(entry*) * (a->n + 1));
  int64_t m = 0;
  for (int64_t k = 0; k < a->n; k++)
    if (entry_visible(a, &a->e[k]) && having_pass(a, h, &a->e[k])) order[m++] = &a->e[k];
  qsort_r(order, (size_t)m, sizeof(entry*), cmp_entry, a);
  owned_entry* rows = (owned_entry*)malloc(sizeof(owned_entry) * (m + 1));
  for (int64_t r = 0; r < m; r++) {
    rows[r].a = a;
    rows[r].x = order[r];
  }
  free(order);
  khip_status st = write_rows(rows, m, out);
  free(rows);
  return st;
}

khip_status oracle_agg_changes(oracle_agg* a, khip_snapshot* out, uint8_t* tombstone) {
  if (!a || !out) return KHIP_E_INVALID;
  owned_entry* rows = (owned_entry*)malloc(sizeof(owned_entry) * (a->n_chg + 1));
  for (int64_t r = 0; r < a->n_chg; r++) {
    rows[r].a = a;
    rows[r].x = &a->e[a->chg[r]];
  }
  khip_status st = write_rows(rows, a->n_chg, out);
  if (st == KHIP_OK && tombstone && a->n_chg) memcpy(tombstone, a->chg_tomb, (size_t)a->n_chg);
  free(rows);
  return st;
}

khip_status oracle_agg_destroy(oracle_agg* a) {
  if (!a) return KHIP_OK;
  free(a->touched);
  free(a->fh_end);
  free(a->fh_idx);
  free(a->fin_emit);
  free(a->chg);
  free(a->chg_tomb);
  if (a->own_stmax) free(a->stmax);
  for (int64_t i = 0; i < a->sk_slots; i++) free(a->sk_list[i]);
  free(a->sk_key); free(a->sk_list); free(a->sk_n); free(a->sk_cap);
  for (int64_t k = 0; k < a->n; k++) free(a->e[k].st);
  free(a->e);
  free(a->slots);
  strdict_free(&a->dict);
  if (a->src_key_type >= 0) strdict_free(&a->src_dict);
  free(a->src_key); free(a->src_live); free(a->src_gvalid); free(a->src_gkey); free(a->src_vals);
  free(a->src_vvalid); free(a->src_slots);
  free(a->col_types);
  free(a->aggs);
  free(a);
  return KHIP_OK;
}

/* ------------------------------------------------- P-thread (key-sharded) restatement
 *
 * The same rules R1-R6 over P shards of the key space, one thread per shard: the multi-core
 * CPU baseline ("P threads over P key-hash partitions") and a faster checker
 * for full-size parity tests.  Results equal oracle_agg_push over the whole batch: a group
 * lives in exactly one shard, and the only cross-record state that is not per group — the
 * task's stream time (R2) — is computed first, sequentially, as the stream time after each
 * record, then every shard applies its own records in arrival order against it. */

static uint32_t shard_of(const oracle_agg* a, const khip_batch* b, int64_t r, int32_t P) {
  uint64_t h;
  if (a->d.key_type == KHIP_KEY_INT64) {
    h = mix64((uint64_t)b->key_i64[r]);
  } else {
    const int64_t o0 = b->key_offsets[r], o1 = b->key_offsets[r + 1];
    h = hash_bytes(b->key_bytes + o0, o1 - o0);
  }
  return (uint32_t)((h >> 32) % (uint64_t)P);
}

typedef struct {
  oracle_agg* a;
  const khip_batch* b;
  const int64_t* idx; /* this shard's records, in arrival order */
  int64_t n;
  const int64_t* st_after; /* stream time after each record (R2), by batch row */
  int64_t applied, late;
} shard_job;

static void* shard_run(void* arg) {
  shard_job* j = (shard_job*)arg;
  oracle_agg* a = j->a;
  const khip_batch* b = j->b;
  const int windowed = a->d.window_kind != KHIP_WINDOW_NONE;
  const int64_t size = a->d.size_ms, adv = a->d.advance_ms;
  for (int64_t k = 0; k < j->n; k++) {
    const int64_t r = j->idx[k];
    const int64_t ts = b->ts[r];
    int64_t key;
    if (a->d.key_type == KHIP_KEY_INT64) {
      key = b->key_i64[r];
    } else {
      const int64_t o0 = b->key_offsets[r], o1 = b->key_offsets[r + 1];
      key = strdict_intern(&a->dict, b->key_bytes + o0, o1 - o0);
    }
    if (!windowed) {
      entry* x = find_or_create(a, key, 0);
      touch(a, x);
      if (ts > x->rowtime) x->rowtime = ts;
      apply_aggs(a, x, b, r);
      j->applied++;
      continue;
    }
    if (a->d.window_kind == KHIP_WINDOW_SESSION) {
      session_apply(a, key, ts, j->st_after[r], b, r, &j->applied, &j->late);
      continue;
    }
    const int64_t close_time = j->st_after[r] - a->grace;
    int64_t lo = ts - size + adv;
    if (lo < 0) lo = 0;
    for (int64_t ws = (lo / adv) * adv; ws <= ts; ws += adv) {
      if (ws + size > close_time) {
        entry* x = find_or_create(a, key, ws);
        touch(a, x);
        if (ts > x->rowtime) x->rowtime = ts;
        apply_aggs(a, x, b, r);
        j->applied++;
        if (ws > a->obs_ws) a->obs_ws = ws;
      } else {
        j->late++;
      }
    }
  }
  return NULL;
}

khip_status oracle_agg_push_sharded(oracle_agg** shards, int32_t P, const khip_batch* b, khip_batch_stats* stats) {
  if (!shards || P < 1 || !b || b->mem != KHIP_MEM_HOST || b->n_rows < 0) return KHIP_E_INVALID;
  oracle_agg* a0 = shards[0];
  if (b->n_cols < a0->d.n_cols) return KHIP_E_INVALID;
  /* SESSION EMIT FINAL: the close time passes every shard's sessions record by record (one task);
   * the sequential oracle_agg_push is its checker */
  if (a0->d.window_kind == KHIP_WINDOW_SESSION && a0->d.emit == KHIP_EMIT_FINAL) return KHIP_E_UNSUPPORTED;
  const int64_t n = b->n_rows;
  khip_batch_stats s;
  memset(&s, 0, sizeof(s));
  s.rows_in = n;
  int64_t* st_after = (int64_t*)malloc(sizeof(int64_t) * (n + 1));
  uint32_t* sh = (uint32_t*)malloc(sizeof(uint32_t) * (n + 1));
  int64_t* cnt = (int64_t*)calloc((size_t)P + 1, sizeof(int64_t));
  int64_t st = a0->stream_time;
  const int64_t st_before = st;
  a0->n_stmax = 0;
  for (int64_t r = 0; r < n; r++) { /* R1 drops and R2 stream time, sequential */
    sh[r] = UINT32_MAX;
    if (!bit_get(b->key_valid, r)) { s.dropped_null_key++; continue; }
    if (!bit_get(b->row_valid, r)) { s.dropped_null_row++; continue; }
    if (b->ts[r] < 0) { s.dropped_bad_ts++; continue; }
    s.rows_accepted++;
    if (b->ts[r] > st) {
      st = b->ts[r];
      stmax_add(a0, st);
    }
    st_after[r] = st;
    sh[r] = shard_of(a0, b, r, P);
    cnt[sh[r] + 1]++;
  }
  for (int32_t p = 0; p < P; p++) cnt[p + 1] += cnt[p];
  int64_t* idx = (int64_t*)malloc(sizeof(int64_t) * (n + 1));
  int64_t* fill = (int64_t*)malloc(sizeof(int64_t) * ((size_t)P + 1));
  memcpy(fill, cnt, sizeof(int64_t) * (size_t)P);
  for (int64_t r = 0; r < n; r++)
    if (sh[r] != UINT32_MAX) idx[fill[sh[r]]++] = r;
  shard_job* jobs = (shard_job*)calloc((size_t)P, sizeof(shard_job));
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)P);
  for (int32_t p = 0; p < P; p++) {
    shards[p]->epoch++;
    shards[p]->n_touched = 0;
    jobs[p].a = shards[p];
    jobs[p].b = b;
    jobs[p].idx = idx + cnt[p];
    jobs[p].n = cnt[p + 1] - cnt[p];
    jobs[p].st_after = st_after;
    pthread_create(&th[p], NULL, shard_run, &jobs[p]);
  }
  for (int32_t p = 0; p < P; p++) {
    pthread_join(th[p], NULL);
    s.windows_applied += jobs[p].applied;
    s.windows_late += jobs[p].late;
    shards[p]->stream_time = st;
  }
  int64_t obs = -1; /* one task, one window store: the largest window start over the shards */
  for (int32_t p = 0; p < P; p++) obs = shards[p]->obs_ws > obs ? shards[p]->obs_ws : obs;
  if (a0->d.window_kind == KHIP_WINDOW_SESSION) obs = st;
  for (int32_t p = 0; p < P; p++) {
    oracle_agg* sp = shards[p];
    sp->obs_ws = obs;
    sp->st_before = st_before;
    if (p) { /* every shard reads the task's stream-time maxima */
      if (sp->own_stmax) free(sp->stmax);
      sp->own_stmax = 0;
      sp->stmax = a0->stmax;
      sp->n_stmax = a0->n_stmax;
    }
    finish_push(sp);
  }
  s.stream_time = st;
  if (stats) *stats = s;
  free(jobs); free(th); free(fill); free(idx); free(cnt); free(sh); free(st_after);
  return KHIP_OK;
}

khip_status oracle_agg_snapshot_size_sharded(oracle_agg** shards, int32_t P, int64_t* n_rows, int64_t* key_bytes) {
  int64_t n = 0, kb = 0;
  for (int32_t p = 0; p < P; p++) {
    int64_t a = 0, k = 0;
    oracle_agg_snapshot_size(shards[p], &a, &k);  /* R9 per shard: obs is shared */
    n += a;
    kb += k;
  }
  if (n_rows) *n_rows = n;
  if (key_bytes) *key_bytes = kb;
  return KHIP_OK;
}

typedef struct {
  oracle_agg* a;
  const khip_having* h;
  int changes; /* 1: the shard's last-push changes instead of its table */
  entry** order;
  uint8_t* tomb; /* changes: tombstone per order[] entry */
  int64_t m;
} sort_job;

static void* sort_run(void* arg) {
  sort_job* j = (sort_job*)arg;
  oracle_agg* a = j->a;
  j->order = (entry**)malloc(sizeof(entry*) * (a->n + 1));
  j->m = 0;
  j->tomb = NULL;
  if (j->changes) { /* the push's emitted rows, already sorted */
    j->tomb = a->chg_tomb;
    for (int64_t k = 0; k < a->n_chg; k++) j->order[j->m++] = &a->e[a->chg[k]];
    return NULL;
  }
  for (int64_t k = 0; k < a->n; k++)
    if (entry_visible(a, &a->e[k]) && having_pass(a, j->h, &a->e[k])) j->order[j->m++] = &a->e[k];
  qsort_r(j->order, (size_t)j->m, sizeof(entry*), cmp_entry, a);
  return NULL;
}

/* Snapshot of the union of the shards: each shard sorted on its own thread, then a P-way
 * merge (binary heap of shard cursors) into (key, ws) order. */
static khip_status merge_sharded(oracle_agg** shards, int32_t P, const khip_having* h, int changes,
                                 khip_snapshot* out, uint8_t* tombstone) {
  sort_job* jobs = (sort_job*)calloc((size_t)P, sizeof(sort_job));
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)P);
  for (int32_t p = 0; p < P; p++) {
    jobs[p].a = shards[p];
    jobs[p].h = h;
    jobs[p].changes = changes;
    pthread_create(&th[p], NULL, sort_run, &jobs[p]);
  }
  int64_t m = 0;
  for (int32_t p = 0; p < P; p++) {
    pthread_join(th[p], NULL);
    m += jobs[p].m;
  }
  owned_entry* rows = (owned_entry*)calloc((size_t)(m + 1), sizeof(owned_entry));
  int64_t* cur = (int64_t*)calloc((size_t)P, sizeof(int64_t));
  int32_t* heap = (int32_t*)malloc(sizeof(int32_t) * (size_t)P);
  int32_t hn = 0;
#define HEAD(p) (jobs[p].order[cur[p]])
#define TOMB(p) (jobs[p].tomb ? (int)jobs[p].tomb[cur[p]] : 0)
#define LESS(p, q) (cmp_row(jobs[p].a, HEAD(p), TOMB(p), jobs[q].a, HEAD(q), TOMB(q)) < 0)
  for (int32_t p = 0; p < P; p++) {
    if (jobs[p].m == 0) continue;
    int32_t i = hn++;
    heap[i] = p;
    while (i > 0 && LESS(heap[i], heap[(i - 1) / 2])) {
      int32_t t = heap[i]; heap[i] = heap[(i - 1) / 2]; heap[(i - 1) / 2] = t;
      i = (i - 1) / 2;
    }
  }
  uint8_t* mtomb = (uint8_t*)malloc((size_t)m + 1);
  for (int64_t r = 0; r < m; r++) {
    const int32_t p = heap[0];
    rows[r].a = jobs[p].a;
    rows[r].x = HEAD(p);
    mtomb[r] = (uint8_t)TOMB(p);
    if (++cur[p] == jobs[p].m) heap[0] = heap[--hn];
    int32_t i = 0;
    for (;;) {
      int32_t l = 2 * i + 1, rr = l + 1, k = i;
      if (l < hn && LESS(heap[l], heap[k])) k = l;
      if (rr < hn && LESS(heap[rr], heap[k])) k = rr;
      if (k == i) break;
      int32_t t = heap[i]; heap[i] = heap[k]; heap[k] = t;
      i = k;
    }
  }
#undef LESS
#undef TOMB
#undef HEAD
  khip_status st = write_rows(rows, m, out);
  if (st == KHIP_OK && tombstone && m) memcpy(tombstone, mtomb, (size_t)m);
  for (int32_t p = 0; p < P; p++) free(jobs[p].order);
  free(rows); free(cur); free(heap); free(jobs); free(th); free(mtomb);
  return st;
}

khip_status oracle_agg_snapshot_sharded(oracle_agg** shards, int32_t P, const khip_having* h, khip_snapshot* out) {
  if (!shards || P < 1 || !out) return KHIP_E_INVALID;
  if (h && (h->agg_index < 0 || h->agg_index >= shards[0]->d.n_aggs)) return KHIP_E_INVALID;
  return merge_sharded(shards, P, h, 0, out, NULL);
}

khip_status oracle_agg_changes_size_sharded(oracle_agg** shards, int32_t P, int64_t* n_rows, int64_t* key_bytes) {
  int64_t n = 0, kb = 0;
  for (int32_t p = 0; p < P; p++) {
    int64_t a = 0, k = 0;
    oracle_agg_changes_size(shards[p], &a, &k);
    n += a;
    kb += k;
  }
  if (n_rows) *n_rows = n;
  if (key_bytes) *key_bytes = kb;
  return KHIP_OK;
}

khip_status oracle_agg_changes_sharded(oracle_agg** shards, int32_t P, khip_snapshot* out, uint8_t* tombstone) {
  if (!shards || P < 1 || !out) return KHIP_E_INVALID;
  return merge_sharded(shards, P, NULL, 1, out, tombstone);
}

/* --------------------------------------------------------------- join table */

struct oracle_table {
  khip_table_desc d;
  int32_t* col_types;
  int64_t* keys;     /* per row slot */
  uint8_t* live;
  int64_t* vals;     /* n_cols values per row, stored as raw 8 bytes */
  uint8_t* nulls;    /* n_cols per row */
  int64_t nrows, cap;
  int64_t* slots;    /* open addressing → row slot or -1 */
  int64_t nslots;
  int64_t nlive;
  strdict dict;      /* KHIP_KEY_UTF8: key bytes → id (the id is the table key) */
};

static void table_rebuild(oracle_table* t, int64_t ns) {
  free(t->slots);
  t->nslots = ns;
  t->slots = (int64_t*)malloc(sizeof(int64_t) * ns);
  for (int64_t i = 0; i < ns; i++) t->slots[i] = -1;
  for (int64_t r = 0; r < t->nrows; r++) {
    int64_t j = (int64_t)(mix64((uint64_t)t->keys[r]) & (uint64_t)(ns - 1));
    while (t->slots[j] >= 0) j = (j + 1) & (ns - 1);
    t->slots[j] = r;
  }
}

khip_status oracle_table_create(const khip_table_desc* desc, oracle_table** out) {
  if (!desc || !out || desc->n_cols < 0) return KHIP_E_INVALID;
  if (desc->key_type != KHIP_KEY_INT64 && desc->key_type != KHIP_KEY_UTF8) return KHIP_E_INVALID;
  oracle_table* t = (oracle_table*)calloc(1, sizeof(oracle_table));
  t->d = *desc;
  strdict_init(&t->dict);
  t->col_types = (int32_t*)malloc(sizeof(int32_t) * (desc->n_cols + 1));
  memcpy(t->col_types, desc->col_types, sizeof(int32_t) * desc->n_cols);
  t->d.col_types = t->col_types;
  table_rebuild(t, 1024);
  *out = t;
  return KHIP_OK;
}

static int64_t table_find(const oracle_table* t, int64_t key) {
  int64_t j = (int64_t)(mix64((uint64_t)key) & (uint64_t)(t->nslots - 1));
  while (t->slots[j] >= 0) {
    if (t->keys[t->slots[j]] == key) return t->slots[j];
    j = (j + 1) & (t->nslots - 1);
  }
  return -1;
}

/* Table key of batch row r: the BIGINT/INT key, or (STRING keys) the id of its UTF-8 bytes —
 * byte equality, as KAFKA STRING keys compare (S/JoinParamsFactory.java:65-84 only requires
 * both sides' key types to match). */
static int64_t table_key(oracle_table* t, const khip_batch* b, int64_t r) {
  if (t->d.key_type != KHIP_KEY_UTF8) return b->key_i64[r];
  const int64_t o0 = b->key_offsets[r], o1 = b->key_offsets[r + 1];
  return strdict_intern(&t->dict, b->key_bytes + o0, o1 - o0);
}

static int64_t read_raw(const khip_batch* b, int c, int type, int64_t r) {
  int64_t v = 0;
  if (type == KHIP_TYPE_INT32) v = ((const int32_t*)b->col_data[c])[r];
  else memcpy(&v, (const char*)b->col_data[c] + 8 * r, 8);
  return v;
}

khip_status oracle_table_upsert(oracle_table* t, const khip_batch* b) {
  if (!t || !b || b->mem != KHIP_MEM_HOST || b->n_cols < t->d.n_cols) return KHIP_E_INVALID;
  const int nc = t->d.n_cols;
  for (int64_t r = 0; r < b->n_rows; r++) {
    if (!bit_get(b->key_valid, r)) continue;
    int64_t key = table_key(t, b, r);
    int64_t row = table_find(t, key);
    if (!bit_get(b->row_valid, r)) { /* tombstone */
      if (row >= 0 && t->live[row]) { t->live[row] = 0; t->nlive--; }
      continue;
    }
    if (row < 0) {
      if (2 * (t->nrows + 1) > t->nslots) table_rebuild(t, t->nslots * 2);
      if (t->nrows == t->cap) {
        t->cap = t->cap ? t->cap * 2 : 1024;
        t->keys = (int64_t*)realloc(t->keys, sizeof(int64_t) * t->cap);
        t->live = (uint8_t*)realloc(t->live, (size_t)t->cap);
        t->vals = (int64_t*)realloc(t->vals, sizeof(int64_t) * t->cap * (nc ? nc : 1));
        t->nulls = (uint8_t*)realloc(t->nulls, (size_t)(t->cap * (nc ? nc : 1)));
      }
      row = t->nrows++;
      t->keys[row] = key;
      t->live[row] = 0;
      int64_t j = (int64_t)(mix64((uint64_t)key) & (uint64_t)(t->nslots - 1));
      while (t->slots[j] >= 0) j = (j + 1) & (t->nslots - 1);
      t->slots[j] = row;
    }
    if (!t->live[row]) { t->live[row] = 1; t->nlive++; }
    for (int c = 0; c < nc; c++) {
      int v = bit_get(b->col_valid ? b->col_valid[c] : NULL, r);
      t->nulls[row * nc + c] = (uint8_t)!v;
      t->vals[row * nc + c] = v ? read_raw(b, c, t->col_types[c], r) : 0;
    }
  }
  return KHIP_OK;
}

khip_status oracle_table_size(oracle_table* t, int64_t* n) {
  if (!t || !n) return KHIP_E_INVALID;
  *n = t->nlive;
  return KHIP_OK;
}

static int where_pass(const oracle_table* t, const khip_where* w, int64_t row) {
  if (!w) return 1;
  if (row < 0) return 0;
  const int nc = t->d.n_cols;
  if (t->nulls[row * nc + w->right_col]) return 0;
  int64_t raw = t->vals[row * nc + w->right_col];
  int c;
  if (t->col_types[w->right_col] == KHIP_TYPE_DOUBLE) {
    double dv;
    memcpy(&dv, &raw, 8);
    if (isnan(dv)) return w->op == KHIP_OP_NE;
    c = dv < w->f64 ? -1 : (dv > w->f64 ? 1 : 0);
  } else {
    c = raw < w->i64 ? -1 : (raw > w->i64 ? 1 : 0);
  }
  switch (w->op) {
    case KHIP_OP_GT: return c > 0;
    case KHIP_OP_GE: return c >= 0;
    case KHIP_OP_LT: return c < 0;
    case KHIP_OP_LE: return c <= 0;
    case KHIP_OP_EQ: return c == 0;
    case KHIP_OP_NE: return c != 0;
  }
  return 0;
}

khip_status oracle_table_probe(oracle_table* t, const khip_batch* b, int32_t join_type,
                               const khip_where* w, khip_join_out* out) {
  if (!t || !b || !out || b->mem != KHIP_MEM_HOST) return KHIP_E_INVALID;
  if (join_type != KHIP_JOIN_LEFT && join_type != KHIP_JOIN_INNER) return KHIP_E_INVALID;
  if (w && (w->right_col < 0 || w->right_col >= t->d.n_cols)) return KHIP_E_INVALID;
  const int nc = t->d.n_cols;
  int64_t m = 0;
  for (int64_t r = 0; r < b->n_rows; r++) {
    if (!bit_get(b->key_valid, r) || !bit_get(b->row_valid, r) || b->ts[r] < 0) continue;
    int64_t row = table_find(t, table_key(t, b, r));
    if (row >= 0 && !t->live[row]) row = -1;
    if (join_type == KHIP_JOIN_INNER && row < 0) continue;
    if (!where_pass(t, w, row)) continue;
    if (m < out->capacity) {
      if (out->stream_row) out->stream_row[m] = r;
      if (out->matched) out->matched[m] = row >= 0;
      for (int c = 0; c < nc; c++) {
        int is_null = row < 0 || t->nulls[row * nc + c];
        if (out->col_null && out->col_null[c]) out->col_null[c][m] = (uint8_t)is_null;
        if (out->col_data && out->col_data[c]) {
          int64_t raw = is_null ? 0 : t->vals[row * nc + c];
          if (t->col_types[c] == KHIP_TYPE_INT32) ((int32_t*)out->col_data[c])[m] = (int32_t)raw;
          else memcpy((char*)out->col_data[c] + 8 * m, &raw, 8);
        }
      }
    }
    m++;
  }
  out->n_rows = m;
  return m > out->capacity ? KHIP_E_BUFFER : KHIP_OK;
}

khip_status oracle_table_destroy(oracle_table* t) {
  if (!t) return KHIP_OK;
  free(t->keys); free(t->live); free(t->vals); free(t->nulls); free(t->slots);
  free(t->col_types);
  strdict_free(&t->dict);
  free(t);
  return KHIP_OK;
}
