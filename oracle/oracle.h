/*
 * oracle.h — CPU restatement of the ksqlDB windowed-aggregate and stream-table
 * join semantics.  TEST INFRASTRUCTURE ONLY: this is the parity checker used by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.  The product
 * path (libksqldb_hip.so) never links, loads or calls it.
 *
 * It reuses the boundary structs of include/ksqldb_hip.h so the oracle and the
 * HIP path are fed byte-identical batches.  All pointers are host pointers.
 *
 * Pinned by the reference's own QTT golden vectors (tests/golden/qtt_*.json,
 * extracted by tests/golden/make_fixtures.py; see oracle.c header for the rules and
 * the reference file:line each rule follows).
 */
#ifndef KSQL_ORACLE_H
#define KSQL_ORACLE_H

#include "../include/ksqldb_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_agg oracle_agg;
typedef struct oracle_table oracle_table;

khip_status oracle_agg_create(const khip_agg_desc* desc, oracle_agg** out);
khip_status oracle_agg_push(oracle_agg* agg, const khip_batch* batch,
                            khip_batch_stats* stats);
khip_status oracle_agg_snapshot_size(oracle_agg* agg, int64_t* n_rows,
                                     int64_t* key_bytes);
khip_status oracle_agg_snapshot(oracle_agg* agg, const khip_having* having,
                                khip_snapshot* out);
khip_status oracle_agg_destroy(oracle_agg* agg);
/* R12 table aggregation; mirrors khip_agg_push_table. */
khip_status oracle_agg_push_table(oracle_agg* agg, const khip_batch* batch, const khip_table_src* src,
                                  khip_batch_stats* stats);

/* Rows the last push emitted (R10), snapshot layout sorted by (key, ws); tombstone[r] = 1
 * for a HAVING delete.  Mirrors khip_agg_changes_size / khip_agg_changes. */
khip_status oracle_agg_changes_size(oracle_agg* agg, int64_t* n_rows, int64_t* key_bytes);
khip_status oracle_agg_changes(oracle_agg* agg, khip_snapshot* out, uint8_t* tombstone);

/* Key-sharded P-thread restatement (same results as oracle_agg_push over the batch): shards[]
 * are P handles created with the same descriptor and only ever pushed together. */
khip_status oracle_agg_push_sharded(oracle_agg** shards, int32_t P, const khip_batch* batch,
                                    khip_batch_stats* stats);
khip_status oracle_agg_snapshot_size_sharded(oracle_agg** shards, int32_t P, int64_t* n_rows,
                                             int64_t* key_bytes);
khip_status oracle_agg_snapshot_sharded(oracle_agg** shards, int32_t P, const khip_having* having,
                                        khip_snapshot* out);
khip_status oracle_agg_changes_size_sharded(oracle_agg** shards, int32_t P, int64_t* n_rows, int64_t* key_bytes);
khip_status oracle_agg_changes_sharded(oracle_agg** shards, int32_t P, khip_snapshot* out, uint8_t* tombstone);

khip_status oracle_table_create(const khip_table_desc* desc, oracle_table** out);
khip_status oracle_table_upsert(oracle_table* t, const khip_batch* rows);
khip_status oracle_table_size(oracle_table* t, int64_t* n_keys);
khip_status oracle_table_probe(oracle_table* t, const khip_batch* stream,
                               int32_t join_type, const khip_where* where,
                               khip_join_out* out);
khip_status oracle_table_destroy(oracle_table* t);

/* Deterministic synthetic generators (splitmix64), identical bit-for-bit to the
 * device generators in ksql_amd/csrc/khip_synth.hip.  Used to build parity
 * inputs on the host for the oracle. */
uint64_t oracle_splitmix64(uint64_t x);

/* R8 repartition routing: the partition Kafka's default partitioner gives a record whose key
 * is serialized in the KAFKA format (Serdes.Integer / Serdes.Long = big-endian 4 / 8 bytes,
 * ksqldb-serde/.../kafka/KafkaSerdeFactory.java:42-43):
 *   toPositive(murmur2(key bytes)) % n_parts          (kafka-clients 7.4.0-ccs, Apache Kafka 3.4:
 *   Utils.murmur2 / Utils.toPositive, BuiltInPartitioner.partitionForKey — third-party, absent
 *   from the reference tree; restated from the published algorithm). */
int32_t oracle_murmur2(const uint8_t* data, int32_t len);
void oracle_kafka_partition(const int64_t* keys, int64_t n, int32_t key_bytes, int32_t n_parts,
                            int32_t* out);

#ifdef __cplusplus
}
#endif

#endif
