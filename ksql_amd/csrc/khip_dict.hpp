// khip_dict.hpp — the device dictionary of serialized STRING keys, shared by the aggregate
// (UTF8 GROUP BY keys) and the stream-table join (STRING-keyed tables).
//
// Group / table identity in the reference is equality of the serialized KAFKA key bytes
// (S/JoinParamsFactory.java:65-84 only requires both join sides' key types to
// match).  The dictionary maps key bytes to a stable int64 id — the byte offset of the key's
// entry in an append-only arena — so every downstream kernel works on 8-byte ids.
//   slot (32 B): [dict word][id | len << 48][first 16 key bytes as two words]
//     dict word: 0 empty | fresh claim: bit63 | fp22 << 40 | batch row (40 bits)
//                        | resident:    bit62 | fp22 << 40 | id / 8
//   arena entry at id o (8-aligned): [u64 hash][i64 len][bytes, padded to 8]
// A map: k_dict_probe (claims, in-place compares, pending rows) → k_dict_commit (per claim) →
// k_dict_resolve (per pending row); kernels in khip_agg.hip.
//
// Inline keys: a key of 0..17 ASCII decimal digits ('0'-'9': card, account and phone numbers,
// numeric ids kept as VARCHAR) has an exact 64-bit form and never enters the dictionary — its id
// is KID_INLINE | length << 57 | its decimal value (10^17 < 2^57; the length keeps leading zeros
// apart: "007" != "7").  Arena offsets stay below 2^48, so the two id spaces are disjoint and id
// equality is still byte equality.  Such a row costs its key bytes and nothing else: no slot
// probe, no arena entry.
#pragma once
#include "khip_inline_id.hpp"
#include "khip_util.hpp"

namespace khip {

__host__ __device__ inline bool kid_inline(int64_t kid) { return kid >= KID_INLINE; }

// The key bytes of an inline id (out: KEY_INLINE_MAX bytes); returns the length.
inline int kid_inline_bytes(int64_t kid, uint8_t* out) {
  const int len = (int)((kid >> 57) & 31);
  uint64_t v = (uint64_t)kid & ((1ULL << 57) - 1);
  for (int j = len - 1; j >= 0; j--) {
    out[j] = (uint8_t)('0' + v % 10);
    v /= 10;
  }
  return len;
}

struct KeyDict {
  DevBuf slots, arena, ctr, lists, retry;
  int64_t dcap = 0, docc = 0, arena_used = 0;
  int64_t last_added = -1;   // keys the last map inserted (-1: no map yet)
  int64_t last_probed = 0;   // rows of the last map that probed the table (not inline)
  int64_t round_probed = 0;  // rows of the last probe round that probed it
  int64_t last_inline = -1;  // inline rows the last inline pass found (-1: none ran yet)
  int64_t round_used = 0, round_keys = 0;  // arena bytes used / keys added after the last good round
  int64_t maps = 0;
};

// Allocate the first 4096 slots.
khip_status dict_init(KeyDict& d, hipStream_t s);

// Batch keys (device offsets[n+1] into device bytes) → ids, inserting unseen keys.  Rows that fail
// kv, rv or ts >= 0 (each check skipped when its pointer is null) get id 0 and are not inserted.
// kid[n] and khash[n] (the key's 64-bit hash; khash may be null) are device outputs.
// key_bytes_total = koff[n].
// Synchronises the stream.
khip_status dict_map(KeyDict& d, hipStream_t s, const int64_t* koff, const uint8_t* kbytes, int64_t key_bytes_total,
                     const uint8_t* kv, const uint8_t* rv, const int64_t* ts, int64_t n, int64_t* kid, int64_t* khash);

// Read-only probe: kid[i] = the id of key i, or -1 when it was never inserted.  Asynchronous.
khip_status dict_find(KeyDict& d, hipStream_t s, const int64_t* koff, const uint8_t* kbytes, int64_t n, int64_t* kid);

// Forget every key (keeps the allocation).  Asynchronous.
khip_status dict_clear(KeyDict& d, hipStream_t s);

void dict_release(KeyDict& d);

}  // namespace khip
