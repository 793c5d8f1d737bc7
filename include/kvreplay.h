/*
 * kvreplay.h — C ABI of the MI355X segment-replay + CRC32-verify engine.
 *
 * Drop-in boundary for the index-rebuild-on-restart path of whispem/mini-kvstore-v2
 * (reference snapshot 0.3.0, read-only at /root/reference):
 *
 *   src/store/engine.rs:53-57   for (_id, path) in &segment_paths {
 *                                   Self::replay_segment(path, &mut values)?;   }
 *   src/store/engine.rs:79-154  replay_segment — the serial per-record walk this ABI replaces
 *   src/volume/storage.rs:27    crc32fast::hash(data) — the CRC-32 definition (ETag)
 *   src/store/index.rs:7        (segment_id, offset, length) — the target index shape
 *
 * The reference has no FFI of its own: the seam is source level.  A Rust
 * caller declares these functions `extern "C"` with #[repr(C)] mirrors of the structs below
 * (INTEGRATION.md shows the binding), sorts segments by id exactly as engine.rs:51 does, hands
 * their bytes over, and folds the returned tuples into its index.
 *
 * Conventions
 *   - All functions are synchronous (KVStore::open is a blocking constructor, engine.rs:24).
 *   - The library never frees caller memory; device scratch belongs to the context.
 *   - A context is not thread-safe; use one per thread (or per GPU).
 *   - Return codes: KVR_OK (0), KVR_CORRUPTED (1, *err filled: the first error in
 *     (segment order, offset) order — exactly the error engine.rs:56 would propagate),
 *     KVR_CAPACITY (2, *n_out = required tuple count), negative = usage / HIP / IO failure.
 */
#ifndef KVREPLAY_H
#define KVREPLAY_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KVR_ABI_VERSION 1

/* ---- status codes --------------------------------------------------------------------- */
#define KVR_OK          0
#define KVR_CORRUPTED   1   /* StoreError::CorruptedData (error.rs:11-12); *err filled     */
#define KVR_CAPACITY    2   /* out[] too small; *n_out = tuples required                     */
#define KVR_EINVAL     (-1) /* bad argument (unsorted segments, NULL pointer, ...)           */
#define KVR_EHIP       (-2) /* HIP runtime failure (no device, launch failure, ...)          */
#define KVR_EIO        (-3) /* host I/O failure                                              */
#define KVR_ENOMEM     (-4) /* host or device allocation failure                             */

/* ---- error kinds: one per CorruptedData site of engine.rs:79-154 (in check order) ------- */
#define KVR_E_NONE      0
#define KVR_E_OPEN      1   /* engine.rs:80-82   "Failed to open segment {path}: {io}"          */
#define KVR_E_KEY_LEN   2   /* engine.rs:96-102  "Failed to read key length in {path}: ..."     */
#define KVR_E_KEY       3   /* engine.rs:107-113 "Failed to read key in {path}: ..."            */
#define KVR_E_UTF8      4   /* engine.rs:114-116 "Invalid UTF-8 key in {path}: {FromUtf8Error}" */
#define KVR_E_VAL_LEN   5   /* engine.rs:121-127 "Failed to read val len in {path}: ..."        */
#define KVR_E_VAL       6   /* engine.rs:130-136 "Failed to read val in {path}: ..."            */
#define KVR_E_OPCODE    7   /* engine.rs:143-149 "Unknown opcode {op} in segment {path}"        */

/* ---- replay flags --------------------------------------------------------------------- */
#define KVR_SEGS_ON_DEVICE      0x1u  /* segs[i].bytes are device pointers on ctx's device      */
#define KVR_OUT_ON_DEVICE       0x2u  /* out is a device pointer (tuples stay resident in HBM)  */
#define KVR_EXPECTED_ON_DEVICE  0x4u  /* expected_crc is a device pointer                        */

/* ---- tuple flags ---------------------------------------------------------------------- */
#define KVR_TF_VERIFIED   0x1u  /* an expected CRC was supplied for this record (SET only)    */
#define KVR_TF_CRC_FAIL   0x2u  /* crc32 != expected: the record fails verification           */

/* One input segment.  Segments must be passed in ascending seg_id (the caller performs the
 * engine.rs:51 sort); each is replayed from offset 0 exactly like replay_segment. */
typedef struct kvr_segment {
    uint64_t       seg_id;   /* id parsed from "segment-<id>.dat" (engine.rs:40-45)           */
    const uint8_t *bytes;    /* segment bytes; host or device pointer (KVR_SEGS_ON_DEVICE)    */
    uint64_t       len;      /* bytes in the file                                              */
} kvr_segment;

/* One record on the replay chain, in (segment, offset) order.  32 bytes, layout frozen.
 * SET: framing [0][klen u32 LE][key][vlen u32 LE][value]  (engine.rs:169-173)
 * DEL: framing [1][klen u32 LE][key]                      (engine.rs:191-193)
 * key bytes live at rec_off + 5, value bytes at rec_off + 9 + key_len. */
typedef struct kvr_tuple {
    uint64_t rec_off;   /* offset of the op byte within the segment                          */
    uint32_t seg_idx;   /* index into the caller's segs[] (map back to seg_id on the host)    */
    uint32_t key_len;
    uint32_t val_len;   /* 0 for DEL                                                          */
    uint32_t crc32;     /* CRC-32/ISO-HDLC of the value bytes = crc32fast::hash (storage.rs:27); 0 for DEL */
    uint32_t key_tag;   /* CRC-32/ISO-HDLC of the key bytes (hash tag for host-side folding)  */
    uint8_t  op;        /* 0 = SET, 1 = DEL                                                    */
    uint8_t  flags;     /* KVR_TF_*                                                            */
    uint16_t reserved;
} kvr_tuple;

/* The first error in (segment, offset) order — the error KVStore::open returns. */
typedef struct kvr_error {
    int32_t  kind;      /* KVR_E_*                                                            */
    uint32_t seg_idx;   /* segment index of the failing record                                */
    uint64_t rec_off;   /* offset of the failing record's op byte                             */
    uint64_t aux;       /* KVR_E_OPCODE: the opcode; KVR_E_UTF8: valid_up_to | (error_len << 32),
                           error_len 0 meaning "incomplete" (Utf8Error::error_len() == None)  */
} kvr_error;

/* Per-call measurements of the last kvr_replay on a context (device timings via hipEvents on
 * the context's stream). */
typedef struct kvr_stats {
    double   ms_total;          /* whole device pipeline, first kernel start -> last kernel end */
    double   ms_replay;         /* the main replay kernel (first pass)                           */
    double   ms_link;           /* stripe linking + re-walk passes                               */
    double   ms_compact;        /* tuple compaction                                              */
    uint64_t bytes_in;          /* segment bytes replayed                                        */
    uint64_t n_records;         /* tuples produced                                               */
    uint64_t n_crc_fail;        /* records whose CRC failed verification                         */
    uint32_t n_stripes;         /* speculation units                                             */
    uint32_t n_tiles;
    uint32_t n_redo;            /* stripes re-walked after a failed speculation                   */
    uint32_t n_link_passes;
} kvr_stats;

typedef struct kvr_ctx kvr_ctx;

/* Context on one HIP device with its own stream and device arenas. */
int  kvr_ctx_create(int device, kvr_ctx **out);
void kvr_ctx_destroy(kvr_ctx *ctx);
/* Run on a caller-provided hipStream_t (e.g. torch.cuda.current_stream().cuda_stream); NULL
 * restores the context's own stream. */
int  kvr_ctx_set_stream(kvr_ctx *ctx, void *hip_stream);
int  kvr_ctx_device(const kvr_ctx *ctx);
/* Tiles (8 KiB each) per stripe, the unit of speculation; 0 = automatic (one stripe per resident
 * wave).  Larger stripes mean fewer speculated entries, smaller ones more parallelism. */
int  kvr_ctx_set_tiles_per_stripe(kvr_ctx *ctx, uint32_t tiles);

/* Replay n_segs segments (ascending seg_id) -> tuples in (segment, offset) order.
 * expected_crc (optional, may be NULL): expected CRC per record in tuple order, e.g. the
 * ETags BlobStorage::put returned (storage.rs:27); records with index < n_expected get
 * KVR_TF_VERIFIED and, on mismatch, KVR_TF_CRC_FAIL.
 * Returns KVR_OK, KVR_CORRUPTED (*err), KVR_CAPACITY (*n_out = required) or < 0.
 * Slots of out past *n_out are unspecified: a call whose linked gather falls back may have written
 * scratch tuples there (always inside out[0..cap)). */
int  kvr_replay(kvr_ctx *ctx, const kvr_segment *segs, size_t n_segs, uint32_t flags,
                const uint32_t *expected_crc, size_t n_expected,
                kvr_tuple *out, size_t cap, size_t *n_out, kvr_error *err);

int  kvr_last_stats(const kvr_ctx *ctx, kvr_stats *out);

/* ---- replay + last-writer fold on the device (SURVEY §8b dedup_last_writer) ----------------
 * kvr_replay, then the fold of engine.rs:137 (insert) / :141 (remove) in HBM (the compaction's
 * hash table over the key bytes): out receives only each live key's final SET tuple, in
 * (segment, offset) order — the records the reference's HashMap holds after open — and
 * *n_out = stats().num_keys (engine.rs:237-259).  Errors as kvr_replay; KVR_CAPACITY with the
 * required count.  flags: KVR_SEGS_ON_DEVICE, KVR_OUT_ON_DEVICE. */
int  kvr_replay_live(kvr_ctx *ctx, const kvr_segment *segs, size_t n_segs, uint32_t flags,
                     kvr_tuple *out, size_t cap, size_t *n_out, kvr_error *err);
/* The same with every key's last record kept, a DEL included (the per-GPU reduction of a sharded
 * store: kvr_replay_live_multi).  In (segment, offset) order; arguments as kvr_replay_live. */
int  kvr_replay_last(kvr_ctx *ctx, const kvr_segment *segs, size_t n_segs, uint32_t flags,
                     kvr_tuple *out, size_t cap, size_t *n_out, kvr_error *err);

/* ---- the open-time index on the device (engine.rs:24-76, index.rs:5-7) ---------------------
 * kvr_replay_index = kvr_replay_live plus a hash table over the live keys built in HBM, so the
 * host receives the reference's HashMap (every live key -> its final SET) as two flat arrays and
 * folds nothing itself:
 *   live[0 .. *n_live)     each live key's final SET tuple, in (segment, offset) order — exactly
 *                          kvr_replay_live's output; *n_live = stats().num_keys
 *   slots[0 .. *n_slots)   the fold's own hash table, entry for entry: slots[h] = 1 + index into
 *                          live[], 0 = free, 0xFFFFFFFF = a key whose last record is a DEL (probe
 *                          on).  *n_slots is a power of two > *n_live (the fold table's size); a
 *                          key's home slot is kvr_index_hash(CRC-32 of the key) & (*n_slots - 1),
 *                          then linear probing.  Which slot a key took may differ between runs;
 *                          lookups do not.
 * flags: KVR_SEGS_ON_DEVICE, KVR_OUT_ON_DEVICE (live and slots are device pointers).
 * Returns as kvr_replay_live; KVR_CAPACITY when live_cap < *n_live or slot_cap < *n_slots — the
 * result then stays in the context until its next call, and kvr_index_fetch copies it out. */
typedef struct kvr_index_stats {
    double   ms_wall;       /* host wall time of the call                                         */
    double   ms_replay;     /* the replay pipeline (device)                                       */
    double   ms_fold;       /* fold rounds, live list and key table (device)                      */
    uint64_t bytes_in;
    uint64_t n_tuples;      /* records replayed                                                   */
    uint64_t n_live;
    uint64_t n_slots;
    uint32_t fold_rounds;   /* probe rounds of the fold (1 + rounds for keys sharing a CRC-32)     */
    uint32_t fold_redo;     /* 1 if the fold table filled up and was redone at 2 n_tuples entries   */
    uint64_t fold_est;      /* distinct-key estimate that sized the table (HyperLogLog; 0: small)   */
    uint64_t fold_slots;    /* fold table entries                                                  */
} kvr_index_stats;

int      kvr_replay_index(kvr_ctx *ctx, const kvr_segment *segs, size_t n_segs, uint32_t flags,
                          kvr_tuple *live, size_t live_cap, uint32_t *slots, uint64_t slot_cap,
                          size_t *n_live, uint64_t *n_slots, kvr_error *err);
int      kvr_index_fetch(kvr_ctx *ctx, uint32_t flags, kvr_tuple *live, size_t live_cap, uint32_t *slots,
                         uint64_t slot_cap);
int      kvr_last_index_stats(const kvr_ctx *ctx, kvr_index_stats *out);
uint64_t kvr_index_slots(uint64_t n_live);     /* max(16, the power of two >= 2 n_live): host tables */
uint32_t kvr_index_hash(uint32_t key_tag);     /* the "lowbias32" integer mix of the tag            */
/* Host lookup of key (klen bytes) in an index whose keys live in segs[] (host bytes): the index
 * into live[] of its final SET, or -1 when the key is not live (engine.rs:200 get -> None). */
int64_t  kvr_index_find(const kvr_tuple *live, const uint32_t *slots, uint64_t n_slots, const kvr_segment *segs,
                        const uint8_t *key, size_t klen);
/* The same table built on the host from a live list (the host-fold path): n_slots a power of two
 * > n_live (kvr_index_slots(n_live) gives the device's size). */
int      kvr_index_build_host(const kvr_tuple *live, size_t n_live, uint32_t *slots, uint64_t n_slots);

/* Key arena (the KVR_EMIT_KEYS option): the key bytes of the live list of the last
 * kvr_replay_live / kvr_replay_index / kvr_ingest_index call on ctx, packed in live-list order —
 * key i is keys[key_off[i] .. key_off[i + 1]), key_off has n_live + 1 entries, *key_bytes = the
 * total.  With the live tuples it is the reference's String-keyed map (engine.rs:114 from_utf8
 * of these bytes, index.rs:7) for a host that does not hold the segment bytes, e.g. a store
 * generated or kept in HBM.  The segments of that call must still be where they were.
 * flags: KVR_OUT_ON_DEVICE.  KVR_CAPACITY (*key_bytes set) when keys_cap or off_cap is short;
 * KVR_EINVAL when ctx holds no live list. */
int  kvr_live_keys(kvr_ctx *ctx, uint32_t flags, uint8_t *keys, uint64_t keys_cap, uint64_t *key_off,
                   size_t off_cap, uint64_t *key_bytes);

/* ---- ingest: the store's files into HBM while they are being read -------------------------
 * kvr_ingest_begin reserves HBM for total_bytes of segments (KVR_ENOMEM when they do not fit:
 * replay them batch-wise with kvr_replay_stream instead).  kvr_ingest_push queues the copy of one
 * segment (ascending seg_id, as engine.rs:51 orders them) on the context's copy stream and returns:
 * pinned bytes (kvr_host_alloc) are DMA'd asynchronously and must stay unchanged until
 * kvr_ingest_index returns.  kvr_ingest_index = kvr_replay_index over the pushed segments once
 * their copies land (seg_idx = push order).  flags: KVR_OUT_ON_DEVICE. */
int  kvr_ingest_begin(kvr_ctx *ctx, uint64_t total_bytes, size_t n_segs);
int  kvr_ingest_push(kvr_ctx *ctx, uint64_t seg_id, const uint8_t *bytes, uint64_t len);
int  kvr_ingest_index(kvr_ctx *ctx, uint32_t flags, kvr_tuple *live, size_t live_cap, uint32_t *slots,
                      uint64_t slot_cap, size_t *n_live, uint64_t *n_slots, kvr_error *err);
/* Abandon an ingest: waits until every copy kvr_ingest_push queued has read its host bytes, then
 * forgets the pushed segments.  A caller that gives up between push and index (a file that
 * vanished while the store was read, engine.rs:80-83) calls it before it frees or unregisters the
 * host buffers it pushed. */
int  kvr_ingest_abort(kvr_ctx *ctx);
/* Pinned (page-locked) host memory for segment bytes: hipHostMalloc / hipHostFree.  Or register
 * existing host memory for DMA (hipHostRegister / hipHostUnregister; cheap once its pages exist)
 * and pass it as pinned. */
int  kvr_host_alloc(uint64_t bytes, void **out);
void kvr_host_free(void *p);
int  kvr_host_register(void *p, uint64_t bytes);
void kvr_host_unregister(void *p);

/* ---- streamed ingest: host segments larger than one transfer ----------
 * The same loop as kvr_replay (engine.rs:55-57) over host-resident segment bytes, e.g. files
 * read (engine.rs:80-83) into memory: consecutive segments are grouped into batches of at most
 * batch_bytes (a larger segment is a batch of its own; 0 = 1 GiB).  While batch b replays, batch
 * b+1 is copied host -> HBM on a second stream into the other of two device slots, so the PCIe
 * transfer and the replay overlap.  With KVR_HOST_PINNED the caller's buffers are pinned
 * (hipHostMalloc / hipHostRegister) and are DMA'd directly; otherwise the library stages them
 * through two pinned buffers of its own.  Output, errors, expected_crc and return codes are
 * exactly those of kvr_replay over the same segs (tuples in (segment, offset) order, seg_idx
 * into segs[]); out is host memory.  kvr_last_stats sums the per-batch device statistics. */
#define KVR_HOST_PINNED         0x8u  /* kvr_replay_stream: segs[i].bytes are pinned host memory */

typedef struct kvr_stream_stats {
    double   ms_wall;     /* host wall time of the whole call: transfers + replays + tuple copies */
    double   ms_device;   /* sum of the batches' device pipelines (kvr_stats.ms_total)            */
    uint64_t bytes_in;    /* segment bytes                                                        */
    uint64_t n_records;   /* tuples produced                                                      */
    uint64_t n_batches;
} kvr_stream_stats;

int  kvr_replay_stream(kvr_ctx *ctx, const kvr_segment *segs, size_t n_segs, uint32_t flags, uint64_t batch_bytes,
                       const uint32_t *expected_crc, size_t n_expected,
                       kvr_tuple *out, size_t cap, size_t *n_out, kvr_error *err);
int  kvr_last_stream_stats(const kvr_ctx *ctx, kvr_stream_stats *out);

/* ---- several GPUs from one process ---------------------------------------------
 * The loop of engine.rs:55-57 over N contexts: segment i of the (sorted) list is replayed by
 * context i mod N, each on its own host thread and stream, no collective; the host merges the
 * shards.  Output, errors, expected_crc and return codes are exactly those of kvr_replay over the
 * same segs on one GPU: tuples in (segment, offset) order with seg_idx into segs[], the first
 * error = the minimum (segment, offset) error over the shards.  devices may repeat an id (several
 * contexts on one GPU).  flags: KVR_SEGS_ON_DEVICE (segment i resident on the device of context
 * i mod N: a sharded store generated or kept in HBM); output to host memory. */
typedef struct kvr_mctx kvr_mctx;
typedef struct kvr_multi_stats {
    double   ms_wall;         /* host wall time of the call: shard threads + merge                 */
    double   ms_device_max;   /* the slowest shard's device pipeline (kvr_stats.ms_total)          */
    uint64_t bytes_in;
    uint64_t n_records;
    uint64_t n_crc_fail;
    uint32_t n_shards;
    uint32_t pad;
} kvr_multi_stats;

int  kvr_mctx_create(const int *devices, int n_devices, kvr_mctx **out);
void kvr_mctx_destroy(kvr_mctx *m);
int  kvr_mctx_size(const kvr_mctx *m);
int  kvr_replay_multi(kvr_mctx *m, const kvr_segment *segs, size_t n_segs, uint32_t flags,
                      const uint32_t *expected_crc, size_t n_expected,
                      kvr_tuple *out, size_t cap, size_t *n_out, kvr_error *err);
int  kvr_last_multi_stats(const kvr_mctx *m, kvr_multi_stats *out);
/* kvr_replay_live over several GPUs: each GPU reduces its shard to every key's
 * last record, tombstones included (a DEL on one GPU may delete a key another GPU SET), only
 * those come back, and the host keeps each key's last record over all shards if it is a SET —
 * exactly kvr_replay_live's output for the whole store.  Every shard exports the key bytes of
 * its last records (kvr_live_keys) and the merge compares those, so the segments may stay on
 * their devices (KVR_SEGS_ON_DEVICE) with no key byte read from host segments.  Replaces the
 * loop of engine.rs:55-57 + the map of engine.rs:137 / :141 on N GPUs. */
int  kvr_replay_live_multi(kvr_mctx *m, const kvr_segment *segs, size_t n_segs, uint32_t flags,
                           kvr_tuple *out, size_t cap, size_t *n_out, kvr_error *err);
/* The key bytes of the last kvr_replay_live_multi output, packed in its order: key i is
 * keys[key_off[i] .. key_off[i + 1]), key_off has n_out + 1 entries, *key_bytes = the total.
 * With the live tuples it is the String-keyed map of engine.rs:114 / index.rs:7 for a store whose
 * bytes live in HBM.  KVR_CAPACITY (*key_bytes set) when a buffer is short, KVR_EINVAL when m
 * holds no live output. */
int  kvr_multi_live_keys(const kvr_mctx *m, uint8_t *keys, uint64_t keys_cap, uint64_t *key_off, size_t off_cap,
                         uint64_t *key_bytes);

/* Host helpers. */
const char *kvr_strerror(int code);
/* CRC-32/ISO-HDLC, identical to crc32fast::hash (storage.rs:27) when crc == 0. */
uint32_t kvr_crc32(uint32_t crc, const uint8_t *data, size_t len);
/* Render the exact engine.rs CorruptedData message (without the "Corrupted data: " prefix of
 * error.rs:11) for err and the segment's path.  Returns the length written (snprintf rules). */
int  kvr_format_error(const kvr_error *err, const char *path, char *buf, size_t cap);

/* ---- live-record rewrite (compaction) -------------------------------------------------
 * The intended KVStore::compact (README.md:283-287: "collect all live keys, write to new
 * segments, delete old segments"; the reference's compaction.rs:9-29 deletes the files without
 * rewriting anything).  Replays segs (ascending seg_id, as kvr_replay), keeps every
 * key's final SET (last writer in (segment, offset) order, engine.rs:137 / :141) and writes those
 * records, byte for byte (the framing of engine.rs:169-173), in (segment, offset) order into out
 * as consecutive new segments.  A new segment starts at the first record whose offset in out is
 * >= k * seg_target (k = 1, 2, ...): segments exceed seg_target by less than one record;
 * seg_target 0 = one segment.  A reference replay of the new segments rebuilds the same map.
 *   out (host, or device with KVR_OUT_ON_DEVICE) receives *out_len bytes; seg_ends[j] = end
 *   offset in out of new segment j, *n_out_segs of them (0 when nothing is live).
 * Returns KVR_OK, KVR_CORRUPTED (*err: the first replay error, as kvr_replay; nothing written),
 * KVR_CAPACITY (out_cap < *out_len or seg_cap < *n_out_segs; both set to what is required) or
 * < 0. */
typedef struct kvr_compact_stats {
    double   ms_replay;     /* the replay pipeline (device time)                              */
    double   ms_fold;       /* last-writer fold, live flags, scans, dense live list           */
    double   ms_gather;     /* byte gather of the live records                                */
    uint64_t n_tuples;      /* records replayed                                               */
    uint64_t n_live;        /* records written                                                */
    uint64_t bytes_in;      /* segment bytes replayed                                         */
    uint64_t bytes_out;     /* bytes written                                                  */
} kvr_compact_stats;

int  kvr_compact(kvr_ctx *ctx, const kvr_segment *segs, size_t n_segs, uint32_t flags, uint64_t seg_target,
                 uint8_t *out, uint64_t out_cap, uint64_t *out_len, uint64_t *seg_ends, size_t seg_cap,
                 size_t *n_out_segs, kvr_error *err);
int  kvr_last_compact_stats(const kvr_ctx *ctx, kvr_compact_stats *out);

/* ---- sharded compaction: one rank of a store whose segments are dealt over several GPUs -----
 * The fold is global (a key's last writer may sit on another rank), so the rewrite runs as
 * three calls per rank around two all-to-all exchanges that the caller performs on device
 * buffers (mini-kvstore-v2_amd/kvreplay/shard.py does it over torch.distributed: RCCL on GPUs).
 *   kvr_compact_stage    replay this rank's segments (segs[i] is global segment gidx[i], the
 *                        position in the store's sorted list), fold locally and build one
 *                        candidate per key (its local last record) addressed to owner rank
 *                        hash(key) mod n_ranks: counts[o] headers and key_bytes[o] key bytes.
 *   kvr_compact_export   copy the candidates to device buffers: headers grouped by owner, key
 *                        bytes grouped by owner (each group's key_off is relative to its group).
 *   kvr_compact_resolve  owner side, over what every rank sent here (headers and keys in sender
 *                        order; hdr_counts[s] / key_counts[s] per sender): d_win[i] = 1 iff header
 *                        i is its key's last writer over all ranks (largest global position).
 *   kvr_compact_finish   d_win = the answers for this rank's own candidates, in export order:
 *                        a record is live iff it is a SET, its key's local last and the winner;
 *                        the live records are written out exactly as kvr_compact does.
 * Every rank's output is disjoint from the others' (one live record per key in the whole store);
 * together they replay to the pre-compaction map.  The staged state shares the context's fold
 * buffers: a kvr_compact / kvr_replay_live / kvr_replay_last / kvr_replay_index call on the same
 * context in between ends it (kvr_compact_export / _finish then return KVR_EINVAL). */
typedef struct kvr_cand {
    uint64_t pos;       /* (global segment index << 40) | rec_off                                */
    uint32_t key_len;
    uint32_t key_tag;   /* CRC-32 of the key                                                    */
    uint32_t key_off;   /* offset of the key bytes within the owner group's key bytes            */
    uint32_t pad;
} kvr_cand;

int  kvr_compact_stage(kvr_ctx *ctx, const kvr_segment *segs, size_t n_segs, uint32_t flags, const uint32_t *gidx,
                       uint32_t n_ranks, uint64_t *counts, uint64_t *key_bytes, kvr_error *err);
int  kvr_compact_export(kvr_ctx *ctx, kvr_cand *d_hdr, uint8_t *d_keys);
int  kvr_compact_resolve(kvr_ctx *ctx, const kvr_cand *d_hdr, const uint8_t *d_keys, const uint64_t *hdr_counts,
                         const uint64_t *key_counts, uint32_t n_ranks, uint8_t *d_win);
int  kvr_compact_finish(kvr_ctx *ctx, const uint8_t *d_win, uint32_t flags, uint64_t seg_target, uint8_t *out,
                        uint64_t out_cap, uint64_t *out_len, uint64_t *seg_ends, size_t seg_cap, size_t *n_out_segs);

/* ---- batch ETag compute / verify --------------------------------------
 * crc_out[i] = crc32fast::hash(data[offs[i] .. offs[i] + lens[i]]) for n blobs of one buffer:
 * the CRC-32/ISO-HDLC that BlobStorage::put renders as the blob's ETag
 * (src/volume/storage.rs:27, format!("{:08x}", ...); kvr_etag_format renders it).  data is host
 * memory, or device memory with KVR_SEGS_ON_DEVICE; crc_out is host memory, or device memory with
 * KVR_OUT_ON_DEVICE; offs / lens are host arrays.  expected (optional; device memory with
 * KVR_EXPECTED_ON_DEVICE): the stored ETags to verify against (a scrub); *n_fail (optional) =
 * blobs whose CRC differs.  Blobs may overlap and sit at any byte offset.  Returns KVR_OK,
 * KVR_EINVAL (a blob outside [0, data_len)) or < 0. */
typedef struct kvr_etag_stats {
    double   ms_chunk;    /* k_etag_chunk: per-4-KiB-chunk CRC registers (the byte pass)      */
    double   ms_join;     /* k_etag_join: chunk registers -> CRC per blob, verification       */
    uint64_t bytes;       /* blob bytes hashed                                                 */
    uint64_t n_blobs;
    uint64_t n_chunks;
    uint64_t n_fail;
} kvr_etag_stats;

int  kvr_etag_batch(kvr_ctx *ctx, const uint8_t *data, uint64_t data_len, const uint64_t *offs, const uint64_t *lens,
                    size_t n, uint32_t flags, const uint32_t *expected, uint32_t *crc_out, uint64_t *n_fail);
int  kvr_last_etag_stats(const kvr_ctx *ctx, kvr_etag_stats *out);
/* out[0..8] = the ETag text "{:08x}" of crc (lowercase hex) and a terminating NUL. */
void kvr_etag_format(uint32_t crc, char *out);

/* ---- synthetic segment generator (device side; byte-identical to kvh_gen_segment) -------- */
typedef struct kvr_gen_params {
    uint64_t seed;
    uint64_t seg_bytes;        /* target size: records are appended while the next one fits  */
    uint32_t key_space_log2;   /* keys are "k%015u" over [0, 2^key_space_log2)                */
    uint32_t key_dist;         /* 0 = uniform, 1 = Zipf-like (log-uniform bucket, P ~ 1/id)    */
    uint32_t val_min;          /* value length: fixed if val_min == val_max, else log-uniform */
    uint32_t val_max;
    uint32_t del_permille;     /* share of DEL records (per mille)                             */
    uint32_t flip_per_million; /* fault injection: one flipped value bit after the manifest    */
} kvr_gen_params;

/* Generate segment number seg_no (0-based) of a synthetic store into device memory d_buf
 * (capacity cap bytes).  *len_out = bytes written; if d_expected != NULL, the manifest
 * (expected CRC per record, 0 for DEL) is written to device memory d_expected (capacity
 * exp_cap entries) and *n_rec_out = records in the segment. */
int  kvr_gen_segment_device(kvr_ctx *ctx, const kvr_gen_params *p, uint64_t seg_no,
                            uint8_t *d_buf, uint64_t cap, uint64_t *len_out,
                            uint32_t *d_expected, uint64_t exp_cap, uint64_t *n_rec_out);

#ifdef __cplusplus
}
#endif
#endif /* KVREPLAY_H */
