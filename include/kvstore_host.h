/*
 * kvstore_host.h — host side of the drop-in: the KVStore::open path of
 * whispem/mini-kvstore-v2 (src/store/engine.rs:24-76) rebuilt around kvr_replay.
 *
 *   kvh_discover      segment discovery + ordering        engine.rs:31-51
 *   kvh_gen_segment   synthetic segments, framing writer  engine.rs:157-198 (byte-identical to
 *                     kvr_gen_segment_device)
 *   kvh_fold          last-writer-wins index fold         engine.rs:137 (insert), :141 (remove)
 *   kvs_open / kvs_get / kvs_stats / kvs_compact / kvs_close
 *                     the crate-public KVStore surface the replay path feeds (lib.rs:2-3,
 *                     engine.rs:24, :200, :232-259); the index has the shape of the reference's
 *                     dead `Index` (src/store/index.rs:7): key -> (segment, offset, length).
 *
 * Status codes and kvr_error are those of kvreplay.h.
 */
#ifndef KVSTORE_HOST_H
#define KVSTORE_HOST_H

#include <stddef.h>
#include <stdint.h>

#include "kvreplay.h"

#ifdef __cplusplus
extern "C" {
#endif

/* CPU generator: same bytes and manifest as kvr_gen_segment_device for (p, seg_no).
 * buf may be NULL to only size the segment (*len_out, *n_rec_out). */
int kvh_gen_segment(const kvr_gen_params *p, uint64_t seg_no, uint8_t *buf, uint64_t cap, uint64_t *len_out,
                    uint32_t *expected, uint64_t exp_cap, uint64_t *n_rec_out);

/* Discovery as engine.rs:31-51: entries of dir named "segment-<id>.dat" whose <id> parses as a
 * Rust u64 (optional '+', ASCII digits, no overflow), in ascending id order (ties by name).
 * Writes up to cap ids to ids[] and NUL-separated full paths into paths (path_cap bytes);
 * *n_out = number of segments found.  Returns KVR_OK, KVR_CAPACITY or KVR_EIO. */
int kvh_discover(const char *dir, uint64_t *ids, size_t cap, char *paths, size_t path_cap, size_t *n_out);

/* Rust `u64::from_str` on [s, s+n): returns 1 and *out on success. */
int kvh_parse_u64(const char *s, size_t n, uint64_t *out);

/* Fold tuples (in (segment, offset) order) by last-writer-wins.  Keys are read from
 * segs[t.seg_idx].bytes + t.rec_off + 5 (host memory).  live[i] = 1 iff tuple i is the final
 * SET of its key.  Returns the number of live keys (stats().num_keys) and *total_bytes
 * (stats().total_bytes, engine.rs:253-255). */
uint64_t kvh_fold(const kvr_segment *segs, const kvr_tuple *t, size_t n, uint8_t *live, uint64_t *total_bytes);
/* The same fold on n_threads host threads (0 = all cores): keys are split by
 * key_tag into one partition per thread (the last writer of a key is its maximal (segment,
 * offset) record, so partitions fold independently).  Same results as kvh_fold. */
uint64_t kvh_fold_parallel(const kvr_segment *segs, const kvr_tuple *t, size_t n, uint32_t n_threads,
                           uint8_t *live, uint64_t *total_bytes);

typedef struct kvs_store kvs_store;

typedef struct kvs_stats {          /* StoreStats, src/store/stats.rs:3-10 */
    uint64_t num_keys;
    uint64_t num_segments;
    uint64_t total_bytes;
    uint64_t active_segment_id;
    uint64_t oldest_segment_id;
} kvs_stats;

/* KVStore::open(dir): create the directory if missing, discover and read the segments,
 * replay them on ctx's GPU, fold the index, create the next active segment file
 * (engine.rs:59-68).  On KVR_CORRUPTED, *err and msg (the exact engine.rs message, without
 * error.rs's "Corrupted data: " prefix) describe the first error. */
int kvs_open(const char *dir, kvr_ctx *ctx, kvs_store **out, kvr_error *err, char *msg, size_t msg_cap);
/* kvs_open with options.  The default path maps every segment file read-only (mmap, populated
 * from the page cache by up to 16 threads: the store's host bytes are the page cache, no copy),
 * registers each mapping for DMA (kvr_host_register) and pushes the segment to HBM
 * (kvr_ingest_push) in store order.  KVS_OPEN_PREAD (or a failed mmap) reads the files instead:
 * 16 threads pread 8-MiB pieces into one arena on 2-MiB pages, and groups of consecutive segments
 * (>= 256 MiB) are registered and pushed as soon as their bytes are in, so reading and PCIe
 * overlap.  Then kvr_ingest_index replays, folds and builds the key table on the GPU and only the
 * live tuples and the table come back.  When the store does not fit in HBM (KVR_ENOMEM) or
 * exceeds the fold's 2^31-tuple limit (KVR_EINVAL), the host-fold path takes over:
 * kvr_replay_stream in batches, kvh_fold_parallel, kvr_index_build_host.  Both give the same index.
 * An unopenable segment k is reported (KVR_E_OPEN) only when segments 0 .. k-1 replay cleanly,
 * as engine.rs:55-57 opens the files one after the other.
 * Segment files must not be truncated by another process while the store is open: a mapped page
 * past the new end of file raises SIGBUS when it is touched (later DMA re-reads, compaction).  The
 * store itself only appends to the active file, and kvs_compact writes new files and unlinks the
 * old ones (an unlinked file's mapping keeps its pages), so its own mappings never lose bytes;
 * KVS_OPEN_PREAD copies the bytes and is immune to outside truncation. */
#define KVS_OPEN_HOST_FOLD  0x1u   /* force the host-fold path                         */
#define KVS_OPEN_NO_PIN     0x2u   /* no kvr_host_register: HIP stages the transfers    */
#define KVS_OPEN_PREAD      0x4u   /* read the files into an arena instead of mapping   */
#define KVS_PATH_DEVICE_INDEX 1u
#define KVS_PATH_HOST_FOLD    2u
#define KVS_LOAD_MMAP  1u
#define KVS_LOAD_PREAD 2u
typedef struct kvs_open_stats {
    double   ms_total;       /* the whole kvs_open_ex call                                        */
    double   ms_register;    /* kvr_host_register calls (inside ms_read)                           */
    double   ms_push;        /* kvr_ingest_push calls (inside ms_read)                             */
    double   ms_read;        /* loading: mapping or reading, registration, pushes                  */
    double   ms_index;       /* after loading -> index ready: transfer tail, replay, fold, copies  */
    uint64_t bytes;          /* segment bytes                                                      */
    uint64_t n_segments;
    uint64_t n_live;         /* stats().num_keys                                                   */
    uint32_t path;           /* KVS_PATH_DEVICE_INDEX or KVS_PATH_HOST_FOLD (last index build)      */
    uint32_t read_threads;
    uint32_t mode;           /* KVS_LOAD_MMAP or KVS_LOAD_PREAD                                     */
    uint32_t pad;
} kvs_open_stats;
/* ctx may be NULL: the store then opens on the host only, which succeeds only when its segments
 * hold no bytes (a new or emptied store); a store with records returns KVR_EINVAL. */
int kvs_open_ex(const char *dir, kvr_ctx *ctx, uint32_t flags, kvs_store **out, kvr_error *err, char *msg,
                size_t msg_cap);
int kvs_last_open_stats(const kvs_store *s, kvs_open_stats *out);
/* KVStore::get (engine.rs:200): 1 and the value bytes if live, 0 if absent. */
int kvs_get(const kvs_store *s, const uint8_t *key, size_t klen, const uint8_t **val, size_t *vlen);
/* Index entry (index.rs:7 shape): segment id, value offset inside that segment file, length. */
int kvs_locate(const kvs_store *s, const uint8_t *key, size_t klen, uint64_t *seg_id, uint64_t *val_off, uint64_t *len);
int kvs_stats_get(const kvs_store *s, kvs_stats *out);
/* KVStore::compact (engine.rs:262-266 -> compaction.rs:9-29) with the intended semantics of
 * README.md:283-287 (the reference deletes every segment without rewriting a key):
 * kvr_compact rewrites the live records into new files segment-<active+1>.dat, ... (segments
 * of about seg_target bytes, 0 = one file), written and fsync'd before every other
 * segment-*.dat is removed (compaction.rs:11-23); then a fresh empty active segment is created
 * (reset_active_segment, engine.rs:209-229) and the index is rebuilt over the new files.  A crash
 * between the writes and the removals leaves old and new files, whose replay gives the same map.
 * Returns KVR_OK, KVR_CORRUPTED (*err) or < 0 (KVR_EIO: a file could not be written/removed). */
int kvs_compact(kvs_store *s, kvr_ctx *ctx, uint64_t seg_target, kvr_error *err);
/* KVStore::list_keys: up to cap keys as (offset, length) pairs into the returned arena. */
size_t kvs_num_keys(const kvs_store *s);
void kvs_close(kvs_store *s);

#ifdef __cplusplus
}
#endif
#endif
