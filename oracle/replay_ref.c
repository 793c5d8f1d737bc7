/*
 * oracle/replay_ref.c — CPU restatement of whispem/mini-kvstore-v2's segment replay.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the HIP engine in
 * mini-kvstore-v2_amd/csrc: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg load it (as liboracle.so via ctypes).  The product never links, calls or falls back to it.
 *
 * What it restates (reference snapshot 0.3.0 at /root/reference, read as text only):
 *   - replay walk ............ src/store/engine.rs:79-154  (oracle_replay)
 *       op byte / clean EOF .. engine.rs:87-92   (any failure to read the op byte ends the segment)
 *       key_len u32 LE ....... engine.rs:95-103  -> KVR_E_KEY_LEN
 *       key bytes ............ engine.rs:106-113 -> KVR_E_KEY
 *       UTF-8 check .......... engine.rs:114-116 -> KVR_E_UTF8 (checked BEFORE the opcode, :118)
 *       SET val_len/value .... engine.rs:119-138 -> KVR_E_VAL_LEN / KVR_E_VAL, then insert (:137)
 *       DEL .................. engine.rs:139-142 (remove; removing an absent key is a no-op)
 *       other opcode ......... engine.rs:143-149 -> KVR_E_OPCODE
 *   - segment order / abort .. engine.rs:51-57 (ascending id; the first error aborts open())
 *   - last-writer-wins fold .. engine.rs:137, :141 (oracle_fold_live)
 *   - CRC-32 ................. crc32fast 1.5.0 (Cargo.lock:252-255) as called at
 *                              src/volume/storage.rs:27: CRC-32/ISO-HDLC, reflected poly
 *                              0xEDB88320, init/xorout 0xFFFFFFFF (crc32fast is a third-party
 *                              crate, absent from /root/reference; its published algorithm is
 *                              restated here and pinned against Python's zlib.crc32)
 *   - UTF-8 validation ....... Rust core::str::from_utf8 (String::from_utf8, engine.rs:114):
 *                              valid_up_to / error_len exactly as Utf8Error reports them
 *   - the reference's cost model for the CPU baseline (oracle_replay_faithful): a BufReader with
 *     the std default 8 KiB buffer (engine.rs:83), two heap allocations per SET (engine.rs:106,
 *     :129), an owning hash map of key -> value (engine.rs:54, :137), plus CRC-32 per value.
 *
 * Pinning: the reference is Rust and cannot be built in this image (no cargo/rustc, SURVEY.md
 * §8c), so this restatement is pinned by the golden vectors in tests/golden/ (restated from the
 * reference's own asserts: examples/persistence.rs, tests/store_integration.rs,
 * examples/compaction.rs, examples/large_dataset.rs) and by zlib.crc32 / Python's UTF-8 decoder
 * (tests/test_oracle_golden.py).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/kvreplay.h"

/* ------------------------------------------------------------------------------------------
 * CRC-32/ISO-HDLC, byte at a time (the table form of crc32fast's baseline algorithm).
 * ---------------------------------------------------------------------------------------- */
static uint32_t g_crc_table[256];
static int g_crc_ready = 0;

static void crc_init(void) {
    if (g_crc_ready) return;
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t c = i;
        for (int k = 0; k < 8; ++k) c = (c & 1u) ? (c >> 1) ^ 0xEDB88320u : (c >> 1);
        g_crc_table[i] = c;
    }
    g_crc_ready = 1;
}

/* crc32fast::Hasher semantics: crc is the running (finalized) value, 0 for a fresh hash. */
uint32_t oracle_crc32(uint32_t crc, const uint8_t *p, size_t n) {
    crc_init();
    uint32_t c = ~crc;
    for (size_t i = 0; i < n; ++i) c = (c >> 8) ^ g_crc_table[(c ^ p[i]) & 0xFFu];
    return ~c;
}

/* ------------------------------------------------------------------------------------------
 * UTF-8 validation with Rust's Utf8Error semantics (core::str::validations::run_utf8_validation).
 * Returns 1 if valid.  Otherwise *valid_up_to = start of the offending sequence and
 * *error_len = 1..3 for an invalid sequence, 0 when the input ends mid-sequence (None).
 * ---------------------------------------------------------------------------------------- */
int oracle_utf8_check(const uint8_t *s, size_t n, uint64_t *valid_up_to, uint32_t *error_len) {
    size_t i = 0;
    while (i < n) {
        const uint8_t b = s[i];
        if (b < 0x80) { ++i; continue; }
        const size_t start = i;
        int width;
        if (b >= 0xC2 && b <= 0xDF) width = 2;
        else if (b >= 0xE0 && b <= 0xEF) width = 3;
        else if (b >= 0xF0 && b <= 0xF4) width = 4;
        else width = 0;
#define FAIL(len_) do { *valid_up_to = start; *error_len = (len_); return 0; } while (0)
#define NEXT(var_) do { if (++i >= n) FAIL(0); (var_) = s[i]; } while (0)
        uint8_t c1, c2, c3;
        switch (width) {
        case 2:
            NEXT(c1);
            if ((c1 & 0xC0) != 0x80) FAIL(1);
            break;
        case 3:
            NEXT(c1);
            if (!((b == 0xE0 && c1 >= 0xA0 && c1 <= 0xBF) ||
                  (b >= 0xE1 && b <= 0xEC && c1 >= 0x80 && c1 <= 0xBF) ||
                  (b == 0xED && c1 >= 0x80 && c1 <= 0x9F) ||
                  (b >= 0xEE && b <= 0xEF && c1 >= 0x80 && c1 <= 0xBF)))
                FAIL(1);
            NEXT(c2);
            if ((c2 & 0xC0) != 0x80) FAIL(2);
            break;
        case 4:
            NEXT(c1);
            if (!((b == 0xF0 && c1 >= 0x90 && c1 <= 0xBF) ||
                  (b >= 0xF1 && b <= 0xF3 && c1 >= 0x80 && c1 <= 0xBF) ||
                  (b == 0xF4 && c1 >= 0x80 && c1 <= 0x8F)))
                FAIL(1);
            NEXT(c2);
            if ((c2 & 0xC0) != 0x80) FAIL(2);
            NEXT(c3);
            if ((c3 & 0xC0) != 0x80) FAIL(3);
            break;
        default:
            FAIL(1);
        }
#undef NEXT
#undef FAIL
        ++i;
    }
    return 1;
}

static inline uint32_t rd_u32le(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

/* ------------------------------------------------------------------------------------------
 * oracle_replay: the engine.rs:53-57 loop over segments + engine.rs:79-154 per segment,
 * emitting one kvr_tuple per record in (segment, offset) order and stopping at the first
 * error (KVStore::open propagates it with `?`, engine.rs:56).
 *   expected/n_expected: optional manifest (tuple order), as in kvr_replay.
 *   Returns KVR_OK, KVR_CORRUPTED (err filled) or KVR_CAPACITY (*n_out = tuples required
 *   for the records seen so far; the walk continues counting).
 * ---------------------------------------------------------------------------------------- */
typedef struct oracle_seg { uint64_t seg_id; const uint8_t *bytes; uint64_t len; } oracle_seg;

int oracle_replay(const oracle_seg *segs, size_t n_segs,
                  const uint32_t *expected, size_t n_expected,
                  kvr_tuple *out, size_t cap, size_t *n_out, kvr_error *err) {
    size_t nt = 0;
    int status = KVR_OK;
    if (err) memset(err, 0, sizeof(*err));
    for (size_t si = 0; si < n_segs; ++si) {
        const uint8_t *b = segs[si].bytes;
        const uint64_t n = segs[si].len;
        uint64_t p = 0;
        for (;;) {
            if (p >= n) break;                                 /* engine.rs:88-91 clean EOF */
            const uint8_t op = b[p];
            kvr_error e = {0, (uint32_t)si, p, 0};
            if (n - p < 5) { e.kind = KVR_E_KEY_LEN; goto fail; }          /* :96-102  */
            const uint64_t klen = rd_u32le(b + p + 1);
            if (n - (p + 5) < klen) { e.kind = KVR_E_KEY; goto fail; }     /* :107-113 */
            {
                uint64_t vu; uint32_t el;
                if (!oracle_utf8_check(b + p + 5, (size_t)klen, &vu, &el)) { /* :114-116 */
                    e.kind = KVR_E_UTF8; e.aux = vu | ((uint64_t)el << 32); goto fail;
                }
            }
            kvr_tuple t;
            memset(&t, 0, sizeof(t));
            t.rec_off = p; t.seg_idx = (uint32_t)si; t.key_len = (uint32_t)klen; t.op = op;
            t.key_tag = oracle_crc32(0, b + p + 5, (size_t)klen);
            uint64_t next;
            if (op == 0) {
                const uint64_t q = p + 5 + klen;
                if (n - q < 4) { e.kind = KVR_E_VAL_LEN; goto fail; }      /* :121-127 */
                const uint64_t vlen = rd_u32le(b + q);
                if (n - (q + 4) < vlen) { e.kind = KVR_E_VAL; goto fail; } /* :130-136 */
                t.val_len = (uint32_t)vlen;
                t.crc32 = oracle_crc32(0, b + q + 4, (size_t)vlen);
                next = q + 4 + vlen;
                if (expected && nt < n_expected) {
                    t.flags |= KVR_TF_VERIFIED;
                    if (expected[nt] != t.crc32) t.flags |= KVR_TF_CRC_FAIL;
                }
            } else if (op == 1) {
                next = p + 5 + klen;                                     /* :139-142 */
            } else {
                e.kind = KVR_E_OPCODE; e.aux = op; goto fail;            /* :143-149 */
            }
            if (out && nt < cap) out[nt] = t;
            ++nt;
            p = next;
            continue;
        fail:
            if (err) *err = e;
            if (n_out) *n_out = nt;
            return KVR_CORRUPTED;
        }
    }
    if (n_out) *n_out = nt;
    if (out && nt > cap) status = KVR_CAPACITY;
    return status;
}

/* ------------------------------------------------------------------------------------------
 * oracle_replay_s16 — the strong CPU baseline (SURVEY §8d ii): oracle_replay's walk and tuples
 * with a slice-by-16 CRC-32 (16 byte tables, 16 bytes per step), for one thread per segment.
 * Same results as oracle_replay (tests/test_oracle_golden.py compares them).
 * ---------------------------------------------------------------------------------------- */
static uint32_t g_s16[16][256];
static int g_s16_ready = 0;

static void s16_init(void) {
    crc_init();
    for (int i = 0; i < 256; ++i) g_s16[0][i] = g_crc_table[i];
    for (int t = 1; t < 16; ++t)
        for (int i = 0; i < 256; ++i) g_s16[t][i] = (g_s16[t - 1][i] >> 8) ^ g_s16[0][g_s16[t - 1][i] & 0xFFu];
    g_s16_ready = 1;
}

uint32_t oracle_crc32_s16(uint32_t crc, const uint8_t *p, size_t n) {
    if (!g_s16_ready) s16_init();
    uint32_t c = ~crc;
    while (n >= 16) {
        const uint32_t a = rd_u32le(p) ^ c, b = rd_u32le(p + 4), d = rd_u32le(p + 8), e = rd_u32le(p + 12);
        c = g_s16[15][a & 255] ^ g_s16[14][(a >> 8) & 255] ^ g_s16[13][(a >> 16) & 255] ^ g_s16[12][a >> 24] ^
            g_s16[11][b & 255] ^ g_s16[10][(b >> 8) & 255] ^ g_s16[9][(b >> 16) & 255] ^ g_s16[8][b >> 24] ^
            g_s16[7][d & 255] ^ g_s16[6][(d >> 8) & 255] ^ g_s16[5][(d >> 16) & 255] ^ g_s16[4][d >> 24] ^
            g_s16[3][e & 255] ^ g_s16[2][(e >> 8) & 255] ^ g_s16[1][(e >> 16) & 255] ^ g_s16[0][e >> 24];
        p += 16;
        n -= 16;
    }
    while (n--) c = (c >> 8) ^ g_s16[0][(c ^ *p++) & 0xFFu];
    return ~c;
}

int oracle_replay_s16(const oracle_seg *segs, size_t n_segs, kvr_tuple *out, size_t cap, size_t *n_out,
                      kvr_error *err) {
    if (!g_s16_ready) s16_init();
    size_t nt = 0;
    if (err) memset(err, 0, sizeof(*err));
    for (size_t si = 0; si < n_segs; ++si) {
        const uint8_t *b = segs[si].bytes;
        const uint64_t n = segs[si].len;
        uint64_t p = 0;
        while (p < n) {                                                   /* engine.rs:88-91 */
            const uint8_t op = b[p];
            kvr_error e = {0, (uint32_t)si, p, 0};
            if (n - p < 5) { e.kind = KVR_E_KEY_LEN; goto fail; }
            const uint64_t klen = rd_u32le(b + p + 1);
            if (n - (p + 5) < klen) { e.kind = KVR_E_KEY; goto fail; }
            {
                uint64_t vu; uint32_t el;
                if (!oracle_utf8_check(b + p + 5, (size_t)klen, &vu, &el)) {
                    e.kind = KVR_E_UTF8; e.aux = vu | ((uint64_t)el << 32); goto fail;
                }
            }
            kvr_tuple t;
            memset(&t, 0, sizeof(t));
            t.rec_off = p; t.seg_idx = (uint32_t)si; t.key_len = (uint32_t)klen; t.op = op;
            t.key_tag = oracle_crc32_s16(0, b + p + 5, (size_t)klen);
            uint64_t next;
            if (op == 0) {
                const uint64_t q = p + 5 + klen;
                if (n - q < 4) { e.kind = KVR_E_VAL_LEN; goto fail; }
                const uint64_t vlen = rd_u32le(b + q);
                if (n - (q + 4) < vlen) { e.kind = KVR_E_VAL; goto fail; }
                t.val_len = (uint32_t)vlen;
                t.crc32 = oracle_crc32_s16(0, b + q + 4, (size_t)vlen);
                next = q + 4 + vlen;
            } else if (op == 1) {
                next = p + 5 + klen;
            } else {
                e.kind = KVR_E_OPCODE; e.aux = op; goto fail;
            }
            if (out && nt < cap) out[nt] = t;
            ++nt;
            p = next;
            continue;
        fail:
            if (err) *err = e;
            if (n_out) *n_out = nt;
            return KVR_CORRUPTED;
        }
    }
    if (n_out) *n_out = nt;
    return (out && nt > cap) ? KVR_CAPACITY : KVR_OK;
}

/* ------------------------------------------------------------------------------------------
 * Last-writer-wins fold (engine.rs:137 insert / :141 remove, segments in id order :55):
 * live[i] = 1 iff tuple i is a SET and no later tuple (in tuple order) names the same key.
 * Keys are compared by bytes (read at rec_off + 5 of their segment).  Returns live count.
 * ---------------------------------------------------------------------------------------- */
typedef struct { uint64_t h; int64_t idx; } slot_t;

static uint64_t key_hash(const uint8_t *k, size_t n) {
    uint64_t h = 1469598103934665603ull;                 /* FNV-1a 64 */
    for (size_t i = 0; i < n; ++i) { h ^= k[i]; h *= 1099511628211ull; }
    return h | 1;                                         /* 0 marks an empty slot */
}

size_t oracle_fold_live(const oracle_seg *segs, const kvr_tuple *t, size_t n, uint8_t *live,
                        uint64_t *total_bytes) {
    size_t cap = 16;
    while (cap < 2 * n + 16) cap <<= 1;
    slot_t *tab = (slot_t *)calloc(cap, sizeof(slot_t));
    if (!tab) return (size_t)-1;
    for (size_t i = 0; i < n; ++i) live[i] = 0;
    for (size_t i = 0; i < n; ++i) {
        const uint8_t *k = segs[t[i].seg_idx].bytes + t[i].rec_off + 5;
        const uint64_t h = key_hash(k, t[i].key_len);
        size_t j = (size_t)(h & (cap - 1));
        for (;;) {
            if (tab[j].h == 0) { tab[j].h = h; tab[j].idx = (int64_t)i; break; }
            if (tab[j].h == h) {
                const kvr_tuple *o = &t[tab[j].idx];
                const uint8_t *ok = segs[o->seg_idx].bytes + o->rec_off + 5;
                if (o->key_len == t[i].key_len && memcmp(ok, k, t[i].key_len) == 0) {
                    tab[j].idx = (int64_t)i; break;               /* later record wins */
                }
            }
            j = (j + 1) & (cap - 1);
        }
    }
    size_t nlive = 0;
    uint64_t tb = 0;
    for (size_t j = 0; j < cap; ++j) {
        if (tab[j].h && t[tab[j].idx].op == 0) {
            live[tab[j].idx] = 1; ++nlive; tb += t[tab[j].idx].val_len;
        }
    }
    free(tab);
    if (total_bytes) *total_bytes = tb;                   /* stats().total_bytes, engine.rs:255 */
    return nlive;                                         /* stats().num_keys,   engine.rs:253 */
}

/* ------------------------------------------------------------------------------------------
 * oracle_compact — the intended KVStore::compact (README.md:283-287: "collect all live keys,
 * write to new segments, delete old segments"; the reference's compaction.rs:9-29 deletes the
 * files without rewriting a key).  Replay (engine.rs:79-154), keep each key's final
 * SET (oracle_fold_live: engine.rs:137 / :141), copy those records byte for byte in tuple order
 * (a record's own bytes are its engine.rs:169-173 framing).  A new segment starts at the first
 * record whose output offset is >= k * seg_target, k = 1, 2, ...; seg_target 0 = one segment.
 * seg_ends[j] = end offset of segment j.  Returns KVR_OK, KVR_CORRUPTED (*err), KVR_CAPACITY
 * (*out_len, *n_out_segs = required) or KVR_ENOMEM.
 * ---------------------------------------------------------------------------------------- */
int oracle_compact(const oracle_seg *segs, size_t n_segs, uint64_t seg_target, uint8_t *out, uint64_t out_cap,
                   uint64_t *out_len, uint64_t *seg_ends, size_t seg_cap, size_t *n_out_segs, kvr_error *err) {
    *out_len = 0;
    *n_out_segs = 0;
    uint64_t total_in = 0;
    for (size_t i = 0; i < n_segs; ++i) total_in += segs[i].len;
    size_t cap = (size_t)(total_in / 5 + 16), nt = 0;
    kvr_tuple *t = (kvr_tuple *)malloc(cap * sizeof(kvr_tuple));
    uint8_t *live = (uint8_t *)malloc(cap + 1);
    if (!t || !live) { free(t); free(live); return KVR_ENOMEM; }
    int rc = oracle_replay(segs, n_segs, NULL, 0, t, cap, &nt, err);
    if (rc != KVR_OK) { free(t); free(live); return rc; }
    oracle_fold_live(segs, t, nt, live, NULL);
    /* output offsets of the live records, then the cuts */
    uint64_t total = 0;
    for (size_t i = 0; i < nt; ++i)
        if (live[i]) total += 9ull + t[i].key_len + t[i].val_len;
    size_t nseg = 0;
    uint64_t next_cut = seg_target, pos = 0;
    int over = total > out_cap;
    for (size_t i = 0; i < nt; ++i) {
        if (!live[i]) continue;
        const uint64_t sz = 9ull + t[i].key_len + t[i].val_len;
        if (seg_target && pos >= next_cut && pos > 0) {      /* this record starts a new segment */
            if (nseg < seg_cap) seg_ends[nseg] = pos;
            ++nseg;
            while (next_cut <= pos) next_cut += seg_target;  /* every k with k * T <= pos is served */
        }
        if (!over) memcpy(out + pos, segs[t[i].seg_idx].bytes + t[i].rec_off, sz);
        pos += sz;
    }
    if (total) {
        if (nseg < seg_cap) seg_ends[nseg] = total;
        ++nseg;
    }
    free(t);
    free(live);
    *out_len = total;
    *n_out_segs = nseg;
    return (over || nseg > seg_cap) ? KVR_CAPACITY : KVR_OK;
}

/* ------------------------------------------------------------------------------------------
 * oracle_replay_faithful — the CPU baseline: the reference's replay cost model, single thread.
 * Reads through an 8 KiB buffered reader (engine.rs:83; large reads bypass the buffer as
 * std's BufReader does), allocates the key and the value per record (engine.rs:106, :129),
 * validates UTF-8, keeps an owning key -> value hash map with replacement/removal
 * (engine.rs:137, :141) and CRC-32s every value (storage.rs:27).  Returns KVR_OK or
 * KVR_CORRUPTED; outputs num_keys / total_bytes (stats(), engine.rs:253-255), the number of
 * records and an order-independent digest of the final map.
 * ---------------------------------------------------------------------------------------- */
typedef struct { const uint8_t *src; uint64_t len, pos; uint8_t buf[8192]; size_t bpos, bfill; } bufrd_t;

static int br_read_exact(bufrd_t *r, uint8_t *dst, size_t n) {
    /* std::io::BufReader::read_exact: serve from the buffer, bypass it for large reads */
    size_t have = r->bfill - r->bpos;
    if (have >= n) { memcpy(dst, r->buf + r->bpos, n); r->bpos += n; return 0; }
    memcpy(dst, r->buf + r->bpos, have); dst += have; n -= have; r->bpos = r->bfill = 0;
    while (n > 0) {
        if (n >= sizeof(r->buf)) {
            uint64_t avail = r->len - r->pos;
            if (avail == 0) return -1;
            size_t k = n < avail ? n : (size_t)avail;
            memcpy(dst, r->src + r->pos, k); r->pos += k; dst += k; n -= k;
        } else {
            uint64_t avail = r->len - r->pos;
            if (avail == 0) return -1;
            size_t k = sizeof(r->buf) < avail ? sizeof(r->buf) : (size_t)avail;
            memcpy(r->buf, r->src + r->pos, k); r->pos += k; r->bfill = k; r->bpos = 0;
            size_t c = n < k ? n : k;
            memcpy(dst, r->buf, c); r->bpos = c; dst += c; n -= c;
        }
    }
    return 0;
}

typedef struct { uint64_t h; uint8_t *key; uint32_t klen; uint8_t *val; uint32_t vlen; int used; } mslot_t;
typedef struct { mslot_t *s; size_t cap, n, tomb; } vmap_t;

static void vm_grow(vmap_t *m);
static mslot_t *vm_find(vmap_t *m, const uint8_t *k, uint32_t kl, uint64_t h, int insert) {
    if (insert && (m->n + m->tomb + 1) * 4 > m->cap * 3) vm_grow(m);
    size_t j = (size_t)(h & (m->cap - 1));
    mslot_t *first_tomb = NULL;
    for (;;) {
        mslot_t *s = &m->s[j];
        if (s->used == 0) {
            if (!insert) return NULL;
            if (first_tomb) { s = first_tomb; m->tomb--; }
            s->used = 1; s->h = h; s->key = NULL; s->klen = kl; s->val = NULL; s->vlen = 0; m->n++;
            return s;
        }
        if (s->used == 2) { if (!first_tomb) first_tomb = s; }
        else if (s->h == h && s->klen == kl && memcmp(s->key, k, kl) == 0) return s;
        j = (j + 1) & (m->cap - 1);
    }
}
static void vm_grow(vmap_t *m) {
    mslot_t *old = m->s; size_t oc = m->cap;
    m->cap = oc ? oc * 2 : 1024; m->s = (mslot_t *)calloc(m->cap, sizeof(mslot_t)); m->n = 0; m->tomb = 0;
    for (size_t i = 0; i < oc; ++i) if (old[i].used == 1) {
        size_t j = (size_t)(old[i].h & (m->cap - 1));
        while (m->s[j].used) j = (j + 1) & (m->cap - 1);
        m->s[j] = old[i]; m->n++;
    }
    free(old);
}

/* the map the last faithful replay built: KVStore::open hands it to the caller (engine.rs:70-75)
 * rather than dropping it, so releasing it is not part of the timed replay */
static vmap_t g_faithful_map = {0};

void oracle_faithful_release(void) {
    vmap_t *m = &g_faithful_map;
    for (size_t i = 0; i < m->cap; ++i) if (m->s[i].used == 1) { free(m->s[i].key); free(m->s[i].val); }
    free(m->s);
    memset(m, 0, sizeof(*m));
}

int oracle_replay_faithful(const oracle_seg *segs, size_t n_segs, uint64_t *num_keys,
                           uint64_t *total_bytes, uint64_t *n_records, uint64_t *digest,
                           kvr_error *err) {
    oracle_faithful_release();
    vmap_t m = {0}; vm_grow(&m);
    bufrd_t *r = (bufrd_t *)malloc(sizeof(bufrd_t));
    uint64_t nrec = 0, crc_acc = 0;
    int status = KVR_OK;
    for (size_t si = 0; si < n_segs && status == KVR_OK; ++si) {
        r->src = segs[si].bytes; r->len = segs[si].len; r->pos = 0; r->bpos = r->bfill = 0;
        uint64_t off = 0;
        for (;;) {
            uint8_t op, lb[4];
            if (br_read_exact(r, &op, 1)) break;
            kvr_error e = {0, (uint32_t)si, off, 0};
            if (br_read_exact(r, lb, 4)) { e.kind = KVR_E_KEY_LEN; goto bad; }
            uint32_t kl = rd_u32le(lb);
            uint8_t *key = (uint8_t *)malloc(kl ? kl : 1);
            if (br_read_exact(r, key, kl)) { free(key); e.kind = KVR_E_KEY; goto bad; }
            uint64_t vu; uint32_t el;
            if (!oracle_utf8_check(key, kl, &vu, &el)) {
                free(key); e.kind = KVR_E_UTF8; e.aux = vu | ((uint64_t)el << 32); goto bad;
            }
            uint64_t h = key_hash(key, kl);
            if (op == 0) {
                if (br_read_exact(r, lb, 4)) { free(key); e.kind = KVR_E_VAL_LEN; goto bad; }
                uint32_t vl = rd_u32le(lb);
                uint8_t *val = (uint8_t *)malloc(vl ? vl : 1);
                if (br_read_exact(r, val, vl)) { free(key); free(val); e.kind = KVR_E_VAL; goto bad; }
                crc_acc += oracle_crc32(0, val, vl);
                mslot_t *s = vm_find(&m, key, kl, h, 1);
                if (s->key) free(key); else s->key = key;         /* HashMap::insert keeps the old key */
                free(s->val); s->val = val; s->vlen = vl;
                off += 9ull + kl + vl;
            } else if (op == 1) {
                mslot_t *s = vm_find(&m, key, kl, h, 0);
                if (s) { free(s->key); free(s->val); s->used = 2; s->key = NULL; s->val = NULL; m.n--; m.tomb++; }
                free(key);
                off += 5ull + kl;
            } else {
                free(key); e.kind = KVR_E_OPCODE; e.aux = op; goto bad;
            }
            ++nrec;
            continue;
        bad:
            if (err) *err = e;
            status = KVR_CORRUPTED;
            break;
        }
    }
    /* stats() (engine.rs:253-255) and a digest from what the walk already computed: the per-value
     * CRCs summed during the replay and the live keys' hashes and lengths (no second pass over
     * the values) */
    uint64_t nk = m.n, tb = 0, dg = crc_acc * 0x9E3779B97F4A7C15ull;
    for (size_t i = 0; i < m.cap; ++i) if (m.s[i].used == 1) {
        tb += m.s[i].vlen;
        dg += (uint64_t)m.s[i].vlen * (m.s[i].h | 1);
    }
    g_faithful_map = m;
    free(r);
    if (num_keys) *num_keys = nk;
    if (total_bytes) *total_bytes = tb;
    if (n_records) *n_records = nrec;
    if (digest) *digest = dg;
    return status;
}
