/*
 * kvr_gen_common.h — the synthetic segment generator's record model, shared by the host
 * generator (kvh_gen_segment, kvr_host.cpp) and the device fill kernel (kvr_replay.hip) so
 * both emit byte-identical segments for the same (seed, segment number).
 *
 * Framing is exactly the reference writer's (src/store/engine.rs:157-198):
 *   SET  [0u8][key_len u32 LE][key][val_len u32 LE][value]     engine.rs:169-173
 *   DEL  [1u8][key_len u32 LE][key]                            engine.rs:191-193
 * Records are appended while the next one fits into seg_bytes, so every segment ends on a
 * record boundary (a clean EOF at an opcode boundary, engine.rs:88-91).
 *
 * Record i of segment s is a pure function of (seed, s, i) through splitmix64, so any record
 * can be produced independently (the device kernel fills records in parallel):
 *   op      DEL with probability del_permille / 1000
 *   key     "k%015llu" of an id: uniform over [0, 2^key_space_log2) or Zipf-like (a uniformly
 *           chosen power-of-two bucket b, then uniform in [2^b - 1, 2^(b+1) - 1): P(id) ~ 1/id)
 *   vlen    fixed (val_min == val_max) or log-uniform: a uniform octave o in [0, nb), then
 *           uniform in [val_min*2^o, val_min*2^(o+1)), nb = max{o : val_min*2^o <= val_max}
 *   value   byte j = byte (j & 7) of mix64(vseed + (j >> 3)), little-endian
 *   fault   with probability flip_per_million / 1e6 one value bit is flipped AFTER the
 *           manifest CRC (the expected ETag, storage.rs:27) has been taken from the clean value
 */
#ifndef KVR_GEN_COMMON_H
#define KVR_GEN_COMMON_H

#include <stdint.h>
#include "../../include/kvreplay.h"

#if defined(__HIPCC__)
#define KVR_HD __host__ __device__ inline
#else
#define KVR_HD static inline
#endif

#define KVR_GEN_KEY_LEN 16u

KVR_HD uint64_t kvr_mix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

KVR_HD uint64_t kvr_gen_sbase(uint64_t seed, uint64_t seg_no) {
    return kvr_mix64(seed ^ kvr_mix64(seg_no ^ 0x5EB5EB5EB5EB5EB5ull));
}

KVR_HD uint64_t kvr_gen_r(uint64_t sbase, uint64_t i, uint32_t k) {
    return kvr_mix64(sbase ^ kvr_mix64((i << 4) | (uint64_t)k));
}

typedef struct kvr_gen_rec {
    uint32_t op;        /* 0 SET, 1 DEL                                 */
    uint32_t vlen;      /* 0 for DEL                                    */
    uint64_t key_id;
    uint64_t vseed;
    int64_t  flip_bit;  /* bit index into the value, -1 = no fault       */
} kvr_gen_rec;

KVR_HD uint32_t kvr_gen_octaves(uint32_t lo, uint32_t hi) {
    uint32_t nb = 0;
    while (nb < 31 && ((uint64_t)lo << (nb + 1)) <= (uint64_t)hi) ++nb;
    return nb;
}

KVR_HD void kvr_gen_record(const kvr_gen_params *p, uint64_t sbase, uint64_t i, kvr_gen_rec *r) {
    r->op = (kvr_gen_r(sbase, i, 0) % 1000u) < p->del_permille ? 1u : 0u;
    const uint32_t ksl = p->key_space_log2 == 0 ? 1u : (p->key_space_log2 > 48 ? 48u : p->key_space_log2);
    if (p->key_dist == 0) {
        r->key_id = kvr_gen_r(sbase, i, 1) & ((1ull << ksl) - 1ull);
    } else {
        const uint32_t b = (uint32_t)(kvr_gen_r(sbase, i, 1) % ksl);
        r->key_id = ((1ull << b) - 1ull) + (kvr_gen_r(sbase, i, 2) & ((1ull << b) - 1ull));
    }
    if (r->op) {
        r->vlen = 0;
    } else if (p->val_min >= p->val_max) {
        r->vlen = p->val_min;
    } else {
        const uint32_t lo = p->val_min ? p->val_min : 1u;
        const uint32_t nb = kvr_gen_octaves(lo, p->val_max);
        if (nb == 0) {
            r->vlen = lo + (uint32_t)(kvr_gen_r(sbase, i, 3) % (uint64_t)(p->val_max - lo + 1u));
        } else {
            const uint32_t o = (uint32_t)(kvr_gen_r(sbase, i, 3) % nb);
            const uint64_t base = (uint64_t)lo << o;
            r->vlen = (uint32_t)(base + kvr_gen_r(sbase, i, 4) % base);
        }
    }
    r->vseed = kvr_gen_r(sbase, i, 5);
    r->flip_bit = -1;
    if (r->vlen && (kvr_gen_r(sbase, i, 6) % 1000000u) < p->flip_per_million)
        r->flip_bit = (int64_t)(kvr_gen_r(sbase, i, 7) % (8ull * r->vlen));
}

KVR_HD uint64_t kvr_gen_rec_size(const kvr_gen_rec *r) {
    return r->op ? 5ull + KVR_GEN_KEY_LEN : 9ull + KVR_GEN_KEY_LEN + r->vlen;
}

/* key bytes: 'k' followed by 15 zero-padded decimal digits of key_id mod 10^15 */
KVR_HD void kvr_gen_key(uint64_t key_id, uint8_t out[KVR_GEN_KEY_LEN]) {
    uint64_t v = key_id % 1000000000000000ull;
    out[0] = 'k';
    for (int d = 15; d >= 1; --d) { out[d] = (uint8_t)('0' + (v % 10u)); v /= 10u; }
}

/* value byte j before fault injection */
KVR_HD uint8_t kvr_gen_vbyte(uint64_t vseed, uint64_t j) {
    return (uint8_t)(kvr_mix64(vseed + (j >> 3)) >> (8u * (uint32_t)(j & 7u)));
}

#endif /* KVR_GEN_COMMON_H */
