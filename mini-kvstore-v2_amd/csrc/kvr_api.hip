/*
 * kvr_api.hip — the C ABI of include/kvreplay.h: contexts, device arenas, the launch
 * pipeline of one replay call, the device-side generator and host helpers.
 *
 * One kvr_replay call:
 *   [H2D of host segments]  k_replay(all stripes)  k_link  k_rewalk(re-walk list)  k_link
 *   k_compact_s  [D2H of tuples]  — one stream, one host synchronisation in the
 *   common case; k_rewalk/k_link rounds only when a speculated stripe entry was wrong (a re-walk
 *   walks on through the wrongly speculated stripes after its own, so one round is the usual case).
 */
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include <hipcub/hipcub.hpp>

#include "kvr_replay_kernel.hip"
#include "kvr_kernels.hip"
#include "kvr_compact.hip"
#include "kvr_etag.hip"

using namespace kvr;

// the replay kernel (kvr_replay_kernel.hip): KR_WPB = stripes per workgroup,
// KR_TILE = tile bytes
#define KR_KERNEL k_replay
static constexpr int KR_RT = RT, KR_WPB = WPB, KR_TILE = TILE, RW_WPB = RT_REWALK / 64;

namespace {

template <class T>
struct DevBuf {
    T *p = nullptr;
    size_t n = 0;
    int ensure(size_t m) {
        if (m <= n && p) return 0;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        if (m == 0) m = 1;
        if (hipMalloc(&p, m * sizeof(T)) != hipSuccess) { p = nullptr; return -1; }
        n = m;
        return 0;
    }
    void release() { if (p) (void)hipFree(p); p = nullptr; n = 0; }
};

constexpr uint32_t REDO_GRID = 1024;
constexpr size_t LC_CTR = 64;                     // Counters' offset in the link + counters block
constexpr size_t LC_BYTES = LC_BLOCK;
static_assert(sizeof(LinkResult) <= LC_CTR && LC_CTR + sizeof(Counters) <= LC_BYTES, "link + counters block");
// stripes up to which k_compact_s links the stripes itself (each workgroup sums the counts before
// its stripe: O(stripes^2) reads in all); more, and k_link runs first
constexpr uint32_t LINKED_MAX_STRIPES = 8192;

// wait for the work queued on st: a host spin on an event for up to 20 ms (a blocking wait wakes
// tens of microseconds after a short pipeline ends), then a blocking wait
hipError_t wait_event(hipEvent_t ev) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        const hipError_t e = hipEventQuery(ev);
        if (e != hipErrorNotReady) return e;
        if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(20)) return hipEventSynchronize(ev);
    }
}
hipError_t wait_stream(hipStream_t st, hipEvent_t ev) {
    hipError_t e = hipEventRecord(ev, st);
    if (e != hipSuccess) return e;
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        e = hipEventQuery(ev);
        if (e != hipErrorNotReady) return e;
        if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(20)) return hipEventSynchronize(ev);
    }
}

// k_replay keeps 32-bit pool slots (the pool and its claim slack stay below 2^32 tuples);
// KVR_POOL_LIMIT lowers the limit (test knob)
uint64_t pool_limit() {
    const char *e = getenv("KVR_POOL_LIMIT");
    return e ? std::max<uint64_t>(strtoull(e, nullptr, 10), 1024) : 0xFFFF0000ull;
}
bool getenv_flag(const char *name) {
    const char *e = getenv(name);
    return e && *e && *e != '0';
}
bool getenv_flag_off(const char *name) {   // set to 0
    const char *e = getenv(name);
    return e && *e == '0';
}
// tuples behind pool_cap that serve a claim past it (k_replay flags the overflow and writes there;
// the host then grows the pool and runs again): one claim of the largest size
constexpr uint64_t POOL_SLACK = (POOL_CHUNK > TILE_RECS ? POOL_CHUNK : TILE_RECS) + 64;

__global__ void k_shift_seg(kvr_tuple *t, uint64_t n, uint32_t by) {   // seg_idx of a batch's tuples
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) t[i].seg_idx += by;
}

}  // namespace

struct kvr_ctx {
    int device = 0;
    int n_cu = 256;
    int wg_per_cu = 1;
    hipStream_t own = nullptr, stream = nullptr;
    hipEvent_t ev[6] = {};
    DevBuf<uint8_t> arena;
    DevBuf<SegDesc> segs;
    DevBuf<StripeDesc> stripes;
    DevBuf<StripeRes> sres;
    DevBuf<TileRes> tres;
    DevBuf<kvr_tuple> pool, dense;
    // key prefixes for the fold: k_replay writes them per pool slot when kout is set, k_compact_s
    // moves them into kout (parallel to the output tuples); compact_front points kout at ckeys
    DevBuf<uint4> kpool, ckeys;
    DevBuf<uint2> ctk;                     // the tuples' (key tag, key length) beside ckeys (k_compact_s):
                                           // k_hll and k_fold_part read these instead of the tuples
    uint4 *kout = nullptr;
    bool ckeys_ok = false;                 // ckeys holds the prefixes of ctup[0, c_nt)
    DevBuf<RedoEnt> redo;
    DevBuf<LinkResult> link;
    DevBuf<Counters> ctr;
    DevBuf<uint32_t> seg_bad, seg_err, expected;
    DevBuf<uint64_t> soff;                 // each stripe's output offset (k_link, for k_compact_s)
    DevBuf<uint32_t> scnt;                 // each stripe's record count, dense (k_replay, for linked k_compact_s)
    DevBuf<PieceHand> hand;                // k_piece -> k_replay: where each stripe's tile loop resumes
    DevBuf<PieceRun> prun;                 // k_piece -> k_compact_s: each stripe's records in run form
    DevBuf<uint2> pcrc;                    // ... their value CRCs and key tags, by pool slot
    DevBuf<uint32_t> crc, kmul, initx;
    DevBuf<GenRecDev> gen;
    // compaction (kvr_compact)
    DevBuf<kvr_tuple> ctup, lout;
    DevBuf<FoldEnt> fent;                  // the fold table (k_fold_claim / k_fold_verify)
    DevBuf<uint32_t> flist, fcnt;          // collision rounds: two tuple lists, their counts
    DevBuf<FPRec> frec;                    // the partitioned fold's records (k_fold_part), per region
    DevBuf<uint32_t> fwoff;                // ... and each region's bucket offsets
    DevBuf<uint32_t> fhot;                 // ... and the hot buckets (k_fold_lds -> k_fold_hot)
    DevBuf<uint32_t> fsz;                  // the fold table's size on the device (k_hll_size)
    bool fold_pending = false;             // deferred rounds launched, not yet checked (fold_settle)
    DevBuf<uint32_t> cslot, cflag, cpos;
    DevBuf<uint8_t> cfl8;                  // kvr_compact: a byte per tuple, live (k_live_ent -> k_dl_*)
    DevBuf<uint32_t> dl_cnt;               // ... per block of DL_CH tuples: live count, then its prefix
    DevBuf<uint64_t> dl_bytes;             // ... and live bytes, then their prefix
    DevBuf<uint64_t> dl_tot;               // fold_derive's totals: live bytes (unused), live records
    DevBuf<uint64_t> csize, coff, l_src, l_off, ctot, ccuts;
    DevBuf<uint8_t> cout, ctmp;
    kvr_compact_stats cstats{};
    uint32_t fold_rounds = 0;              // probe rounds of the last fold (1 = no tag collision)
    uint32_t fold_redo = 0;                // folds redone at full size (the estimate was low)
    uint64_t fold_est = 0, fold_slots = 0;  // distinct-key estimate, table entries used
    DevBuf<uint8_t> hpart, hreg;           // HyperLogLog registers per workgroup, merged
    size_t c_nt = 0;                       // tuples of the last compaction front half
    uint32_t c_ranks = 0;                  // sharded compaction state (kvr_compact_stage .. finish)
    bool c_staged = false;
    uint64_t c_ncand = 0, c_nkey = 0;
    DevBuf<uint32_t> c_gidx, c_own, c_sidx;
    DevBuf<uint64_t> c_val, c_scan, c_gstart;
    DevBuf<kvr_cand> c_hdr;
    DevBuf<uint8_t> c_keys;
    DevBuf<uint32_t> r_rep, r_slot;
    DevBuf<uint64_t> r_best, r_hk;
    LinkResult *h_link = nullptr;
    Counters *h_ctr = nullptr;
    // link result and counters share one device block (one memset, one copy back per call) and one
    // pinned host block.  There are two device blocks: a call uses block lc_cur, and the linked
    // k_compact_s clears the other one for the next call
    DevBuf<uint8_t> lcbuf;
    uint32_t lc_cur = 0;
    uint8_t *h_lc = nullptr;
    std::vector<SegDesc> h_segs;
    std::vector<StripeDesc> h_stripes;
    // the descriptors last uploaded to segs / stripes: a call over the same segments skips the copy
    std::vector<SegDesc> up_segs;
    std::vector<StripeDesc> up_stripes;
    const void *up_segs_p = nullptr, *up_stripes_p = nullptr;
    uint64_t up_tps = 0;                   // the tiles per stripe of the uploaded stripes
    bool h_stripes_up = false;             // h_stripes holds exactly the uploaded stripes
    bool lc_zero = false;                  // lcbuf is known to be zero (cleared at the end of the last call)
    uint64_t pool_hint = 0;
    uint32_t piece_skip = 0;               // calls left that skip k_piece (see replay_one: KVR_PIECE_ADAPT)
    uint64_t pool_need = 0;                // > 0: the last replay needed more than 32-bit pool slots
    uint32_t tps_override = 0;
    kvr_stats stats{};
    // streamed ingest (kvr_replay_stream): two HBM batch slots filled on a copy stream, two pinned
    // staging slots for pageable callers
    hipStream_t copy = nullptr;
    hipEvent_t ev_copy[2] = {};
    DevBuf<uint8_t> slot[2];
    uint8_t *h_stage[2] = {};
    uint64_t h_stage_cap[2] = {};
    kvr_stream_stats sstats{};
    // batch ETag (kvr_etag_batch)
    DevBuf<uint32_t> e_x, e_cb, e_creg, e_out, e_exp;
    DevBuf<uint64_t> e_cpre, e_offs, e_lens, e_fail, e_cdesc;
    DevBuf<uint8_t> e_data;
    kvr_etag_stats estats{};
    uint32_t e_wg_per_cu = 0;
    // open-time index (kvr_replay_index) and ingest (kvr_ingest_*): the live list stays in lout,
    // the key table in islots, until the next call
    DevBuf<uint32_t> islots;
    DevBuf<uint64_t> koff, klen;           // key arena (kvr_live_keys): offsets, lengths
    DevBuf<uint8_t> kbuf;
    uint64_t ix_live = 0, ix_slots = 0;
    bool ix_valid = false;
    kvr_index_stats istats{};
    DevBuf<uint8_t> ing;                   // the store's segment bytes, resident in HBM
    uint64_t ing_off = 0;
    std::vector<kvr_segment> ing_segs;     // device pointers into ing, in push order
};

// a HIP failure returns KVR_EHIP and says which call failed on stderr (KVR_QUIET=1 silences it)
#define HIPCHK(x)                                                                              \
    do {                                                                                       \
        const hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                                \
            if (!getenv("KVR_QUIET")) fprintf(stderr, "kvr: %s failed: %s (%s:%d)\n", #x,      \
                                              hipGetErrorName(e_), __FILE__, __LINE__);        \
            return KVR_EHIP;                                                                   \
        }                                                                                      \
    } while (0)

// ---------------------------------------------------------------------------------------
// tables: slice-by-16 CRC tables and the shift operators X(n) = x^(8n) mod P
// ---------------------------------------------------------------------------------------
static void build_tables(std::vector<uint32_t> &crc, std::vector<uint32_t> &kmul, std::vector<uint32_t> &initx) {
    crc.assign(16 * 256, 0);
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t c = i;
        for (int k = 0; k < 8; ++k) c = (c & 1u) ? (c >> 1) ^ POLY : (c >> 1);
        crc[i] = c;
    }
    for (int t = 1; t < 16; ++t)
        for (int i = 0; i < 256; ++i) {
            const uint32_t prev = crc[(t - 1) * 256 + i];
            crc[t * 256 + i] = (prev >> 8) ^ crc[prev & 0xFF];
        }
    // X(n) = x^(8n) mod P (reflected): "push the register through n zero bytes"
    std::vector<uint32_t> X(SC + 1);
    X[0] = GF_ONE;
    for (int i = 1; i <= SC; ++i) X[i] = gf_mul(X[i - 1], 0x00800000u);   // * x^8
    initx.assign(NIX + 3, 0);
    for (int j = 0; j < NIX; ++j) initx[j] = gf_mul(0xFFFFFFFFu, X[j]);
    // nibble tables of "multiply by a constant": kmul[t][i][n] = (n << 4i) * K_t, with
    //   K_t = X(SC * 2^t)        for t < KSET_Q          (in-row steps of the segmented scan)
    //   K_t = X(4 (t - KSET_Q))  for KSET_Q <= t < KSET_R (a register pushed through 4q bytes)
    //   K_t = X(SC (t - KSET_R + 1)) for t >= KSET_R     (cross-row steps of the scan)
    kmul.assign(KMUL_SETS * 8 * 16, 0);
    uint32_t K = X[SC], R = X[SC];
    for (int t = 0; t < KMUL_SETS; ++t) {
        uint32_t Kt;
        if (t < KSET_Q) { Kt = K; K = gf_mul(K, K); }
        else if (t < KSET_R) Kt = X[4 * (t - KSET_Q)];
        else { Kt = R; R = gf_mul(R, X[SC]); }
        for (int i = 0; i < 8; ++i)
            for (uint32_t n = 0; n < 16; ++n) kmul[(t * 8 + i) * 16 + n] = gf_mul(n << (4 * i), Kt);
    }
}

extern "C" {

const char *kvr_strerror(int code) {
    switch (code) {
    case KVR_OK: return "ok";
    case KVR_CORRUPTED: return "corrupted data";
    case KVR_CAPACITY: return "output capacity too small";
    case KVR_EINVAL: return "invalid argument";
    case KVR_EHIP: return "HIP runtime error";
    case KVR_EIO: return "I/O error";
    case KVR_ENOMEM: return "out of memory";
    default: return "unknown status";
    }
}

uint32_t kvr_crc32(uint32_t crc, const uint8_t *data, size_t len) {
    static uint32_t T[256];
    static bool ready = false;
    if (!ready) {
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t c = i;
            for (int k = 0; k < 8; ++k) c = (c & 1u) ? (c >> 1) ^ POLY : (c >> 1);
            T[i] = c;
        }
        ready = true;
    }
    uint32_t c = ~crc;
    for (size_t i = 0; i < len; ++i) c = (c >> 8) ^ T[(c ^ data[i]) & 0xFFu];
    return ~c;
}

int kvr_format_error(const kvr_error *e, const char *path, char *buf, size_t cap) {
    if (!e || !buf) return -1;
    if (!path) path = "";
    static const char *eof = "failed to fill whole buffer";   // std::io read_exact UnexpectedEof
    switch (e->kind) {
    case KVR_E_OPEN: {
        const int code = (int)e->aux;
        return snprintf(buf, cap, "Failed to open segment %s: %s (os error %d)", path, strerror(code), code);
    }
    case KVR_E_KEY_LEN: return snprintf(buf, cap, "Failed to read key length in %s: %s", path, eof);
    case KVR_E_KEY: return snprintf(buf, cap, "Failed to read key in %s: %s", path, eof);
    case KVR_E_UTF8: {
        const unsigned long long vu = e->aux & 0xFFFFFFFFull;
        const unsigned el = (unsigned)(e->aux >> 32);
        if (el)
            return snprintf(buf, cap, "Invalid UTF-8 key in %s: invalid utf-8 sequence of %u bytes from index %llu",
                            path, el, vu);
        return snprintf(buf, cap, "Invalid UTF-8 key in %s: incomplete utf-8 byte sequence from index %llu", path, vu);
    }
    case KVR_E_VAL_LEN: return snprintf(buf, cap, "Failed to read val len in %s: %s", path, eof);
    case KVR_E_VAL: return snprintf(buf, cap, "Failed to read val in %s: %s", path, eof);
    case KVR_E_OPCODE: return snprintf(buf, cap, "Unknown opcode %u in segment %s", (unsigned)e->aux, path);
    default: return snprintf(buf, cap, "no error");
    }
}

// point link / ctr at device block b of lcbuf
static void lc_select(kvr_ctx *c, uint32_t b) {
    c->lc_cur = b;
    c->link.p = reinterpret_cast<LinkResult *>(c->lcbuf.p + b * LC_BYTES);
    c->link.n = 1;
    c->ctr.p = reinterpret_cast<Counters *>(c->lcbuf.p + b * LC_BYTES + LC_CTR);
    c->ctr.n = 1;
}

int kvr_ctx_create(int device, kvr_ctx **out) {
    if (!out) return KVR_EINVAL;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return KVR_EHIP;
    if (device < 0 || device >= ndev) return KVR_EINVAL;
    HIPCHK(hipSetDevice(device));
    kvr_ctx *c = new kvr_ctx();
    c->device = device;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0) c->n_cu = prop.multiProcessorCount;
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, KR_KERNEL, KR_RT, 0) == hipSuccess && occ > 0) c->wg_per_cu = occ;
    if (hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess) { delete c; return KVR_EHIP; }
    c->stream = c->own;
    for (auto &e : c->ev) if (hipEventCreate(&e) != hipSuccess) { delete c; return KVR_EHIP; }
    // (fine-grained: k_link writes it and k_compact_s adds to it from the device, see replay_one)
    if (hipHostMalloc(reinterpret_cast<void **>(&c->h_lc), LC_BYTES, hipHostMallocCoherent) != hipSuccess) {
        delete c;
        return KVR_ENOMEM;
    }
    c->h_link = reinterpret_cast<LinkResult *>(c->h_lc);
    c->h_ctr = reinterpret_cast<Counters *>(c->h_lc + LC_CTR);
    std::vector<uint32_t> crc, kmul, initx;
    build_tables(crc, kmul, initx);
    if (c->crc.ensure(crc.size()) || c->kmul.ensure(kmul.size()) || c->initx.ensure(initx.size()) ||
        c->lcbuf.ensure(2 * LC_BYTES)) {
        kvr_ctx_destroy(c);
        return KVR_ENOMEM;
    }
    lc_select(c, 0);
    if (hipMemcpy(c->crc.p, crc.data(), crc.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->kmul.p, kmul.data(), kmul.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->initx.p, initx.data(), initx.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
        kvr_ctx_destroy(c);
        return KVR_EHIP;
    }
    *out = c;
    return KVR_OK;
}

void kvr_ctx_destroy(kvr_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    c->arena.release(); c->segs.release(); c->stripes.release(); c->sres.release(); c->tres.release();
    c->pool.release(); c->dense.release(); c->redo.release();
    c->link.p = nullptr; c->ctr.p = nullptr;   // (inside lcbuf)
    c->lcbuf.release();
    c->seg_bad.release(); c->seg_err.release(); c->expected.release(); c->soff.release(); c->scnt.release(); c->hand.release();
    c->crc.release(); c->kmul.release(); c->initx.release(); c->gen.release();
    c->kpool.release(); c->ckeys.release(); c->ctk.release();
    c->ctup.release(); c->lout.release(); c->fent.release(); c->flist.release(); c->fcnt.release(); c->fsz.release();
    c->frec.release(); c->fwoff.release(); c->fhot.release();
    c->cslot.release(); c->cflag.release(); c->cfl8.release(); c->dl_cnt.release(); c->dl_bytes.release(); c->dl_tot.release(); c->islots.release(); c->ing.release(); c->hpart.release(); c->hreg.release();
    c->koff.release(); c->klen.release(); c->kbuf.release();
    c->cpos.release(); c->csize.release(); c->coff.release(); c->l_src.release();
    c->l_off.release(); c->ctot.release(); c->ccuts.release(); c->cout.release(); c->ctmp.release();
    c->c_gidx.release(); c->c_own.release(); c->c_sidx.release(); c->c_val.release(); c->c_scan.release();
    c->c_gstart.release(); c->c_hdr.release(); c->c_keys.release(); c->r_rep.release(); c->r_slot.release();
    c->r_best.release(); c->r_hk.release();
    c->e_x.release(); c->e_cb.release(); c->e_creg.release(); c->e_out.release(); c->e_exp.release();
    c->e_cpre.release(); c->e_offs.release(); c->e_lens.release(); c->e_fail.release(); c->e_data.release();
    c->e_cdesc.release();
    if (c->copy) (void)hipStreamSynchronize(c->copy);
    for (int i = 0; i < 2; ++i) {
        c->slot[i].release();
        if (c->h_stage[i]) (void)hipHostFree(c->h_stage[i]);
        if (c->ev_copy[i]) (void)hipEventDestroy(c->ev_copy[i]);
    }
    if (c->copy) (void)hipStreamDestroy(c->copy);
    if (c->h_lc) (void)hipHostFree(c->h_lc);
    for (auto &e : c->ev) if (e) (void)hipEventDestroy(e);
    if (c->own) (void)hipStreamDestroy(c->own);
    delete c;
}

int kvr_ctx_set_stream(kvr_ctx *c, void *s) {
    if (!c) return KVR_EINVAL;
    c->stream = s ? reinterpret_cast<hipStream_t>(s) : c->own;
    return KVR_OK;
}

int kvr_ctx_device(const kvr_ctx *c) { return c ? c->device : -1; }

int kvr_ctx_set_tiles_per_stripe(kvr_ctx *c, uint32_t tiles) {
    if (!c) return KVR_EINVAL;
    c->tps_override = tiles;
    return KVR_OK;
}

int kvr_last_stats(const kvr_ctx *c, kvr_stats *out) {
    if (!c || !out) return KVR_EINVAL;
    *out = c->stats;
    return KVR_OK;
}

static float ev_ms(hipEvent_t a, hipEvent_t b) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, a, b) != hipSuccess) return 0.f;
    return ms;
}

static int replay_one(kvr_ctx *c, const kvr_segment *segs, size_t n, uint32_t flags, const uint32_t *expected,
                      size_t n_expected, kvr_tuple *out, size_t cap, size_t *n_out, kvr_error *err);

// a replay whose tuples exceed the pool's 32-bit slots (dense small records: more than about
// 4 G records in one call) runs as consecutive batches of whole segments, each its own
// pipeline, the tuples appended in order — the same output, errors and return codes.  When a
// fold or the compaction's gather reads the segments afterwards, host segments are first copied
// into the arena all at once (the batches then replay them in place), so that every segment stays
// resident and, at the end, the segment descriptors on the device describe the whole input: the
// fold, the key arena and the gather read keys and records of any batch.  A plain replay stages
// each batch on its own (no more HBM than one batch).  Key prefixes (kout) are appended per batch
// like the tuples.
static int replay_batched(kvr_ctx *c, const kvr_segment *segs, size_t n, uint32_t flags, const uint32_t *expected,
                          size_t n_expected, kvr_tuple *out, size_t cap, size_t *n_out, kvr_error *err, uint64_t need) {
    uint64_t total = 0;
    for (size_t i = 0; i < n; ++i) total += segs[i].len;
    const uint64_t parts = need / (pool_limit() / 2) + 1;
    const uint64_t budget = total / parts + 1;
    HIPCHK(hipSetDevice(c->device));
    std::vector<kvr_segment> dsegs(segs, segs + n);
    // host segments go resident all at once only when something reads them after the replay: a
    // fold (key prefixes requested, c->kout) or a device-side consumer of the output (the
    // compaction's gather, KVR_OUT_ON_DEVICE); a plain replay stages each batch's segments itself
    const bool resident = !(flags & KVR_SEGS_ON_DEVICE) && (c->kout || (flags & KVR_OUT_ON_DEVICE));
    if (resident) {
        uint64_t arena = 256;
        for (size_t i = 0; i < n; ++i) arena += (segs[i].len + 255) & ~255ull;
        if (c->arena.ensure(arena)) return KVR_ENOMEM;
        uint64_t off = 0;
        for (size_t i = 0; i < n; ++i) {
            dsegs[i].bytes = c->arena.p + off;
            if (segs[i].len)
                HIPCHK(hipMemcpyAsync(c->arena.p + off, segs[i].bytes, segs[i].len, hipMemcpyHostToDevice, c->stream));
            off += (segs[i].len + 255) & ~255ull;
        }
        flags |= KVR_SEGS_ON_DEVICE;
    }
    uint4 *const kout = (flags & KVR_OUT_ON_DEVICE) ? c->kout : nullptr;
    size_t done = 0;
    kvr_stats sum{};
    for (size_t s0 = 0; s0 < n;) {
        size_t s1 = s0;
        uint64_t b = 0;
        while (s1 < n && (s1 == s0 || b + segs[s1].len <= budget)) b += segs[s1++].len;
        if (s1 - s0 == n) return KVR_ENOMEM;   // one segment alone is too dense to split here
        const size_t e0 = std::min(done, n_expected);
        const size_t room = done < cap ? cap - done : 0;
        size_t nb = 0;
        kvr_error e{};
        c->kout = kout && room ? kout + done : nullptr;
        const int rc = kvr_replay(c, dsegs.data() + s0, s1 - s0, flags, expected ? expected + e0 : nullptr,
                                  expected ? n_expected - e0 : 0, room ? out + done : nullptr, room, &nb, &e);
        sum.ms_total += c->stats.ms_total; sum.ms_replay += c->stats.ms_replay; sum.ms_link += c->stats.ms_link;
        sum.ms_compact += c->stats.ms_compact; sum.bytes_in += c->stats.bytes_in; sum.n_records += c->stats.n_records;
        sum.n_crc_fail += c->stats.n_crc_fail; sum.n_stripes += c->stats.n_stripes; sum.n_tiles += c->stats.n_tiles;
        sum.n_redo += c->stats.n_redo; sum.n_link_passes += c->stats.n_link_passes;
        if (rc == KVR_CORRUPTED) {   // batches run in (segment, offset) order: the store's first error
            if (err) { *err = e; err->seg_idx += (uint32_t)s0; }
            c->stats = sum;
            c->kout = kout;
            return rc;
        }
        if (rc != KVR_OK && rc != KVR_CAPACITY) { c->kout = kout; return rc; }
        if (s0 && !(flags & KVR_OUT_ON_DEVICE)) {   // seg_idx into the caller's segs[]
            for (size_t t = 0, m = std::min(nb, room); t < m; ++t) out[done + t].seg_idx += (uint32_t)s0;
        } else if (s0 && nb) {
            hipLaunchKernelGGL(k_shift_seg, dim3((uint32_t)((std::min(nb, room) + 255) / 256)), dim3(256), 0, c->stream,
                               out + done, (uint64_t)std::min(nb, room), (uint32_t)s0);
            HIPCHK(hipStreamSynchronize(c->stream));
        }
        done += nb;
        s0 = s1;
    }
    c->kout = done <= cap ? kout : nullptr;   // (prefixes past the output's room were not written)
    if (!(flags & KVR_SEGS_ON_DEVICE)) {   // staged per batch: nothing describes the whole input
        c->up_segs_p = nullptr;
        c->up_stripes_p = nullptr;
        c->h_stripes_up = false;
        c->stats = sum;
        *n_out = done;
        return done > cap ? KVR_CAPACITY : KVR_OK;
    }
    // the descriptors of every segment (only base and len are read after the replay), and the
    // per-call upload caches invalidated
    if (c->segs.ensure(n)) return KVR_ENOMEM;
    std::vector<SegDesc> all(n);
    for (size_t i = 0; i < n; ++i) {
        all[i] = SegDesc{};
        all[i].base = dsegs[i].bytes;
        all[i].len = dsegs[i].len;
        all[i].d0 = (uint32_t)(reinterpret_cast<uintptr_t>(dsegs[i].bytes) & 15u);
    }
    HIPCHK(hipMemcpyAsync(c->segs.p, all.data(), n * sizeof(SegDesc), hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    c->up_segs_p = nullptr;
    c->up_stripes_p = nullptr;
    c->h_stripes_up = false;
    c->stats = sum;
    *n_out = done;
    return done > cap ? KVR_CAPACITY : KVR_OK;
}

int kvr_replay(kvr_ctx *c, const kvr_segment *segs, size_t n, uint32_t flags, const uint32_t *expected,
               size_t n_expected, kvr_tuple *out, size_t cap, size_t *n_out, kvr_error *err) {
    if (!c || (!segs && n) || !n_out || (cap && !out)) return KVR_EINVAL;
    uint64_t need = 0;
    const int rc = replay_one(c, segs, n, flags, expected, n_expected, out, cap, n_out, err);
    if (rc != KVR_ENOMEM || !c->pool_need) return rc;
    need = c->pool_need;   // the pool this input needs exceeds 32-bit slots: batch it
    c->pool_need = 0;
    c->pool_hint = 0;
    return replay_batched(c, segs, n, flags, expected, n_expected, out, cap, n_out, err, need);
}

static int replay_one(kvr_ctx *c, const kvr_segment *segs, size_t n, uint32_t flags, const uint32_t *expected,
                      size_t n_expected, kvr_tuple *out, size_t cap, size_t *n_out, kvr_error *err) {
    if (err) memset(err, 0, sizeof(*err));
    *n_out = 0;
    memset(&c->stats, 0, sizeof(c->stats));
    c->ix_valid = false;   // the segment descriptors and the pool change: an earlier live list is stale
    if (n == 0) return KVR_OK;
    if (n >= 0xFFFFFFFFull) return KVR_EINVAL;
    for (size_t i = 0; i < n; ++i) {
        if (i && segs[i].seg_id < segs[i - 1].seg_id) return KVR_EINVAL;   // caller sorts (engine.rs:51)
        if (segs[i].len && !segs[i].bytes) return KVR_EINVAL;
    }
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = c->stream;

    // 1. segment bytes in HBM
    std::vector<const uint8_t *> dptr(n);
    uint64_t total_bytes = 0;
    for (size_t i = 0; i < n; ++i) total_bytes += segs[i].len;
    if (flags & KVR_SEGS_ON_DEVICE) {
        for (size_t i = 0; i < n; ++i) dptr[i] = segs[i].bytes;
    } else {
        uint64_t need = 256;
        for (size_t i = 0; i < n; ++i) need += (segs[i].len + 255) & ~255ull;
        if (c->arena.ensure(need)) return KVR_ENOMEM;
        uint64_t off = 0;
        for (size_t i = 0; i < n; ++i) {
            dptr[i] = c->arena.p + off;
            if (segs[i].len) HIPCHK(hipMemcpyAsync(c->arena.p + off, segs[i].bytes, segs[i].len, hipMemcpyHostToDevice, st));
            off += (segs[i].len + 255) & ~255ull;
        }
    }

    // 2. tiles and stripes
    c->h_segs.assign(n, SegDesc{});
    uint64_t total_tiles = 0;
    for (size_t i = 0; i < n; ++i) {
        SegDesc &g = c->h_segs[i];
        g.base = dptr[i];
        g.len = segs[i].len;
        g.d0 = (uint32_t)(reinterpret_cast<uintptr_t>(dptr[i]) & 15u);
        g.n_tiles = g.len ? (uint32_t)((g.len + g.d0 + KR_TILE - 1) / KR_TILE) : 0u;
        g.tile0 = (uint32_t)total_tiles;
        total_tiles += g.n_tiles;
    }
    if (total_tiles >= 0xFFFFFFFFull) return KVR_EINVAL;
    // one stripe per resident wave, one round (k_replay: WPB stripes per workgroup).  Measured
    // (tools/tps_sweep.py): one round beats two by 5 % on cfg2 and 14 % on cfg5, and stripe counts
    // between whole rounds leave a ragged tail
    const uint64_t target = (uint64_t)c->n_cu * (uint64_t)c->wg_per_cu * KR_WPB;
    const uint64_t tps = c->tps_override ? c->tps_override : std::max<uint64_t>(1, (total_tiles + target - 1) / target);
    // the same segment layout and stripe length as the last uploaded call: the stripes are the
    // uploaded ones (h_stripes still holds them), only their per-segment indices are copied
    bool same_layout = c->h_stripes_up && c->up_tps == tps && c->up_segs.size() == n && c->up_stripes_p != nullptr;
    for (size_t i = 0; same_layout && i < n; ++i) {
        const SegDesc &a = c->h_segs[i], &b = c->up_segs[i];
        same_layout = a.base == b.base && a.len == b.len && a.d0 == b.d0 && a.n_tiles == b.n_tiles && a.tile0 == b.tile0;
    }
    const bool same_layout_call = same_layout && (flags & KVR_SEGS_ON_DEVICE);
    if (same_layout) {
        for (size_t i = 0; i < n; ++i) {
            c->h_segs[i].stripe0 = c->up_segs[i].stripe0;
            c->h_segs[i].n_stripes = c->up_segs[i].n_stripes;
        }
    } else {
        c->h_stripes_up = false;
        c->h_stripes.clear();
        for (size_t i = 0; i < n; ++i) {
            SegDesc &g = c->h_segs[i];
            g.stripe0 = (uint32_t)c->h_stripes.size();
            const uint64_t ns = g.n_tiles ? (g.n_tiles + tps - 1) / tps : 0;
            for (uint64_t j = 0; j < ns; ++j)
                c->h_stripes.push_back(StripeDesc{(uint32_t)i, (uint32_t)(j * g.n_tiles / ns),
                                                  (uint32_t)((j + 1) * g.n_tiles / ns), j == 0 ? 1u : 0u});
            g.n_stripes = (uint32_t)ns;
        }
    }
    const uint32_t n_stripes = (uint32_t)c->h_stripes.size();
    const uint32_t n_tiles = (uint32_t)total_tiles;
    c->stats.bytes_in = total_bytes;
    c->stats.n_stripes = n_stripes;
    c->stats.n_tiles = n_tiles;
    if (n_stripes == 0) return KVR_OK;   // only empty segments: nothing to replay

    if (c->segs.ensure(n) || c->stripes.ensure(n_stripes) || c->sres.ensure(n_stripes) ||
        c->tres.ensure(n_tiles) || c->redo.ensure(std::max<uint32_t>(n_stripes, REDO_GRID)) ||
        c->seg_bad.ensure(n) || c->seg_err.ensure(n) || c->soff.ensure(n_stripes) || c->scnt.ensure(n_stripes) || c->hand.ensure(n_stripes) || c->prun.ensure(n_stripes))
        return KVR_ENOMEM;
    // (the same segments as the last call: the descriptors on the device are still these)
    if (c->up_segs_p != c->segs.p || c->up_segs.size() != n ||
        memcmp(c->up_segs.data(), c->h_segs.data(), n * sizeof(SegDesc)) != 0) {
        HIPCHK(hipMemcpyAsync(c->segs.p, c->h_segs.data(), n * sizeof(SegDesc), hipMemcpyHostToDevice, st));
        c->up_segs = c->h_segs;
        c->up_segs_p = c->segs.p;
    }
    if (c->up_stripes_p != c->stripes.p || c->up_stripes.size() != n_stripes ||
        (!same_layout && memcmp(c->up_stripes.data(), c->h_stripes.data(), n_stripes * sizeof(StripeDesc)) != 0)) {
        c->up_stripes_p = nullptr;   // (invalid until the copy is queued)
        HIPCHK(hipMemcpyAsync(c->stripes.p, c->h_stripes.data(), n_stripes * sizeof(StripeDesc), hipMemcpyHostToDevice, st));
        c->up_stripes = c->h_stripes;
        c->up_stripes_p = c->stripes.p;
    }
    c->up_tps = tps;
    c->h_stripes_up = true;


    const uint32_t *d_exp = nullptr;
    if (expected && n_expected) {
        if (flags & KVR_EXPECTED_ON_DEVICE) {
            d_exp = expected;
        } else {
            if (c->expected.ensure(n_expected)) return KVR_ENOMEM;
            HIPCHK(hipMemcpyAsync(c->expected.p, expected, n_expected * 4, hipMemcpyHostToDevice, st));
            d_exp = c->expected.p;
        }
    }

    const Tables tb{c->crc.p, c->kmul.p, c->initx.p};
    for (int attempt = 0; attempt < 10; ++attempt) {
        // each workgroup claims pool space in chunks of >= pool_chunk tuples: budget one partly
        // used chunk per stripe on top of the expected record count
        const uint32_t pool_chunk = POOL_CHUNK;
        const uint64_t pool_cap = std::max<uint64_t>(
            c->pool_hint, std::max<uint64_t>(65536, total_bytes / 192 + n + (uint64_t)n_stripes * pool_chunk));
        if (pool_cap > pool_limit()) {   // k_replay keeps 32-bit pool slots in LDS: kvr_replay batches
            c->pool_need = pool_cap;
            return KVR_ENOMEM;
        }
        if (c->pool.ensure(pool_cap + POOL_SLACK) || c->pcrc.ensure(pool_cap + POOL_SLACK)) return KVR_ENOMEM;
        uint4 *kp = nullptr;               // key prefixes (calls that fold, device output only)
        if (c->kout && (flags & KVR_OUT_ON_DEVICE)) {
            if (c->kpool.ensure(pool_cap + POOL_SLACK)) return KVR_ENOMEM;
            kp = c->kpool.p;
        }
        // (key tag, key length) beside the prefixes (ctk parallels ckeys, where compact_front points kout)
        uint2 *ktk = nullptr;
        if (kp && c->kout >= c->ckeys.p && c->kout < c->ckeys.p + c->ckeys.n && c->ctk.n >= c->ckeys.n)
            ktk = c->ctk.p + (c->kout - c->ckeys.p);
        kvr_tuple *d_out;
        uint64_t out_cap;
        if (flags & KVR_OUT_ON_DEVICE) {
            d_out = out;
            out_cap = cap;
        } else {
            if (c->dense.ensure(pool_cap)) return KVR_ENOMEM;
            d_out = c->dense.p;
            out_cap = pool_cap;
        }
        // the ordered gather pool -> output: one workgroup per stripe from the stripe offsets k_link
        // computes
        // linked: k_compact_s links the stripes itself (no k_link launch); KVR_LINK_KERNEL=1 keeps
        // k_link first (test and timing knob)
        const bool linked = n_stripes <= LINKED_MAX_STRIPES && !getenv_flag("KVR_LINK_KERNEL");
        uint8_t *const lc = reinterpret_cast<uint8_t *>(c->link.p);   // this call's device block
        uint4 *const lc_next = reinterpret_cast<uint4 *>(c->lcbuf.p + (c->lc_cur ^ 1u) * LC_BYTES);
        // the kernels' own start / end timestamps (the dispatch packets' completion signals, as
        // rocprofv3 reads them) time k_replay and the pipeline: no marker packets between the
        // kernels.  KVR_EVENT_MARKERS=1 records separate events instead (timing knob)
        const bool markers = getenv_flag("KVR_EVENT_MARKERS");
        // k_piece takes every stripe first (runs of equal SETs, value-aligned) and hands the rest of a
        // stripe to k_replay's tile loop; ms_replay spans both
        // (a device-resident store that k_piece left entirely to k_replay on the last call with the same
        // segment layout -- cfg4's SET/DEL mix, cfg5's mixed values -- skips it for the next 7 calls:
        // its launch, table staging and entry checks cost such a store 2-3 %; KVR_PIECE_ADAPT=0 keeps
        // it on every call.  Either way the tuples are the same: k_replay takes any stripe)
        const bool piece = !getenv_flag("KVR_NO_PIECE") && !(c->piece_skip && same_layout_call);
        if (c->piece_skip) --c->piece_skip;
        auto launch_compact = [&](bool lk, hipEvent_t stop) {
            hipExtLaunchKernelGGL(k_compact_s, dim3(n_stripes), dim3(CT), 0, st, nullptr, markers ? nullptr : stop, 0u,
                               c->segs.p, c->stripes.p, c->sres.p, c->soff.p,
                               c->tres.p, c->pool.p, pool_cap, d_out, out_cap, d_exp,
                               (uint64_t)(d_exp ? n_expected : 0), c->ctr.p, c->link.p, kp, kp ? c->kout : nullptr,
                               kp ? reinterpret_cast<uint32_t *>(ktk) : nullptr, c->h_ctr,
                               lk ? c->scnt.p : nullptr, n_stripes, (uint32_t)KR_TILE, lc_next,
                               piece ? c->prun.p : nullptr, c->pcrc.p);
        };
        auto launch_link = [&]() {
            hipLaunchKernelGGL(k_link, dim3(1), dim3(LT), 0, st, c->segs.p, (uint32_t)n, c->stripes.p, n_stripes, c->sres.p,
                               c->redo.p, (uint32_t)c->redo.n, c->link.p, c->seg_bad.p, c->seg_err.p, (uint32_t)KR_TILE,
                               c->soff.p, c->ctr.p, c->h_link, c->h_ctr);
        };
        // counters and link result start at zero (the last successful call cleared them behind its
        // results, so this memset usually runs only on a context's first call or after an error)
        if (!c->lc_zero || attempt) HIPCHK(hipMemsetAsync(lc, 0, LC_BYTES, st));
        c->lc_zero = false;
        if (linked) {   // the host mirror the linked k_compact_s writes into (no kernel of this context runs)
            c->h_ctr->unlinked = 0;
            c->h_ctr->crc_fail = 0;
            c->h_ctr->overflow = 0;
        }
        if (markers) HIPCHK(hipEventRecord(c->ev[0], st));
        if (piece) {
            hipExtLaunchKernelGGL(k_piece, dim3((n_stripes + KR_WPB - 1) / KR_WPB), dim3(PNT), 0, st,
                                  markers ? nullptr : c->ev[0], nullptr, 0u, c->segs.p, c->stripes.p, n_stripes, c->sres.p,
                                  c->tres.p, c->pool.p, pool_cap, c->ctr.p, tb, pool_chunk, kp, c->scnt.p, c->hand.p,
                                  c->pcrc.p, c->prun.p);
            HIPCHK(hipGetLastError());
        }
        hipExtLaunchKernelGGL(KR_KERNEL, dim3((n_stripes + KR_WPB - 1) / KR_WPB), dim3(KR_RT), 0, st,
                              markers || piece ? nullptr : c->ev[0], markers ? nullptr : c->ev[1], 0u, c->segs.p, c->stripes.p,
                              n_stripes, c->sres.p, c->tres.p, c->pool.p, pool_cap, c->ctr.p, tb, pool_chunk, kp, c->scnt.p,
                              piece ? c->hand.p : nullptr);
        HIPCHK(hipGetLastError());
        if (markers) HIPCHK(hipEventRecord(c->ev[1], st));
        if (!linked) {
            launch_link();
            HIPCHK(hipGetLastError());
            HIPCHK(hipEventRecord(c->ev[2], st));
        }
        // compaction is launched right away: it does nothing unless linking succeeded (status 0),
        // which is the common case; otherwise the host re-walks and compacts again below
        launch_compact(linked, c->ev[3]);
        HIPCHK(hipGetLastError());
        if (markers) HIPCHK(hipEventRecord(c->ev[3], st));
        // link result + counters: k_link (or the linked k_compact_s) writes them into the pinned
        // mirror h_lc (and clears a device block after a clean pass), k_compact_s adds its CRC
        // failures there; when the call did not end cleanly the device block is copied as it is
        HIPCHK(wait_event(c->ev[3]));
        bool lc_switch = false;   // a clean linked pass: the next call uses the other (cleared) block
        bool relinked = false;    // the linked gather gave up: k_link and the plain gather ran after it
        if (linked) {
            if (c->h_ctr->overflow) {
                c->h_link->status = 0;   // (the pool is grown below)
            } else if (c->h_ctr->unlinked) {
                // a stripe did not link on its own (an error, a wrong speculation, a pass-through
                // stripe it could not check): k_link and the plain gather, as without linking.  The
                // stats then time the pipeline to this gather's end, k_link included.
                HIPCHK(hipEventRecord(c->ev[2], st));
                launch_link();
                HIPCHK(hipEventRecord(c->ev[4], st));
                launch_compact(false, c->ev[3]);
                HIPCHK(hipGetLastError());
                if (markers) HIPCHK(hipEventRecord(c->ev[3], st));   // (no dispatch stamp in markers mode)
                HIPCHK(wait_stream(st, c->ev[5]));
                relinked = true;
            } else {
                c->h_link->status = 0;
                c->h_link->n_redo = 0;
                c->h_link->passes = 1;
                lc_switch = true;
            }
        }
        const bool clean = c->h_link->status == 0 && !c->h_ctr->overflow;
        if (!clean) {
            HIPCHK(hipMemcpyAsync(c->h_lc, lc, LC_BYTES, hipMemcpyDeviceToHost, st));
            HIPCHK(hipStreamSynchronize(st));
        }
        c->stats.ms_replay = ev_ms(c->ev[0], c->ev[1]);
        c->stats.ms_link = relinked ? ev_ms(c->ev[2], c->ev[4]) : linked ? 0.0f : ev_ms(c->ev[1], c->ev[2]);
        c->stats.ms_compact = relinked ? ev_ms(c->ev[4], c->ev[3]) : ev_ms(linked ? c->ev[1] : c->ev[2], c->ev[3]);
        c->stats.ms_total = ev_ms(c->ev[0], c->ev[3]);

        // rare: more re-walk rounds (a speculated entry was wrong twice in a row)
        uint32_t guard = 0;
        bool recompact = false;
        const bool dbg = getenv("KVR_DEBUG") != nullptr;
        if (dbg) {
            fprintf(stderr, "kvr: pass1 status=%d n_redo=%u first_problem=%u passes=%u overflow=%u\n",
                    c->h_link->status, c->h_link->n_redo, c->h_link->first_problem_seg, c->h_link->passes,
                    c->h_ctr->overflow);
            std::vector<RedoEnt> rl(c->h_link->n_redo);
            std::vector<StripeRes> sr(n_stripes);
            (void)hipMemcpy(rl.data(), c->redo.p, rl.size() * sizeof(RedoEnt), hipMemcpyDeviceToHost);
            (void)hipMemcpy(sr.data(), c->sres.p, sr.size() * sizeof(StripeRes), hipMemcpyDeviceToHost);
            for (size_t q = 0; q < rl.size() && q < 40; ++q) {
                const uint32_t s = rl[q].stripe;
                const StripeDesc &d = c->h_stripes[s];
                fprintf(stderr, "   p1 redo stripe %u seg %u tiles [%u,%u) true-entry %llu | spec entry %lld exit %lld err %u@%lld"
                        " | pred entry %lld exit %lld\n", s, d.seg, d.t_begin, d.t_end, (unsigned long long)rl[q].entry,
                        (long long)sr[s].entry, (long long)sr[s].exit, sr[s].err_kind, (long long)sr[s].err_pos,
                        s ? (long long)sr[s - 1].entry : -9, s ? (long long)sr[s - 1].exit : -9);
            }
        }
        if (c->h_ctr->overflow & 1u) {   // pool too small: grow to what this pass needed and run again
            c->pool_hint = std::max<uint64_t>(c->h_ctr->pool_cursor, pool_cap) * 2;
            continue;
        }
        while (c->h_link->status == 3 && guard++ < n_stripes + 4) {
            hipLaunchKernelGGL(k_rewalk, dim3((std::max(1u, std::min(c->h_link->n_redo, (uint32_t)c->redo.n)) + RW_WPB - 1) / RW_WPB), dim3(RT_REWALK),
                               0, st, c->segs.p, c->stripes.p, n_stripes, c->sres.p, c->tres.p, c->pool.p, pool_cap, c->ctr.p,
                               tb, c->redo.p, c->link.p, pool_chunk, kp);
            hipLaunchKernelGGL(k_link, dim3(1), dim3(LT), 0, st, c->segs.p, (uint32_t)n, c->stripes.p, n_stripes,
                               c->sres.p, c->redo.p, (uint32_t)c->redo.n, c->link.p, c->seg_bad.p, c->seg_err.p, (uint32_t)KR_TILE,
                               c->soff.p, c->ctr.p, nullptr, nullptr);
            HIPCHK(hipGetLastError());
            HIPCHK(hipMemcpyAsync(c->h_link, c->link.p, sizeof(LinkResult), hipMemcpyDeviceToHost, st));
            HIPCHK(hipMemcpyAsync(c->h_ctr, c->ctr.p, sizeof(Counters), hipMemcpyDeviceToHost, st));
            HIPCHK(hipStreamSynchronize(st));
            recompact = true;
            if (c->h_ctr->overflow) break;
            if (dbg) {
                fprintf(stderr, "kvr: round %u status=%d n_redo=%u first_problem=%u\n", guard, c->h_link->status,
                        c->h_link->n_redo, c->h_link->first_problem_seg);
                if (guard < 6 || guard % 50 == 0) {
                    std::vector<RedoEnt> rl(c->h_link->n_redo);
                    std::vector<StripeRes> sr(n_stripes);
                    (void)hipMemcpy(rl.data(), c->redo.p, rl.size() * sizeof(RedoEnt), hipMemcpyDeviceToHost);
                    (void)hipMemcpy(sr.data(), c->sres.p, sr.size() * sizeof(StripeRes), hipMemcpyDeviceToHost);
                    for (auto &r : rl) {
                        const StripeDesc &d = c->h_stripes[r.stripe];
                        fprintf(stderr, "   redo stripe %u seg %u tiles [%u,%u) forced %llu | now entry %lld exit %lld err %u@%lld\n",
                                r.stripe, d.seg, d.t_begin, d.t_end, (unsigned long long)r.entry,
                                (long long)sr[r.stripe].entry, (long long)sr[r.stripe].exit, sr[r.stripe].err_kind,
                                (long long)sr[r.stripe].err_pos);
                    }
                }
            }
        }
        c->stats.n_redo = guard;
        if (c->h_ctr->overflow & 4u) {   // bug trap: an imposed entry before its stripe
            fprintf(stderr, "kvr: stripe re-walk got an entry before the stripe\n");
            return KVR_EHIP;
        }
        if (c->h_link->status == 3 && !(c->h_ctr->overflow & 1u)) {   // cannot happen: each round fixes one stripe (bug trap)
            fprintf(stderr, "kvr: stripe linking did not converge after %u rounds\n", guard);
            return KVR_EHIP;
        }
        const bool cleared = clean;   // k_link cleared the block after a clean first pass (or, linked, the
                                      // other block is clear: lc_switch)
        if (recompact && c->h_link->status == 0 && !c->h_ctr->overflow) {
            c->h_ctr->crc_fail = 0;
            launch_compact(false, nullptr);   // (its CRC failures go to h_ctr)
            HIPCHK(hipGetLastError());
            HIPCHK(hipStreamSynchronize(st));
        }
        c->stats.n_link_passes = c->h_link->passes;
        if (c->h_ctr->overflow & 2u) {   // stitch did not converge (bug trap)
            fprintf(stderr, "kvr: tile stitch did not converge\n");
            return KVR_EHIP;
        }
        if (c->h_ctr->overflow & 1u) {   // pool too small: grow to what this pass needed and run again
            c->pool_hint = std::max<uint64_t>(c->h_ctr->pool_cursor, pool_cap) * 2;
            continue;
        }
        if (c->h_link->status == 1) {
            if (err) {
                err->kind = (int32_t)c->h_link->err_kind;
                err->seg_idx = c->h_link->err_seg;
                err->rec_off = c->h_link->err_pos;
                err->aux = c->h_link->err_aux;
            }
            return KVR_CORRUPTED;
        }
        const uint64_t total = c->h_ctr->total_tuples;
        if (piece && linked && (flags & KVR_SEGS_ON_DEVICE) && !getenv_flag_off("KVR_PIECE_ADAPT"))
            c->piece_skip = c->h_ctr->piece_done ? 0u : 7u;
        c->stats.n_records = total;
        c->stats.n_crc_fail = c->h_ctr->crc_fail;
        *n_out = total;
        // the block is clear for the next call (else clear it now, behind this call's work)
        if (lc_switch) lc_select(c, c->lc_cur ^ 1u);
        if (cleared) c->lc_zero = true;
        else if (hipMemsetAsync(c->link.p, 0, LC_BYTES, st) == hipSuccess) c->lc_zero = true;
        if (!(flags & KVR_OUT_ON_DEVICE) && cap) {
            const uint64_t m = std::min<uint64_t>(total, cap);
            if (m) {
                HIPCHK(hipMemcpyAsync(out, c->dense.p, m * sizeof(kvr_tuple), hipMemcpyDeviceToHost, st));
                HIPCHK(hipStreamSynchronize(st));
            }
        }
        return total > cap ? KVR_CAPACITY : KVR_OK;
    }
    return KVR_ENOMEM;
}

// ---------------------------------------------------------------------------------------
// live-record rewrite (kvr_compact.hip): replay -> fold -> live list -> gather -> cuts
// ---------------------------------------------------------------------------------------
// replay + the local last-writer fold (k_fold_claim / k_fold_verify): the front half of every
// compaction and of kvr_replay_live / kvr_replay_index.  It reuses the buffers of a staged
// sharded compaction, so it ends one (kvr_compact_export / _finish then return KVR_EINVAL until
// the next kvr_compact_stage).  rewrite: also size the buffers of the byte rewrite
// (compact_back).  cs: the statistics this call fills (the caller's, so a live replay leaves
// kvr_last_compact_stats alone).
static int fold_launch(kvr_ctx *c, size_t nt, bool deferred);
static int compact_front(kvr_ctx *c, const kvr_segment *segs, size_t n, uint32_t flags, kvr_error *err, size_t *nt_out,
                         bool rewrite, kvr_compact_stats *cs, bool deferred = false) {
    *nt_out = 0;
    c->ix_valid = false;
    c->c_staged = false;
    c->c_nt = 0;
    c->fold_rounds = 0;
    c->fold_redo = 0;
    c->fold_est = 0;
    memset(cs, 0, sizeof(*cs));
    if (err) memset(err, 0, sizeof(*err));
    uint64_t bytes_in = 0;
    for (size_t i = 0; i < n; ++i) bytes_in += segs[i].len;
    cs->bytes_in = bytes_in;
    if (n == 0) return KVR_OK;
    // 1. replay into context-resident tuples; the segment bytes stay in HBM (c->segs)
    size_t nt = 0;
    c->ckeys_ok = false;
    if (c->ctup.ensure(bytes_in / 64 + 1024) || c->ckeys.ensure(c->ctup.n) || c->ctk.ensure(c->ckeys.n)) return KVR_ENOMEM;
    const uint32_t rflags = (flags & KVR_SEGS_ON_DEVICE) | KVR_OUT_ON_DEVICE;
    c->kout = c->ckeys.p;   // the tuples' key prefixes alongside them (k_fold_claim / k_fold_verify)
    int rc = kvr_replay(c, segs, n, rflags, nullptr, 0, c->ctup.p, c->ctup.n, &nt, err);
    if (rc == KVR_CAPACITY) {
        if (c->ctup.ensure(nt) || c->ckeys.ensure(c->ctup.n) || c->ctk.ensure(c->ckeys.n)) { c->kout = nullptr; return KVR_ENOMEM; }
        c->kout = c->ckeys.p;
        rc = kvr_replay(c, segs, n, rflags, nullptr, 0, c->ctup.p, c->ctup.n, &nt, err);
    }
    c->ckeys_ok = c->kout != nullptr;   // (a batched replay past the output capacity drops them)
    c->kout = nullptr;
    if (rc != KVR_OK) return rc;
    cs->ms_replay = c->stats.ms_total;
    cs->n_tuples = nt;
    *nt_out = nt;
    if (nt == 0) return KVR_OK;
    if (nt >= 0x7FFFFFFFull) return KVR_EINVAL;   // 32-bit tuple indices in the fold table
    c->c_nt = nt;
    hipStream_t st = c->stream;
    if (c->cflag.ensure(nt) || c->cpos.ensure(nt) || c->csize.ensure(nt)) return KVR_ENOMEM;
    if (rewrite && (c->coff.ensure(nt) || c->l_src.ensure(nt) || c->l_off.ensure(nt + 1) || c->ctot.ensure(2)))
        return KVR_ENOMEM;
    size_t t1 = 0, t2 = 0;
    if (rewrite) HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, t1, c->csize.p, c->coff.p, (int)nt, st));
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, t2, c->cflag.p, c->cpos.p, (int)nt, st));
    if (c->ctmp.ensure(std::max(t1, t2))) return KVR_ENOMEM;
    HIPCHK(hipEventRecord(c->ev[0], st));
    return fold_launch(c, nt, deferred);
}

// the grid of the kernels that walk the fold table (grid-stride over its size on the device)
static uint32_t fold_grid(const kvr_ctx *c) {
    return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((c->fent.n + 255) / 256, 4096));
}

// 2. the key's last tuple (open addressing over the key bytes, kvr_compact.hip) of c->ctup[0, nt).
// The table is sized for the distinct keys (HyperLogLog estimate, load <= 0.63) rather than the
// tuples, so it stays in the caches; the size is computed and used on the device (no host round
// trip between the estimate and the claims); a table that fills up is redone at 2 n entries.
// deferred: round 0 and FOLD_SPEC_ROUNDS - 1 further collision rounds (each of at most
// FOLD_SPEC_CAP tuples, their sizes read on the device) are launched without a host sync; the
// caller syncs once for everything and calls fold_settle, which redoes the fold synchronously in
// the rare case that this was not enough.  Otherwise the rounds run with one sync each.
constexpr uint32_t FOLD_SPEC_ROUNDS = 3, FOLD_SPEC_CAP = 65536, FOLD_CNT = 2;
constexpr int FOLD_REDONE = 1000;   // internal (compact_back): the deferred fold was redone
static int fold_launch(kvr_ctx *c, size_t nt, bool deferred) {
    hipStream_t st = c->stream;
    uint64_t full_slots = 1;
    while (full_slots < 2 * (uint64_t)nt) full_slots <<= 1;
    if (c->fent.ensure(full_slots) || c->cslot.ensure(nt) || c->flist.ensure(2 * nt) ||
        c->fcnt.ensure(FOLD_CNT * FOLD_SPEC_ROUNDS + 1) || c->fsz.ensure(4))
        return KVR_ENOMEM;
    c->fold_rounds = 0;
    c->fold_redo = 0;
    c->fold_est = 0;
    c->fold_pending = false;
    const bool tiny = getenv("KVR_FOLD_TINY_TABLE") != nullptr;   // test knob: force the full-size redo
    const uint2 *tk = (c->ckeys_ok && c->ctk.n >= nt) ? c->ctk.p : nullptr;   // (key tag, key length) per tuple
    if (tiny) {
        hipLaunchKernelGGL(k_fold_setsize, dim3(1), dim3(1), 0, st, c->fsz.p, 15u);
    } else if (nt >= 65536) {
        const uint32_t hb = (uint32_t)std::min<uint64_t>((nt + HLL_T - 1) / HLL_T, 2ull * (uint64_t)c->n_cu);
        if (c->hpart.ensure((uint64_t)hb * HLL_M) || c->hreg.ensure(HLL_M)) return KVR_ENOMEM;
        // (from the key tags k_compact_s wrote beside the prefixes: 8 B a tuple instead of 32)
        hipLaunchKernelGGL(k_hll, dim3(hb), dim3(HLL_T), 0, st, c->ctup.p, tk, (uint64_t)nt, c->hpart.p);
        hipLaunchKernelGGL(k_hll_merge, dim3(HLL_M / 16 / HLL_MG), dim3(HLL_MERGE_T), 0, st, c->hpart.p, hb, c->hreg.p);
        hipLaunchKernelGGL(k_hll_size, dim3(1), dim3(HLL_SIZE_T), 0, st, c->hreg.p, full_slots, c->fsz.p);
    } else {
        hipLaunchKernelGGL(k_fold_setsize, dim3(1), dim3(1), 0, st, c->fsz.p, (uint32_t)(full_slots - 1));
    }
    HIPCHK(hipGetLastError());
    static const bool pre = getenv("KVR_CLAIM_PRELOAD") && atoi(getenv("KVR_CLAIM_PRELOAD"));   // timing knob
    const bool nokeys = getenv("KVR_FOLD_SEGKEYS") != nullptr;   // test/timing knob: keys from the segments
    const uint4 *kd = (c->ckeys_ok && !nokeys) ? c->ckeys.p : nullptr;
    // one probe round over m tuples (list: null = all, in round 0); counters cnt[0] tuples left for
    // the next round, cnt[1] claims that found the table full
    auto round = [&](uint64_t m, const uint32_t *n_dev, const uint32_t *list, uint32_t *next, uint32_t *cnt) {
        const uint32_t g = (uint32_t)((m + 255) / 256);
        if (pre)
            hipLaunchKernelGGL(k_fold_claim<true>, dim3(g), dim3(256), 0, st, c->ctup.p, m, n_dev, list, c->segs.p,
                               c->fent.p, c->fsz.p, c->cslot.p, cnt + 1, kd);
        else
            hipLaunchKernelGGL(k_fold_claim<false>, dim3(g), dim3(256), 0, st, c->ctup.p, m, n_dev, list, c->segs.p,
                               c->fent.p, c->fsz.p, c->cslot.p, cnt + 1, kd);
        hipLaunchKernelGGL(k_fold_verify, dim3(g), dim3(256), 0, st, c->ctup.p, m, n_dev, list, c->segs.p, c->fent.p,
                           c->fsz.p, c->cslot.p, next, cnt, kd);
    };
    // round 0: the partitioned fold (k_fold_part / k_fold_lds) when the buckets of the largest
    // table fit the LDS histogram, its overflow tuples being round 1's list; else the global claims
    // over every tuple (KVR_FOLD_GLOBAL forces them: A/B and test knob)
    // (test knobs: KVR_FOLD_RANGE, a smaller range (a power of two >= 16), and KVR_FOLD_BUCKET, at
    // most that many records of a bucket folded in LDS (the rest through k_fold_hot), send many
    // tuples on to the global rounds)
    uint32_t s_lim = FP_S, cap_lim = 0;
    if (const char *e = getenv("KVR_FOLD_RANGE")) {
        const uint32_t v = (uint32_t)atoi(e);
        if (v >= 16 && v <= FP_S && (v & (v - 1)) == 0) s_lim = v;
    }
    if (const char *e = getenv("KVR_FOLD_BUCKET")) cap_lim = (uint32_t)atoi(e);
    const uint64_t p_host = std::max<uint64_t>(1, full_slots / s_lim);   // >= the ranges of any table size
    const uint64_t nwg = (nt + FP_CH - 1) / FP_CH;                       // k_fold_part's regions
    const bool part = p_host <= FP_PMAX && nwg <= FP_WMAX && getenv("KVR_FOLD_GLOBAL") == nullptr;
    const uint64_t hot_max = p_host / 4 + 2;   // hot buckets (cnt > cap >= 4 nt / P) and their run arrays
    if (part && (c->frec.ensure(nwg * FP_CH) || c->fwoff.ensure(nwg * (p_host + 1)) ||
                 c->fhot.ensure(hot_max * 2 + hot_max * 2 * (nwg + 1))))
        return KVR_ENOMEM;
again:
    HIPCHK(hipMemsetAsync(c->fcnt.p, 0, (FOLD_CNT * FOLD_SPEC_ROUNDS + 1) * sizeof(uint32_t), st));
    if (part) {
        hipLaunchKernelGGL(k_fold_part, dim3((uint32_t)nwg), dim3(FP_T), 0, st, c->ctup.p, (uint64_t)nt, c->segs.p, kd,
                           tk, c->fsz.p, s_lim, c->frec.p, c->fwoff.p);
        // (a synced fold serves kvr_compact_stage, whose k_cand reads every tuple's entry)
        hipLaunchKernelGGL(k_fold_lds, dim3((uint32_t)p_host), dim3(FP_T), 0, st, c->ctup.p, c->segs.p, c->fsz.p, s_lim,
                           c->frec.p, c->fwoff.p, (uint32_t)nwg, c->fent.p, c->flist.p, c->fcnt.p, c->cslot.p,
                           deferred ? 0u : 1u, (uint64_t)nt, cap_lim, c->fhot.p, c->fhot.p + hot_max * 2,
                           c->fcnt.p + FOLD_CNT * FOLD_SPEC_ROUNDS, (uint32_t)hot_max);
        hipLaunchKernelGGL(k_fold_hot, dim3((uint32_t)c->n_cu * 4), dim3(256), 0, st, c->ctup.p, c->segs.p, c->fsz.p,
                           c->frec.p, (uint32_t)nwg, c->fent.p, c->fhot.p, c->fhot.p + hot_max * 2,
                           c->fcnt.p + FOLD_CNT * FOLD_SPEC_ROUNDS, c->flist.p, c->fcnt.p, c->cslot.p,
                           deferred ? 0u : 1u, (uint32_t)hot_max);
    } else {
        hipLaunchKernelGGL(k_fent_clear, dim3(fold_grid(c)), dim3(256), 0, st, c->fent.p, c->fsz.p);
        round(nt, nullptr, nullptr, c->flist.p, c->fcnt.p);
    }
    HIPCHK(hipGetLastError());
    if (deferred) {
        for (uint32_t r = 1; r < FOLD_SPEC_ROUNDS; ++r)
            round(FOLD_SPEC_CAP, c->fcnt.p + FOLD_CNT * (r - 1), c->flist.p + (uint64_t)((r - 1) & 1u) * nt,
                  c->flist.p + (uint64_t)(r & 1u) * nt, c->fcnt.p + FOLD_CNT * r);
        HIPCHK(hipGetLastError());
        c->fold_pending = true;
        return KVR_OK;
    }
    const uint32_t *list = c->flist.p;
    uint64_t m = 0;
    for (uint32_t r = 0;; ++r) {
        uint32_t *next = c->flist.p + (uint64_t)(r & 1u) * nt;
        if (r > 0) {
            HIPCHK(hipMemsetAsync(c->fcnt.p, 0, FOLD_CNT * sizeof(uint32_t), st));
            round(m, nullptr, list, next, c->fcnt.p);
            HIPCHK(hipGetLastError());
        }
        uint32_t cnt[2] = {0, 0};   // tuples left for the next round, claims that found the table full
        uint32_t fs[4] = {0, 0, 0, 0};
        HIPCHK(hipMemcpyAsync(cnt, c->fcnt.p, 8, hipMemcpyDeviceToHost, st));
        if (r == 0) HIPCHK(hipMemcpyAsync(fs, c->fsz.p, 16, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        if (r == 0) {
            c->fold_slots = (uint64_t)fs[0] + 1;
            c->fold_est = (uint64_t)fs[2] | ((uint64_t)fs[3] << 32);
        }
        c->fold_rounds = r + 1;
        if (cnt[1]) {
            if (c->fold_slots == full_slots) return KVR_EHIP;   // cannot happen: 2 n entries hold every tuple
            hipLaunchKernelGGL(k_fold_setsize, dim3(1), dim3(1), 0, st, c->fsz.p, (uint32_t)(full_slots - 1));
            ++c->fold_redo;
            goto again;
        }
        if (cnt[0] == 0) break;
        // tuples whose tag another key holds: each round moves every one of them at least one
        // entry on, so (table size) rounds bound the loop (a few in practice)
        if (r > c->fold_slots) return KVR_EHIP;
        list = next;
        m = cnt[0];
    }
    return KVR_OK;
}

// the counters of deferred rounds, read back with the caller's own sync (fold_check_*)
struct FoldCheck {
    uint32_t cnt[FOLD_CNT * FOLD_SPEC_ROUNDS];
    uint32_t fs[4];
};
static hipError_t fold_check_enqueue(kvr_ctx *c, FoldCheck *fc) {
    if (!c->fold_pending) return hipSuccess;
    hipError_t e = hipMemcpyAsync(fc->cnt, c->fcnt.p, sizeof(fc->cnt), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(fc->fs, c->fsz.p, sizeof(fc->fs), hipMemcpyDeviceToHost, c->stream);
    return e;
}
// after that sync: true when the deferred rounds finished the fold (statistics filled in)
static bool fold_check_eval(kvr_ctx *c, const FoldCheck &fc) {
    if (!c->fold_pending) return true;
    c->fold_pending = false;
    c->fold_slots = (uint64_t)fc.fs[0] + 1;
    c->fold_est = (uint64_t)fc.fs[2] | ((uint64_t)fc.fs[3] << 32);
    bool ok = true;
    uint32_t rounds = 1;
    for (uint32_t r = 0; r < FOLD_SPEC_ROUNDS; ++r) {
        const uint32_t left = fc.cnt[FOLD_CNT * r], full = fc.cnt[FOLD_CNT * r + 1];
        if (full) ok = false;
        if (left) {
            if (r + 1 == FOLD_SPEC_ROUNDS || left > FOLD_SPEC_CAP) ok = false;
            else rounds = r + 2;
        }
    }
    c->fold_rounds = rounds;
    return ok;
}

// after the caller's sync point: did the deferred rounds finish the fold?  Reads the counters
// (and, when n_live is given, the live count fold_derive's scan left in dl_tot[1]) with one sync;
// if the fold was not complete it is redone synchronously and *redone is set (the caller then
// redoes what it derived from the table).
static int fold_settle(kvr_ctx *c, size_t nt, bool *redone, uint64_t *n_live) {
    (void)nt;
    *redone = false;
    hipStream_t st = c->stream;
    FoldCheck fc{};
    HIPCHK(fold_check_enqueue(c, &fc));
    if (n_live) HIPCHK(hipMemcpyAsync(n_live, c->dl_tot.p + 1, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (fold_check_eval(c, fc)) return KVR_OK;
    *redone = true;
    return fold_launch(c, nt, false);
}

// live flags (and, for a rewrite, record sizes) of the tuples from the fold table
// (keep_del: the last record of every key, tombstones included)
// (sparse: a byte per tuple in cfl8 instead, for kvr_compact's dense list, k_dl_*)
static hipError_t live_flags(kvr_ctx *c, size_t nt, bool sizes, bool keep_del = false, bool sparse = false) {
    hipStream_t st = c->stream;
    const uint64_t nfl = (nt + DL_CH - 1) / DL_CH * DL_CH;
    if (sparse && c->cfl8.ensure(nfl)) return hipErrorOutOfMemory;
    hipError_t e = sparse ? hipMemsetAsync(c->cfl8.p, 0, nfl, st) : hipMemsetAsync(c->cflag.p, 0, nt * 4, st);
    if (e == hipSuccess && sizes && !sparse) e = hipMemsetAsync(c->csize.p, 0, nt * 8, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_live_ent, dim3(fold_grid(c)), dim3(256), 0, st, c->fent.p, c->fsz.p, c->ctup.p,
                       (sizes && !sparse) ? c->csize.p : nullptr, sparse ? nullptr : c->cflag.p,
                       sparse ? c->cfl8.p : nullptr, keep_del ? 1u : 0u);
    return hipGetLastError();
}
// kvr_compact's dense live list from byte flags (k_dl_count / k_dl_scan / k_dl_fill); the two scans
// over every tuple (sizes, live flags) remain as a test and timing knob
static bool compact_packed(const kvr_ctx *c, size_t nt) {
    (void)c; (void)nt;
    return getenv("KVR_COMPACT_TWO_SCANS") == nullptr;
}

// sizes and live flags are in csize / cflag: scans, dense live list, cuts, gather, output
static int compact_back(kvr_ctx *c, uint32_t flags, uint64_t seg_target, uint8_t *out, uint64_t out_cap,
                        uint64_t *out_len, uint64_t *seg_ends, size_t seg_cap, size_t *n_out_segs,
                        bool packed = false) {
    const size_t nt = c->c_nt;
    const uint64_t bytes_in = c->cstats.bytes_in;
    hipStream_t st = c->stream;
    const uint32_t g = (uint32_t)((nt + 255) / 256);
    size_t tb = c->ctmp.n;
    const uint32_t nb = (uint32_t)((nt + DL_CH - 1) / DL_CH);
    if (packed) {
        if (c->dl_cnt.ensure(nb) || c->dl_bytes.ensure(nb)) return KVR_ENOMEM;
        hipLaunchKernelGGL(k_dl_count, dim3(nb), dim3(DL_T), 0, st, c->cfl8.p, c->ctup.p, c->dl_cnt.p, c->dl_bytes.p);
        hipLaunchKernelGGL(k_dl_scan, dim3(1), dim3(DL_ST), 0, st, c->dl_cnt.p, c->dl_bytes.p, nb, c->l_off.p, c->ctot.p);
    } else {
        HIPCHK(hipcub::DeviceScan::ExclusiveSum(c->ctmp.p, tb, c->csize.p, c->coff.p, (int)nt, st));
        tb = c->ctmp.n;
        HIPCHK(hipcub::DeviceScan::ExclusiveSum(c->ctmp.p, tb, c->cflag.p, c->cpos.p, (int)nt, st));
        hipLaunchKernelGGL(k_ctotals, dim3(1), dim3(64), 0, st, c->csize.p, c->coff.p, c->cflag.p, c->cpos.p,
                           (uint64_t)nt, c->l_off.p, c->ctot.p);
    }
    HIPCHK(hipGetLastError());
    // the live bytes are at most the segment bytes: size everything by that bound, so the rest of
    // the pipeline runs without a host round trip (the kernels read the true sizes on device)
    const uint64_t max_cuts = seg_target ? bytes_in / seg_target + 1 : 1;
    if (c->ccuts.ensure(max_cuts)) return KVR_ENOMEM;
    if (packed)
        hipLaunchKernelGGL(k_dl_fill, dim3(nb), dim3(DL_T), 0, st, c->cfl8.p, c->ctup.p, c->segs.p, c->dl_cnt.p,
                           c->dl_bytes.p, c->l_src.p, c->l_off.p);
    else
        hipLaunchKernelGGL(k_scatter, dim3(g), dim3(256), 0, st, c->ctup.p, (uint64_t)nt, c->segs.p, c->csize.p,
                           c->coff.p, c->cflag.p, c->cpos.p, c->l_src.p, c->l_off.p);
    HIPCHK(hipGetLastError());
    if (seg_target) {
        hipLaunchKernelGGL(k_cuts, dim3((uint32_t)std::min<uint64_t>((max_cuts + 255) / 256, 1024)), dim3(256), 0, st,
                           c->l_off.p, c->ctot.p, seg_target, c->ccuts.p);
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipEventRecord(c->ev[1], st));
    // gather straight into a device output when it is 8-B aligned, else through staging
    const bool direct = (flags & KVR_OUT_ON_DEVICE) && !(reinterpret_cast<uintptr_t>(out) & 7u);
    uint8_t *d_out = out;
    uint64_t d_cap = out_cap;
    if (!direct) {
        if (c->cout.ensure(bytes_in + 8)) return KVR_ENOMEM;
        d_out = c->cout.p;
        d_cap = bytes_in;
    }
    hipLaunchKernelGGL(k_gather_r, dim3((uint32_t)c->n_cu * 16), dim3(CT_GATHER), 0, st, c->l_src.p, c->l_off.p,
                       c->ctot.p, d_out, d_cap);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(c->ev[2], st));
    uint64_t tot[2] = {0, 0};
    HIPCHK(hipMemcpyAsync(tot, c->ctot.p, sizeof(tot), hipMemcpyDeviceToHost, st));
    std::vector<uint64_t> cuts(seg_target ? max_cuts : 0);
    if (seg_target) HIPCHK(hipMemcpyAsync(cuts.data(), c->ccuts.p, max_cuts * 8, hipMemcpyDeviceToHost, st));
    FoldCheck fc{};
    HIPCHK(fold_check_enqueue(c, &fc));   // a deferred fold is checked with this same sync
    HIPCHK(hipStreamSynchronize(st));
    if (!fold_check_eval(c, fc)) {        // rare: redo the fold with synced rounds, then the caller
        const int rc = fold_launch(c, nt, false);   // redoes the rewrite
        return rc == KVR_OK ? FOLD_REDONE : rc;
    }
    c->cstats.ms_fold = ev_ms(c->ev[0], c->ev[1]);
    c->cstats.ms_gather = ev_ms(c->ev[1], c->ev[2]);
    const uint64_t total = tot[0], n_live = tot[1];
    c->cstats.n_live = n_live;
    c->cstats.bytes_out = total;
    // new-segment boundaries: the distinct cut offsets, then the end
    std::vector<uint64_t> ends;
    if (total) {
        const uint64_t n_cuts = (seg_target && total > seg_target) ? (total - 1) / seg_target : 0;
        for (uint64_t k = 0; k < n_cuts; ++k)
            if (cuts[k] < total && (ends.empty() || cuts[k] > ends.back())) ends.push_back(cuts[k]);
        ends.push_back(total);
    }
    *out_len = total;
    *n_out_segs = ends.size();
    if (total > out_cap || ends.size() > seg_cap) return KVR_CAPACITY;
    for (size_t j = 0; j < ends.size(); ++j) seg_ends[j] = ends[j];
    if (total && !direct) {
        HIPCHK(hipMemcpyAsync(out, d_out, total, (flags & KVR_OUT_ON_DEVICE) ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
    }
    return KVR_OK;
}

int kvr_compact(kvr_ctx *c, const kvr_segment *segs, size_t n, uint32_t flags, uint64_t seg_target, uint8_t *out,
                uint64_t out_cap, uint64_t *out_len, uint64_t *seg_ends, size_t seg_cap, size_t *n_out_segs,
                kvr_error *err) {
    if (!c || (!segs && n) || !out_len || !n_out_segs || (out_cap && !out) || (seg_cap && !seg_ends)) return KVR_EINVAL;
    *out_len = 0;
    *n_out_segs = 0;
    size_t nt = 0;
    const int rc = compact_front(c, segs, n, flags, err, &nt, true, &c->cstats, true);   // deferred rounds
    if (rc != KVR_OK || nt == 0) return rc;
    const bool packed = compact_packed(c, nt);
    HIPCHK(live_flags(c, nt, true, false, packed));
    int rb = compact_back(c, flags, seg_target, out, out_cap, out_len, seg_ends, seg_cap, n_out_segs, packed);
    if (rb == FOLD_REDONE) {
        HIPCHK(live_flags(c, nt, true, false, packed));
        rb = compact_back(c, flags, seg_target, out, out_cap, out_len, seg_ends, seg_cap, n_out_segs, packed);
    }
    return rb;
}

int kvr_compact_stage(kvr_ctx *c, const kvr_segment *segs, size_t n, uint32_t flags, const uint32_t *gidx,
                      uint32_t n_ranks, uint64_t *counts, uint64_t *key_bytes, kvr_error *err) {
    if (!c || (!segs && n) || (n && !gidx) || n_ranks == 0 || !counts || !key_bytes) return KVR_EINVAL;
    for (uint32_t o = 0; o < n_ranks; ++o) counts[o] = key_bytes[o] = 0;
    c->c_ranks = n_ranks;
    size_t nt = 0;
    const int rc = compact_front(c, segs, n, flags, err, &nt, true, &c->cstats);
    if (rc != KVR_OK) return rc;
    c->c_staged = true;
    if (nt == 0) return KVR_OK;
    hipStream_t st = c->stream;
    const uint32_t g = (uint32_t)((nt + 255) / 256);
    if (c->c_gidx.ensure(n) || c->c_own.ensure(nt) || c->c_sidx.ensure(nt) || c->c_val.ensure(nt) ||
        c->c_scan.ensure(nt) || c->c_gstart.ensure(2 * (n_ranks + 1)) || c->c_hdr.ensure(nt) ||
        c->c_keys.ensure(c->cstats.bytes_in + 8))
        return KVR_ENOMEM;
    size_t t3 = 0;
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, t3, c->c_val.p, c->c_scan.p, (int)nt, st));
    if (c->ctmp.n < t3 && c->ctmp.ensure(t3)) return KVR_ENOMEM;
    HIPCHK(hipMemcpyAsync(c->c_gidx.p, gidx, n * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemsetAsync(c->c_gstart.p, 0, 2 * (n_ranks + 1) * 8, st));
    hipLaunchKernelGGL(k_cand, dim3(g), dim3(256), 0, st, c->ctup.p, (uint64_t)nt, c->fent.p, c->cslot.p, n_ranks,
                       c->c_own.p);
    for (uint32_t o = 0; o < n_ranks; ++o) {   // one group per owner rank, in owner order
        hipLaunchKernelGGL(k_cand_val, dim3(g), dim3(256), 0, st, c->ctup.p, (uint64_t)nt, c->c_own.p, o, c->c_val.p);
        size_t tb = c->ctmp.n;
        HIPCHK(hipcub::DeviceScan::ExclusiveSum(c->ctmp.p, tb, c->c_val.p, c->c_scan.p, (int)nt, st));
        hipLaunchKernelGGL(k_cand_total, dim3(1), dim3(64), 0, st, c->c_scan.p, c->c_val.p, (uint64_t)nt, o, n_ranks,
                           c->c_gstart.p);
        hipLaunchKernelGGL(k_cand_place, dim3(g), dim3(256), 0, st, c->ctup.p, (uint64_t)nt, c->segs.p, c->c_gidx.p,
                           c->c_own.p, o, n_ranks, c->c_scan.p, c->c_gstart.p, c->c_hdr.p, c->c_keys.p, c->c_sidx.p);
        HIPCHK(hipGetLastError());
    }
    std::vector<uint64_t> gs(2 * (n_ranks + 1));
    HIPCHK(hipMemcpyAsync(gs.data(), c->c_gstart.p, gs.size() * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    for (uint32_t o = 0; o < n_ranks; ++o) {
        counts[o] = gs[o + 1] - gs[o];
        key_bytes[o] = gs[n_ranks + 1 + o + 1] - gs[n_ranks + 1 + o];
    }
    c->c_ncand = gs[n_ranks];
    c->c_nkey = gs[2 * n_ranks + 1];
    return KVR_OK;
}

int kvr_compact_export(kvr_ctx *c, kvr_cand *d_hdr, uint8_t *d_keys) {
    if (!c || !c->c_staged) return KVR_EINVAL;
    hipStream_t st = c->stream;
    if (c->c_ncand) HIPCHK(hipMemcpyAsync(d_hdr, c->c_hdr.p, c->c_ncand * sizeof(kvr_cand), hipMemcpyDeviceToDevice, st));
    if (c->c_nkey) HIPCHK(hipMemcpyAsync(d_keys, c->c_keys.p, c->c_nkey, hipMemcpyDeviceToDevice, st));
    HIPCHK(hipStreamSynchronize(st));
    return KVR_OK;
}

int kvr_compact_resolve(kvr_ctx *c, const kvr_cand *d_hdr, const uint8_t *d_keys, const uint64_t *hdr_counts,
                        const uint64_t *key_counts, uint32_t n_ranks, uint8_t *d_win) {
    if (!c || !hdr_counts || !key_counts || n_ranks == 0) return KVR_EINVAL;
    std::vector<uint64_t> hk(2 * (n_ranks + 1), 0);   // header starts, then key bases, per sender
    for (uint32_t s2 = 0; s2 < n_ranks; ++s2) {
        hk[s2 + 1] = hk[s2] + hdr_counts[s2];
        hk[n_ranks + 1 + s2 + 1] = hk[n_ranks + 1 + s2] + key_counts[s2];
    }
    const uint64_t m = hk[n_ranks];
    if (m == 0) return KVR_OK;
    if (m >= 0x7FFFFFFFull) return KVR_EINVAL;
    uint64_t slots = 1;
    while (slots < 2 * m) slots <<= 1;
    hipStream_t st = c->stream;
    if (c->r_rep.ensure(slots) || c->r_best.ensure(slots) || c->r_slot.ensure(m) || c->r_hk.ensure(hk.size()))
        return KVR_ENOMEM;
    HIPCHK(hipMemcpyAsync(c->r_hk.p, hk.data(), hk.size() * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemsetAsync(c->r_rep.p, 0xFF, slots * 4, st));
    HIPCHK(hipMemsetAsync(c->r_best.p, 0, slots * 8, st));
    const uint32_t g = (uint32_t)((m + 255) / 256);
    hipLaunchKernelGGL(k_res_insert, dim3(g), dim3(256), 0, st, d_hdr, m, d_keys, c->r_hk.p, c->r_hk.p + n_ranks + 1,
                       n_ranks, c->r_rep.p, reinterpret_cast<unsigned long long *>(c->r_best.p), (uint32_t)(slots - 1),
                       c->r_slot.p);
    hipLaunchKernelGGL(k_res_flag, dim3(g), dim3(256), 0, st, d_hdr, m,
                       reinterpret_cast<const unsigned long long *>(c->r_best.p), c->r_slot.p, d_win);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(st));
    return KVR_OK;
}

int kvr_compact_finish(kvr_ctx *c, const uint8_t *d_win, uint32_t flags, uint64_t seg_target, uint8_t *out,
                       uint64_t out_cap, uint64_t *out_len, uint64_t *seg_ends, size_t seg_cap, size_t *n_out_segs) {
    if (!c || !c->c_staged || !out_len || !n_out_segs || (out_cap && !out) || (seg_cap && !seg_ends)) return KVR_EINVAL;
    *out_len = 0;
    *n_out_segs = 0;
    const size_t nt = c->c_nt;
    if (nt == 0) return KVR_OK;
    hipLaunchKernelGGL(k_live_global, dim3((uint32_t)((nt + 255) / 256)), dim3(256), 0, c->stream, c->ctup.p,
                       (uint64_t)nt, c->fent.p, c->cslot.p, c->c_sidx.p, d_win, c->csize.p, c->cflag.p);
    HIPCHK(hipGetLastError());
    return compact_back(c, flags, seg_target, out, out_cap, out_len, seg_ends, seg_cap, n_out_segs);
}

int kvr_last_compact_stats(const kvr_ctx *c, kvr_compact_stats *out) {
    if (!c || !out) return KVR_EINVAL;
    *out = c->cstats;
    return KVR_OK;
}

// diagnostic build only (-DKVR_PROF): per-phase cycle sums of k_replay's tile loop
int kvr_prof_read(unsigned long long *out, int reset) {
#ifdef KVR_PROF
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_prof), 16 * 8) != hipSuccess) return KVR_EHIP;
    if (reset) {
        unsigned long long z[16] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_prof), z, sizeof(z)) != hipSuccess) return KVR_EHIP;
    }
    return KVR_OK;
#else
    (void)out; (void)reset;
    return KVR_EINVAL;
#endif
}

// diagnostic build only: k_piece's per-stripe (start, end, HW_ID, XCC_ID), 4 x n words (not in the header)
int kvr_prof_stripes(unsigned long long *out, int n) {
#ifdef KVR_PROF
    if (n > 16384) n = 16384;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pst), (size_t)n * 32) == hipSuccess ? KVR_OK : KVR_EHIP;
#else
    (void)out; (void)n;
    return KVR_EINVAL;
#endif
}

int kvr_gen_segment_device(kvr_ctx *c, const kvr_gen_params *p, uint64_t seg_no, uint8_t *d_buf, uint64_t cap,
                           uint64_t *len_out, uint32_t *d_expected, uint64_t exp_cap, uint64_t *n_rec_out) {
    if (!c || !p || !len_out) return KVR_EINVAL;
    HIPCHK(hipSetDevice(c->device));
    const uint64_t sbase = kvr_gen_sbase(p->seed, seg_no);
    std::vector<GenRecDev> recs;
    uint64_t off = 0;
    for (uint64_t i = 0;; ++i) {
        kvr_gen_rec r;
        kvr_gen_record(p, sbase, i, &r);
        const uint64_t sz = kvr_gen_rec_size(&r);
        if (off + sz > p->seg_bytes) break;
        recs.push_back(GenRecDev{off, r.key_id, r.vseed, r.flip_bit, r.op, r.vlen});
        off += sz;
    }
    *len_out = off;
    if (n_rec_out) *n_rec_out = recs.size();
    if (off > cap || !d_buf) return KVR_CAPACITY;
    if (d_expected && recs.size() > exp_cap) return KVR_CAPACITY;
    if (recs.empty()) return KVR_OK;
    if (c->gen.ensure(recs.size())) return KVR_ENOMEM;
    hipStream_t st = c->stream;
    HIPCHK(hipMemcpyAsync(c->gen.p, recs.data(), recs.size() * sizeof(GenRecDev), hipMemcpyHostToDevice, st));
    const uint32_t grid = (uint32_t)std::min<uint64_t>(recs.size(), 65536);
    hipLaunchKernelGGL(k_gen_fill, dim3(grid), dim3(256), 0, st, c->gen.p, (uint64_t)recs.size(), d_buf);
    HIPCHK(hipGetLastError());
    if (d_expected) {
        const uint32_t g2 = (uint32_t)std::min<uint64_t>((recs.size() + 255) / 256, 65536);
        hipLaunchKernelGGL(k_gen_manifest, dim3(g2), dim3(256), 0, st, c->gen.p, (uint64_t)recs.size(), c->crc.p, d_expected);
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipStreamSynchronize(st));
    return KVR_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------------------
// streamed ingest: host segments -> HBM in batches on a copy stream, the
// transfer of batch b+1 overlapping the replay of batch b (engine.rs:55-57 over host bytes)
// ---------------------------------------------------------------------------------------
namespace {
struct StreamBatch {
    size_t s0, s1;     // segments [s0, s1)
    uint64_t bytes;    // padded bytes in the HBM slot
    uint64_t raw;      // segment bytes
};
}  // namespace

// Fill HBM slot k with batch b on the copy stream (runs on a helper thread while the caller's
// thread replays the previous batch).  Pageable bytes go through pinned staging slot k first,
// one segment at a time, so the memcpy of segment i+1 overlaps the DMA of segment i.
static int stream_fill(kvr_ctx *c, const kvr_segment *segs, const StreamBatch &b, int k, uint32_t flags) {
    HIPCHK(hipSetDevice(c->device));
    const bool pinned = (flags & KVR_HOST_PINNED) != 0;
    uint64_t off = 0;
    for (size_t i = b.s0; i < b.s1; ++i) {
        const uint64_t len = segs[i].len;
        if (len) {
            const uint8_t *src = segs[i].bytes;
            if (!pinned) {
                memcpy(c->h_stage[k] + off, src, len);
                src = c->h_stage[k] + off;
            }
            HIPCHK(hipMemcpyAsync(c->slot[k].p + off, src, len, hipMemcpyHostToDevice, c->copy));
        }
        off += (len + 255) & ~255ull;
    }
    HIPCHK(hipEventRecord(c->ev_copy[k], c->copy));
    return KVR_OK;
}

extern "C" {

int kvr_replay_stream(kvr_ctx *c, const kvr_segment *segs, size_t n, uint32_t flags, uint64_t batch_bytes,
                      const uint32_t *expected, size_t n_expected, kvr_tuple *out, size_t cap, size_t *n_out,
                      kvr_error *err) {
    if (!c || (!segs && n) || !n_out || (cap && !out)) return KVR_EINVAL;
    if (flags & ~KVR_HOST_PINNED) return KVR_EINVAL;   // host bytes in, host tuples out
    if (err) memset(err, 0, sizeof(*err));
    *n_out = 0;
    memset(&c->sstats, 0, sizeof(c->sstats));
    memset(&c->stats, 0, sizeof(c->stats));
    if (n == 0) return KVR_OK;
    if (n >= 0xFFFFFFFFull) return KVR_EINVAL;
    for (size_t i = 0; i < n; ++i) {
        if (i && segs[i].seg_id < segs[i - 1].seg_id) return KVR_EINVAL;   // caller sorts (engine.rs:51)
        if (segs[i].len && !segs[i].bytes) return KVR_EINVAL;
    }
    const auto t0 = std::chrono::steady_clock::now();
    if (batch_bytes == 0) batch_bytes = 1ull << 30;
    // batches: consecutive segments while their padded sizes fit batch_bytes (a larger segment
    // is a batch of its own)
    std::vector<StreamBatch> bs;
    StreamBatch cur{0, 0, 0, 0};
    uint64_t slot_need = 256;
    for (size_t i = 0; i < n; ++i) {
        const uint64_t padded = (segs[i].len + 255) & ~255ull;
        if (cur.s1 > cur.s0 && cur.bytes + padded > batch_bytes) {
            bs.push_back(cur);
            cur = StreamBatch{i, i, 0, 0};
        }
        cur.s1 = i + 1;
        cur.bytes += padded;
        cur.raw += segs[i].len;
        slot_need = std::max(slot_need, cur.bytes);
    }
    bs.push_back(cur);
    HIPCHK(hipSetDevice(c->device));
    if (!c->copy) {
        HIPCHK(hipStreamCreateWithFlags(&c->copy, hipStreamNonBlocking));
        for (auto &e : c->ev_copy) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    for (int k = 0; k < 2 && k < (int)bs.size(); ++k) {
        if (c->slot[k].ensure(slot_need)) return KVR_ENOMEM;
        if (!(flags & KVR_HOST_PINNED) && c->h_stage_cap[k] < slot_need) {
            if (c->h_stage[k]) (void)hipHostFree(c->h_stage[k]);
            c->h_stage[k] = nullptr;
            c->h_stage_cap[k] = 0;
            if (hipHostMalloc(reinterpret_cast<void **>(&c->h_stage[k]), slot_need) != hipSuccess) {
                c->h_stage[k] = nullptr;
                return KVR_ENOMEM;
            }
            c->h_stage_cap[k] = slot_need;
        }
    }
    auto drain = [&](int rc) {
        (void)hipStreamSynchronize(c->copy);
        return rc;
    };
    int rc = stream_fill(c, segs, bs[0], 0, flags);
    if (rc != KVR_OK) return drain(rc);
    kvr_stats tot{};
    size_t done = 0;   // tuples of the finished batches (counted on past cap: the required size)
    std::vector<kvr_segment> loc;
    for (size_t b = 0; b < bs.size(); ++b) {
        const int k = (int)(b & 1);
        const StreamBatch &B = bs[b];
        // the replay of batch b waits for its transfer on the device, not on the host
        HIPCHK(hipStreamWaitEvent(c->stream, c->ev_copy[k], 0));
        int rc_next = KVR_OK;
        std::thread filler;
        if (b + 1 < bs.size())   // slot k^1 held batch b-1, whose replay has returned
            filler = std::thread([&, b, k] { rc_next = stream_fill(c, segs, bs[b + 1], k ^ 1, flags); });
        loc.resize(B.s1 - B.s0);
        uint64_t off = 0;
        for (size_t j = 0; j < loc.size(); ++j) {
            const kvr_segment &s = segs[B.s0 + j];
            loc[j] = kvr_segment{s.seg_id, c->slot[k].p + off, s.len};
            off += (s.len + 255) & ~255ull;
        }
        // expected CRCs are per record in tuple order; a batch holds at most raw/5 + 1 records
        const size_t e0 = std::min(done, n_expected);
        const size_t ne = expected ? std::min<uint64_t>(n_expected - e0, B.raw / 5 + 1) : 0;
        const size_t room = done < cap ? cap - done : 0;
        size_t nb = 0;
        kvr_error e{};
        rc = kvr_replay(c, loc.data(), loc.size(), KVR_SEGS_ON_DEVICE, ne ? expected + e0 : nullptr, ne,
                        room ? out + done : nullptr, room, &nb, &e);
        if (filler.joinable()) filler.join();
        tot.ms_total += c->stats.ms_total;
        tot.ms_replay += c->stats.ms_replay;
        tot.ms_link += c->stats.ms_link;
        tot.ms_compact += c->stats.ms_compact;
        tot.bytes_in += c->stats.bytes_in;
        tot.n_records += c->stats.n_records;
        tot.n_crc_fail += c->stats.n_crc_fail;
        tot.n_stripes += c->stats.n_stripes;
        tot.n_tiles += c->stats.n_tiles;
        tot.n_redo += c->stats.n_redo;
        tot.n_link_passes += c->stats.n_link_passes;
        if (rc == KVR_CORRUPTED) {   // batches run in (segment, offset) order: this is the first error
            if (err) {
                *err = e;
                err->seg_idx += (uint32_t)B.s0;
            }
            return drain(rc);
        }
        if (rc != KVR_OK && rc != KVR_CAPACITY) return drain(rc);
        if (B.s0) {   // seg_idx into the caller's segs[]
            const size_t m = std::min(nb, room);
            for (size_t t = 0; t < m; ++t) out[done + t].seg_idx += (uint32_t)B.s0;
        }
        done += nb;
        if (rc_next != KVR_OK) return drain(rc_next);
    }
    c->stats = tot;
    *n_out = done;
    c->sstats.n_batches = bs.size();
    c->sstats.bytes_in = tot.bytes_in;
    c->sstats.n_records = done;
    c->sstats.ms_device = tot.ms_total;
    c->sstats.ms_wall = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return done > cap ? KVR_CAPACITY : KVR_OK;
}

int kvr_last_stream_stats(const kvr_ctx *c, kvr_stream_stats *out) {
    if (!c || !out) return KVR_EINVAL;
    *out = c->sstats;
    return KVR_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------------------
// batch ETag compute / verify (kvr_etag.hip; SURVEY §8f rank 4, storage.rs:27)
// ---------------------------------------------------------------------------------------
extern "C" {

int kvr_etag_batch(kvr_ctx *c, const uint8_t *data, uint64_t data_len, const uint64_t *offs, const uint64_t *lens,
                   size_t n, uint32_t flags, const uint32_t *expected, uint32_t *crc_out, uint64_t *n_fail) {
    if (!c || (n && (!offs || !lens || !crc_out)) || (data_len && !data)) return KVR_EINVAL;
    if (flags & ~(KVR_SEGS_ON_DEVICE | KVR_OUT_ON_DEVICE | KVR_EXPECTED_ON_DEVICE)) return KVR_EINVAL;
    memset(&c->estats, 0, sizeof(c->estats));
    if (n_fail) *n_fail = 0;
    if (n == 0) return KVR_OK;
    if (n >= 0xFFFFFFFFull) return KVR_EINVAL;
    std::vector<uint64_t> cpre(n + 1);
    uint64_t nch = 0, bytes = 0;
    for (size_t i = 0; i < n; ++i) {
        if (offs[i] > data_len || lens[i] > data_len - offs[i]) return KVR_EINVAL;   // blob outside data
        cpre[i] = nch;
        nch += (lens[i] + ETAG_CH - 1) / ETAG_CH;
        bytes += lens[i];
    }
    cpre[n] = nch;
    if (nch >= 0xFFFFFFFFull || data_len >= (1ull << 48)) return KVR_EINVAL;   // (k_etag_map's packed descriptors)
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = c->stream;
    if (!c->e_x.p) {   // XT[t] = x^(8t) for t <= CH, XC[l] = x^(8 l CH) for l < 64, x^(8 * 64 CH)
        std::vector<uint32_t> x(ETAG_NX);
        x[0] = GF_ONE;
        for (uint32_t t = 1; t <= ETAG_CH; ++t) x[t] = gf_mul(x[t - 1], 0x00800000u);
        uint32_t *xc = x.data() + ETAG_CH + 1;
        xc[0] = GF_ONE;
        for (int l = 1; l <= 64; ++l) xc[l] = gf_mul(xc[l - 1], x[ETAG_CH]);
        // KL: per lane, nibble tables of the full-chunk lane shift x^(8 (CH - 64 (lane + 1)))
        x.resize(ETAG_NX + ETAG_NKL);
        for (uint32_t l = 0; l < 64; ++l)
            for (uint32_t i = 0; i < 8; ++i)
                for (uint32_t nb = 0; nb < 16; ++nb)
                    x[ETAG_NX + l * 128 + i * 16 + nb] = gf_mul(nb << (4 * i), x[ETAG_CH - 64 * (l + 1)]);
        if (c->e_x.ensure(x.size())) return KVR_ENOMEM;
        HIPCHK(hipMemcpyAsync(c->e_x.p, x.data(), x.size() * 4, hipMemcpyHostToDevice, st));
        HIPCHK(hipStreamSynchronize(st));   // x is a local
    }
    const uint8_t *d_data = data;
    if (!(flags & KVR_SEGS_ON_DEVICE)) {
        if (c->e_data.ensure(data_len + 256)) return KVR_ENOMEM;
        if (data_len) HIPCHK(hipMemcpyAsync(c->e_data.p, data, data_len, hipMemcpyHostToDevice, st));
        d_data = c->e_data.p;
    }
    if (c->e_cpre.ensure(n + 1) || c->e_offs.ensure(n) || c->e_lens.ensure(n) || c->e_cdesc.ensure(nch + 1) ||
        c->e_creg.ensure(nch) || c->e_fail.ensure(1))
        return KVR_ENOMEM;
    HIPCHK(hipMemcpyAsync(c->e_cpre.p, cpre.data(), (n + 1) * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(c->e_offs.p, offs, n * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(c->e_lens.p, lens, n * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemsetAsync(c->e_fail.p, 0, 8, st));
    uint32_t *d_out = crc_out;
    if (!(flags & KVR_OUT_ON_DEVICE)) {
        if (c->e_out.ensure(n)) return KVR_ENOMEM;
        d_out = c->e_out.p;
    }
    const uint32_t *d_exp = expected;
    if (expected && !(flags & KVR_EXPECTED_ON_DEVICE)) {
        if (c->e_exp.ensure(n)) return KVR_ENOMEM;
        HIPCHK(hipMemcpyAsync(c->e_exp.p, expected, n * 4, hipMemcpyHostToDevice, st));
        d_exp = c->e_exp.p;
    }
    const uint32_t mgrid = (uint32_t)std::min<uint64_t>((nch + 255) / 256, 65536);
    if (nch)
        hipLaunchKernelGGL(k_etag_map, dim3(mgrid), dim3(256), 0, st, c->e_cpre.p, (uint64_t)n, c->e_offs.p, c->e_lens.p,
                           nch, c->e_cdesc.p);
    HIPCHK(hipEventRecord(c->ev[0], st));
    if (nch) {
        const uint64_t per = (uint64_t)ETAG_WPB * (KVR_ETAG_DB ? ETAG_NC_DB : ETAG_NC);
        if (!c->e_wg_per_cu) {   // persistent grid: exactly the resident workgroups
            int occ = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_etag_chunk, 64 * ETAG_WPB, 0) != hipSuccess || occ < 1)
                occ = 1;
            c->e_wg_per_cu = (uint32_t)occ;
        }
        const uint64_t g = std::min<uint64_t>((nch + per - 1) / per, (uint64_t)c->n_cu * c->e_wg_per_cu);
        hipLaunchKernelGGL(k_etag_chunk, dim3((uint32_t)g), dim3(64 * ETAG_WPB), 0, st, d_data, data_len, c->e_cdesc.p,
                           nch, c->crc.p, c->e_x.p, c->e_creg.p);
    }
    HIPCHK(hipEventRecord(c->ev[1], st));
    hipLaunchKernelGGL(k_etag_join, dim3((uint32_t)((n + ETAG_WPB - 1) / ETAG_WPB)), dim3(64 * ETAG_WPB), 0, st,
                       c->e_lens.p, c->e_cpre.p, (uint64_t)n, c->e_creg.p, c->e_x.p, d_exp, d_out,
                       reinterpret_cast<unsigned long long *>(c->e_fail.p));
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(c->ev[2], st));
    uint64_t fails = 0;
    HIPCHK(hipMemcpyAsync(&fails, c->e_fail.p, 8, hipMemcpyDeviceToHost, st));
    if (!(flags & KVR_OUT_ON_DEVICE)) HIPCHK(hipMemcpyAsync(crc_out, d_out, n * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(wait_stream(st, c->ev[5]));
    float a = 0.f, b = 0.f;
    (void)hipEventElapsedTime(&a, c->ev[0], c->ev[1]);
    (void)hipEventElapsedTime(&b, c->ev[1], c->ev[2]);
    c->estats.ms_chunk = a;
    c->estats.ms_join = b;
    c->estats.bytes = bytes;
    c->estats.n_blobs = n;
    c->estats.n_chunks = nch;
    c->estats.n_fail = expected ? fails : 0;
    if (n_fail) *n_fail = c->estats.n_fail;
    return KVR_OK;
}

int kvr_last_etag_stats(const kvr_ctx *c, kvr_etag_stats *out) {
    if (!c || !out) return KVR_EINVAL;
    *out = c->estats;
    return KVR_OK;
}

void kvr_etag_format(uint32_t crc, char *out) {
    if (out) snprintf(out, 9, "%08x", crc);
}

}  // extern "C"

#include "kvr_index.hip"
#include "kvr_multi.hip"
