/*
 * kvr_host.cpp — host side of the drop-in (include/kvstore_host.h): discovery, the CPU
 * generator, the last-writer-wins fold and a KVStore mirror whose open() replays on the GPU.
 * Built with g++ into libkvhost.so, linked against libkvreplay.so.
 */
#include <dirent.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/kvreplay.h"
#include "../../include/kvstore_host.h"
#include "kvr_gen_common.h"

namespace {

uint32_t crc_table[256];
bool crc_ready = false;

uint32_t crc32_update(uint32_t crc, const uint8_t *p, size_t n) {
    if (!crc_ready) {
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t c = i;
            for (int k = 0; k < 8; ++k) c = (c & 1u) ? (c >> 1) ^ 0xEDB88320u : (c >> 1);
            crc_table[i] = c;
        }
        crc_ready = true;
    }
    uint32_t c = ~crc;
    for (size_t i = 0; i < n; ++i) c = (c >> 8) ^ crc_table[(c ^ p[i]) & 0xFFu];
    return ~c;
}

bool utf8_valid(const uint8_t *s, size_t n) {   // std::str::from_utf8 acceptance (valid or not)
    size_t i = 0;
    while (i < n) {
        const uint8_t b = s[i];
        if (b < 0x80) { ++i; continue; }
        int w = (b >= 0xC2 && b <= 0xDF) ? 2 : (b >= 0xE0 && b <= 0xEF) ? 3 : (b >= 0xF0 && b <= 0xF4) ? 4 : 0;
        if (!w || i + w > n) return false;
        const uint8_t c1 = s[i + 1];
        bool ok = (c1 & 0xC0) == 0x80;
        if (w == 3) ok = (b == 0xE0) ? (c1 >= 0xA0 && c1 <= 0xBF) : (b == 0xED) ? (c1 >= 0x80 && c1 <= 0x9F) : ok;
        if (w == 4) ok = (b == 0xF0) ? (c1 >= 0x90 && c1 <= 0xBF) : (b == 0xF4) ? (c1 >= 0x80 && c1 <= 0x8F) : ok;
        if (!ok) return false;
        for (int k = 2; k < w; ++k) if ((s[i + k] & 0xC0) != 0x80) return false;
        i += w;
    }
    return true;
}

struct KeyRef {   // key bytes inside a resident segment
    const uint8_t *p;
    uint32_t n;
    uint32_t tag;
};
struct KeyHash {
    size_t operator()(const KeyRef &k) const { return (size_t)k.tag * 0x9E3779B97F4A7C15ull; }
};
struct KeyEq {
    bool operator()(const KeyRef &a, const KeyRef &b) const { return a.n == b.n && memcmp(a.p, b.p, a.n) == 0; }
};

}  // namespace

struct kvs_store {
    std::string dir;
    std::vector<uint64_t> ids;
    std::vector<std::vector<uint8_t>> bytes;
    struct Ent { uint32_t seg_idx; uint64_t val_off; uint32_t len; };
    std::unordered_map<KeyRef, Ent, KeyHash, KeyEq> index;
    uint64_t total_bytes = 0;
    uint64_t active_id = 0;
};

extern "C" {

int kvh_parse_u64(const char *s, size_t n, uint64_t *out) {
    if (n == 0) return 0;
    size_t i = 0;
    if (s[0] == '+') {   // u64::from_str accepts one leading '+' (not alone)
        if (n == 1) return 0;
        i = 1;
    }
    uint64_t v = 0;
    for (; i < n; ++i) {
        const unsigned d = (unsigned char)s[i] - '0';
        if (d > 9) return 0;
        if (v > (UINT64_MAX - d) / 10) return 0;   // overflow -> Err
        v = v * 10 + d;
    }
    *out = v;
    return 1;
}

int kvh_gen_segment(const kvr_gen_params *p, uint64_t seg_no, uint8_t *buf, uint64_t cap, uint64_t *len_out,
                    uint32_t *expected, uint64_t exp_cap, uint64_t *n_rec_out) {
    if (!p || !len_out) return KVR_EINVAL;
    const uint64_t sbase = kvr_gen_sbase(p->seed, seg_no);
    uint64_t off = 0, i = 0;
    for (;; ++i) {   // size pass
        kvr_gen_rec r;
        kvr_gen_record(p, sbase, i, &r);
        const uint64_t sz = kvr_gen_rec_size(&r);
        if (off + sz > p->seg_bytes) break;
        off += sz;
    }
    *len_out = off;
    if (n_rec_out) *n_rec_out = i;
    if (!buf) return KVR_OK;
    if (off > cap || (expected && i > exp_cap)) return KVR_CAPACITY;
    uint64_t o = 0;
    for (uint64_t k = 0; k < i; ++k) {
        kvr_gen_rec r;
        kvr_gen_record(p, sbase, k, &r);
        uint8_t *q = buf + o;
        q[0] = (uint8_t)r.op;   // engine.rs:169 / :191
        q[1] = (uint8_t)KVR_GEN_KEY_LEN; q[2] = 0; q[3] = 0; q[4] = 0;
        kvr_gen_key(r.key_id, q + 5);
        if (r.op == 0) {
            uint8_t *v = q + 9 + KVR_GEN_KEY_LEN;
            q[5 + KVR_GEN_KEY_LEN] = (uint8_t)r.vlen;
            q[6 + KVR_GEN_KEY_LEN] = (uint8_t)(r.vlen >> 8);
            q[7 + KVR_GEN_KEY_LEN] = (uint8_t)(r.vlen >> 16);
            q[8 + KVR_GEN_KEY_LEN] = (uint8_t)(r.vlen >> 24);
            for (uint64_t j = 0; j < r.vlen; ++j) v[j] = kvr_gen_vbyte(r.vseed, j);
            if (expected) expected[k] = crc32_update(0, v, r.vlen);   // manifest before the fault
            if (r.flip_bit >= 0) v[(uint64_t)r.flip_bit >> 3] ^= (uint8_t)(1u << (r.flip_bit & 7));
        } else if (expected) {
            expected[k] = 0;
        }
        o += kvr_gen_rec_size(&r);
    }
    return KVR_OK;
}

int kvh_discover(const char *dir, uint64_t *ids, size_t cap, char *paths, size_t path_cap, size_t *n_out) {
    if (!dir || !n_out) return KVR_EINVAL;
    DIR *d = opendir(dir);
    if (!d) return KVR_EIO;
    std::vector<std::pair<uint64_t, std::string>> found;
    static const char pre[] = "segment-", suf[] = ".dat";
    while (struct dirent *e = readdir(d)) {
        const char *name = e->d_name;
        const size_t n = strlen(name);
        if (!utf8_valid(reinterpret_cast<const uint8_t *>(name), n)) continue;   // to_str() == None
        if (n < 8 || memcmp(name, pre, 8) != 0) continue;                          // engine.rs:40
        if (n < 4 || memcmp(name + n - 4, suf, 4) != 0) continue;
        if (n < 12) continue;
        uint64_t id;
        if (!kvh_parse_u64(name + 8, n - 12, &id)) continue;                       // engine.rs:43
        std::string full = std::string(dir) + "/" + name;                          // base_dir.join(name)
        found.emplace_back(id, full);
    }
    closedir(d);
    std::stable_sort(found.begin(), found.end(), [](const auto &a, const auto &b) {   // engine.rs:51
        return a.first != b.first ? a.first < b.first : a.second < b.second;
    });
    *n_out = found.size();
    if (found.size() > cap) return KVR_CAPACITY;
    size_t po = 0;
    for (size_t i = 0; i < found.size(); ++i) {
        if (ids) ids[i] = found[i].first;
        if (paths) {
            const size_t L = found[i].second.size() + 1;
            if (po + L > path_cap) return KVR_CAPACITY;
            memcpy(paths + po, found[i].second.c_str(), L);
            po += L;
        }
    }
    return KVR_OK;
}

uint64_t kvh_fold(const kvr_segment *segs, const kvr_tuple *t, size_t n, uint8_t *live, uint64_t *total_bytes) {
    std::unordered_map<KeyRef, size_t, KeyHash, KeyEq> last;
    last.reserve(n / 2 + 16);
    for (size_t i = 0; i < n; ++i) {
        const KeyRef k{segs[t[i].seg_idx].bytes + t[i].rec_off + 5, t[i].key_len, t[i].key_tag};
        auto it = last.find(k);
        if (it == last.end()) last.emplace(k, i);
        else it->second = i;                   // later record wins (engine.rs:137, :141)
    }
    if (live) memset(live, 0, n);
    uint64_t nk = 0, tb = 0;
    for (const auto &kv : last) {
        if (t[kv.second].op == 0) {
            if (live) live[kv.second] = 1;
            ++nk;
            tb += t[kv.second].val_len;
        }
    }
    if (total_bytes) *total_bytes = tb;
    return nk;
}

// Parallel fold: the last writer of a key is its maximal (segment, offset)
// record, so the keys can be split by hash into independent partitions.  Phase 1 counts each
// chunk's tuples per partition, phase 2 scatters the tuple indices partition-major (chunk order
// kept, so each partition stays in (segment, offset) order), phase 3 folds every partition into
// its own open-addressing table (key_tag as the hash, key bytes compared on a tag match).
uint64_t kvh_fold_parallel(const kvr_segment *segs, const kvr_tuple *t, size_t n, uint32_t n_threads,
                           uint8_t *live, uint64_t *total_bytes) {
    if (total_bytes) *total_bytes = 0;
    if (n == 0) return 0;
    if (n_threads == 0) n_threads = std::max(1u, std::thread::hardware_concurrency());
    n_threads = std::min<uint32_t>(n_threads, 256);
    if (n >= 0xFFFFFFFFull || n_threads == 1) return kvh_fold(segs, t, n, live, total_bytes);
    const uint32_t P = n_threads;                       // one partition per thread
    const size_t chunk = (n + P - 1) / P;
    auto part = [P](uint32_t tag) { return (uint32_t)(((uint64_t)(tag * 0x9E3779B1u) * P) >> 32); };
    std::vector<uint64_t> cnt((size_t)P * P, 0);         // cnt[chunk * P + partition]
    std::vector<std::thread> th;
    auto run = [&](auto fn) {
        th.clear();
        for (uint32_t w = 0; w < P; ++w) th.emplace_back(fn, w);
        for (auto &x : th) x.join();
    };
    run([&](uint32_t c) {
        const size_t a = std::min(n, c * chunk), b = std::min(n, a + chunk);
        uint64_t *h = &cnt[(size_t)c * P];
        for (size_t i = a; i < b; ++i) ++h[part(t[i].key_tag)];
    });
    std::vector<uint64_t> pstart(P + 1, 0), cur((size_t)P * P);
    for (uint32_t p = 0; p < P; ++p) {
        uint64_t s = pstart[p];
        for (uint32_t c = 0; c < P; ++c) { cur[(size_t)c * P + p] = s; s += cnt[(size_t)c * P + p]; }
        pstart[p + 1] = s;
    }
    std::vector<uint32_t> idx(n);
    run([&](uint32_t c) {
        const size_t a = std::min(n, c * chunk), b = std::min(n, a + chunk);
        uint64_t *o = &cur[(size_t)c * P];
        for (size_t i = a; i < b; ++i) idx[o[part(t[i].key_tag)]++] = (uint32_t)i;
    });
    if (live) memset(live, 0, n);
    std::vector<uint64_t> nk(P, 0), tb(P, 0);
    run([&](uint32_t p) {
        const uint64_t a = pstart[p], b = pstart[p + 1];
        if (a == b) return;
        uint64_t cap = 16;
        while (cap < 2 * (b - a)) cap <<= 1;
        // slot = key_tag << 32 | tuple index of the key's latest record: probes compare tags in
        // the table and touch the tuple and the key bytes only on a tag match
        constexpr uint64_t EMPTY = ~0ull;
        std::vector<uint64_t> slot(cap, EMPTY);
        const uint64_t mask = cap - 1;
        for (uint64_t j = a; j < b; ++j) {
            const uint32_t i = idx[j];
            const kvr_tuple &x = t[i];
            const uint64_t tag = (uint64_t)x.key_tag << 32;
            for (uint64_t h = ((uint64_t)x.key_tag * 0x9E3779B97F4A7C15ull) >> 20;; ++h) {
                uint64_t &s = slot[h & mask];
                if (s == EMPTY) { s = tag | i; break; }
                if ((s & 0xFFFFFFFF00000000ull) != tag) continue;
                const kvr_tuple &y = t[(uint32_t)s];
                if (y.key_len == x.key_len &&
                    memcmp(segs[y.seg_idx].bytes + y.rec_off + 5, segs[x.seg_idx].bytes + x.rec_off + 5,
                           x.key_len) == 0) {
                    s = tag | i;                      // later record wins (engine.rs:137, :141)
                    break;
                }
            }
        }
        for (uint64_t s : slot) {
            if (s == EMPTY) continue;
            const kvr_tuple &y = t[(uint32_t)s];
            if (y.op != 0) continue;
            if (live) live[(uint32_t)s] = 1;
            ++nk[p];
            tb[p] += y.val_len;
        }
    });
    uint64_t k = 0, bytes = 0;
    for (uint32_t p = 0; p < P; ++p) { k += nk[p]; bytes += tb[p]; }
    if (total_bytes) *total_bytes = bytes;
    return k;
}

static int read_file(const std::string &path, std::vector<uint8_t> &out, int *os_err) {
    const int fd = open(path.c_str(), O_RDONLY);
    if (fd < 0) { *os_err = errno; return -1; }   // engine.rs:80-82: open failure -> CorruptedData
    struct stat st;
    if (fstat(fd, &st) == 0 && S_ISDIR(st.st_mode)) {   // read() fails -> treated as EOF (engine.rs:88)
        close(fd);
        out.clear();
        return 0;
    }
    out.clear();
    uint8_t buf[1 << 16];
    for (;;) {
        const ssize_t r = read(fd, buf, sizeof(buf));
        if (r < 0) { if (errno == EINTR) continue; break; }   // a read error ends the segment like EOF
        if (r == 0) break;
        out.insert(out.end(), buf, buf + r);
    }
    close(fd);
    return 0;
}

// replay the store's resident segments on ctx's GPU and fold the index (engine.rs:53-57, :137, :141)
static int build_index(kvs_store *s, kvr_ctx *ctx, kvr_error *err, char *msg, size_t msg_cap,
                       const std::vector<std::string> *paths) {
    const size_t n = s->ids.size();
    s->index.clear();
    s->total_bytes = 0;
    std::vector<kvr_segment> segs(n);
    uint64_t total = 0;
    for (size_t i = 0; i < n; ++i) {
        segs[i] = kvr_segment{s->ids[i], s->bytes[i].data(), s->bytes[i].size()};
        total += s->bytes[i].size();
    }
    // the replay and the last-writer fold (engine.rs:137, :141) both run on the GPU
    // (kvr_replay_live): only each live key's final SET comes back
    std::vector<kvr_tuple> tuples(std::max<size_t>(16, total / 256));
    size_t nt = 0;
    kvr_error e{};
    int rc = n ? kvr_replay_live(ctx, segs.data(), n, 0, tuples.data(), tuples.size(), &nt, &e) : KVR_OK;
    if (rc == KVR_CAPACITY) {
        tuples.resize(nt);
        rc = kvr_replay_live(ctx, segs.data(), n, 0, tuples.data(), tuples.size(), &nt, &e);
    }
    if (rc == KVR_CORRUPTED) {
        if (err) *err = e;
        if (msg && paths) kvr_format_error(&e, (*paths)[e.seg_idx].c_str(), msg, msg_cap);
        return rc;
    }
    if (rc != KVR_OK) return rc;
    s->index.reserve(nt + 16);
    for (size_t i = 0; i < nt; ++i) {   // one live SET per key, already folded
        const kvr_tuple &t = tuples[i];
        const KeyRef k{segs[t.seg_idx].bytes + t.rec_off + 5, t.key_len, t.key_tag};
        s->index[k] = kvs_store::Ent{t.seg_idx, t.rec_off + 9 + t.key_len, t.val_len};
    }
    for (const auto &kv : s->index) s->total_bytes += kv.second.len;
    return KVR_OK;
}

static bool is_segment_name(const char *name) {   // compaction.rs:41-43
    const size_t n = strlen(name);
    return n >= 12 && memcmp(name, "segment-", 8) == 0 && memcmp(name + n - 4, ".dat", 4) == 0;
}

static int write_file_sync(const std::string &path, const uint8_t *p, size_t n) {
    const int fd = open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (fd < 0) return -1;
    size_t o = 0;
    while (o < n) {
        const ssize_t w = write(fd, p + o, n - o);
        if (w < 0) { if (errno == EINTR) continue; close(fd); return -1; }
        o += (size_t)w;
    }
    const int rc = fsync(fd);
    close(fd);
    return rc;
}

int kvs_open(const char *dir, kvr_ctx *ctx, kvs_store **out, kvr_error *err, char *msg, size_t msg_cap) {
    if (!dir || !ctx || !out) return KVR_EINVAL;
    *out = nullptr;
    if (err) memset(err, 0, sizeof(*err));
    if (msg && msg_cap) msg[0] = 0;
    struct stat st;
    if (stat(dir, &st) != 0 && mkdir(dir, 0777) != 0 && errno != EEXIST) return KVR_EIO;   // engine.rs:26-28
    size_t n = 0;
    int rc = kvh_discover(dir, nullptr, 0, nullptr, 0, &n);
    if (rc != KVR_OK && rc != KVR_CAPACITY) return rc;
    std::vector<uint64_t> ids(n);
    std::vector<char> pbuf(n * 4200 + 16);
    rc = kvh_discover(dir, ids.data(), n, pbuf.data(), pbuf.size(), &n);
    if (rc != KVR_OK) return rc;
    kvs_store *s = new kvs_store();
    s->dir = dir;
    s->ids = ids;
    s->bytes.resize(n);
    std::vector<std::string> paths(n);
    size_t po = 0;
    for (size_t i = 0; i < n; ++i) { paths[i] = std::string(pbuf.data() + po); po += paths[i].size() + 1; }
    for (size_t i = 0; i < n; ++i) {
        int e = 0;
        if (read_file(paths[i], s->bytes[i], &e) != 0) {
            if (err) { err->kind = KVR_E_OPEN; err->seg_idx = (uint32_t)i; err->aux = (uint64_t)e; }
            if (msg && err) kvr_format_error(err, paths[i].c_str(), msg, msg_cap);
            delete s;
            return KVR_CORRUPTED;
        }
    }
    std::vector<std::string> *pp = &paths;
    rc = build_index(s, ctx, err, msg, msg_cap, pp);
    if (rc != KVR_OK) { delete s; return rc; }
    // engine.rs:59-68: next id = max + 1, create the (empty) active segment for appends
    s->active_id = (n ? ids[n - 1] : 0) + 1;
    const std::string ap = std::string(dir) + "/segment-" + std::to_string(s->active_id) + ".dat";
    const int fd = open(ap.c_str(), O_WRONLY | O_CREAT | O_APPEND, 0644);
    if (fd >= 0) close(fd);
    *out = s;
    return KVR_OK;
}

int kvs_get(const kvs_store *s, const uint8_t *key, size_t klen, const uint8_t **val, size_t *vlen) {
    if (!s) return KVR_EINVAL;
    const KeyRef k{key, (uint32_t)klen, crc32_update(0, key, klen)};
    auto it = s->index.find(k);
    if (it == s->index.end()) return 0;
    if (val) *val = s->bytes[it->second.seg_idx].data() + it->second.val_off;
    if (vlen) *vlen = it->second.len;
    return 1;
}

int kvs_locate(const kvs_store *s, const uint8_t *key, size_t klen, uint64_t *seg_id, uint64_t *val_off, uint64_t *len) {
    if (!s) return KVR_EINVAL;
    const KeyRef k{key, (uint32_t)klen, crc32_update(0, key, klen)};
    auto it = s->index.find(k);
    if (it == s->index.end()) return 0;
    if (seg_id) *seg_id = s->ids[it->second.seg_idx];
    if (val_off) *val_off = it->second.val_off;
    if (len) *len = it->second.len;
    return 1;
}

int kvs_stats_get(const kvs_store *s, kvs_stats *out) {
    if (!s || !out) return KVR_EINVAL;
    out->num_keys = s->index.size();
    uint64_t nseg = 0;   // engine.rs:239-250: entries named segment-*.dat, parse or not
    if (DIR *d = opendir(s->dir.c_str())) {
        while (struct dirent *e = readdir(d)) {
            const size_t n = strlen(e->d_name);
            if (n >= 8 && memcmp(e->d_name, "segment-", 8) == 0 && n >= 4 && memcmp(e->d_name + n - 4, ".dat", 4) == 0 &&
                utf8_valid(reinterpret_cast<const uint8_t *>(e->d_name), n))
                ++nseg;
        }
        closedir(d);
    }
    out->num_segments = nseg;
    out->total_bytes = s->total_bytes;
    out->active_segment_id = s->active_id;
    out->oldest_segment_id = 0;   // engine.rs:257
    return KVR_OK;
}

size_t kvs_num_keys(const kvs_store *s) { return s ? s->index.size() : 0; }

int kvs_compact(kvs_store *s, kvr_ctx *ctx, uint64_t seg_target, kvr_error *err) {
    if (!s || !ctx) return KVR_EINVAL;
    if (err) memset(err, 0, sizeof(*err));
    const size_t n = s->ids.size();
    std::vector<kvr_segment> segs(n);
    uint64_t bytes_in = 0;
    for (size_t i = 0; i < n; ++i) {
        segs[i] = kvr_segment{s->ids[i], s->bytes[i].data(), s->bytes[i].size()};
        bytes_in += s->bytes[i].size();
    }
    // 1. the live records, re-framed into new segments, on the GPU
    std::vector<uint8_t> out(std::max<uint64_t>(bytes_in, 1));
    std::vector<uint64_t> ends(seg_target ? bytes_in / seg_target + 2 : 1);
    uint64_t out_len = 0;
    size_t n_new = 0;
    int rc = KVR_OK;
    if (n) {
        rc = kvr_compact(ctx, segs.data(), n, 0, seg_target, out.data(), out.size(), &out_len, ends.data(),
                         ends.size(), &n_new, err);
        if (rc == KVR_CAPACITY) {
            out.resize(out_len);
            ends.resize(n_new);
            rc = kvr_compact(ctx, segs.data(), n, 0, seg_target, out.data(), out.size(), &out_len, ends.data(),
                             ends.size(), &n_new, err);
        }
        if (rc != KVR_OK) return rc;
    }
    // 2. new files first (ids after the active segment), durable before anything is removed
    std::vector<uint64_t> new_ids(n_new);
    std::vector<std::vector<uint8_t>> new_bytes(n_new);
    std::vector<std::string> new_names(n_new);
    uint64_t prev = 0;
    for (size_t j = 0; j < n_new; ++j) {
        new_ids[j] = s->active_id + 1 + j;
        new_names[j] = "segment-" + std::to_string(new_ids[j]) + ".dat";
        new_bytes[j].assign(out.begin() + (ptrdiff_t)prev, out.begin() + (ptrdiff_t)ends[j]);
        if (write_file_sync(s->dir + "/" + new_names[j], new_bytes[j].data(), new_bytes[j].size()) != 0) return KVR_EIO;
        prev = ends[j];
    }
    // 3. every other segment-*.dat goes (compaction.rs:11-23; NotFound is not an error)
    if (DIR *d = opendir(s->dir.c_str())) {
        std::vector<std::string> victims;
        while (struct dirent *e = readdir(d)) {
            if (!is_segment_name(e->d_name)) continue;
            if (std::find(new_names.begin(), new_names.end(), std::string(e->d_name)) != new_names.end()) continue;
            victims.push_back(s->dir + "/" + e->d_name);
        }
        closedir(d);
        for (const auto &v : victims)
            if (unlink(v.c_str()) != 0 && errno != ENOENT) return KVR_EIO;
    } else {
        return KVR_EIO;
    }
    // 4. reset_active_segment (engine.rs:209-229): the next id, an empty file
    s->active_id = s->active_id + n_new + 1;
    const std::string ap = s->dir + "/segment-" + std::to_string(s->active_id) + ".dat";
    const int fd = open(ap.c_str(), O_WRONLY | O_CREAT | O_APPEND, 0644);
    if (fd < 0) return KVR_EIO;
    close(fd);
    // 5. the store now reads the new files; the index is rebuilt over them (same map)
    s->ids = new_ids;
    s->bytes = std::move(new_bytes);
    return build_index(s, ctx, err, nullptr, 0, nullptr);
}

void kvs_close(kvs_store *s) { delete s; }

}  // extern "C"
