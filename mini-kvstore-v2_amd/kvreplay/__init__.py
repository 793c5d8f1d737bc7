"""kvreplay — Python bindings over the C ABI (include/kvreplay.h, include/kvstore_host.h).

This mirrors the reference's replay surface (whispem/mini-kvstore-v2):
  KVStore.open(dir)   -> src/store/engine.rs:24   (index rebuild on restart, replay on the GPU)
  KVStore.get(key)    -> engine.rs:200
  KVStore.stats()     -> engine.rs:237-259 (StoreStats, src/store/stats.rs:3-10)
  CorruptedData       -> StoreError::CorruptedData (src/store/error.rs:11-12), same messages
and exposes the engine itself (Context.replay) plus the synthetic generator.

The native libraries are required: importing a function that needs them raises if
lib/libkvreplay.so / lib/libkvhost.so are missing (there is no Python fallback).
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_LIB = os.path.join(_PKG, "lib")

# ---- status / kinds (kvreplay.h) -------------------------------------------------------------
OK, CORRUPTED, CAPACITY = 0, 1, 2
EINVAL, EHIP, EIO, ENOMEM = -1, -2, -3, -4
E_NONE, E_OPEN, E_KEY_LEN, E_KEY, E_UTF8, E_VAL_LEN, E_VAL, E_OPCODE = range(8)
KIND_NAMES = {0: "NONE", 1: "OPEN", 2: "KEY_LEN", 3: "KEY", 4: "UTF8", 5: "VAL_LEN", 6: "VAL", 7: "OPCODE"}
SEGS_ON_DEVICE, OUT_ON_DEVICE, EXPECTED_ON_DEVICE, HOST_PINNED = 0x1, 0x2, 0x4, 0x8
TF_VERIFIED, TF_CRC_FAIL = 0x1, 0x2

TUPLE_DTYPE = np.dtype([("rec_off", "<u8"), ("seg_idx", "<u4"), ("key_len", "<u4"), ("val_len", "<u4"),
                        ("crc32", "<u4"), ("key_tag", "<u4"), ("op", "u1"), ("flags", "u1"),
                        ("reserved", "<u2")])
assert TUPLE_DTYPE.itemsize == 32


class Segment(C.Structure):
    _fields_ = [("seg_id", C.c_uint64), ("bytes", C.c_void_p), ("len", C.c_uint64)]


class Error(C.Structure):
    _fields_ = [("kind", C.c_int32), ("seg_idx", C.c_uint32), ("rec_off", C.c_uint64), ("aux", C.c_uint64)]


class Stats(C.Structure):
    _fields_ = [("ms_total", C.c_double), ("ms_replay", C.c_double), ("ms_link", C.c_double),
                ("ms_compact", C.c_double), ("bytes_in", C.c_uint64), ("n_records", C.c_uint64),
                ("n_crc_fail", C.c_uint64), ("n_stripes", C.c_uint32), ("n_tiles", C.c_uint32),
                ("n_redo", C.c_uint32), ("n_link_passes", C.c_uint32)]


class StreamStats(C.Structure):
    _fields_ = [("ms_wall", C.c_double), ("ms_device", C.c_double), ("bytes_in", C.c_uint64),
                ("n_records", C.c_uint64), ("n_batches", C.c_uint64)]


class MultiStats(C.Structure):
    _fields_ = [("ms_wall", C.c_double), ("ms_device_max", C.c_double), ("bytes_in", C.c_uint64),
                ("n_records", C.c_uint64), ("n_crc_fail", C.c_uint64), ("n_shards", C.c_uint32),
                ("pad", C.c_uint32)]


class EtagStats(C.Structure):
    _fields_ = [("ms_chunk", C.c_double), ("ms_join", C.c_double), ("bytes", C.c_uint64),
                ("n_blobs", C.c_uint64), ("n_chunks", C.c_uint64), ("n_fail", C.c_uint64)]


class GenParams(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("seg_bytes", C.c_uint64), ("key_space_log2", C.c_uint32),
                ("key_dist", C.c_uint32), ("val_min", C.c_uint32), ("val_max", C.c_uint32),
                ("del_permille", C.c_uint32), ("flip_per_million", C.c_uint32)]


class StoreStats(C.Structure):
    _fields_ = [("num_keys", C.c_uint64), ("num_segments", C.c_uint64), ("total_bytes", C.c_uint64),
                ("active_segment_id", C.c_uint64), ("oldest_segment_id", C.c_uint64)]


CAND_BYTES = 24   # sizeof(kvr_cand)


class CompactStats(C.Structure):
    _fields_ = [("ms_replay", C.c_double), ("ms_fold", C.c_double), ("ms_gather", C.c_double),
                ("n_tuples", C.c_uint64), ("n_live", C.c_uint64), ("bytes_in", C.c_uint64),
                ("bytes_out", C.c_uint64)]


class IndexStats(C.Structure):
    _fields_ = [("ms_wall", C.c_double), ("ms_replay", C.c_double), ("ms_fold", C.c_double),
                ("bytes_in", C.c_uint64), ("n_tuples", C.c_uint64), ("n_live", C.c_uint64),
                ("n_slots", C.c_uint64), ("fold_rounds", C.c_uint32), ("fold_redo", C.c_uint32),
                ("fold_est", C.c_uint64), ("fold_slots", C.c_uint64)]


class OpenStats(C.Structure):
    _fields_ = [("ms_total", C.c_double), ("ms_register", C.c_double), ("ms_push", C.c_double),
                ("ms_read", C.c_double),
                ("ms_index", C.c_double), ("bytes", C.c_uint64), ("n_segments", C.c_uint64),
                ("n_live", C.c_uint64), ("path", C.c_uint32), ("read_threads", C.c_uint32),
                ("mode", C.c_uint32), ("pad", C.c_uint32)]


OPEN_HOST_FOLD, OPEN_NO_PIN, OPEN_PREAD = 0x1, 0x2, 0x4
LOAD_MMAP, LOAD_PREAD = 1, 2
PATH_DEVICE_INDEX, PATH_HOST_FOLD = 1, 2


# ---- library loading ---------------------------------------------------------------------------
_rep = None
_host = None


def lib_paths():
    # KVREPLAY_VARIANT: a diagnostic build pair under lib/vpair (build.py build_variant_pair),
    # timing tools only
    v = os.environ.get("KVREPLAY_VARIANT")
    d = os.path.join(_LIB, "vpair", v) if v else _LIB
    return os.path.join(d, "libkvreplay.so"), os.path.join(d, "libkvhost.so")


def _load():
    global _rep, _host
    if _rep is not None:
        return _rep, _host
    rp, hp = lib_paths()
    if not (os.path.exists(rp) and os.path.exists(hp)):
        raise RuntimeError(f"kvreplay native libraries missing ({rp}); run __graft_entry__.build()")
    rep = C.CDLL(rp, mode=C.RTLD_GLOBAL)
    host = C.CDLL(hp)
    P, U64, U32, SZ, I = C.c_void_p, C.c_uint64, C.c_uint32, C.c_size_t, C.c_int
    rep.kvr_ctx_create.argtypes = [I, C.POINTER(P)]
    rep.kvr_ctx_destroy.argtypes = [P]
    rep.kvr_ctx_destroy.restype = None
    rep.kvr_ctx_set_stream.argtypes = [P, P]
    rep.kvr_ctx_device.argtypes = [P]
    rep.kvr_ctx_set_tiles_per_stripe.argtypes = [P, U32]
    rep.kvr_replay.argtypes = [P, C.POINTER(Segment), SZ, U32, P, SZ, P, SZ, C.POINTER(SZ), C.POINTER(Error)]
    rep.kvr_last_stats.argtypes = [P, C.POINTER(Stats)]
    rep.kvr_mctx_create.argtypes = [P, I, C.POINTER(P)]
    rep.kvr_mctx_destroy.argtypes = [P]
    rep.kvr_mctx_destroy.restype = None
    rep.kvr_mctx_size.argtypes = [P]
    rep.kvr_replay_multi.argtypes = [P, C.POINTER(Segment), SZ, U32, P, SZ, P, SZ, C.POINTER(SZ), C.POINTER(Error)]
    rep.kvr_replay_live_multi.argtypes = [P, C.POINTER(Segment), SZ, U32, P, SZ, C.POINTER(SZ), C.POINTER(Error)]
    rep.kvr_multi_live_keys.argtypes = [P, P, U64, P, SZ, C.POINTER(U64)]
    rep.kvr_replay_last.argtypes = [P, C.POINTER(Segment), SZ, U32, P, SZ, C.POINTER(SZ), C.POINTER(Error)]
    rep.kvr_last_multi_stats.argtypes = [P, C.POINTER(MultiStats)]
    rep.kvr_replay_stream.argtypes = [P, C.POINTER(Segment), SZ, U32, U64, P, SZ, P, SZ, C.POINTER(SZ),
                                      C.POINTER(Error)]
    rep.kvr_replay_live.argtypes = [P, C.POINTER(Segment), SZ, U32, P, SZ, C.POINTER(SZ), C.POINTER(Error)]
    rep.kvr_last_stream_stats.argtypes = [P, C.POINTER(StreamStats)]
    rep.kvr_replay_index.argtypes = [P, C.POINTER(Segment), SZ, U32, P, SZ, P, U64, C.POINTER(SZ), C.POINTER(U64),
                                     C.POINTER(Error)]
    rep.kvr_index_fetch.argtypes = [P, U32, P, SZ, P, U64]
    rep.kvr_live_keys.argtypes = [P, U32, P, U64, P, SZ, C.POINTER(U64)]
    rep.kvr_last_index_stats.argtypes = [P, C.POINTER(IndexStats)]
    rep.kvr_index_slots.argtypes = [U64]
    rep.kvr_index_slots.restype = U64
    rep.kvr_index_hash.argtypes = [U32]
    rep.kvr_index_hash.restype = U32
    rep.kvr_index_find.argtypes = [P, P, U64, C.POINTER(Segment), P, SZ]
    rep.kvr_index_find.restype = C.c_int64
    rep.kvr_index_build_host.argtypes = [P, SZ, P, U64]
    rep.kvr_ingest_begin.argtypes = [P, U64, SZ]
    rep.kvr_ingest_push.argtypes = [P, U64, P, U64]
    rep.kvr_ingest_index.argtypes = [P, U32, P, SZ, P, U64, C.POINTER(SZ), C.POINTER(U64), C.POINTER(Error)]
    rep.kvr_host_alloc.argtypes = [U64, C.POINTER(P)]
    rep.kvr_host_free.argtypes = [P]
    rep.kvr_host_free.restype = None
    rep.kvr_host_register.argtypes = [P, U64]
    rep.kvr_host_unregister.argtypes = [P]
    rep.kvr_host_unregister.restype = None
    rep.kvr_etag_batch.argtypes = [P, P, U64, P, P, SZ, U32, P, P, C.POINTER(U64)]
    rep.kvr_last_etag_stats.argtypes = [P, C.POINTER(EtagStats)]
    rep.kvr_etag_format.argtypes = [U32, C.c_char_p]
    rep.kvr_etag_format.restype = None
    rep.kvr_compact.argtypes = [P, C.POINTER(Segment), SZ, U32, U64, P, U64, C.POINTER(U64), P, SZ, C.POINTER(SZ),
                                C.POINTER(Error)]
    rep.kvr_last_compact_stats.argtypes = [P, C.POINTER(CompactStats)]
    rep.kvr_compact_stage.argtypes = [P, C.POINTER(Segment), SZ, U32, P, U32, P, P, C.POINTER(Error)]
    rep.kvr_compact_export.argtypes = [P, P, P]
    rep.kvr_compact_resolve.argtypes = [P, P, P, P, P, U32, P]
    rep.kvr_compact_finish.argtypes = [P, P, U32, U64, P, U64, C.POINTER(U64), P, SZ, C.POINTER(SZ)]
    rep.kvr_strerror.argtypes = [I]
    rep.kvr_strerror.restype = C.c_char_p
    rep.kvr_crc32.argtypes = [U32, P, SZ]
    rep.kvr_crc32.restype = U32
    rep.kvr_format_error.argtypes = [C.POINTER(Error), C.c_char_p, C.c_char_p, SZ]
    rep.kvr_gen_segment_device.argtypes = [P, C.POINTER(GenParams), U64, P, U64, C.POINTER(U64), P, U64,
                                           C.POINTER(U64)]
    host.kvh_gen_segment.argtypes = [C.POINTER(GenParams), U64, P, U64, C.POINTER(U64), P, U64, C.POINTER(U64)]
    host.kvh_discover.argtypes = [C.c_char_p, P, SZ, P, SZ, C.POINTER(SZ)]
    host.kvh_parse_u64.argtypes = [C.c_char_p, SZ, C.POINTER(U64)]
    host.kvh_fold.argtypes = [C.POINTER(Segment), P, SZ, P, C.POINTER(U64)]
    host.kvh_fold.restype = U64
    host.kvh_fold_parallel.argtypes = [C.POINTER(Segment), P, SZ, U32, P, C.POINTER(U64)]
    host.kvh_fold_parallel.restype = U64
    host.kvs_open.argtypes = [C.c_char_p, P, C.POINTER(P), C.POINTER(Error), C.c_char_p, SZ]
    host.kvs_open_ex.argtypes = [C.c_char_p, P, U32, C.POINTER(P), C.POINTER(Error), C.c_char_p, SZ]
    host.kvs_last_open_stats.argtypes = [P, C.POINTER(OpenStats)]
    host.kvs_get.argtypes = [P, P, SZ, C.POINTER(P), C.POINTER(SZ)]
    host.kvs_locate.argtypes = [P, P, SZ, C.POINTER(U64), C.POINTER(U64), C.POINTER(U64)]
    host.kvs_stats_get.argtypes = [P, C.POINTER(StoreStats)]
    host.kvs_num_keys.argtypes = [P]
    host.kvs_num_keys.restype = SZ
    host.kvs_compact.argtypes = [P, P, U64, C.POINTER(Error)]
    host.kvs_close.argtypes = [P]
    host.kvs_close.restype = None
    _rep, _host = rep, host
    return rep, host


def native():
    """(libkvreplay, libkvhost) ctypes handles; raises if they are not built."""
    return _load()


# ---- errors ------------------------------------------------------------------------------------
class CorruptedData(Exception):
    """StoreError::CorruptedData (src/store/error.rs:11-12)."""

    def __init__(self, kind, seg_idx, rec_off, aux, message=""):
        self.kind, self.seg_idx, self.rec_off, self.aux = kind, seg_idx, rec_off, aux
        self.message = message
        super().__init__(f"Corrupted data: {message}" if message else
                         f"Corrupted data: {KIND_NAMES.get(kind, kind)} in segment #{seg_idx} at {rec_off}")


class NativeError(RuntimeError):
    pass


def format_error(kind, seg_idx, rec_off, aux, path):
    rep, _ = _load()
    e = Error(kind, seg_idx, rec_off, aux)
    buf = C.create_string_buffer(8192)
    rep.kvr_format_error(C.byref(e), path.encode(), buf, len(buf))
    return buf.value.decode()


def crc32(data: bytes, crc: int = 0) -> int:
    rep, _ = _load()
    a = np.frombuffer(bytes(data), dtype=np.uint8)
    return int(rep.kvr_crc32(crc, a.ctypes.data if a.size else None, a.size))


def etag_format(crc: int) -> str:
    """The ETag text BlobStorage::put returns: format!("{:08x}", crc) (storage.rs:27)."""
    rep, _ = _load()
    buf = C.create_string_buffer(9)
    rep.kvr_etag_format(crc, buf)
    return buf.value.decode()


# ---- generator ---------------------------------------------------------------------------------
@dataclass
class GenSpec:
    seed: int = 0x6B767265706C6179
    seg_bytes: int = 64 << 20
    key_space_log2: int = 20
    key_dist: int = 0
    val_min: int = 1024
    val_max: int = 1024
    del_permille: int = 0
    flip_per_million: int = 0

    def c(self):
        return GenParams(self.seed, self.seg_bytes, self.key_space_log2, self.key_dist, self.val_min,
                         self.val_max, self.del_permille, self.flip_per_million)


def gen_segment_cpu(spec: GenSpec, seg_no: int):
    """(bytes as uint8 ndarray, manifest uint32 ndarray) — byte-identical to the device generator."""
    _, host = _load()
    p = spec.c()
    ln, nr = C.c_uint64(), C.c_uint64()
    rc = host.kvh_gen_segment(C.byref(p), seg_no, None, 0, C.byref(ln), None, 0, C.byref(nr))
    if rc != OK:
        raise NativeError(rc)
    buf = np.zeros(max(ln.value, 1), dtype=np.uint8)
    exp = np.zeros(max(nr.value, 1), dtype=np.uint32)
    rc = host.kvh_gen_segment(C.byref(p), seg_no, buf.ctypes.data, buf.size, C.byref(ln), exp.ctypes.data,
                              exp.size, C.byref(nr))
    if rc != OK:
        raise NativeError(rc)
    return buf[:ln.value], exp[:nr.value]


def parse_u64(s: str):
    _, host = _load()
    b = s.encode()
    out = C.c_uint64()
    return int(out.value) if host.kvh_parse_u64(b, len(b), C.byref(out)) else None


def discover(dirpath: str):
    _, host = _load()
    n = C.c_size_t()
    host.kvh_discover(dirpath.encode(), None, 0, None, 0, C.byref(n))
    ids = np.zeros(max(n.value, 1), dtype=np.uint64)
    pbuf = C.create_string_buffer(max(n.value, 1) * 4200)
    rc = host.kvh_discover(dirpath.encode(), ids.ctypes.data, ids.size, pbuf, len(pbuf), C.byref(n))
    if rc != OK:
        raise NativeError(rc)
    paths = pbuf.raw.split(b"\0")[: n.value]
    return [(int(ids[i]), paths[i].decode()) for i in range(n.value)]


def fold(segments, tuples, threads=None, pinned=False):
    """Native last-writer-wins fold: (live mask, num_keys, total_bytes).  threads=None runs
    kvh_fold (one thread), else kvh_fold_parallel on that many threads (0 = all cores).
    segments are bytes / uint8 arrays, or (ptr, len) host pairs with pinned=True."""
    _, host = _load()
    if pinned:
        segs = (Segment * max(len(segments), 1))(*[Segment(i, p, ln) for i, (p, ln) in enumerate(segments)])
        t = np.ascontiguousarray(tuples, dtype=TUPLE_DTYPE)
        live = np.zeros(max(len(t), 1), dtype=np.uint8)
        tb = C.c_uint64()
        nk = host.kvh_fold_parallel(segs, t.ctypes.data if len(t) else None, len(t), threads or 0,
                                    live.ctypes.data, C.byref(tb))
        return live[: len(t)].astype(bool), int(nk), int(tb.value)
    arrs = [np.ascontiguousarray(np.frombuffer(s, dtype=np.uint8) if isinstance(s, (bytes, bytearray)) else s)
            for s in segments]
    segs = (Segment * max(len(arrs), 1))(*[Segment(i, a.ctypes.data if a.size else None, a.size)
                                            for i, a in enumerate(arrs)])
    t = np.ascontiguousarray(tuples, dtype=TUPLE_DTYPE)
    live = np.zeros(max(len(t), 1), dtype=np.uint8)
    tb = C.c_uint64()
    if threads is None:
        nk = host.kvh_fold(segs, t.ctypes.data if len(t) else None, len(t), live.ctypes.data, C.byref(tb))
    else:
        nk = host.kvh_fold_parallel(segs, t.ctypes.data if len(t) else None, len(t), threads, live.ctypes.data,
                                    C.byref(tb))
    return live[: len(t)].astype(bool), int(nk), int(tb.value)


# ---- the engine --------------------------------------------------------------------------------
@dataclass
class ReplayResult:
    status: int
    tuples: np.ndarray | None
    n: int
    error: Error | None
    stats: Stats


class CompactResult:
    def __init__(self, status, data, seg_ends, out_len, n_segs, error, stats):
        self.status, self.data, self.seg_ends, self.out_len, self.n_segs = status, data, seg_ends, out_len, n_segs
        self.error, self.stats = error, stats

    def segments(self):
        """The new segment files' bytes (host output)."""
        out, s = [], 0
        for e in self.seg_ends:
            out.append(self.data[s:e])
            s = e
        return out


class MultiContext:
    """kvr_mctx: one context per entry of devices (ids may repeat), segments dealt round-robin,
    shards replayed concurrently on host threads, merged on the host (kvr_replay_multi)."""

    def __init__(self, devices):
        rep, _ = _load()
        self._rep = rep
        d = (C.c_int * len(devices))(*devices)
        h = C.c_void_p()
        rc = rep.kvr_mctx_create(d, len(devices), C.byref(h))
        if rc != OK:
            raise NativeError(f"kvr_mctx_create({list(devices)}) failed: {rep.kvr_strerror(rc).decode()} ({rc})")
        self.h, self.devices = h, list(devices)

    def close(self):
        if getattr(self, "h", None):
            self._rep.kvr_mctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def last_stats(self) -> MultiStats:
        s = MultiStats()
        self._rep.kvr_last_multi_stats(self.h, C.byref(s))
        return s

    def replay(self, segments, seg_ids=None, expected=None, cap=None, live=False, on_device=False):
        """Same contract as Context.replay; returns ReplayResult (stats: MultiStats).
        live=True: kvr_replay_live_multi (each GPU reduces its shard to every key's last record,
        tombstones included; the host keeps the live keys' final SETs).  on_device: segments are
        (ptr, len) pairs, segment i resident on the device of context i mod N."""
        keep = []
        n = len(segments)
        segs = (Segment * max(n, 1))()
        total = 0
        for i, s in enumerate(segments):
            sid = seg_ids[i] if seg_ids is not None else i
            if on_device:
                ptr, ln = s
            else:
                a = np.frombuffer(s, dtype=np.uint8) if isinstance(s, (bytes, bytearray)) else np.ascontiguousarray(s)
                keep.append(a)
                ptr, ln = (a.ctypes.data if a.size else None), a.size
            segs[i] = Segment(sid, ptr, ln)
            total += ln
        exp_ptr, n_exp = None, 0
        if expected is not None:
            e = np.ascontiguousarray(expected, dtype=np.uint32)
            keep.append(e)
            exp_ptr, n_exp = (e.ctypes.data if e.size else None), e.size
        if cap is None:
            cap = max(1024, total // 24 + n)
        out_arr = np.zeros(max(cap, 1), dtype=TUPLE_DTYPE)
        n_out = C.c_size_t()
        err = Error()
        fl = SEGS_ON_DEVICE if on_device else 0
        if live:
            rc = self._rep.kvr_replay_live_multi(self.h, segs, n, fl, out_arr.ctypes.data, cap, C.byref(n_out),
                                                 C.byref(err))
        else:
            rc = self._rep.kvr_replay_multi(self.h, segs, n, fl, exp_ptr, n_exp, out_arr.ctypes.data, cap,
                                            C.byref(n_out), C.byref(err))
        if rc == CAPACITY:
            return self.replay(segments, seg_ids, expected, cap=n_out.value + 16, live=live, on_device=on_device)
        if rc < 0:
            raise NativeError(f"kvr_replay_multi: {self._rep.kvr_strerror(rc).decode()} ({rc})")
        tuples = out_arr[: n_out.value] if rc == OK else None
        return ReplayResult(rc, tuples, n_out.value, err if rc == CORRUPTED else None, self.last_stats())

    def live_keys(self, n_live):
        """Key bytes of the last replay(live=True) output of n_live tuples (kvr_multi_live_keys)
        -> (packed key bytes uint8 array, offsets: n_live + 1 uint64)."""
        kb = C.c_uint64()
        offs = np.zeros(n_live + 1, dtype=np.uint64)
        rc = self._rep.kvr_multi_live_keys(self.h, None, 0, offs.ctypes.data, offs.size, C.byref(kb))
        if rc not in (OK, CAPACITY):
            raise NativeError(f"kvr_multi_live_keys: {rc}")
        keys = np.zeros(max(kb.value, 1), dtype=np.uint8)
        rc = self._rep.kvr_multi_live_keys(self.h, keys.ctypes.data, keys.size, offs.ctypes.data, offs.size,
                                           C.byref(kb))
        if rc != OK:
            raise NativeError(f"kvr_multi_live_keys: {rc}")
        return keys[: kb.value], offs


class SegmentList:
    """A segment list marshaled once into the kvr_segment array of the C ABI, for callers that
    replay the same segments repeatedly (Context.replay accepts it in place of a list; the
    segment bytes must stay alive and unchanged).  on_device: (ptr, len) pairs in HBM."""

    def __init__(self, segments, seg_ids=None, on_device=False):
        self.n = len(segments)
        self.on_device = on_device
        self.keep = []
        self.arr = (Segment * max(self.n, 1))()
        self.total = 0
        for i, s in enumerate(segments):
            sid = seg_ids[i] if seg_ids is not None else i
            if on_device:
                ptr, ln = s
            else:
                a = np.frombuffer(s, dtype=np.uint8) if isinstance(s, (bytes, bytearray)) else np.ascontiguousarray(s)
                self.keep.append(a)
                ptr, ln = (a.ctypes.data if a.size else None), a.size
            self.arr[i] = Segment(sid, ptr, ln)
            self.total += ln

    def __len__(self):
        return self.n


class Context:
    """One kvr_ctx on one HIP device."""

    def __init__(self, device: int = 0):
        rep, _ = _load()
        self._rep = rep
        h = C.c_void_p()
        rc = rep.kvr_ctx_create(device, C.byref(h))
        if rc != OK:
            raise NativeError(f"kvr_ctx_create({device}) failed: {rep.kvr_strerror(rc).decode()} ({rc})")
        self.h = h
        self.device = device

    def close(self):
        if getattr(self, "h", None):
            self._rep.kvr_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_tiles_per_stripe(self, tiles: int):
        self._rep.kvr_ctx_set_tiles_per_stripe(self.h, tiles)

    def set_stream(self, stream_ptr: int | None):
        self._rep.kvr_ctx_set_stream(self.h, stream_ptr)

    def last_stats(self) -> Stats:
        s = Stats()
        self._rep.kvr_last_stats(self.h, C.byref(s))
        return s

    def replay(self, segments, seg_ids=None, expected=None, cap=None, on_device=False, out_ptr=None,
               expected_on_device=False):
        """Replay host segments (list of bytes / uint8 arrays), or device segments given as
        (ptr, len) pairs with on_device=True.  Returns ReplayResult; tuples is a numpy
        TUPLE_DTYPE array unless out_ptr (device memory) is given.  segments may be a
        SegmentList (marshaled once; its on_device flag applies)."""
        if not isinstance(segments, SegmentList):
            segments = SegmentList(segments, seg_ids, on_device)
        n, segs, total, on_device = segments.n, segments.arr, segments.total, segments.on_device
        keep = [segments]
        flags = (SEGS_ON_DEVICE if on_device else 0)
        exp_ptr, n_exp = None, 0
        if expected is not None:
            if expected_on_device:
                exp_ptr, n_exp = expected
                flags |= EXPECTED_ON_DEVICE
            else:
                e = np.ascontiguousarray(expected, dtype=np.uint32)
                keep.append(e)
                exp_ptr, n_exp = (e.ctypes.data if e.size else None), e.size
        if cap is None:
            cap = max(1024, total // 24 + n)
        out_arr = None
        if out_ptr is not None:
            flags |= OUT_ON_DEVICE
            outp = out_ptr
        else:
            out_arr = np.zeros(cap, dtype=TUPLE_DTYPE)
            outp = out_arr.ctypes.data
        n_out = C.c_size_t()
        err = Error()
        rc = self._rep.kvr_replay(self.h, segs, n, flags, exp_ptr, n_exp, outp, cap, C.byref(n_out), C.byref(err))
        if rc == CAPACITY and out_ptr is None:
            return self.replay(segments, seg_ids, expected, cap=n_out.value + 16, on_device=on_device,
                               expected_on_device=expected_on_device)
        if rc < 0:
            raise NativeError(f"kvr_replay: {self._rep.kvr_strerror(rc).decode()} ({rc})")
        tuples = out_arr[: n_out.value] if out_arr is not None and rc == OK else None
        return ReplayResult(rc, tuples, n_out.value, err if rc == CORRUPTED else None, self.last_stats())

    def replay_stream(self, segments, seg_ids=None, expected=None, cap=None, batch_bytes=0, pinned=False):
        """Streamed ingest (kvr_replay_stream): host segments go to HBM in batches of batch_bytes
        on a copy stream, overlapping the replay of the previous batch.  segments are bytes /
        uint8 arrays, or (ptr, len) pairs of pinned host memory with pinned=True.  Returns
        ReplayResult with the same tuples and errors as replay() on the same segments; the
        streaming statistics are in .stream_stats."""
        segs, keep, total = self._segments(segments, seg_ids, pinned)
        flags = HOST_PINNED if pinned else 0
        exp_ptr, n_exp = None, 0
        if expected is not None:
            e = np.ascontiguousarray(expected, dtype=np.uint32)
            keep.append(e)
            exp_ptr, n_exp = (e.ctypes.data if e.size else None), e.size
        if cap is None:
            cap = max(1024, total // 24 + len(segments))
        out_arr = np.zeros(max(cap, 1), dtype=TUPLE_DTYPE)
        n_out = C.c_size_t()
        err = Error()
        rc = self._rep.kvr_replay_stream(self.h, segs, len(segments), flags, batch_bytes, exp_ptr, n_exp,
                                         out_arr.ctypes.data, cap, C.byref(n_out), C.byref(err))
        if rc == CAPACITY:
            return self.replay_stream(segments, seg_ids, expected, cap=n_out.value + 16, batch_bytes=batch_bytes,
                                      pinned=pinned)
        if rc < 0:
            raise NativeError(f"kvr_replay_stream: {self._rep.kvr_strerror(rc).decode()} ({rc})")
        ss = StreamStats()
        self._rep.kvr_last_stream_stats(self.h, C.byref(ss))
        tuples = out_arr[: n_out.value] if rc == OK else None
        r = ReplayResult(rc, tuples, n_out.value, err if rc == CORRUPTED else None, self.last_stats())
        r.stream_stats = ss
        return r

    def replay_live(self, segments, seg_ids=None, on_device=False, out_ptr=None, cap=None):
        """Replay + last-writer fold on the device (kvr_replay_live): only the live keys' final
        SET tuples, in (segment, offset) order.  Returns ReplayResult (tuples None with out_ptr)."""
        segs, keep, total = self._segments(segments, seg_ids, on_device)
        if cap is None:
            cap = max(1024, total // 24 + len(segments))
        flags = SEGS_ON_DEVICE if on_device else 0
        out_arr = None
        if out_ptr is not None:
            flags |= OUT_ON_DEVICE
            outp = out_ptr
        else:
            out_arr = np.zeros(max(cap, 1), dtype=TUPLE_DTYPE)
            outp = out_arr.ctypes.data
        n_out = C.c_size_t()
        err = Error()
        rc = self._rep.kvr_replay_live(self.h, segs, len(segments), flags, outp, cap, C.byref(n_out), C.byref(err))
        if rc == CAPACITY and out_ptr is None:
            return self.replay_live(segments, seg_ids, on_device, None, n_out.value + 16)
        if rc < 0:
            raise NativeError(f"kvr_replay_live: {self._rep.kvr_strerror(rc).decode()} ({rc})")
        tuples = out_arr[: n_out.value] if out_arr is not None and rc == OK else None
        return ReplayResult(rc, tuples, n_out.value, err if rc == CORRUPTED else None, self.last_stats())

    def replay_index(self, segments, seg_ids=None, on_device=False):
        """Replay + fold + key table on the device (kvr_replay_index) -> Index (live tuples in
        (segment, offset) order and the slot table; lookups through Index.find)."""
        segs, keep, total = self._segments(segments, seg_ids, on_device)
        flags = SEGS_ON_DEVICE if on_device else 0
        nl, ns = C.c_size_t(), C.c_uint64()
        err = Error()
        rc = self._rep.kvr_replay_index(self.h, segs, len(segments), flags, None, 0, None, 0, C.byref(nl),
                                        C.byref(ns), C.byref(err))
        if rc == CORRUPTED:
            return ReplayResult(rc, None, 0, err, self.last_stats())
        live = np.zeros(max(nl.value, 1), dtype=TUPLE_DTYPE)
        slots = np.zeros(max(ns.value, 1), dtype=np.uint32)
        if rc == CAPACITY:
            rc = self._rep.kvr_index_fetch(self.h, 0, live.ctypes.data, nl.value, slots.ctypes.data, ns.value)
        if rc != OK:
            raise NativeError(f"kvr_replay_index: {self._rep.kvr_strerror(rc).decode()} ({rc})")
        st = IndexStats()
        self._rep.kvr_last_index_stats(self.h, C.byref(st))
        return Index(live[: nl.value], slots[: ns.value], None if on_device else keep, st)

    def ingest_index(self, segments, seg_ids=None, pinned=False, host_ptrs=False):
        """The open path's device calls: kvr_ingest_begin, one kvr_ingest_push per segment (host
        bytes; pinned=True stages them in kvr_host_alloc memory first; host_ptrs=True: segments
        are (pointer, length) pairs into host memory the caller keeps), kvr_ingest_index."""
        n = len(segments)
        if host_ptrs:
            class _P:   # (pointer, length) with the ndarray attributes used below
                def __init__(self, p, ln):
                    self.size, self.ctypes = ln, type("c", (), {"data": p})()
            arrs = [_P(p, ln) for p, ln in segments]
        else:
            arrs = [np.frombuffer(s, dtype=np.uint8) if isinstance(s, (bytes, bytearray)) else np.ascontiguousarray(s)
                    for s in segments]
        total = sum((a.size + 255) & ~255 for a in arrs)
        host_mem = None
        if pinned and not host_ptrs:
            hp = C.c_void_p()
            if self._rep.kvr_host_alloc(total + 256, C.byref(hp)) != OK:
                raise NativeError("kvr_host_alloc failed")
            host_mem = hp.value
            staged, o = [], 0
            for a in arrs:
                v = np.ctypeslib.as_array((C.c_uint8 * max(a.size, 1)).from_address(host_mem + o))[: a.size]
                v[:] = a
                staged.append(v)
                o += (a.size + 255) & ~255
            arrs = staged
        try:
            rc = self._rep.kvr_ingest_begin(self.h, total, n)
            if rc != OK:
                raise NativeError(f"kvr_ingest_begin: {rc}")
            for i, a in enumerate(arrs):
                sid = seg_ids[i] if seg_ids is not None else i
                rc = self._rep.kvr_ingest_push(self.h, sid, a.ctypes.data if a.size else None, a.size)
                if rc != OK:
                    raise NativeError(f"kvr_ingest_push: {rc}")
            nl, ns = C.c_size_t(), C.c_uint64()
            err = Error()
            rc = self._rep.kvr_ingest_index(self.h, 0, None, 0, None, 0, C.byref(nl), C.byref(ns), C.byref(err))
            if rc == CORRUPTED:
                return ReplayResult(rc, None, 0, err, self.last_stats())
            live = np.zeros(max(nl.value, 1), dtype=TUPLE_DTYPE)
            slots = np.zeros(max(ns.value, 1), dtype=np.uint32)
            if rc == CAPACITY:
                rc = self._rep.kvr_index_fetch(self.h, 0, live.ctypes.data, nl.value, slots.ctypes.data, ns.value)
            if rc != OK:
                raise NativeError(f"kvr_ingest_index: {rc}")
            st = IndexStats()
            self._rep.kvr_last_index_stats(self.h, C.byref(st))
            return Index(live[: nl.value], slots[: ns.value], None if host_ptrs else [np.array(a) for a in arrs], st)
        finally:
            if host_mem:
                self._rep.kvr_host_free(host_mem)

    def live_keys(self, n_live):
        """Key arena of the last replay_live / replay_index / ingest_index (kvr_live_keys), whose
        live list has n_live tuples -> (packed key bytes uint8 array, offsets: n_live + 1 uint64)."""
        kb = C.c_uint64()
        offs = np.zeros(n_live + 1, dtype=np.uint64)
        rc = self._rep.kvr_live_keys(self.h, 0, None, 0, offs.ctypes.data, offs.size, C.byref(kb))
        if rc not in (OK, CAPACITY):
            raise NativeError(f"kvr_live_keys: {rc}")
        keys = np.zeros(max(kb.value, 1), dtype=np.uint8)
        rc = self._rep.kvr_live_keys(self.h, 0, keys.ctypes.data, keys.size, offs.ctypes.data, offs.size, C.byref(kb))
        if rc != OK:
            raise NativeError(f"kvr_live_keys: {rc}")
        return keys[: kb.value], offs

    def etag_batch(self, data, offs, lens, expected=None, on_device=False, data_len=None):
        """Batch ETag (kvr_etag_batch): CRC-32 of data[offs[i]:offs[i]+lens[i]] for every i.
        data is bytes / a uint8 array, or a device pointer with on_device=True (then data_len).
        Returns (crc uint32 array, n_fail, EtagStats)."""
        if on_device:
            dptr, dlen = data, data_len
            keep = None
        else:
            keep = np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray)) else \
                np.ascontiguousarray(data, dtype=np.uint8)
            dptr, dlen = (keep.ctypes.data if keep.size else None), keep.size
        o = np.ascontiguousarray(offs, dtype=np.uint64)
        ln = np.ascontiguousarray(lens, dtype=np.uint64)
        n = len(o)
        out = np.zeros(max(n, 1), dtype=np.uint32)
        ep = None
        if expected is not None:
            e = np.ascontiguousarray(expected, dtype=np.uint32)
            ep = e.ctypes.data
        nf = C.c_uint64()
        rc = self._rep.kvr_etag_batch(self.h, dptr, dlen, o.ctypes.data if n else None, ln.ctypes.data if n else None,
                                      n, SEGS_ON_DEVICE if on_device else 0, ep, out.ctypes.data, C.byref(nf))
        if rc != OK:
            raise NativeError(f"kvr_etag_batch: {self._rep.kvr_strerror(rc).decode()} ({rc})")
        st = EtagStats()
        self._rep.kvr_last_etag_stats(self.h, C.byref(st))
        del keep
        return out[:n], int(nf.value), st

    def _segments(self, segments, seg_ids, on_device):
        keep, n = [], len(segments)
        segs = (Segment * max(n, 1))()
        total = 0
        for i, s in enumerate(segments):
            sid = seg_ids[i] if seg_ids is not None else i
            if on_device:
                ptr, ln = s
            else:
                a = np.frombuffer(s, dtype=np.uint8) if isinstance(s, (bytes, bytearray)) else np.ascontiguousarray(s)
                keep.append(a)
                ptr, ln = (a.ctypes.data if a.size else None), a.size
            segs[i] = Segment(sid, ptr, ln)
            total += ln
        return segs, keep, total

    def compact(self, segments, seg_target=0, seg_ids=None, on_device=False, out_ptr=None, out_cap=0):
        """Live-record rewrite (kvr_compact).  Returns CompactResult: data (bytes, host output)
        unless out_ptr (device memory of out_cap bytes) is given; seg_ends = end offsets of the
        new segments in the output."""
        segs, keep, total = self._segments(segments, seg_ids, on_device)
        flags = SEGS_ON_DEVICE if on_device else 0
        out_arr = None
        if out_ptr is not None:
            flags |= OUT_ON_DEVICE
            outp, cap = out_ptr, out_cap
        else:
            cap = max(total, 1)
            out_arr = np.zeros(cap, dtype=np.uint8)
            outp = out_arr.ctypes.data
        n_ends = (total // seg_target + 2) if seg_target else 1
        ends = np.zeros(n_ends, dtype=np.uint64)
        out_len, n_segs = C.c_uint64(), C.c_size_t()
        err = Error()
        rc = self._rep.kvr_compact(self.h, segs, len(segments), flags, seg_target, outp, cap, C.byref(out_len),
                                   ends.ctypes.data, ends.size, C.byref(n_segs), C.byref(err))
        if rc < 0:
            raise NativeError(f"kvr_compact: {self._rep.kvr_strerror(rc).decode()} ({rc})")
        st = CompactStats()
        self._rep.kvr_last_compact_stats(self.h, C.byref(st))
        data = out_arr[: out_len.value].tobytes() if out_arr is not None and rc == OK else None
        return CompactResult(rc, data, [int(x) for x in ends[: n_segs.value]] if rc == OK else [], out_len.value,
                             n_segs.value, err if rc == CORRUPTED else None, st)

    # ---- sharded compaction (kvreplay.shard.compact_sharded drives these around the exchange) ----
    def compact_stage(self, segments, gidx, n_ranks, on_device=False):
        """Replay + local fold + candidates by owner rank -> (counts[n_ranks], key_bytes[n_ranks])."""
        segs, keep, total = self._segments(segments, None, on_device)
        g = np.ascontiguousarray(gidx, dtype=np.uint32)
        counts = np.zeros(n_ranks, dtype=np.uint64)
        kb = np.zeros(n_ranks, dtype=np.uint64)
        err = Error()
        rc = self._rep.kvr_compact_stage(self.h, segs, len(segments), SEGS_ON_DEVICE if on_device else 0,
                                         g.ctypes.data if g.size else None, n_ranks, counts.ctypes.data,
                                         kb.ctypes.data, C.byref(err))
        if rc == CORRUPTED:
            raise CorruptedData(err.kind, err.seg_idx, err.rec_off, err.aux)
        if rc != OK:
            raise NativeError(f"kvr_compact_stage: {rc}")
        self._stage_total = total
        return counts.astype(np.int64), kb.astype(np.int64)

    def compact_export(self, d_hdr: int, d_keys: int):
        rc = self._rep.kvr_compact_export(self.h, d_hdr, d_keys)
        if rc != OK:
            raise NativeError(f"kvr_compact_export: {rc}")

    def compact_resolve(self, d_hdr: int, d_keys: int, hdr_counts, key_counts, d_win: int):
        hc = np.ascontiguousarray(hdr_counts, dtype=np.uint64)
        kc = np.ascontiguousarray(key_counts, dtype=np.uint64)
        rc = self._rep.kvr_compact_resolve(self.h, d_hdr, d_keys, hc.ctypes.data, kc.ctypes.data, hc.size, d_win)
        if rc != OK:
            raise NativeError(f"kvr_compact_resolve: {rc}")

    def compact_finish(self, d_win: int, seg_target=0):
        """This rank's live records (host bytes) and new-segment ends."""
        cap = max(getattr(self, "_stage_total", 0), 1)
        out = np.zeros(cap, dtype=np.uint8)
        n_ends = (cap // seg_target + 2) if seg_target else 1
        ends = np.zeros(n_ends, dtype=np.uint64)
        ol, ns = C.c_uint64(), C.c_size_t()
        rc = self._rep.kvr_compact_finish(self.h, d_win, 0, seg_target, out.ctypes.data, out.size, C.byref(ol),
                                          ends.ctypes.data, ends.size, C.byref(ns))
        if rc != OK:
            raise NativeError(f"kvr_compact_finish: {rc}")
        return out[: ol.value].tobytes(), [int(x) for x in ends[: ns.value]]

    def gen_segment_device(self, spec: GenSpec, seg_no: int, d_buf: int, cap: int, d_expected=None,
                           exp_cap=0):
        p = spec.c()
        ln, nr = C.c_uint64(), C.c_uint64()
        rc = self._rep.kvr_gen_segment_device(self.h, C.byref(p), seg_no, d_buf, cap, C.byref(ln), d_expected,
                                              exp_cap, C.byref(nr))
        if rc != OK:
            raise NativeError(f"kvr_gen_segment_device: {rc} (len {ln.value}, records {nr.value})")
        return ln.value, nr.value


def gen_segment_size(spec: GenSpec, seg_no: int):
    _, host = _load()
    p = spec.c()
    ln, nr = C.c_uint64(), C.c_uint64()
    host.kvh_gen_segment(C.byref(p), seg_no, None, 0, C.byref(ln), None, 0, C.byref(nr))
    return ln.value, nr.value


class Index:
    """The open-time index (kvr_replay_index): live tuples + the key table over them."""

    def __init__(self, live, slots, segments, stats):
        self.live, self.slots, self.stats = live, slots, stats
        self.status = OK
        self._segs = segments

    def find(self, key, segments=None):
        """Index into live[] of key's final SET, or -1 (kvr_index_find)."""
        rep, _ = _load()
        segs = segments if segments is not None else self._segs
        arrs = [np.frombuffer(s, dtype=np.uint8) if isinstance(s, (bytes, bytearray)) else np.ascontiguousarray(s)
                for s in segs]
        cs = (Segment * max(len(arrs), 1))(*[Segment(i, a.ctypes.data if a.size else None, a.size)
                                             for i, a in enumerate(arrs)])
        kb = key.encode() if isinstance(key, str) else bytes(key)
        k = np.frombuffer(kb, dtype=np.uint8)
        if len(self.live) == 0:
            return -1
        return int(rep.kvr_index_find(self.live.ctypes.data, self.slots.ctypes.data, len(self.slots), cs,
                                      k.ctypes.data if k.size else None, k.size))


def index_build_host(live):
    """kvr_index_build_host: the device table's layout built on the host from a live list."""
    rep, _ = _load()
    live = np.ascontiguousarray(live, dtype=TUPLE_DTYPE)
    ns = int(rep.kvr_index_slots(len(live)))
    slots = np.zeros(ns, dtype=np.uint32)
    rc = rep.kvr_index_build_host(live.ctypes.data if len(live) else None, len(live), slots.ctypes.data, ns)
    if rc != OK:
        raise NativeError(f"kvr_index_build_host: {rc}")
    return slots


def index_hash(tag):
    rep, _ = _load()
    return int(rep.kvr_index_hash(tag))


# ---- KVStore mirror ----------------------------------------------------------------------------
class KVStore:
    """The reference's KVStore::open / get / stats path with replay on the GPU."""

    def __init__(self, handle, ctx):
        self._h = handle
        self._ctx = ctx
        _, self._host = _load()

    @classmethod
    def open(cls, dirpath: str, ctx: Context | None = None, flags: int = 0):
        """flags: OPEN_HOST_FOLD (the batch path with the host fold), OPEN_NO_PIN (kvs_open_ex)."""
        _, host = _load()
        ctx = ctx or Context(0)
        h = C.c_void_p()
        err = Error()
        msg = C.create_string_buffer(8192)
        rc = host.kvs_open_ex(str(dirpath).encode(), ctx.h, flags, C.byref(h), C.byref(err), msg, len(msg))
        if rc == CORRUPTED:
            raise CorruptedData(err.kind, err.seg_idx, err.rec_off, err.aux, msg.value.decode())
        if rc != OK:
            raise NativeError(f"kvs_open: {rc}")
        return cls(h, ctx)

    def get(self, key):
        kb = key.encode() if isinstance(key, str) else bytes(key)
        a = np.frombuffer(kb, dtype=np.uint8)
        vp, vl = C.c_void_p(), C.c_size_t()
        found = self._host.kvs_get(self._h, a.ctypes.data if a.size else None, a.size, C.byref(vp), C.byref(vl))
        if not found:
            return None
        return C.string_at(vp.value, vl.value) if vl.value else b""

    def locate(self, key):
        kb = key.encode() if isinstance(key, str) else bytes(key)
        a = np.frombuffer(kb, dtype=np.uint8)
        sid, off, ln = C.c_uint64(), C.c_uint64(), C.c_uint64()
        if not self._host.kvs_locate(self._h, a.ctypes.data if a.size else None, a.size, C.byref(sid),
                                     C.byref(off), C.byref(ln)):
            return None
        return int(sid.value), int(off.value), int(ln.value)

    def stats(self):
        s = StoreStats()
        self._host.kvs_stats_get(self._h, C.byref(s))
        return s

    def open_stats(self):
        s = OpenStats()
        self._host.kvs_last_open_stats(self._h, C.byref(s))
        return s

    def compact(self, seg_target: int = 0):
        """KVStore::compact with the intended semantics (README.md:283-287): live records are
        rewritten into new segment files, the old ones removed, the index rebuilt over them."""
        err = Error()
        rc = self._host.kvs_compact(self._h, self._ctx.h, seg_target, C.byref(err))
        if rc == CORRUPTED:
            raise CorruptedData(err.kind, err.seg_idx, err.rec_off, err.aux)
        if rc != OK:
            raise NativeError(f"kvs_compact: {rc}")

    def close(self):
        if self._h:
            self._host.kvs_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
