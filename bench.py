"""bench.py — device-resident segment replay + CRC32 verification on MI355X.

Workload (BASELINE.json configs[1], the metric's 1-GPU configuration): per GPU, 64 synthetic
segments of 64 MiB with 1 KiB values (uniform keys over 2^20, no deletes), generated directly
into HBM by the device generator (byte-identical to the CPU generator), plus the manifest of
expected CRCs.  One step = one kvr_replay over all of the rank's segments: parse + CRC32 +
verify + ordered tuples left in HBM.  Weak scaling: rank r replays its own 64 segments
(segments shard by construction, no collective on the data path; torch.distributed is used
only for the barrier and the max-over-ranks timing).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg2|cfg3|cfg4|cfg5]
                                     --gpus N > 1 without WORLD_SIZE in the environment: the parent
                                     (which never touches a GPU) launches N ranks with
                                     torch.distributed.run and exits with their status; under a
                                     launcher WORLD_SIZE must equal N
  python bench.py --dry-run          the same launch / barrier / max-over-ranks path on CPU (gloo), a
                                     sleep standing in for the replay (tests/test_bench_launch.py)
  python bench.py --mode etag        batch ETag compute/verify in cfg3's volume-server
                                     shape: 131072 blobs of 64 KiB (8 GiB) resident in HBM, one step =
                                     one kvr_etag_batch (CRC-32 per blob + verify against stored ETags)
  python bench.py --mode compact     the compaction live-record rewrite on
                                     cfg4's per-GPU shard (50 % DEL): one step = one kvr_compact
                                     (replay + last-writer fold + gather of the live records into
                                     new segments), input and output resident in HBM; 1 GPU
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mini-kvstore-v2_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

METRIC = "device-resident segment-replay GiB/s + CRC32-verified records/s, 1/2/4/8 GPU"
PEAK_HBM_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
CONFIGS = {
    # name: (segments per GPU, segment bytes, spec kwargs, description)
    "cfg2": (64, 64 << 20, dict(val_min=1024, val_max=1024, key_space_log2=20),
             "{n} x 64 MiB segments, 1 KiB values, uniform keys over 2^20, 0% DEL"),
    "cfg3": (8, 1 << 30, dict(val_min=65536, val_max=65536, key_space_log2=20),
             "{n} x 1 GiB segments, 64 KiB values (volume-server blob shape)"),
    "cfg4": (64, 64 << 20, dict(val_min=1024, val_max=1024, key_space_log2=20, del_permille=500),
             "{n} x 64 MiB segments per GPU (512 over 8 GPUs at 64), 1 KiB values, 50% DEL"),
    "cfg5": (64, 512 << 20, dict(val_min=16, val_max=1 << 20, key_space_log2=24, key_dist=1, del_permille=100),
             "{n} x 512 MiB segments per GPU (256 GiB over 8 GPUs at 64), Zipf-like keys over 2^24, 16 B-1 MiB values, 10% DEL"),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default=None, choices=list(CONFIGS))
    ap.add_argument("--mode", default="replay", choices=["replay", "compact", "etag"])
    ap.add_argument("--segments", type=int, default=0, help="override segments per GPU")
    ap.add_argument("--cpu-segs", type=int, default=0,
                    help="CPU baseline sample in segments (default: about 2 GiB of the shard)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-stream", action="store_true", help="skip the pinned-host streamed (H2D-inclusive) leg")
    ap.add_argument("--no-open", action="store_true", help="skip the kvs_open-from-files leg")
    ap.add_argument("--stream-batch", type=int, default=512 << 20, help="kvr_replay_stream batch bytes")
    ap.add_argument("--dry-run", action="store_true", help="CPU rehearsal of the launch and timing path (gloo)")
    args = ap.parse_args()
    if args.config is None:
        args.config = "cfg4" if args.mode == "compact" else "cfg2"

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return spawn_ranks(args.gpus)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: one rank per GPU")
    if args.dry_run:
        return dry_run(args, world, rank)

    import numpy as np
    import torch
    import torch.distributed as dist
    import kvreplay as K

    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if args.mode == "etag":
        return bench_etag(args, K, torch, dev, world, rank)

    nseg, seg_bytes, kw, desc = CONFIGS[args.config]
    if args.segments:
        nseg = args.segments
    desc = desc.format(n=nseg)   # the workload label names the segments actually replayed
    spec = K.GenSpec(seed=0x6B767265706C6179 + int(args.config[3:]), seg_bytes=seg_bytes, **kw)
    ctx = K.Context(local)

    # ---- generate this rank's shard directly into HBM -------------------------------------
    # round-robin sharding of the store's segment list (segment i -> GPU i mod N):
    # rank r owns global segments r, r + N, r + 2N, ...
    seg_nos = [rank + world * i for i in range(nseg)]
    sizes = [K.gen_segment_size(spec, s) for s in seg_nos]
    offs, tot = [], 0
    for ln, _ in sizes:
        offs.append(tot)
        tot += (ln + 255) & ~255
    n_rec = sum(nr for _, nr in sizes)
    data = torch.empty(tot + 256, dtype=torch.uint8, device=dev)
    manifest = torch.empty(n_rec + 1, dtype=torch.int32, device=dev)
    eo = 0
    for s, (ln, nr), o in zip(seg_nos, sizes, offs):
        ctx.gen_segment_device(spec, s, data.data_ptr() + o, ln, manifest.data_ptr() + 4 * eo, nr)
        eo += nr
    torch.cuda.synchronize()
    segs = [(data.data_ptr() + o, ln) for (ln, _), o in zip(sizes, offs)]
    seg_total = sum(ln for ln, _ in sizes)
    out = torch.empty((n_rec + 1024) * 32, dtype=torch.uint8, device=dev)
    if args.mode == "compact":
        return bench_compact(args, ctx, segs, seg_nos, seg_total, n_rec, desc, nseg, seg_bytes, world)

    # the segment list is marshaled into the C ABI's kvr_segment array once (a native caller hands
    # over its array; rebuilding 64 ctypes structs per call is harness time, not replay time)
    seg_list = K.SegmentList(segs, seg_ids=seg_nos, on_device=True)

    def step():
        r = ctx.replay(seg_list, expected=(manifest.data_ptr(), n_rec), expected_on_device=True,
                       out_ptr=out.data_ptr(), cap=n_rec + 1024)
        if r.status != 0:
            raise RuntimeError(f"replay failed: status {r.status} error {r.error and r.error.kind}")
        return r

    for _ in range(args.warmup):
        r = step()
    # correctness of the timed work: every record present and CRC-verified against the manifest
    assert r.n == n_rec, (r.n, n_rec)
    assert r.stats.n_crc_fail == 0

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    k_ms = []
    for _ in range(args.steps):
        r = step()
        k_ms.append((r.stats.ms_replay, r.stats.ms_total))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    per_rank = None
    if world > 1:
        from kvreplay.shard import max_over_ranks
        per_rank = gather_per_rank(dt, seg_total, args.steps)
        dt = max_over_ranks(dt)

    ms_replay = float(np.mean([a for a, _ in k_ms]))
    ms_pipe = float(np.mean([b for _, b in k_ms]))
    total_bytes = seg_total * world * args.steps
    total_recs = n_rec * world * args.steps
    gib_s = total_bytes / dt / 2 ** 30
    alg_bytes = seg_total + 32 * n_rec          # segment bytes read once + 32-B tuple writes
    achieved = alg_bytes / (ms_replay / 1e3) / 1e9

    cpu = e2e = cpu_par = cpu_all = None
    if rank == 0 and world == 1 and not args.no_cpu:
        import oracle_py as O   # the checker / CPU baseline only
        # the faithful port runs about 0.5 GiB/s on one core: a sample of about 2 GiB (32 of cfg2's
        # 64 segments, 4 of cfg5's 512-MiB segments, 2 of cfg3's 1-GiB segments) keeps it near 5 s
        cs = min(args.cpu_segs or max(1, (2 << 30) // seg_bytes), nseg)
        hall = data[:tot].cpu().numpy()   # the shard's bytes (byte-identical to kvh_gen_segment's)
        all_segs = [hall[o:o + ln] for (ln, _), o in zip(sizes, offs)]
        host_segs = all_segs[:cs]
        sb = sum(len(h) for h in host_segs)
        t1 = time.perf_counter()
        rc, nk, tb, nr, dg, err = O.replay_faithful(host_segs, release=False)
        ct = time.perf_counter() - t1
        O.faithful_release()   # the reference's open() returns the map; dropping it is not replay work
        assert rc == 0 and nr == sum(nr_ for _, nr_ in sizes[:cs])
        # end-to-end from host memory (the path's real start and end): the same sample
        # replayed from pageable host buffers, H2D of segment bytes + kernels + D2H of the tuples
        ctx.replay(host_segs, seg_ids=seg_nos[:cs])
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        rh = ctx.replay(host_segs, seg_ids=seg_nos[:cs])
        et = time.perf_counter() - t2
        assert rh.status == 0 and rh.n == nr
        e2e = {"value": round(sb / et / 2 ** 30, 3), "unit": "GiB/s", "sample": f"{cs} segments ({sb / 2**30:.2f} GiB) "
               "from pageable host memory: H2D of segment bytes + replay + D2H of the tuples, one call"}
        # strong CPU baseline (SURVEY §8d ii): the oracle's parse + slice-by-16 CRC + tuple walk (no
        # owning map) over the whole shard, one segment per thread on every core this process may use
        from concurrent.futures import ThreadPoolExecutor
        host = host_cpu_info()

        def strong(threads):
            pts = []
            for _ in range(3):
                t3 = time.perf_counter()
                with ThreadPoolExecutor(threads) as ex:
                    pr = list(ex.map(lambda h: O.replay_s16([h]), all_segs))
                pts.append(time.perf_counter() - t3)
                assert all(r[0] == 0 for r in pr) and sum(len(r[1]) for r in pr) == n_rec
            return min(pts)

        def strong_line(pt, threads, what):
            return {"value": round(seg_total / pt / 2 ** 30, 4), "unit": "GiB/s", "cores": threads, "kind": "port",
                    "records_per_s": round(n_rec / pt, 1), "nproc": host["nproc"], "affinity": host["affinity"],
                    "cpu_model": host["model"],
                    "sample": f"all {nseg} segments ({seg_total / 2**30:.2f} GiB): oracle_replay_s16 (framing walk, "
                              f"UTF-8 check, slice-by-16 CRC-32 of every key and value, 32-B tuples; no owning map), "
                              f"one segment per thread (the framing is serial within a segment, engine.rs:85), "
                              f"{threads} threads = {what}, best of 3"}
        cpu_par = strong_line(strong(host["threads"]), host["threads"], "this job's CPU share per GPU")
        all_threads = min(host["affinity"], nseg)
        cpu_all = strong_line(strong(all_threads), all_threads,
                              f"every core of the affinity set ({host['affinity']}) the {nseg} segments can use")
        del hall, all_segs, host_segs
        cpu = {"value": round(sb / ct / 2 ** 30, 4), "unit": "GiB/s", "cores": 1, "kind": "port",
               "records_per_s": round(nr / ct, 1), "nproc": host["nproc"], "cpu_model": host["model"],
               "sample": f"{cs} of the {nseg} segments ({sb / 2**30:.2f} GiB), oracle_replay_faithful: "
                         f"8 KiB buffered reads, per-record allocations, owning key->value map, CRC-32 per value "
                         f"(engine.rs:79-154 cost model), 1 thread, warm memory; the map is released after the clock"}

    stream = None
    if rank == 0 and world == 1 and not args.no_stream:
        # H2D-inclusive rate (SURVEY §8d end-to-end, §8f rank 2): the whole shard in pinned host
        # memory, streamed through kvr_replay_stream (batch b+1's DMA overlapping batch b's replay),
        # tuples back in host memory with the CRC verification; wall clock of the whole call
        pin = torch.empty(tot + 256, dtype=torch.uint8, pin_memory=True)
        pin.copy_(data)
        man = manifest[:n_rec].cpu().numpy().view(np.uint32)
        hsegs = [(pin.data_ptr() + o, ln) for (ln, _), o in zip(sizes, offs)]
        torch.cuda.synchronize()
        walls = []
        for i in range(3):
            rs = ctx.replay_stream(hsegs, seg_ids=seg_nos, expected=man, cap=n_rec + 1024,
                                   batch_bytes=args.stream_batch, pinned=True)
            assert rs.status == 0 and rs.n == n_rec and rs.stats.n_crc_fail == 0
            if i:
                walls.append(rs.stream_stats.ms_wall)
        w = min(walls) / 1e3
        # the host index fold of those tuples: kvh_fold_parallel, keys read
        # from the pinned segment bytes; 16 threads (the GPU box's CPU share per GPU)
        fold_s = []
        for i in range(2):
            tf = time.perf_counter()
            live, nk, tb = K.fold(hsegs, rs.tuples, threads=16, pinned=True)
            fold_s.append(time.perf_counter() - tf)
        # the open path's index from the same pinned bytes (kvr_ingest_begin / _push / _index):
        # every segment DMA'd into HBM, replay + fold + key table on the device, live tuples and
        # the table back — what kvs_open does once the files are read
        ix_s = []
        for i in range(3):
            tf = time.perf_counter()
            ix = ctx.ingest_index(hsegs, seg_ids=seg_nos, host_ptrs=True)
            if i:
                ix_s.append(time.perf_counter() - tf)
            assert ix.status == 0 and len(ix.live) == nk
        ixs = ix.stats
        stream = {"value": round(seg_total / w / 2 ** 30, 3), "unit": "GiB/s",
                  "records_per_s": round(n_rec / w, 1), "batch_bytes": args.stream_batch,
                  "n_batches": int(rs.stream_stats.n_batches),
                  "ms_device_sum": round(rs.stream_stats.ms_device, 3),
                  "host_fold_ms": round(min(fold_s) * 1e3, 3), "host_fold_threads": 16, "live_keys": nk,
                  "index_rebuild_host_fold_GiB_s": round(seg_total / (w + min(fold_s)) / 2 ** 30, 3),
                  "index_rebuild_GiB_s": round(seg_total / min(ix_s) / 2 ** 30, 3),
                  "index_rebuild_ms": round(min(ix_s) * 1e3, 3),
                  "index_device_ms": {"replay": round(ixs.ms_replay, 3), "fold_live_table": round(ixs.ms_fold, 3),
                                      "fold_rounds": int(ixs.fold_rounds)},
                  "sample": f"all {nseg} segments ({seg_total / 2**30:.2f} GiB) from pinned host memory: "
                            "value = kvr_replay_stream wall time (pinned H2D on a copy stream overlapping replay + "
                            "CRC verify + D2H of the tuples to host), best of 2; index_rebuild = kvr_ingest_* wall "
                            "time (H2D of every segment, replay, device fold, key table, D2H of the live tuples "
                            "and the table), best of 2; index_rebuild_host_fold = the stream plus kvh_fold_parallel"}
        del pin

    live_idx = None
    if rank == 0 and world == 1 and not args.no_stream:
        # the index built on the device (kvr_replay_live: replay + last-writer fold in HBM, only
        # the live keys' final tuples written), device-resident in and out
        lo = torch.empty((n_rec + 1024) * 32, dtype=torch.uint8, device=dev)
        lms = []
        for i in range(3):
            torch.cuda.synchronize()
            t4 = time.perf_counter()
            rl = ctx.replay_live(segs, seg_ids=seg_nos, on_device=True, out_ptr=lo.data_ptr(), cap=n_rec + 1024)
            torch.cuda.synchronize()
            assert rl.status == 0
            if i:
                lms.append(time.perf_counter() - t4)
        live_idx = {"value": round(seg_total / min(lms) / 2 ** 30, 3), "unit": "GiB/s", "live_keys": rl.n,
                    "ms": round(min(lms) * 1e3, 3),
                    "sample": "kvr_replay_live on the device-resident shard: replay + last-writer fold in HBM, "
                              "live tuples out (the index of engine.rs:137/:141), wall time, best of 2"}
        del lo

    open_files = None
    if rank == 0 and world == 1 and not args.no_open:
        # KVStore::open from files (engine.rs:24-76): the shard written as segment-<id>.dat files
        # (page cache warm), then kvs_open_ex: parallel pread into pinned memory, per-segment DMA
        # into HBM as each file lands, replay + fold + key table on the device; best of 2
        import shutil
        import tempfile
        tmpd = tempfile.mkdtemp(prefix="kvr_open_", dir=os.environ.get("TMPDIR", "/tmp"))
        try:
            hall = data[:tot].cpu().numpy()
            for (ln, _), o, sid in zip(sizes, offs, seg_nos):
                with open(os.path.join(tmpd, f"segment-{sid}.dat"), "wb") as f:
                    f.write(memoryview(hall[o:o + ln]))
            del hall
            best = None
            for i in range(3):
                for n in os.listdir(tmpd):   # the active segment kvs_open creates is empty: drop it
                    if os.path.getsize(os.path.join(tmpd, n)) == 0:
                        os.unlink(os.path.join(tmpd, n))
                t5 = time.perf_counter()
                st_ = K.KVStore.open(tmpd, ctx)
                wall = time.perf_counter() - t5
                o_ = st_.open_stats()
                assert st_.stats().num_keys == live_idx["live_keys"] if live_idx else True
                st_.close()
                if i and (best is None or wall < best[0]):
                    best = (wall, o_)
            wall, o_ = best
            open_files = {"value": round(seg_total / wall / 2 ** 30, 3), "unit": "GiB/s", "ms": round(wall * 1e3, 2),
                          "load": "mmap" if o_.mode == K.LOAD_MMAP else "pread", "ms_load": round(o_.ms_read, 2),
                          "ms_register_in_load": round(o_.ms_register, 2), "ms_push_in_load": round(o_.ms_push, 2),
                          "ms_index_after_load": round(o_.ms_index, 2), "read_threads": int(o_.read_threads),
                          "path": "device-index" if o_.path == K.PATH_DEVICE_INDEX else "host-fold",
                          "live_keys": int(o_.n_live),
                          "sample": f"kvs_open_ex over {nseg} segment files ({seg_total / 2**30:.2f} GiB, page cache "
                                    "warm): discovery, every file mmap'd (populated from the page cache, 16 threads) "
                                    "and registered for DMA, pushed to HBM in store order, device replay + fold + key table, wall time, best of 2"}
        finally:
            shutil.rmtree(tmpd, ignore_errors=True)

    traffic = None   # HBM bytes per replay (k_piece + k_replay) from PMC (tools/pmc_traffic.py), if measured on this build
    tj = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tj):
        import hashlib
        pm = json.load(open(tj))
        lib = os.path.join(ROOT, "mini-kvstore-v2_amd", "lib", "libkvreplay.so")
        if (pm.get("lib_sha256_16") == hashlib.sha256(open(lib, "rb").read()).hexdigest()[:16]
                and args.config == "cfg2" and nseg == CONFIGS["cfg2"][0]):
            traffic = round(pm["hbm_bytes"])

    res = {
        "metric": METRIC, "value": round(gib_s, 3), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic (device generator, seeded)",
        "config": {"workload": f"{args.config}: {desc}, device-resident", "segments_per_gpu": nseg,
                   "segment_bytes": seg_bytes, "bytes_per_gpu": seg_total, "records_per_gpu": n_rec,
                   "parallelism": f"shard-segments x{world} (no collective)"},
        "records_per_s": round(total_recs / dt, 1),
        "crc_verified_records_per_s": round(total_recs / dt, 1),
        "ms_kernel_replay": round(ms_replay, 4), "ms_device_pipeline": round(ms_pipe, 4),
        "roofline": {"bound": "hbm", "kernel": "k_piece + k_replay (k_piece's start to k_replay's end)",
                     "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS,
                     "unit": "GB/s", "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": traffic,
                     "alg_bytes_per_launch": alg_bytes},
        "cpu_baseline": cpu,
        "cpu_baseline_parallel": cpu_par,
        "cpu_baseline_allcores": cpu_all,
        "e2e_host": e2e,
        "e2e_stream_pinned": stream,
        "live_index_device": live_idx,
        "open_from_files": open_files,
    }
    if per_rank is not None:
        res["per_rank"] = per_rank
    if rank == 0:
        print(json.dumps(res))
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


def bench_compact(args, ctx, segs, seg_nos, seg_total, n_rec, desc, nseg, seg_bytes, world):
    """kvr_compact over the rank's shard, in and out of HBM.  Per step: the replay pipeline, the
    fold (hash insert, live flags, scans, dense list) and the gather of the live records."""
    import numpy as np
    import torch
    import kvreplay as K
    target = 64 << 20
    if world > 1:
        return bench_compact_sharded(args, ctx, segs, seg_nos, seg_total, n_rec, desc, nseg, seg_bytes, world, target)
    out = torch.empty(seg_total + 4096, dtype=torch.uint8, device="cuda")

    def step():
        r = ctx.compact(segs, target, seg_ids=seg_nos, on_device=True, out_ptr=out.data_ptr(), out_cap=out.numel())
        if r.status != 0:
            raise RuntimeError(f"compact failed: status {r.status}")
        return r

    for _ in range(args.warmup):
        r = step()
    # self-check (size-independent): the new segments replay cleanly to exactly the live records
    starts = [0] + r.seg_ends[:-1]
    new = [(out.data_ptr() + a, b - a) for a, b in zip(starts, r.seg_ends)]
    rr = ctx.replay(new, on_device=True)
    assert rr.status == 0 and rr.n == r.stats.n_live, (rr.status, rr.n, r.stats.n_live)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    st = []
    for _ in range(args.steps):
        r = step()
        st.append((r.stats.ms_replay, r.stats.ms_fold, r.stats.ms_gather))
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ms_rep, ms_fold, ms_gat = (float(np.mean([x[i] for x in st])) for i in range(3))
    live_bytes, n_live = r.stats.bytes_out, r.stats.n_live
    # the pipeline's algorithmic HBM bytes per step: every segment byte read once by
    # the replay, its 32-B tuples written once and read once by the fold, the live records read once
    # and written once by the gather
    alg = seg_total + 2 * 32 * n_rec + 2 * live_bytes
    # per step, wall clock (launch gaps, scans and host work between the phases included)
    ms_step = dt / args.steps * 1e3
    achieved = alg / (ms_step / 1e3) / 1e9
    phases = {"replay": round(ms_rep, 4), "fold": round(ms_fold, 4), "gather": round(ms_gat, 4)}
    res = {
        "metric": "device-resident compaction live-record rewrite GiB/s (segment bytes in)",
        "value": round(seg_total * args.steps / dt / 2 ** 30, 3), "unit": "GiB/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (device generator, seeded)",
        "config": {"workload": f"{args.config}: {desc}, device-resident, compaction into ~64 MiB segments",
                   "segments_per_gpu": nseg, "segment_bytes": seg_bytes, "bytes_per_gpu": seg_total,
                   "records_per_gpu": n_rec, "live_records": n_live, "live_bytes": live_bytes,
                   "new_segments": len(r.seg_ends), "parallelism": "1 GPU"},
        "ms_replay": round(ms_rep, 4), "ms_fold": round(ms_fold, 4), "ms_gather": round(ms_gat, 4),
        "roofline": {"bound": "hbm", "kernel": "compaction pipeline (k_replay, fold kernels, k_gather_r)",
                     "dominant_kernel": "k_replay" if ms_rep >= max(ms_fold, ms_gat) else
                                        ("fold" if ms_fold >= ms_gat else "k_gather_r"),
                     "ms_by_phase": phases, "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS,
                     "unit": "GB/s", "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": None,
                     "alg_bytes_per_step": alg, "time_base": "ms_per_step"},
    }
    print(json.dumps(res))
    ctx.close()


def bench_compact_sharded(args, ctx, segs, seg_nos, seg_total, n_rec, desc, nseg, seg_bytes, world, target):
    """N ranks, segments round-robin: the global last-writer fold needs the candidate exchange
    (kvreplay.shard.compact_sharded: two all-to-alls over RCCL); one step = the whole sharded
    compaction, timed with barriers and the max over ranks."""
    import numpy as np
    import torch
    import torch.distributed as dist
    from kvreplay import shard as SH
    eng = SH.DeviceCompactEngine(ctx, torch.device("cuda", torch.cuda.current_device()))
    rank = dist.get_rank()

    def step():
        return SH.compact_sharded(eng, segs, seg_nos, seg_target=target, on_device=True)

    for _ in range(args.warmup):
        data, ends = step()
    n_live = torch.tensor([ctx_live(ctx)], dtype=torch.int64, device="cuda")
    dist.all_reduce(n_live)
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    dt = SH.max_over_ranks(time.perf_counter() - t0)
    res = {
        "metric": "device-resident compaction live-record rewrite GiB/s (segment bytes in)",
        "value": round(seg_total * world * args.steps / dt / 2 ** 30, 3), "unit": "GiB/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (device generator, seeded)",
        "config": {"workload": f"{args.config}: {desc}, device-resident input, sharded compaction "
                               f"(round-robin), each rank's output copied to host",
                   "segments_per_gpu": nseg, "segment_bytes": seg_bytes, "bytes_per_gpu": seg_total,
                   "records_per_gpu": n_rec, "live_records_total": int(n_live.item()),
                   "parallelism": f"shard-segments x{world}, candidate all-to-all (RCCL)"},
    }
    if rank == 0:
        print(json.dumps(res))
    ctx.close()
    dist.destroy_process_group()


def ctx_live(ctx):
    import ctypes as C
    import kvreplay as K
    st = K.CompactStats()
    K.native()[0].kvr_last_compact_stats(ctx.h, C.byref(st))
    return int(st.n_live)



def bench_etag(args, K, torch, dev, world, rank):
    """kvr_etag_batch over 8 GiB of 64-KiB blobs in HBM (volume-server shape, cfg3), verified
    against the stored ETags every step; a sample is checked against zlib.crc32 first."""
    import zlib
    import numpy as np
    import torch.distributed as dist
    n_blob, blob = 131072, 65536
    ctx = K.Context(dev.index or 0)
    g = torch.Generator(device=dev)
    g.manual_seed(0x6B767265 + rank)
    data = torch.randint(0, 256, (n_blob * blob,), dtype=torch.uint8, device=dev, generator=g)
    offs = np.arange(n_blob, dtype=np.uint64) * blob
    lens = np.full(n_blob, blob, dtype=np.uint64)
    torch.cuda.synchronize()
    stored, _, _ = ctx.etag_batch(data.data_ptr(), offs, lens, on_device=True, data_len=data.numel())
    for i in (0, 1, n_blob // 2, n_blob - 1):
        assert int(stored[i]) == zlib.crc32(data[i * blob:(i + 1) * blob].cpu().numpy().tobytes())
    ms = []
    for _ in range(args.warmup):
        ctx.etag_batch(data.data_ptr(), offs, lens, expected=stored, on_device=True, data_len=data.numel())
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        crc, nf, st = ctx.etag_batch(data.data_ptr(), offs, lens, expected=stored, on_device=True,
                                     data_len=data.numel())
        assert nf == 0
        ms.append((st.ms_chunk, st.ms_join))
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        from kvreplay.shard import max_over_ranks
        dt = max_over_ranks(dt)
    total = n_blob * blob
    mc = float(np.mean([a for a, _ in ms]))
    mj = float(np.mean([b for _, b in ms]))
    alg = total + 4 * (total // 4096) + 4 * n_blob      # blob bytes once + chunk registers + CRCs
    res = {"metric": "batch ETag compute+verify GiB/s (SURVEY §8f rank 4)", "value": round(total * world * args.steps / dt / 2 ** 30, 3),
           "unit": "GiB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": round(dt / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "u8", "data": "synthetic (torch.randint on device, seeded)",
           "config": {"workload": f"{n_blob} x 64 KiB blobs (8 GiB, volume-server shape) in HBM, CRC-32 + verify",
                      "blobs_per_gpu": n_blob, "blob_bytes": blob},
           "blobs_per_s": round(n_blob * world * args.steps / dt, 1),
           "ms_kernel_chunk": round(mc, 4), "ms_kernel_join": round(mj, 4),
           "roofline": {"bound": "hbm", "kernel": "k_etag_chunk", "achieved": round(alg / (mc / 1e3) / 1e9, 1),
                        "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": round(alg / (mc / 1e3) / 1e9 / PEAK_HBM_GBS, 4),
                        "traffic": None, "alg_bytes_per_launch": alg}}
    if rank == 0:
        print(json.dumps(res))
    ctx.close()

def host_cpu_info():
    """The CPU the baselines ran on: nproc, this process's affinity, the thread count used (the
    affinity set, capped by OMP_NUM_THREADS, which the GPU box sets to this job's 16-core share) and
    the model name (lscpu's "Model name", read from /proc/cpuinfo)."""
    aff = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    threads = min(aff, int(omp)) if omp and omp.isdigit() and int(omp) > 0 else aff
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"nproc": os.cpu_count(), "affinity": aff, "threads": threads, "model": model}


def spawn_ranks(n):
    """One process per GPU: run this script under torch.distributed.run as a child process (this
    parent has made no HIP call, so nothing is exec'd over an initialised GPU) and exit with its
    status.  Rendezvous on 127.0.0.1 (the container hostname may not resolve)."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def gather_per_rank(dt, bytes_per_rank, steps):
    """Every rank's own wall time and rate, on rank 0 (None elsewhere)."""
    import torch.distributed as dist
    mine = {"rank": dist.get_rank(), "seconds": round(dt, 6),
            "GiB_s": round(bytes_per_rank * steps / dt / 2 ** 30, 3) if dt > 0 else None}
    out = [None] * dist.get_world_size() if dist.get_rank() == 0 else None
    dist.gather_object(mine, out, dst=0)
    return out


def dry_run(args, world, rank):
    """The launch, barrier and max-over-ranks logic of the replay leg on CPU (gloo): a sleep of
    (rank + 1) ms stands in for one replay step, so the whole-job time must be the slowest rank's."""
    import torch.distributed as dist
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo")
    bytes_per_rank = 1 << 30
    for _ in range(args.warmup):
        time.sleep(0.001 * (rank + 1))
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        time.sleep(0.001 * (rank + 1))
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    per_rank = None
    if world > 1:
        from kvreplay.shard import max_over_ranks
        per_rank = gather_per_rank(dt, bytes_per_rank, args.steps)
        dt = max_over_ranks(dt)
    if rank == 0:
        print(json.dumps({"metric": METRIC + " (dry run: no GPU, sleep steps)", "value": round(
            bytes_per_rank * world * args.steps / dt / 2 ** 30, 3), "unit": "GiB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "none (dry run)", "config": {"workload": "dry run", "parallelism": f"shard-segments x{world}"},
            "per_rank": per_rank}))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
