"""Full-size GPU tests at BASELINE.json's shapes: the segments are generated
in HBM by the device generator exactly as bench.py does, replayed through the C ABI, and checked

  cfg2  64 x 64 MiB, 1 KiB values          tuple for tuple against the oracle (one segment per host
  cfg3  8 x 1 GiB, 64 KiB values           thread over the D2H copy of the same bytes) + manifest
  cfg4  64 x 64 MiB, 50 % DEL (one GPU's   the compaction (kvr_compact) output byte for byte against
        shard of the compaction config)    oracle_compact, and its replay against the oracle's
  cfg5  64 x 512 MiB (one GPU's 32 GiB     size-independent properties: records = generator count,
        shard of the 256 GiB store)        every CRC verified against the manifest with 0 failures,
                                           stripe re-walks reported; every segment against the oracle
"""
import numpy as np
import pytest
import torch

import kvreplay as K
import oracle_py as O

pytestmark = pytest.mark.gpu

SPECS = {   # bench.py CONFIGS (seed = 0x6B767265706C6179 + config number)
    "cfg2": (64, 64 << 20, dict(val_min=1024, val_max=1024, key_space_log2=20)),
    "cfg3": (8, 1 << 30, dict(val_min=65536, val_max=65536, key_space_log2=20)),
    "cfg4": (64, 64 << 20, dict(val_min=1024, val_max=1024, key_space_log2=20, del_permille=500)),
    "cfg5": (64, 512 << 20, dict(val_min=16, val_max=1 << 20, key_space_log2=24, key_dist=1, del_permille=100)),
}


def _generate(ctx, cfg):
    nseg, seg_bytes, kw = SPECS[cfg]
    spec = K.GenSpec(seed=0x6B767265706C6179 + int(cfg[3:]), seg_bytes=seg_bytes, **kw)
    sizes = [K.gen_segment_size(spec, s) for s in range(nseg)]
    offs, tot = [], 0
    for ln, _ in sizes:
        offs.append(tot)
        tot += (ln + 255) & ~255
    n_rec = sum(nr for _, nr in sizes)
    data = torch.empty(tot + 256, dtype=torch.uint8, device="cuda")
    man = torch.empty(n_rec + 1, dtype=torch.int32, device="cuda")
    eo = 0
    for s, ((ln, nr), o) in enumerate(zip(sizes, offs)):
        ctx.gen_segment_device(spec, s, data.data_ptr() + o, ln, man.data_ptr() + 4 * eo, nr)
        eo += nr
    torch.cuda.synchronize()
    return data, offs, sizes, man, n_rec


def _replay_to_host(ctx, data, offs, sizes, man, n_rec):
    segs = [(data.data_ptr() + o, ln) for (ln, _), o in zip(sizes, offs)]
    out = torch.empty((n_rec + 1024) * 32, dtype=torch.uint8, device="cuda")
    r = ctx.replay(segs, expected=(man.data_ptr(), n_rec), expected_on_device=True, on_device=True,
                   out_ptr=out.data_ptr(), cap=n_rec + 1024)
    torch.cuda.synchronize()
    t = out[: r.n * 32].cpu().numpy().view(K.TUPLE_DTYPE) if r.status == 0 else None
    return r, t


@pytest.mark.parametrize("cfg", ["cfg2", "cfg3"])
def test_full_size_bit_exact(gctx, cfg):
    data, offs, sizes, man, n_rec = _generate(gctx, cfg)
    r, t = _replay_to_host(gctx, data, offs, sizes, man, n_rec)
    assert r.status == 0 and r.n == n_rec and r.stats.n_crc_fail == 0
    host = data.cpu().numpy()
    segs = [host[o: o + ln] for (ln, _), o in zip(sizes, offs)]
    del data
    rc, ref, _ = O.replay_parallel(segs, threads=16)
    assert rc == 0 and len(ref) == n_rec
    ref["flags"] |= np.where(ref["op"] == 0, K.TF_VERIFIED, 0).astype(np.uint8)   # the manifest matches
    if not np.array_equal(t, ref):
        bad = np.nonzero(t != ref)[0][:5]
        raise AssertionError(f"{cfg}: tuple mismatch at {bad}: gpu={t[bad]} oracle={ref[bad]}")


def test_cfg5_shard_properties(gctx):
    data, offs, sizes, man, n_rec = _generate(gctx, "cfg5")
    assert sum(ln for ln, _ in sizes) > 31 << 30           # the full 32-GiB shard of one GPU
    r, t = _replay_to_host(gctx, data, offs, sizes, man, n_rec)
    assert r.status == 0
    assert r.n == n_rec                                     # every generated record, no more
    assert r.stats.n_crc_fail == 0                          # every value CRC = the manifest's ETag
    assert int(np.count_nonzero(t["flags"] & K.TF_VERIFIED)) == int(np.count_nonzero(t["op"] == 0))
    assert r.stats.n_redo >= 0 and r.stats.n_stripes > 0
    # per-segment record counts match the generator, and all 64 segments (32 GiB, one segment per
    # host thread) match the oracle tuple for tuple
    counts = np.bincount(t["seg_idx"], minlength=len(sizes))
    assert [int(c) for c in counts] == [nr for _, nr in sizes]
    host = data.cpu().numpy()
    segs = [host[o: o + ln] for (ln, _), o in zip(sizes, offs)]
    del data
    rc, ref, _ = O.replay_parallel(segs, threads=16)
    assert rc == 0 and len(ref) == n_rec
    ref["flags"] |= np.where(ref["op"] == 0, K.TF_VERIFIED, 0).astype(np.uint8)   # the manifest matches
    if not np.array_equal(t, ref):
        bad = np.nonzero(t != ref)[0][:5]
        raise AssertionError(f"cfg5: tuple mismatch at {bad}: gpu={t[bad]} oracle={ref[bad]}")


def test_full_size_cfg4_compaction(gctx):
    """BASELINE config 4's compaction at one GPU's full shard (64 x 64 MiB, 1 KiB values, 50 % DEL
    of earlier-SET keys): kvr_compact with input and output in HBM, exactly as bench.py --mode
    compact runs it.  The output bytes and the new segment boundaries equal oracle_compact's
    (compaction.rs:9-29 with the intended live rewrite, README.md:283-287), and a replay of the new
    segments on the GPU equals the oracle's replay of them, tuple for tuple (the pre-compaction
    map, tests/store_integration.rs:20-31, now across a reopen)."""
    data, offs, sizes, man, n_rec = _generate(gctx, "cfg4")
    segs = [(data.data_ptr() + o, ln) for (ln, _), o in zip(sizes, offs)]
    total = sum(ln for ln, _ in sizes)
    target = 64 << 20
    out = torch.empty(total + 4096, dtype=torch.uint8, device="cuda")
    r = gctx.compact(segs, target, on_device=True, out_ptr=out.data_ptr(), out_cap=out.numel())
    assert r.status == 0 and r.out_len == r.stats.bytes_out
    torch.cuda.synchronize()
    got = out[: r.out_len].cpu().numpy().tobytes()
    host = data.cpu().numpy()
    hsegs = [host[o: o + ln] for (ln, _), o in zip(sizes, offs)]
    del data, out
    rc, want, ends, _ = O.compact(hsegs, seg_target=target)
    assert rc == 0
    assert len(got) == len(want) and got == want
    assert r.seg_ends == ends
    news = O.split_segments(want, ends)
    rco, ro, _ = O.replay(news)
    rg = gctx.replay(news)
    assert rco == rg.status == 0 and np.array_equal(rg.tuples, ro)
    # every record of the new segments is a SET, and there is exactly one per live key
    assert (ro["op"] == 0).all() and len(ro) == r.stats.n_live


def test_replay_past_the_pool_slot_limit(gctx):
    """kvr_replay over more records than the pool's 32-bit slots hold (the real limit, 2^32 - 2^16
    tuples, not lowered): 4.5 G five-byte DEL records of the empty key ([1][0 0 0 0], a valid record:
    engine.rs:96-114 accepts an empty UTF-8 key, :141 removes it) in 15 segments of 1.5 GB, between
    two generated segments.  kvr_replay batches the input into whole-segment pipelines; the tuples
    (in HBM, 144 GB) are checked on the device against their exact expected values (rec_off = 5 j,
    seg_idx, key_len = val_len = crc32 = key_tag = 0, op = 1), the generated segments tuple for
    tuple against the oracle, and a torn last segment gives the oracle's first error.
    (The fold caps one call at 2^31 tuples, below this limit, so the folding callers never batch at
    the real limit; they are run batched at full cfg4 size below with the limit lowered.)"""
    spec = K.GenSpec(seed=109, seg_bytes=1 << 20, key_space_log2=12, val_min=0, val_max=3000, del_permille=200)
    small = [K.gen_segment_cpu(spec, s)[0] for s in range(2)]
    n_big, rec_big = 15, 300_000_000
    big_len = 5 * rec_big
    n_rec = n_big * rec_big
    assert n_rec > 0xFFFF0000
    data = torch.zeros(n_big * big_len + 2 * (1 << 20) + 4096, dtype=torch.uint8, device="cuda")
    data[: n_big * big_len].view(-1, 5)[:, 0] = 1
    tail = data[n_big * big_len:]
    o0 = 0
    tail[o0: o0 + len(small[0])] = torch.from_numpy(np.asarray(small[0])).cuda()
    o1 = ((len(small[0]) + 255) // 256) * 256
    tail[o1: o1 + len(small[1])] = torch.from_numpy(np.asarray(small[1])).cuda()
    tb = tail.data_ptr()
    segs = ([(tb + o0, len(small[0]))] + [(data.data_ptr() + i * big_len, big_len) for i in range(n_big)] +
            [(tb + o1, len(small[1]))])
    rc0, ref0, _ = O.replay([small[0]])
    rc1, ref1, _ = O.replay([small[1]])
    assert rc0 == rc1 == 0
    total = n_rec + len(ref0) + len(ref1)
    out = torch.empty((total + 1024) * 32, dtype=torch.uint8, device="cuda")
    r = gctx.replay(segs, on_device=True, out_ptr=out.data_ptr(), cap=total + 1024)
    torch.cuda.synchronize()
    assert r.status == 0 and r.n == total
    t64 = out.view(torch.int64)
    # the generated segments against the oracle
    got0 = out[: len(ref0) * 32].cpu().numpy().view(K.TUPLE_DTYPE)
    assert np.array_equal(got0, ref0)
    b1 = (len(ref0) + n_rec) * 32
    got1 = out[b1: b1 + len(ref1) * 32].cpu().numpy().view(K.TUPLE_DTYPE).copy()
    assert (got1["seg_idx"] == n_big + 1).all()
    got1["seg_idx"] = 0
    assert np.array_equal(got1, ref1)
    # the big segments: every tuple equals its expected value, checked on the device in chunks
    step = 50_000_000
    base = len(ref0)
    for s in range(n_big):
        for j0 in range(0, rec_big, step):
            m = min(step, rec_big - j0)
            rows = t64[4 * (base + s * rec_big + j0): 4 * (base + s * rec_big + j0 + m)].view(m, 4)
            want_off = torch.arange(j0, j0 + m, device="cuda", dtype=torch.int64) * 5
            assert torch.equal(rows[:, 0], want_off)
            assert bool((rows[:, 1] == s + 1).all())          # seg_idx s + 1, key_len 0
            assert bool((rows[:, 2] == 0).all())              # val_len 0, crc32 0
            assert bool((rows[:, 3] == (1 << 32)).all())      # key_tag 0, op 1, flags 0
            del rows, want_off
    # a torn last segment: the first error is the oracle's, found in the last batch
    torn = small[1][: len(small[1]) - 3]
    rce, _, err = O.replay([torn])
    assert rce == K.CORRUPTED
    segs[-1] = (tb + o1, len(torn))
    r = gctx.replay(segs, on_device=True, out_ptr=out.data_ptr(), cap=total + 1024)
    assert r.status == K.CORRUPTED
    assert (r.error.kind, r.error.seg_idx, r.error.rec_off, r.error.aux) == (err.kind, n_big + 1, err.rec_off, err.aux)


def test_full_size_cfg4_fold_batched(gctx, monkeypatch):
    """The folding callers batched at full size: one GPU's cfg4 shard (64 x 64 MiB, 8 M records,
    50 % DEL) with the pool-slot limit lowered to 16 M tuples (above the 8.4 M slots of claim slack
    the 4096 stripes reserve), so kvr_replay_live and kvr_compact run their replay as four
    whole-segment batches, then fold all of them (the path a
    mid-round-3 bug once broke with status 0).  The live list equals the oracle's fold and the
    compaction output equals oracle_compact byte for byte."""
    data, offs, sizes, man, n_rec = _generate(gctx, "cfg4")
    segs = [(data.data_ptr() + o, ln) for (ln, _), o in zip(sizes, offs)]
    host = data.cpu().numpy()
    hsegs = [host[o: o + ln] for (ln, _), o in zip(sizes, offs)]
    rc, t, _ = O.replay_parallel(hsegs, threads=16)
    assert rc == 0 and len(t) == n_rec
    live, nk, _ = O.fold_live(hsegs, t)
    monkeypatch.setenv("KVR_POOL_LIMIT", "16000000")
    r = gctx.replay_live(segs, on_device=True)
    assert r.status == 0 and r.n == nk and np.array_equal(r.tuples, t[live])
    total = sum(ln for ln, _ in sizes)
    target = 64 << 20
    out = torch.empty(total + 4096, dtype=torch.uint8, device="cuda")
    rcmp = gctx.compact(segs, target, on_device=True, out_ptr=out.data_ptr(), out_cap=out.numel())
    assert rcmp.status == 0
    torch.cuda.synchronize()
    got = out[: rcmp.out_len].cpu().numpy().tobytes()
    del data, out
    rco, want, ends, _ = O.compact(hsegs, seg_target=target)
    assert rco == 0 and got == want and rcmp.seg_ends == ends
