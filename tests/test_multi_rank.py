"""Multi-rank (N > 1) path on CPU: world_size-2 gloo processes shard the segment list round-robin,
replay their shards, gather on rank 0 and merge.  The per-shard replay here is the CPU oracle
standing in for the GPU (no GPU in this container); the GPU shard path is covered by
tests/test_gpu_parity.py::test_sharded_replay_matches_single and by bench.py --gpus N.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import kvreplay as K
from kvreplay import shard as SH
import oracle_py as O

SPEC = K.GenSpec(seed=0xD15C, seg_bytes=60_000, val_min=8, val_max=700, del_permille=500, key_space_log2=9)
N_SEGS = 7


def _segments(corrupt=()):
    segs = [K.gen_segment_cpu(SPEC, s)[0].tobytes() for s in range(N_SEGS)]
    for i in corrupt:                      # a torn tail inside the last record
        segs[i] = segs[i][:-3]
    return segs


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, corrupt, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        segs = _segments(corrupt)
        idx = SH.shard_round_robin(len(segs), world, rank)
        rc, t, e = O.replay([segs[i] for i in idx])            # stand-in for Context.replay on this rank's GPU
        err = (e.kind, e.seg_idx, e.rec_off, e.aux) if rc == K.CORRUPTED else None
        part = SH.localize(idx, rc, t if rc == K.OK else None, err)
        parts = SH.gather_shards(part)
        slowest = SH.max_over_ranks(0.25 * (rank + 1))
        if rank == 0:
            st, merged, first = SH.merge_shards(parts)
            np.save(os.path.join(outdir, "merged.npy"), merged)
            with open(os.path.join(outdir, "meta.txt"), "w") as f:
                f.write(f"{st} {first} {slowest}\n")
    finally:
        dist.destroy_process_group()


def _run(world, corrupt, tmp_path):
    mp.start_processes(_rank_main, args=(world, _free_port(), corrupt, str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    st, rest = open(tmp_path / "meta.txt").read().split(" ", 1)
    return int(st), np.load(tmp_path / "merged.npy"), rest


def test_round_robin_assignment():
    assert SH.shard_round_robin(7, 2, 0) == [0, 2, 4, 6]
    assert SH.shard_round_robin(7, 2, 1) == [1, 3, 5]
    owned = sorted(i for r in range(8) for i in SH.shard_round_robin(512, 8, r))
    assert owned == list(range(512))


def test_two_rank_gloo_merge_matches_single(tmp_path):
    st, merged, rest = _run(2, (), tmp_path)
    segs = _segments()
    rc, ref, _ = O.replay(segs)
    assert st == K.OK and rc == K.OK
    assert np.array_equal(merged, ref)                        # same tuples, same (seg, off) order
    live_m, nk_m, tb_m = K.fold(segs, merged)
    live_r, nk_r, tb_r = K.fold(segs, ref)
    assert (nk_m, tb_m) == (nk_r, tb_r) and np.array_equal(live_m, live_r)
    assert float(rest.split()[-1]) == 0.5                     # max over ranks, not rank 0's own time


def test_eight_rank_gloo_merge_matches_single(tmp_path):
    """The target width (8 ranks, one per GPU of a node) with fewer segments than ranks would leave
    ranks empty: N_SEGS = 7 over 8 ranks, so rank 7 owns nothing and still joins the gather."""
    st, merged, rest = _run(8, (), tmp_path)
    rc, ref, _ = O.replay(_segments())
    assert st == K.OK and rc == K.OK and np.array_equal(merged, ref)
    assert float(rest.split()[-1]) == 2.0                     # the slowest of 8 ranks (0.25 * 8)


def test_two_rank_gloo_first_error_is_global_minimum(tmp_path):
    # segment 3 (rank 1) and segment 4 (rank 0) are both torn: the store's error is segment 3's
    st, _, rest = _run(2, (3, 4), tmp_path)
    segs = _segments((3, 4))
    rc, _, e = O.replay(segs)
    assert st == K.CORRUPTED and rc == K.CORRUPTED
    assert rest.split(")")[0] + ")" == str((e.kind, e.seg_idx, e.rec_off, e.aux))
    assert e.seg_idx == 3


# ---- sharded compaction: the one step with a real exchange (kvreplay.shard.compact_sharded) ----
def _compact_rank_main(rank, world, port, target, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from compact_cpu_engine import HostCompactEngine   # stand-in for DeviceCompactEngine (no GPU here)
        segs = _segments()
        idx = SH.shard_round_robin(len(segs), world, rank)
        data, ends = SH.compact_sharded(HostCompactEngine(), [segs[i] for i in idx], idx, seg_target=target)
        with open(os.path.join(outdir, f"r{rank}.bin"), "wb") as f:
            f.write(data)
        np.save(os.path.join(outdir, f"r{rank}_ends.npy"), np.array(ends, dtype=np.uint64))
    finally:
        dist.destroy_process_group()


def _expected_split(segs, world):
    """Per rank: the global last record of every key when it is a SET and lives in that rank's
    shard, in (segment, offset) order (engine.rs:137/:141 over the whole store)."""
    rc, t, _ = O.replay(segs)
    assert rc == 0
    last = {}
    for i, r in enumerate(t):
        s = segs[r["seg_idx"]]
        last[s[r["rec_off"] + 5: r["rec_off"] + 5 + r["key_len"]]] = i
    out = [bytearray() for _ in range(world)]
    for i in sorted(last.values()):
        r = t[i]
        if r["op"] == 0:
            s = segs[r["seg_idx"]]
            out[r["seg_idx"] % world] += s[r["rec_off"]: r["rec_off"] + 9 + r["key_len"] + r["val_len"]]
    return [bytes(b) for b in out]


@pytest.mark.parametrize("world,target", [(2, 0), (2, 5000), (3, 0), (8, 0)])
def test_sharded_compaction_gloo(world, target, tmp_path):
    mp.start_processes(_compact_rank_main, args=(world, _free_port(), target, str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    segs = _segments()
    exp = _expected_split(segs, world)
    outs = [open(tmp_path / f"r{r}.bin", "rb").read() for r in range(world)]
    assert outs == exp
    # every rank's new segments, replayed together, rebuild the store's map
    new = []
    for r in range(world):
        ends = [int(e) for e in np.load(tmp_path / f"r{r}_ends.npy")]
        new += O.split_segments(outs[r], ends)
        if target and ends:
            starts = [0] + ends[:-1]
            assert all(s // target < (e - 1) // target + 1 for s, e in zip(starts, ends))
    rc, t, _ = O.replay(new)
    live, nk, _ = O.fold_live(new, t)
    rc0, t0, _ = O.replay(segs)
    live0, nk0, tb0 = O.fold_live(segs, t0)
    assert nk == nk0 == len(t) and live.all()
