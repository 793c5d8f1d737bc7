"""GPU parity of the streamed ingest (kvr_replay_stream) against the CPU oracle.

The batching (segments grouped into HBM slots, batch b+1 copied while batch b replays) must be
invisible: the tuples, the seg_idx numbering, the expected-CRC verification and the first error
equal the oracle's replay of the same segments (engine.rs:55-57 in segment order), for pageable
callers (library staging) and pinned ones (direct DMA).
"""
import numpy as np
import pytest

import kvreplay as K
import oracle_py as O

pytestmark = pytest.mark.gpu


def _segments(spec, n):
    gen = [K.gen_segment_cpu(spec, s) for s in range(n)]
    return [g[0] for g in gen], np.concatenate([g[1] for g in gen])


def _check(rs, ro):
    assert rs.status == ro[0], (rs.status, ro[0])
    if ro[0] == 0:
        assert rs.n == len(ro[1])
        assert np.array_equal(rs.tuples, ro[1]), "streamed tuples differ from the oracle"
    else:
        eo, eg = ro[2], rs.error
        assert (eg.kind, eg.seg_idx, eg.rec_off, eg.aux) == (eo.kind, eo.seg_idx, eo.rec_off, eo.aux)


# batch sizes: one segment per batch, several per batch, everything in one batch, and a size
# below every segment (each segment becomes its own oversized batch)
@pytest.mark.parametrize("batch", [300_000, 1_000_000, 1 << 30, 4096])
def test_stream_matches_oracle(gctx, batch):
    spec = K.GenSpec(seed=81, seg_bytes=300_000, val_min=16, val_max=9000, del_permille=200,
                     flip_per_million=20_000)
    segs, exp = _segments(spec, 7)
    segs.insert(3, np.zeros(0, dtype=np.uint8))   # an empty segment inside a batch
    ro = O.replay(segs, expected=exp)
    rs = gctx.replay_stream(segs, expected=exp, batch_bytes=batch)
    _check(rs, ro)
    assert rs.stream_stats.n_records == len(ro[1])
    assert rs.stream_stats.bytes_in == sum(len(s) for s in segs)
    assert int(np.count_nonzero(rs.tuples["flags"] & K.TF_CRC_FAIL)) > 0   # the flips were seen
    # identical to the one-call replay of the same bytes
    rg = gctx.replay(segs, expected=exp)
    assert np.array_equal(rg.tuples, rs.tuples)


def test_stream_pinned_host_buffers(gctx):
    torch = pytest.importorskip("torch")
    spec = K.GenSpec(seed=82, seg_bytes=1 << 20, val_min=1024, val_max=1024, del_permille=100)
    segs, exp = _segments(spec, 6)
    pinned = []
    for s in segs:
        t = torch.empty(len(s), dtype=torch.uint8, pin_memory=True)
        t.numpy()[:] = s
        pinned.append(t)
    ro = O.replay(segs, expected=exp)
    rs = gctx.replay_stream([(t.data_ptr(), t.numel()) for t in pinned], expected=exp,
                            batch_bytes=2 << 20, pinned=True)
    _check(rs, ro)
    assert rs.stream_stats.n_batches == 3


@pytest.mark.parametrize("where", [0, 4, 6])
def test_stream_first_error_in_later_batch(gctx, where):
    spec = K.GenSpec(seed=83, seg_bytes=200_000, val_min=16, val_max=4000, del_permille=100)
    segs, _ = _segments(spec, 7)
    segs[where] = segs[where][:-3]   # a truncated tail: the first error is in segment `where`
    if where < 6:
        segs[6] = segs[6][:-1]       # a later error that must not be reported
    ro = O.replay(segs)
    rs = gctx.replay_stream(segs, batch_bytes=450_000)
    _check(rs, ro)
    assert rs.error.seg_idx == where


def test_stream_capacity_retry_and_seg_ids(gctx):
    spec = K.GenSpec(seed=84, seg_bytes=250_000, val_min=0, val_max=64, del_permille=300)
    segs, _ = _segments(spec, 5)
    ids = [3, 9, 10, 44, 100]
    ro = O.replay(segs, seg_ids=ids)
    rs = gctx.replay_stream(segs, seg_ids=ids, cap=100, batch_bytes=260_000)   # forces KVR_CAPACITY first
    _check(rs, ro)


def test_stream_empty(gctx):
    rs = gctx.replay_stream([])
    assert rs.status == 0 and rs.n == 0
