"""Multi-GPU replay by sharding segments.

Segments are independent parse units (framing never crosses files, engine.rs:80-85), so the
store's segment list — sorted by id as engine.rs:51 sorts it — is dealt round-robin to the GPUs
(segment i -> GPU i mod N).  Each GPU replays its shard with no collective on the data path; the
host gathers the per-GPU tuple arrays and merges them back into (segment, offset) order, which is
the order engine.rs:55-57 applies records in.  The first error of the whole store is the minimum
(segment, offset) error over the shards: a shard that fails at segment i says nothing about the
segments other shards replayed after i, and engine.rs:56 would have stopped at i.

Works with one process driving several contexts (ShardedReplay) or one process per GPU
(torch.distributed, any backend: gather_shards()).

Compaction of a sharded store (compact_sharded) is the one step with a real exchange: a key's
last writer may sit on another rank.  Each rank folds its shard locally and sends every key's
local last record (a candidate: global position + key bytes) to the key's owner rank
(hash(key) mod N) with an all-to-all; owners keep the largest position per key and answer with
one flag per candidate through a second all-to-all; each rank then writes out its winners that
are SETs.  Over RCCL (backend "nccl") the buffers are device tensors.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import CORRUPTED, OK, TUPLE_DTYPE, Context


def shard_round_robin(n_segments: int, world: int, rank: int) -> list[int]:
    """Global segment indices owned by `rank` (segment i -> rank i mod world)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    return list(range(rank, n_segments, world))


@dataclass
class ShardResult:
    """One shard's replay: tuples with seg_idx already mapped to the GLOBAL segment index."""
    status: int
    tuples: np.ndarray
    error: tuple | None          # (kind, global seg_idx, rec_off, aux) when status == CORRUPTED


def localize(global_idx: list[int], status: int, tuples, error) -> ShardResult:
    """Map a shard's local seg_idx (index into its own segment list) back to global indices."""
    gmap = np.asarray(global_idx, dtype=np.uint32)
    t = np.array(tuples if tuples is not None else np.zeros(0, TUPLE_DTYPE), dtype=TUPLE_DTYPE, copy=True)
    if len(t):
        t["seg_idx"] = gmap[t["seg_idx"]]
    err = None
    if status == CORRUPTED and error is not None:
        kind, seg, off, aux = error
        err = (int(kind), int(gmap[seg]), int(off), int(aux))
    return ShardResult(status, t, err)


def merge_shards(parts: list[ShardResult]) -> tuple[int, np.ndarray, tuple | None]:
    """Merge shard results into the single-GPU answer: (status, tuples in (seg, off) order, error)."""
    errs = [p.error for p in parts if p.status == CORRUPTED and p.error is not None]
    if errs:
        first = min(errs, key=lambda e: (e[1], e[2]))
        return CORRUPTED, np.zeros(0, TUPLE_DTYPE), first
    for p in parts:
        if p.status != OK:
            raise RuntimeError(f"shard failed with status {p.status}")
    allt = np.concatenate([p.tuples for p in parts]) if parts else np.zeros(0, TUPLE_DTYPE)
    order = np.lexsort((allt["rec_off"], allt["seg_idx"]))
    return OK, allt[order], None


def gather_shards(local: ShardResult, group=None) -> list[ShardResult] | None:
    """Gather every rank's ShardResult on rank 0 over torch.distributed (host objects; any backend).
    Returns the list on rank 0 and None elsewhere."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    payload = (local.status, local.tuples.tobytes(), local.error)
    out = [None] * world if rank == 0 else None
    dist.gather_object(payload, out, dst=0, group=group)
    if rank != 0:
        return None
    return [ShardResult(s, np.frombuffer(b, dtype=TUPLE_DTYPE).copy(), e) for s, b, e in out]


class ShardedReplay:
    """Replay a store's segments over several GPUs from one process (one Context per device)."""

    def __init__(self, devices: list[int] | None = None, contexts: list[Context] | None = None):
        if contexts is None:
            contexts = [Context(d) for d in (devices or [0])]
        self.ctxs = contexts

    def replay(self, segments, seg_ids=None, expected=None, on_device=False):
        """Same contract as Context.replay over the whole (sorted) segment list."""
        n = len(segments)
        world = len(self.ctxs)
        exp_parts = _split_expected(segments, expected, world) if expected is not None else [None] * world
        def one(r):
            idx = shard_round_robin(n, world, r)
            if not idx:
                return None
            res = self.ctxs[r].replay([segments[i] for i in idx],
                                      seg_ids=None if seg_ids is None else [seg_ids[i] for i in idx],
                                      expected=exp_parts[r], on_device=on_device)
            e = res.error
            err = (e.kind, e.seg_idx, e.rec_off, e.aux) if (res.status == CORRUPTED and e is not None) else None
            return localize(idx, res.status, res.tuples if res.status == OK else None, err)

        # one host thread per context: the native calls release the GIL, so the GPUs run concurrently
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(max_workers=world) as ex:
            parts = [p for p in ex.map(one, range(world)) if p is not None]
        return merge_shards(parts)


def _split_expected(segments, expected, world):
    """The manifest is in global tuple order; shard it by record counts per segment (the caller
    supplies per-segment record counts as expected = (crcs, counts))."""
    crcs, counts = expected
    starts = np.concatenate([[0], np.cumsum(counts)])
    out = []
    for r in range(world):
        idx = shard_round_robin(len(segments), world, r)
        out.append(np.concatenate([crcs[starts[i]:starts[i + 1]] for i in idx]) if idx else None)
    return out


def max_over_ranks(x: float, group=None) -> float:
    """Whole-job time = the slowest rank's (bench.py contract); works on gloo (CPU) and nccl."""
    import torch
    import torch.distributed as dist
    dev = "cuda" if dist.get_backend(group) == "nccl" else "cpu"
    t = torch.tensor([float(x)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


class DeviceCompactEngine:
    """kvr_compact_stage / _export / _resolve / _finish on one Context (device buffers)."""

    def __init__(self, ctx: Context, device):
        self.ctx, self.device = ctx, device

    def stage(self, segments, gidx, n_ranks, on_device=False):
        import torch
        counts, kb = self.ctx.compact_stage(segments, gidx, n_ranks, on_device=on_device)
        from . import CAND_BYTES
        hdr = torch.empty(max(int(counts.sum()) * CAND_BYTES, 1), dtype=torch.uint8, device=self.device)
        keys = torch.empty(max(int(kb.sum()), 1), dtype=torch.uint8, device=self.device)
        self.ctx.compact_export(hdr.data_ptr(), keys.data_ptr())
        return counts, kb, hdr[: int(counts.sum()) * CAND_BYTES], keys[: int(kb.sum())]

    def resolve(self, hdr, keys, hdr_counts, key_counts):
        import torch
        win = torch.zeros(max(int(np.sum(hdr_counts)), 1), dtype=torch.uint8, device=self.device)
        self.ctx.compact_resolve(hdr.data_ptr() if hdr.numel() else 0, keys.data_ptr() if keys.numel() else 0,
                                 hdr_counts, key_counts, win.data_ptr())
        return win[: int(np.sum(hdr_counts))]

    def finish(self, win, seg_target):
        return self.ctx.compact_finish(win.data_ptr() if win.numel() else 0, seg_target)


def _a2a(out, inp, out_splits, in_splits, group):
    import torch.distributed as dist
    dist.all_to_all_single(out, inp, [int(x) for x in out_splits], [int(x) for x in in_splits], group=group)


def compact_sharded(engine, segments, gidx, seg_target=0, group=None, on_device=False):
    """This rank's share of the compaction of a sharded store (every rank calls it): returns the
    live records this rank holds, as new segment bytes and their end offsets.  engine provides
    stage / resolve / finish (DeviceCompactEngine on GPUs; the CPU tests bring a host one)."""
    import torch
    import torch.distributed as dist
    from . import CAND_BYTES
    world = dist.get_world_size(group)
    counts, kb, hdr, keys = engine.stage(segments, gidx, world, on_device=on_device)
    dev = hdr.device
    # 1. how much each rank sends each other rank
    mine = torch.tensor(np.stack([counts, kb], axis=1).reshape(-1), dtype=torch.int64, device=dev)
    theirs = torch.empty_like(mine)
    _a2a(theirs, mine, [2] * world, [2] * world, group)
    th = theirs.cpu().numpy().reshape(world, 2)
    rc_counts, rc_keys = th[:, 0], th[:, 1]
    # 2. candidates to their owners (exact sizes: the splits must add up to the tensors)
    hdr_in = torch.empty(int(rc_counts.sum()) * CAND_BYTES, dtype=torch.uint8, device=dev)
    keys_in = torch.empty(int(rc_keys.sum()), dtype=torch.uint8, device=dev)
    _a2a(hdr_in, hdr, rc_counts * CAND_BYTES, counts * CAND_BYTES, group)
    _a2a(keys_in, keys, rc_keys, kb, group)
    # 3. owners decide; the answers go back in the senders' order
    win_in = engine.resolve(hdr_in, keys_in, rc_counts, rc_keys)
    win_mine = torch.zeros(int(counts.sum()), dtype=torch.uint8, device=dev)
    _a2a(win_mine, win_in, counts, rc_counts, group)
    return engine.finish(win_mine, seg_target)
