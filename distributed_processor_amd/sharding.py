"""Multi-GPU sharding of emulated shots.

Shots are independent units: a shot's C cores interact only through fproc
and sync, which live inside one wavefront (csrc/interp.hip).  So N ranks --
one process per GPU, ``torch.distributed`` over RCCL/xGMI -- split the
global shot range with no exchange on the data path.  Every random counter
is keyed by the *global* shot index (Philox ctr = shot, core, m), so a shard
produces exactly the lanes the single-GPU run would, for any N.

The path's only collective is the outcome histogram: ``all_reduce(SUM)`` of
an int64 [n_groups, 2^C] tensor (100 x 256 x 8 B = 200 KB at config 2).  An
optional validation gather brings a fixed-size sample of lanes (summaries or
event slots) to every rank with ``all_gather`` -- equal-size tensors, so one
RCCL ring call rather than per-rank send/recv.

Nothing here depends on the backend: the same calls run under ``gloo`` on
CPU tensors (tests/test_dist.py) and ``nccl`` (= RCCL on ROCm) on GPU.
"""

from __future__ import annotations

from typing import Tuple

import numpy as np


def shard_range(n_total: int, rank: int, world: int) -> Tuple[int, int]:
    """(shot_begin, n_shots) of ``rank`` for strong scaling: contiguous
    blocks, the first ``n_total % world`` ranks one shot longer."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError('rank {} outside world {}'.format(rank, world))
    if n_total < 0:
        raise ValueError('n_total must be >= 0')
    q, r = divmod(int(n_total), int(world))
    begin = rank * q + min(rank, r)
    return begin, q + (1 if rank < r else 0)


def weak_shard(shots_per_rank: int, rank: int) -> Tuple[int, int]:
    """(shot_begin, n_shots) for weak scaling: every rank runs the same
    number of shots, rank r owning global shots [r*n, (r+1)*n)."""
    return int(rank) * int(shots_per_rank), int(shots_per_rank)


def _dist():
    import torch.distributed as dist
    return dist if dist.is_available() and dist.is_initialized() else None


def world_size(group=None) -> int:
    dist = _dist()
    return dist.get_world_size(group) if dist is not None else 1


def allreduce_histogram(hist, group=None, async_op=False):
    """Sum the int64 outcome histogram over ranks, in place (no-op on one
    rank).  ``hist``: torch.int64 tensor on the backend's device.  With
    ``async_op`` the collective is only enqueued (on RCCL's stream, after the
    work already queued on the current stream) and its work handle returned
    (None on one rank): ``handle.wait()`` orders later work on the current
    stream after it, so the exchange of one batch overlaps the next batch's
    kernel."""
    import torch
    if hist.dtype != torch.int64:
        raise TypeError('histogram must be int64, got {}'.format(hist.dtype))
    if world_size(group) > 1:
        dist = _dist()
        work = dist.all_reduce(hist, op=dist.ReduceOp.SUM, group=group, async_op=async_op)
        return work if async_op else hist
    return None if async_op else hist


class HistogramPipeline:
    """Per-batch launches with the histogram exchange overlapped (bench.py).

    Batch k's kernel writes its outcome histogram into buffer k % n_buffers;
    the buffer's all-reduce is enqueued asynchronously right after the launch
    (on RCCL's stream, ordered after the kernel), so batch k's exchange runs
    while batch k + 1's kernel does.  Before a buffer is reused, the exchange
    that last used it is waited for; it is then zeroed, unless ``zero`` is
    False because the launch assigns the histogram (dpemu_config.hist_assign:
    the library's reduce kernel stores the counts, one launch fewer per batch).
    ``clear_next``: the launch is ``launch(hist, hist_next)`` and its kernel
    zeroes ``hist_next`` (dpemu_outputs.hist_next), the buffer of batch k + 1,
    in passing -- accumulating runs with no zeroing launch at all.  That needs
    three buffers: batch k's kernel clears the buffer batch k - 2 exchanged
    (waited for first), while batch k - 1's exchange may still run.
    ``drain()`` waits for every pending exchange; ``result()`` is then the
    histogram of the last batch, summed over ranks.  One rank: no
    collectives, the same call sequence.
    """

    def __init__(self, hist, n_buffers=2, group=None, zero=True, clear_next=False):
        import torch
        if n_buffers < 1:
            raise ValueError('n_buffers must be >= 1')
        if clear_next:
            if zero:
                raise ValueError('clear_next: the kernels zero the buffers (zero=False)')
            n_buffers = max(n_buffers, 3)
            hist.zero_()                              # batch 0's buffer; later ones the kernels clear
        self.bufs = [hist] + [torch.zeros_like(hist) for _ in range(n_buffers - 1)]
        self.pending = [None] * n_buffers
        self.group = group
        self.zero = zero
        self.clear_next = clear_next
        self.k = 0

    def _wait(self, b):
        if self.pending[b] is not None:
            self.pending[b].wait()                    # this buffer's previous exchange is done
            self.pending[b] = None

    def step(self, launch):
        """launch(hist) (clear_next: launch(hist, hist_next)): enqueue one
        batch writing into (accumulating on) hist"""
        n = len(self.bufs)
        b = self.k % n
        self.k += 1
        self._wait(b)
        h = self.bufs[b]
        if self.clear_next:
            nb = (b + 1) % n
            self._wait(nb)                            # the kernel is about to zero it
            launch(h, self.bufs[nb])
        else:
            if self.zero:
                h.zero_()
            launch(h)
        self.pending[b] = allreduce_histogram(h, group=self.group, async_op=True)
        return h

    def drain(self):
        for b, w in enumerate(self.pending):
            if w is not None:
                w.wait()
                self.pending[b] = None

    def result(self):
        """the last batch's rank-summed histogram (after drain)"""
        if self.k == 0:
            raise RuntimeError('no batch has run')
        return self.bufs[(self.k - 1) % len(self.bufs)]


def gather_sample(t, group=None):
    """Every rank's equal-shape tensor ``t`` stacked along a new leading rank
    axis (one all_gather).  Collects a sampled subset of lanes' timelines or
    summaries for validation."""
    import torch
    if world_size(group) == 1:
        return t.unsqueeze(0)
    dist = _dist()
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size(group))]
    dist.all_gather(parts, t.contiguous(), group=group)
    return torch.stack(parts)


def max_over_ranks(value: float, device=None, group=None) -> float:
    """The largest ``value`` of any rank (bench timing: the job ends when the
    slowest rank ends)."""
    import torch
    if world_size(group) == 1:
        return float(value)
    dist = _dist()
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def sample_lanes(n_shots: int, cores_per_shot: int, n_sample: int, lane_order: int = 0) -> np.ndarray:
    """Local lane indices of ``n_sample`` whole shots spread evenly over a
    shard of ``n_shots`` (every core of each chosen shot, in the run's lane
    order: core-major L = core * n_shots + shot, or shot-major
    L = shot * C + core), ordered shot by shot.  The same count on every
    rank keeps gather_sample's tensors equal-shaped."""
    if n_shots <= 0 or n_sample <= 0:
        return np.zeros(0, np.int64)
    k = min(int(n_sample), int(n_shots))
    shots = (np.arange(k, dtype=np.int64) * n_shots) // k
    cores = np.arange(cores_per_shot, dtype=np.int64)[None, :]
    if lane_order == 1:                                  # _abi.LANES_SHOT_MAJOR
        return (shots[:, None] * int(cores_per_shot) + cores).reshape(-1)
    return (cores * int(n_shots) + shots[:, None]).reshape(-1)
