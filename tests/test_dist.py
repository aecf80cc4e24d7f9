"""The N > 1 path on CPU: world-size-2 ``gloo`` process group.

Each rank emulates its shard of the global shot range and the ranks combine
outcome histograms with ``sharding.allreduce_histogram`` and a sampled lane
gather with ``sharding.gather_sample`` -- the same calls bench.py makes over
RCCL on GPUs -- and bench.py's batch loop itself, ``sharding.HistogramPipeline``
(double-buffered, asynchronous exchange), runs here with a CPU stand-in for the
kernel.  The per-rank emulation is oracle_fast (the checker: no GPU in this
container); the GPU kernel is pinned to it bit for bit by
tests/test_gpu_parity.py, including sharding-invariance tests at 10^6 shots.
Rank 0 checks the combined result against one unsharded run.
"""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from distributed_processor_amd import _abi, sharding, workloads
from distributed_processor_amd.emulator import ProgramSet

N_TOTAL = 1001          # odd: uneven shards
N_SAMPLE = 7
N_BATCH, N_BATCHES = 301, 5


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _workload():
    ps = ProgramSet(workloads.config3_active_reset(8))
    cfg = _abi.make_config(8, n_groups=ps.n_groups, max_cycles=50000, event_cap=16, meas_cap=4,
                           meas_latency=workloads.CONFIG3_MEAS_LATENCY, p1=0.37, seed=0xABCD)
    return ps, cfg


def _rank_main(rank, world, port, out_dir):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        ps, cfg = _workload()
        begin, n = sharding.shard_range(N_TOTAL, rank, world)
        out = oracle.fast_run(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, begin, n, threads=1,
                              want=('summary', 'hist'))
        hist = torch.from_numpy(out['hist'].astype(np.int64))
        h2 = hist.clone()
        work = sharding.allreduce_histogram(h2, async_op=True)     # the bench's overlapped form
        sharding.allreduce_histogram(hist)
        work.wait()
        assert torch.equal(h2, hist)
        lanes = sharding.sample_lanes(n, cfg.cores_per_shot, N_SAMPLE)
        sample = torch.from_numpy(out['summary'][lanes].astype(np.int64))
        gathered = sharding.gather_sample(sample)
        slowest = sharding.max_over_ranks(float(rank + 1))
        # bench.py's batch loop: batch b = global shots [b * N_BATCH, (b + 1) * N_BATCH),
        # this rank's share of it emulated by the stand-in "kernel" (oracle_fast
        # assigning the pipeline's buffer, as the GPU kernel does with hist_assign:
        # no zeroing between batches)
        pipe = sharding.HistogramPipeline(torch.zeros_like(hist), zero=False)
        for b in range(N_BATCHES):
            b0, bn = sharding.shard_range(N_BATCH, rank, world)

            def launch(h, b=b, b0=b0, bn=bn):
                o = oracle.fast_run(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, b * N_BATCH + b0, bn,
                                    threads=1, want=('hist',))
                h.copy_(torch.from_numpy(o['hist'].astype(np.int64)))
            pipe.step(launch)
        pipe.drain()
        last_two = torch.stack([pipe.bufs[(N_BATCHES - 2) % 2], pipe.result()])
        # the accumulating form (dpemu_outputs.hist_next): the stand-in kernel
        # adds into its buffer and zeroes the next batch's
        cn = sharding.HistogramPipeline(torch.full_like(hist, 3), zero=False, clear_next=True)
        for b in range(N_BATCHES):
            b0, bn = sharding.shard_range(N_BATCH, rank, world)

            def launch_cn(h, h_next, b=b, b0=b0, bn=bn):
                o = oracle.fast_run(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, b * N_BATCH + b0, bn,
                                    threads=1, want=('hist',))
                h_next.zero_()
                h.add_(torch.from_numpy(o['hist'].astype(np.int64)))
            cn.step(launch_cn)
        cn.drain()
        assert torch.equal(cn.result(), last_two[1])
        assert torch.equal(cn.bufs[(N_BATCHES - 2) % 3], last_two[0])
        if rank == 0:
            np.save(os.path.join(out_dir, 'hist.npy'), hist.numpy())
            np.save(os.path.join(out_dir, 'gathered.npy'), gathered.numpy())
            np.save(os.path.join(out_dir, 'slowest.npy'), np.array([slowest]))
            np.save(os.path.join(out_dir, 'pipeline.npy'), last_two.numpy())
    finally:
        dist.destroy_process_group()


def test_shard_range_partitions():
    for total in (0, 1, 7, 1000, 1001):
        for world in (1, 2, 3, 8):
            spans = [sharding.shard_range(total, r, world) for r in range(world)]
            assert sum(n for _, n in spans) == total
            pos = 0
            for b, n in spans:
                assert b == pos
                pos += n
            assert max(n for _, n in spans) - min(n for _, n in spans) <= 1
    assert sharding.weak_shard(10 ** 6, 3) == (3 * 10 ** 6, 10 ** 6)
    with pytest.raises(ValueError):
        sharding.shard_range(10, 2, 2)


def test_sample_lanes_whole_shots():
    lanes = sharding.sample_lanes(100, 8, 5)          # core-major lanes: L = core * 100 + shot
    assert len(lanes) == 40
    shots = lanes.reshape(5, 8) % 100
    assert (shots == shots[:, :1]).all() and len(set(shots[:, 0])) == 5
    assert (lanes.reshape(5, 8) // 100 == np.arange(8)).all()
    assert len(sharding.sample_lanes(0, 8, 5)) == 0
    sm = sharding.sample_lanes(100, 8, 5, lane_order=1)     # shot-major lanes: L = shot * 8 + core
    np.testing.assert_array_equal(sm % 8, lanes // 100)
    np.testing.assert_array_equal(sm // 8, lanes % 100)


def test_single_rank_collectives_are_identity():
    h = torch.arange(6, dtype=torch.int64)
    assert sharding.allreduce_histogram(h) is h and h.tolist() == list(range(6))
    assert sharding.allreduce_histogram(h, async_op=True) is None        # one rank: nothing to wait for
    assert sharding.gather_sample(h).shape == (1, 6)
    assert sharding.max_over_ranks(2.5) == 2.5
    with pytest.raises(TypeError):
        sharding.allreduce_histogram(torch.zeros(3, dtype=torch.int32))


def test_two_rank_gloo_matches_unsharded(tmp_path):
    world = 2
    mp.start_processes(_rank_main, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                       join=True, start_method='spawn')
    ps, cfg = _workload()
    full = oracle.fast_run(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, 0, N_TOTAL, threads=2,
                           want=('summary', 'hist'))
    hist = np.load(tmp_path / 'hist.npy')
    assert hist.sum() == N_TOTAL
    np.testing.assert_array_equal(hist, full['hist'].astype(np.int64))
    gathered = np.load(tmp_path / 'gathered.npy')
    assert gathered.shape == (world, N_SAMPLE * 8, 8)
    for r in range(world):
        begin, n = sharding.shard_range(N_TOTAL, r, world)
        loc = sharding.sample_lanes(n, 8, N_SAMPLE)
        lanes = (loc // n) * N_TOTAL + begin + loc % n          # the same (shot, core) in the unsharded run
        np.testing.assert_array_equal(gathered[r], full['summary'][lanes].astype(np.int64))
    assert float(np.load(tmp_path / 'slowest.npy')[0]) == float(world)
    # the pipeline's last two batches, summed over ranks = the unsharded batches
    last_two = np.load(tmp_path / 'pipeline.npy')
    for j, b in enumerate((N_BATCHES - 2, N_BATCHES - 1)):
        ref = oracle.fast_run(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, b * N_BATCH, N_BATCH, threads=2,
                              want=('hist',))['hist'].astype(np.int64)
        np.testing.assert_array_equal(last_two[j], ref)


def test_pipeline_single_rank_and_buffer_reuse():
    """one rank: the pipeline is the plain batch loop; a buffer is zeroed
    before its reuse, so every batch's histogram is that batch alone"""
    h = torch.zeros(4, dtype=torch.int64)
    pipe = sharding.HistogramPipeline(h, n_buffers=2)
    for b in range(5):
        pipe.step(lambda t, b=b: t.add_(b + 1))
    pipe.drain()
    assert pipe.result().tolist() == [5] * 4 and pipe.bufs[1 - (5 - 1) % 2].tolist() == [4] * 4
    with pytest.raises(RuntimeError):
        sharding.HistogramPipeline(h).result()


def test_pipeline_assigning_launch_skips_zeroing():
    """zero=False: the launch assigns the buffer (hist_assign), the pipeline
    launches nothing else; an accumulating launch would then see old counts"""
    h = torch.full((4,), 99, dtype=torch.int64)
    pipe = sharding.HistogramPipeline(h, n_buffers=2, zero=False)
    for b in range(5):
        pipe.step(lambda t, b=b: t.fill_(b + 1))
    pipe.drain()
    assert pipe.result().tolist() == [5] * 4 and pipe.bufs[1 - (5 - 1) % 2].tolist() == [4] * 4
    acc = sharding.HistogramPipeline(torch.full((2,), 7, dtype=torch.int64), n_buffers=1, zero=False)
    acc.step(lambda t: t.add_(1))
    assert acc.result().tolist() == [8, 8]


def test_pipeline_clear_next_rotation():
    """clear_next: three buffers; batch k's launch gets batch k + 1's buffer
    to zero and accumulates into its own, which batch k - 1 zeroed (batch 0's
    the pipeline zeroes once)"""
    h = torch.full((4,), 99, dtype=torch.int64)
    pipe = sharding.HistogramPipeline(h, zero=False, clear_next=True)
    assert len(pipe.bufs) == 3 and h.tolist() == [0] * 4
    seen = []

    def launch(t, nxt, b):
        assert t.tolist() == [0] * 4 and nxt is not t
        seen.append((t.data_ptr(), nxt.data_ptr()))
        nxt.zero_()                      # as the kernel does (hist_next)
        t.add_(b + 1)
    for b in range(7):
        pipe.step(lambda t, nxt, b=b: launch(t, nxt, b))
    pipe.drain()
    assert pipe.result().tolist() == [7] * 4 and pipe.bufs[(7 - 2) % 3].tolist() == [6] * 4
    ptrs = [x.data_ptr() for x in pipe.bufs]
    assert seen == [(ptrs[k % 3], ptrs[(k + 1) % 3]) for k in range(7)]
    with pytest.raises(ValueError):
        sharding.HistogramPipeline(h, clear_next=True)          # zero=True would add a launch back


def _settle_main(rank, world, port, out_dir):
    """bench.settle on both ranks with a step that enqueues a collective and
    runs at a different speed per rank: the ranks must agree on the step count
    (a mismatch deadlocks the collectives, as an uneven wall-time loop did)"""
    import sys
    import time
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        import bench
        t = torch.zeros(1)
        count = [0]

        def step():
            time.sleep(0.002 * (rank + 1))
            dist.all_reduce(t)
            count[0] += 1
        n = bench.settle(step, lambda: None, seconds=0.1, sync=lambda: None, device='cpu')
        dist.barrier()
        np.save(os.path.join(out_dir, 'settle{}.npy'.format(rank)), np.array([n, count[0]]))
    finally:
        dist.destroy_process_group()


def test_bench_settle_same_step_count_on_every_rank(tmp_path):
    world = 2
    mp.start_processes(_settle_main, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                       join=True, start_method='spawn')
    got = [np.load(tmp_path / 'settle{}.npy'.format(r)) for r in range(world)]
    assert got[0][0] == got[1][0] == got[0][1] == got[1][1] > 3
