"""BASELINE configs at their stated per-GPU sizes, the whole launch against
the oracle (config 4 at full size: tests/test_gpu_rb.py).

* config 2 (BASELINE configs[1]): 8-core Ramsey, 100 delay points, 10^6
  shots on one GPU -- every output array of the bench's launch (summaries,
  events, measurements, histogram) equal to oracle_fast over the same 10^6
  shots, bit for bit;
* config 3 (configs[2]): active reset, 10^7 shots over 8 GPUs = 1.25 * 10^6
  shots per GPU -- rank 0's and rank 7's shards (global shot offsets, the
  RNG keyed by global shot index) each equal to oracle_fast in full, and the
  eight shards' histograms (two of them run) consistent with the outcome law;
* configs 2 and 3 also in the bench's own launch shape: shot-major lanes
  (DPEMU_LANES_SHOT_MAJOR); config 2 accumulating while it clears the next
  run's histogram (dpemu_outputs.hist_next), config 3 with hist_assign;
* config 5 (configs[4]): DDS of 128 RB timelines x 16 channels at 16
  samples / clock, the bench's full-size launch (2048 channels x 209,952
  samples): every channel over its whole length equal to oracle_dds (in
  chunks of 256 channels).

oracle_fast / oracle_dds run with the job's CPU share (OMP_NUM_THREADS, 16
on the GPU box)."""

import os

import numpy as np
import pytest

import oracle
from distributed_processor_amd import _abi, workloads
from distributed_processor_amd.dds import ChannelPlan
from distributed_processor_amd.emulator import Emulator, ProgramSet, alloc_device_outputs

pytestmark = pytest.mark.gpu

THREADS = int(os.environ.get('OMP_NUM_THREADS', '0') or 0) or min(16, os.cpu_count() or 1)


@pytest.fixture(scope='module')
def emu():
    e = Emulator(0)
    yield e
    e.close()


def run_full(emu, ps, cfg, n, shot0, want, clear_next=False):
    import torch
    emu.load(ps)
    out = alloc_device_outputs(cfg, n, want=want)
    if clear_next:
        out['hist_next'] = torch.full_like(out['hist'], 0x5A5A5A5A)
    for k, t in out.items():
        if k == 'hist_next':
            continue
        if k == 'hist' and cfg.hist_assign:
            t.fill_(0x5A5A5A5A)   # hist_assign overwrites: stale counts must not survive
        else:
            t.zero_()                 # slots past a lane's count stay 0, as in the oracle's arrays
    emu.run_device(cfg, n, shot0, out)
    torch.cuda.synchronize()
    g = {k: v.cpu().numpy() for k, v in out.items()}
    if clear_next:
        assert not g.pop('hist_next').any(), 'hist_next not cleared'
    del out
    torch.cuda.empty_cache()
    f = oracle.fast_run(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, shot0, n, threads=THREADS, want=want)
    for k in want:
        a = g[k].view(f[k].dtype).reshape(f[k].shape)
        if not np.array_equal(a, f[k]):
            bad = np.argwhere(a != f[k])
            raise AssertionError('{}: {} mismatches, first at {}'.format(k, len(bad), bad[0].tolist()))
    return g


BENCH_SHAPE = dict(lane_order=_abi.LANES_SHOT_MAJOR, hist_assign=True)


@pytest.mark.parametrize('bench_shape', [False, True], ids=['core_major', 'bench_shape'])
def test_config2_full_launch_bit_exact(emu, bench_shape):
    ps = ProgramSet(workloads.config2_ramsey(n_cores=8, n_points=100))
    cfg = _abi.make_config(8, n_groups=ps.n_groups, max_cycles=1 << 20, event_cap=8, trace_cap=0, meas_cap=2,
                           meas_latency=64, seed=0x5EED, p1=0.5,
                           lane_order=_abi.LANES_SHOT_MAJOR if bench_shape else _abi.LANES_CORE_MAJOR)
    n = 10 ** 6
    g = run_full(emu, ps, cfg, n, 0, ('summary', 'events', 'meas', 'hist'), clear_next=bench_shape)
    s = _abi.unpack_summary(g['summary'].view(np.uint32))
    assert (s['status'] == _abi.ST_DONE).all() and (s['flags'] == 0).all()
    assert int(g['hist'].sum()) == n


@pytest.mark.parametrize('rank,shape', [(0, {}), (7, BENCH_SHAPE)], ids=['rank0_core_major', 'rank7_bench_shape'])
def test_config3_shard_bit_exact(emu, rank, shape):
    ps = ProgramSet(workloads.config3_active_reset(8))
    cfg = _abi.make_config(8, n_groups=ps.n_groups, max_cycles=50000, event_cap=16, trace_cap=0, meas_cap=4,
                           meas_latency=workloads.CONFIG3_MEAS_LATENCY, seed=0x5EED, p1=0.5, **shape)
    n = 1250000
    g = run_full(emu, ps, cfg, n, rank * n, ('summary', 'events', 'meas', 'hist'))
    s = _abi.unpack_summary(g['summary'].view(np.uint32))
    assert (s['status'] == _abi.ST_DONE).all()
    assert int(g['hist'].sum()) == n
    # the conditional X180 pair ran exactly where the first outcome was 1
    flip = (s['meas_bits'] & 1).astype(bool)
    assert (s['n_events'][flip] == s['n_events'][~flip].min() + 2).all()
    assert abs(flip.mean() - 0.5) < 0.01


def config5_timelines(emu, workload='rb2q'):
    """the bench's config-5 inputs: 128 8-core RB timelines (depth 200) on the
    device -- two-qubit Clifford RB on four qubit pairs (the bench default,
    ~560-720 drive strobes per lane: the dense-channel LDS plan) or the
    RB-shaped generator (the 20-KiB plan) -- the 2048-channel plan and the
    sample count"""
    import torch
    n_seq = 128
    if workload == 'rb2q':
        ps = workloads.config4_rb2q_set(n_seq, 200, n_cores=8)
    else:
        ps = ProgramSet(workloads.config4_rb(n_seq=n_seq, depth=200, n_cores=8))
    ops = ps.words[:, 3] >> 28
    strobes = np.add.reduceat(((ops == 0x9) | (ops == 0xB)).astype(np.int64), ps.offsets.astype(np.int64))
    cfg = _abi.make_config(8, n_groups=ps.n_groups, max_cycles=1 << 20, event_cap=max(512, int(strobes.max()) + 1),
                           meas_cap=4, meas_latency=64, seed=0x5EED)
    emu.load(ps)
    ev = alloc_device_outputs(cfg, n_seq, want=('summary', 'events'))
    ev['events'].zero_()
    emu.run_device(cfg, n_seq, 0, ev)
    torch.cuda.synchronize()
    n_samples = ((int(ev['summary'][:, 0].max().item()) + 8) * 16 + 3) // 4 * 4
    params = {i: (e['samples_per_clk'], e['interp_ratio']) for i, e in enumerate(workloads.ELEMS)}
    chans = [(q, c, e) for q in range(n_seq) for c in range(8) for e in (workloads.QDRV, workloads.RDRV)]
    plan = ChannelPlan(ps, cfg, 0, n_seq, chans, params)
    assert plan.n_channels == 2048 and n_samples > 200000
    return cfg, ev, plan, n_samples


@pytest.mark.parametrize('workload', ['rb2q', 'rb'])
def test_config5_full_launch_all_channels(emu, workload):
    import torch
    cfg, ev, plan, n_samples = config5_timelines(emu, workload)
    iq = emu.synthesize(plan, ev, n_samples)
    torch.cuda.synchronize()
    summ, events = ev['summary'].cpu().numpy(), ev['events'].cpu().numpy()
    plays = np.zeros(plan.n_channels, bool)
    CH = 256
    for c0 in range(0, plan.n_channels, CH):
        got = iq[c0:c0 + CH].cpu().numpy().view(np.uint32)
        ref = oracle.dds(plan.desc[c0:c0 + CH], summ, events, plan.env, plan.freq, n_samples, cfg.event_cap,
                         threads=THREADS)
        if not np.array_equal(got, ref):
            bad = np.argwhere(got != ref)
            raise AssertionError('{} mismatching samples, first at channel {} sample {}'.format(
                len(bad), c0 + int(bad[0][0]), int(bad[0][1])))
        plays[c0:c0 + CH] = (ref != 0).any(axis=1)
    assert plays.all()                                   # every qdrv and rdrv channel plays


@pytest.mark.parametrize('shape', [{}, BENCH_SHAPE], ids=['core_major', 'bench_shape'])
def test_config3_lut_full_shard_bit_exact(emu, shape):
    """config 3 through the fproc_lut back end (workloads.config3_lut: every
    core waits on the syndrome LUT, hdl/fproc_lut.sv) at the per-GPU shard
    size, rank 3's shard: branch_kernel with the LUT FSM, every output equal
    to oracle_fast"""
    ps = ProgramSet(workloads.config3_lut(8))
    cfg = _abi.make_config(8, n_groups=ps.n_groups, max_cycles=50000, event_cap=16, trace_cap=0, meas_cap=4,
                           fproc_mode=_abi.FPROC_LUT, meas_latency=workloads.CONFIG3_MEAS_LATENCY, lut_mask=0xFF,
                           lut_table=workloads.config3_lut_table(8), seed=0x5EED, p1=0.5, **shape)
    n = 1250000
    g = run_full(emu, ps, cfg, n, 3 * n, ('summary', 'events', 'meas', 'hist'))
    assert emu.last_kernel().startswith('branch_kernel<'), emu.last_kernel()
    s = _abi.unpack_summary(g['summary'].view(np.uint32))
    assert (s['status'] == _abi.ST_DONE).all()
    assert int(g['hist'].sum()) == n


def test_config3_cross_core_reads_full_shard(emu):
    """config 3 with every core conditioning on ANOTHER core's outcome
    (fproc_meas id = (c + 3) % 8: the cross-lane lookup through LDS of
    branch_kernel), rank 5's 1.25 * 10^6-shot shard in the bench's launch
    shape, every output equal to oracle_fast; the X90 pair ran exactly where
    the read core's first outcome was 1"""
    ps = ProgramSet(workloads.config3_active_reset(8, read_shift=3))
    cfg = _abi.make_config(8, n_groups=ps.n_groups, max_cycles=50000, event_cap=16, trace_cap=0, meas_cap=4,
                           meas_latency=workloads.CONFIG3_MEAS_LATENCY, seed=0x5EED, p1=0.5, **BENCH_SHAPE)
    n = 1250000
    g = run_full(emu, ps, cfg, n, 5 * n, ('summary', 'events', 'meas', 'hist'))
    assert emu.last_kernel().startswith('branch_kernel<'), emu.last_kernel()
    s = _abi.unpack_summary(g['summary'].view(np.uint32))
    assert (s['status'] == _abi.ST_DONE).all()
    first = (s['meas_bits'] & 1).astype(bool).reshape(n, 8)        # shot-major lanes
    flip = np.roll(first, -3, axis=1)                              # core c reads core (c + 3) % 8
    ne = s['n_events'].reshape(n, 8)
    assert (ne[flip] == ne[~flip].min() + 2).all()



def test_config3_eight_shards_equal_one_launch(emu):
    """config 3 at its stated total, 10^7 shots x 8 cores (BASELINE configs[2]):
    the eight 1.25 * 10^6-shot shards that eight GPUs would run (global shot
    offsets, bench launch shape) sum to the histogram of ONE 10^7-shot launch,
    and that histogram equals oracle_fast's over the same 10^7 shots"""
    import torch
    ps = ProgramSet(workloads.config3_active_reset(8))
    cfg = _abi.make_config(8, n_groups=ps.n_groups, max_cycles=50000, event_cap=16, trace_cap=0, meas_cap=4,
                           meas_latency=workloads.CONFIG3_MEAS_LATENCY, seed=0x5EED, p1=0.5, **BENCH_SHAPE)
    emu.load(ps)
    n, G = 1250000, 8
    out = alloc_device_outputs(cfg, n * G, want=('hist',))
    emu.run_device(cfg, n * G, 0, out)
    full = out['hist'].clone()
    total = torch.zeros_like(full)
    for r in range(G):
        emu.run_device(cfg, n, r * n, out)
        total += out['hist']
    torch.cuda.synchronize()
    assert torch.equal(total, full)
    assert int(full.sum().item()) == n * G
    f = oracle.fast_run(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, 0, n * G, threads=THREADS, want=('hist',))
    assert np.array_equal(full.cpu().numpy().view(f['hist'].dtype).reshape(f['hist'].shape), f['hist'])
