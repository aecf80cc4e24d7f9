"""The readout demodulation model (meas_model DEMOD, include/dpemu.h) on the
GPU through the C ABI, bit for bit against oracle_fast (itself pinned to the
per-clock oracle_rtl, tests/test_fast_vs_rtl.py::test_fuzz_demod_model, and
to float math, tests/test_demod.py):

* fuzzed programs (jumps, fproc_meas / fproc_lut, sync, register programs,
  pulse-only programs) with random drive / LO elements, windows, delays,
  discriminators and per-program frequency tables, every output array
  including the accumulated {I, Q} (dpemu_outputs.acc), on branch_kernel<DEMOD>
  and on the general interpreter;
* config 3 (active reset) with the demodulation model at the per-GPU shard
  size, 1.25 * 10^6 shots x 8 cores, in both lane orders;
* the physics on the GPU's own outputs: the LO rotated by pi flips the
  assignment, a detuned LO collapses the state separation."""

import math
import os
import random

import numpy as np
import pytest

import oracle
from distributed_processor_amd import _abi, workloads
from distributed_processor_amd._native import DpemuError
from distributed_processor_amd.emulator import Emulator, ProgramSet, alloc_device_outputs
from tests.progfuzz import random_case, shaped_case
from tests.test_fast_vs_rtl import demod_params

pytestmark = pytest.mark.gpu

THREADS = int(os.environ.get('OMP_NUM_THREADS', '0') or 0) or min(16, os.cpu_count() or 1)
OUT = ('summary', 'events', 'trace', 'meas', 'regs', 'hist', 'acc')


@pytest.fixture(scope='module')
def emu():
    e = Emulator(0)
    yield e
    e.close()


def random_tables(rng, n_programs):
    lens = [rng.choice([0, 1, 3, 600]) for _ in range(2 * n_programs)]
    words = np.array([rng.getrandbits(32) for _ in range(sum(lens))], np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint32)
    return (words, offs[0::2], np.array(lens[0::2], np.uint32), offs[1::2], np.array(lens[1::2], np.uint32))


def compare(g, f, ctx):
    for k in OUT:
        if k in f:
            a, b = np.asarray(g[k]), np.asarray(f[k])
            if not np.array_equal(a, b):
                bad = np.argwhere(a != b)
                raise AssertionError('{} {}: {} mismatches, first at {}: gpu {} ref {}'.format(
                    ctx, k, len(bad), bad[0].tolist(), a[tuple(bad[0])], b[tuple(bad[0])]))


def run_pair(emu, ps, cfg, n_shots, shot0, tables):
    emu.load(ps)
    emu.load_readout_freqs(cfg.ro_drv_elem, cfg.meas_elem, tables=tables)
    g = emu.run(n_shots, shot0, cfg=cfg, outputs=OUT).arrays
    assert emu.last_kernel().startswith('branch_kernel<'), emu.last_kernel()
    assert int(emu.last_kernel().split('=')[1].split(',')[0].rstrip('>'), 16) & 0x40   # FEAT_DEMOD
    f = oracle.fast_run(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, shot0, n_shots, want=OUT, ro=tables)
    base = cfg.exec_flags
    for flags in (_abi.X_GENERAL | _abi.X_PROG_LDS, _abi.X_PROG_MAJOR | _abi.X_HIST_DIRECT, _abi.X_PROG_LDS):
        cfg.exec_flags = flags
        g2 = emu.run(n_shots, shot0, cfg=cfg, outputs=OUT).arrays
        compare(g2, g, 'execution variant {:#x}'.format(flags))
    cfg.exec_flags = base
    return g, f


@pytest.mark.parametrize('seed', range(24))
def test_fuzz_demod_gpu_vs_fast(emu, seed):
    rng = random.Random(70000 + seed)
    kind = seed % 4
    C = [1, 2, 4, 8][(seed // 4) % 4]
    if kind == 2:
        case = shaped_case(71000 + seed, C, n_groups=1 + seed % 3)
    else:
        case = random_case(72000 + seed, ncores=C, mode=['meas', 'lut', 'meas', 'meas'][kind], allow_late=True,
                           allow_hang=True, linear=kind == 3)
    mode = _abi.FPROC_MEAS if case['mode'] == 'meas' else _abi.FPROC_LUT
    groups = [[case['progs'][case['table'][g * C + c]] for c in range(C)] for g in range(case['n_groups'])]
    ps = ProgramSet(groups, cores_per_shot=C)
    meas_elem = seed % 4
    cfg = _abi.make_config(C, n_groups=ps.n_groups, max_cycles=6000 + 20000 * (seed % 2), event_cap=64,
                           trace_cap=32, meas_cap=16, fproc_mode=mode, meas_latency=1 + seed % 23,
                           sync_latency=1 + seed % 3, seed=seed, meas_elem=meas_elem,
                           lane_order=seed % 2, demod=demod_params(rng, C, meas_elem))
    g, f = run_pair(emu, ps, cfg, 333 + 111 * (seed % 3), seed * 1000, random_tables(rng, ps.n_programs))
    compare(g, f, 'seed {}'.format(seed))


def test_demod_needs_tables_and_acc_needs_demod(emu):
    """a DEMOD run without frequency tables and an acc output on another
    model are refused at the C ABI (no silent zero words, no stale buffer)"""
    import ctypes as C
    ps = ProgramSet(workloads.config1_linear())
    emu.load(ps)
    cfg = _abi.make_config(1, max_cycles=10000, event_cap=8, meas_cap=2, demod=dict(drv_elem=1))
    arrays = _abi.alloc_host_outputs(cfg, 4, ('summary', 'acc'))
    o = _abi.outputs_struct(arrays)
    rc = emu._L.dpemu_run_host(emu._h, C.addressof(cfg), 0, 4, C.addressof(o))
    assert rc == -22 and b'dpemu_load_readout_freqs' in emu._L.dpemu_last_error(emu._h)
    cfg2 = _abi.make_config(1, max_cycles=10000, event_cap=8, meas_cap=2)
    rc = emu._L.dpemu_run_host(emu._h, C.addressof(cfg2), 0, 4, C.addressof(o))
    assert rc == -22 and b'acc' in emu._L.dpemu_last_error(emu._h)
    with pytest.raises(DpemuError):
        emu.load_readout_freqs(1, 2, tables=(np.zeros(1, np.uint32),) + (np.zeros(3, np.uint32),) * 4)


def config3_demod_cfg(ps, **kw):
    return _abi.make_config(8, n_groups=ps.n_groups, max_cycles=50000, event_cap=16, trace_cap=0, meas_cap=4,
                            meas_latency=workloads.CONFIG3_DEMOD_LATENCY, seed=0x5EED, p1=0.5,
                            demod=workloads.config3_demod(ps), **kw)


@pytest.mark.parametrize('rank,shape', [(2, {}), (6, dict(lane_order=_abi.LANES_SHOT_MAJOR, hist_assign=True))],
                         ids=['rank2_core_major', 'rank6_bench_shape'])
def test_config3_demod_full_shard_bit_exact(emu, rank, shape):
    """config 3 with the demodulation readout at the per-GPU shard size
    (1.25 * 10^6 shots x 8 cores): summaries, events, meas_valid cycles and
    outcomes, accumulated {I, Q} and the histogram equal oracle_fast; the
    conditional X90 pair ran exactly where the first readout said 1, and
    the calibrated discriminator assigns ~99 % of shots their prepared state"""
    import torch
    ps = ProgramSet(workloads.config3_active_reset(8))
    cfg = config3_demod_cfg(ps, **shape)
    emu.load(ps)
    n = 1250000
    want = ('summary', 'events', 'meas', 'hist', 'acc')
    out = alloc_device_outputs(cfg, n, want=want)
    for k, t in out.items():
        t.zero_()
    emu.run_device(cfg, n, rank * n, out)
    torch.cuda.synchronize()
    assert emu.last_kernel().startswith('branch_kernel<'), emu.last_kernel()
    g = {k: v.cpu().numpy() for k, v in out.items()}
    del out
    torch.cuda.empty_cache()
    f = oracle.fast_run(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, rank * n, n, threads=THREADS, want=want,
                        ro=ps.readout_freqs(cfg.ro_drv_elem, cfg.meas_elem))
    for k in want:
        a = g[k].view(f[k].dtype).reshape(f[k].shape)
        if not np.array_equal(a, f[k]):
            bad = np.argwhere(a != f[k])
            raise AssertionError('{}: {} mismatches, first at {}'.format(k, len(bad), bad[0].tolist()))
    s = _abi.unpack_summary(g['summary'].view(np.uint32))
    assert (s['status'] == _abi.ST_DONE).all() and int(g['hist'].sum()) == n
    flip = (s['meas_bits'] & 1).astype(bool)
    assert (s['n_events'][flip] == s['n_events'][~flip].min() + 2).all()
    # prepared state of the first readout: Philox word 0 of (shot, core, m = 0) < 2^31
    shots = np.arange(rank * n, rank * n + 4096, dtype=np.uint64)
    st = np.array([[oracle.lib().oracle_philox_u32(0x5EED, int(sh), c, 0) < (1 << 31) for sh in shots]
                   for c in range(8)])
    lanes = np.array([[_abi.lane_index(int(sh) - rank * n, c, n, 8, cfg.lane_order) for sh in shots]
                      for c in range(8)])
    assert (flip[lanes] == st).mean() > 0.97


def _read_prog(ph_lo):
    from tests.test_demod import ro_program
    return ro_program([dict(A=40000, ph_d=0, ph_lo=ph_lo, L_d=250, L_lo=250, lo_at=300)])


def _assign_gpu(emu, ph_lo=0, f_lo=0x12345678, sigma=60.0, n=20000, p1=0.5):
    f_d = 0x12345678
    ps = ProgramSet([[_read_prog(ph_lo)]], cores_per_shot=1)
    ax = ((-f_d * 300) % 2 ** 32) * 2 * math.pi / 2 ** 32
    cfg = _abi.make_config(1, max_cycles=20000, event_cap=8, meas_cap=2, meas_latency=32, p1=p1,
                           demod=dict(drv_elem=1, cpw=4, delay=300, theta=(math.pi, 0.0), axis=ax, sigma=sigma))
    tables = (np.array([f_d, f_lo], np.uint32), np.array([0], np.uint32), np.array([1], np.uint32),
              np.array([1], np.uint32), np.array([1], np.uint32))
    emu.load(ps)
    emu.load_readout_freqs(1, 2, tables=tables)
    g = emu.run(n, 0, cfg=cfg, outputs=('summary', 'meas', 'acc')).arrays
    f = oracle.fast_run(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, 0, n, want=('summary', 'meas', 'acc'),
                        ro=tables)
    compare(g, f, 'assign')
    st = np.array([oracle.lib().oracle_philox_u32(0x5EED, s, 0, 0) < (1 << 31) for s in range(n)])
    return g, st


def test_gpu_pi_rotated_lo_flips_assignment(emu):
    g, st = _assign_gpu(emu)
    assert (g['meas'][0, :, 1] == st).mean() > 0.98
    g2, _ = _assign_gpu(emu, ph_lo=2 ** 16)
    assert (g2['meas'][0, :, 1] == st).mean() < 0.02
    a, _ = _assign_gpu(emu, sigma=0.0, n=256)
    b, _ = _assign_gpu(emu, ph_lo=2 ** 16, sigma=0.0, n=256)
    assert np.abs(a['acc'][0].astype(np.int64) + b['acc'][0]).max() <= 2


def test_gpu_detuned_lo_collapses_separation(emu):
    det = int(0.01 * 2 ** 32)
    means = {}
    for name, f_lo in (('tuned', 0x12345678), ('detuned', (0x12345678 - det) & 0xFFFFFFFF)):
        m = [_assign_gpu(emu, f_lo=f_lo, sigma=0.0, n=64, p1=p)[0]['acc'][0].astype(np.float64).mean(axis=0)
             for p in (0.0, 1.0)]
        means[name] = float(np.hypot(*(m[1] - m[0])))
    assert means['detuned'] < 0.01 * means['tuned']
    g, st = _assign_gpu(emu, f_lo=(0x12345678 - det) & 0xFFFFFFFF)
    assert 0.45 < (g['meas'][0, :, 1] == st).mean() < 0.55


def test_demod_sharding_invariance(emu):
    """shards of a DEMOD run (global shot offsets) equal the unsharded run in
    every output, the accumulated I/Q included: the noise and state draws are
    keyed by the global shot index, as for the other models"""
    ps = ProgramSet(workloads.config3_active_reset(8))
    cfg = config3_demod_cfg(ps)
    emu.load(ps)
    outs = ('summary', 'events', 'meas', 'acc')
    whole = emu.run(3000, 500, cfg=cfg, outputs=outs).arrays
    parts = [emu.run(n, s0, cfg=cfg, outputs=outs).arrays for s0, n in ((500, 1000), (1500, 1200), (2700, 800))]
    for k in outs:
        lane_axis = 0 if k == 'summary' else 1
        per = [_abi.by_shot(p[k], 8, axis=lane_axis) for p in parts]          # (..., core, shot, ...)
        got = np.concatenate(per, axis=lane_axis + 1)
        np.testing.assert_array_equal(got, _abi.by_shot(whole[k], 8, axis=lane_axis), err_msg=k)
