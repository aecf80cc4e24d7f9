"""HIP interpreter (libdpemu.so, through the C ABI) vs oracle_fast, bit for bit.

oracle_fast is itself pinned to the per-clock RTL restatement
(tests/test_fast_vs_rtl.py), which is pinned to the reference's cocotb
known-answer tests (tests/test_rtl_kat.py).  Every output array -- lane
summaries, events, amplitudes, register/qclk traces, measurements, final
registers, histograms -- must be identical.  At full BASELINE sizes the
checks are size-independent properties (sharding invariance, histogram
totals, per-group determinism).
"""

import numpy as np
import pytest

import oracle
from distributed_processor_amd import _abi, workloads
from distributed_processor_amd.emulator import Emulator, ProgramSet
from tests.progfuzz import pack_programs, random_case, shaped_case

pytestmark = pytest.mark.gpu

ALL_OUT = ('summary', 'events', 'trace', 'meas', 'regs', 'hist')


@pytest.fixture(scope='module')
def emu():
    e = Emulator(0)
    yield e
    e.close()


def compare_all(gpu, ref, ctx=''):
    for k in ALL_OUT:
        if k in ref:
            assert k in gpu, k
            a, b = np.asarray(gpu[k]), np.asarray(ref[k])
            if not np.array_equal(a, b):
                bad = np.argwhere(a != b)
                raise AssertionError('{} {}: {} mismatches, first at {}: gpu {} ref {}'.format(
                    ctx, k, len(bad), bad[0].tolist(), a[tuple(bad[0])], b[tuple(bad[0])]))


def run_pair(emu, ps, cfg, n_shots, shot0=0):
    """GPU run and oracle; the execution variants (LDS-staged programs,
    histogram strategy, program-major fetch, the general interpreter for
    branch-free programs, the per-lane macro fetch instead of the staged
    macro chunks, nontemporal event rows) must produce the same bytes"""
    emu.load(ps)
    g = emu.run(n_shots, shot0, cfg=cfg, outputs=ALL_OUT)
    f = oracle.fast_run(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, shot0, n_shots, want=ALL_OUT)
    base = cfg.exec_flags
    for flags in (_abi.X_PROG_LDS | _abi.X_HIST_REPL, _abi.X_HIST_DIRECT | _abi.X_PROG_MAJOR,
                  _abi.X_GENERAL | _abi.X_PROG_LDS, _abi.X_MACRO_DIRECT, _abi.X_STREAM_EVENTS):
        cfg.exec_flags = flags
        g2 = emu.run(n_shots, shot0, cfg=cfg, outputs=ALL_OUT)
        compare_all(g2.arrays, g.arrays, 'execution variant {:#x}'.format(flags))
    cfg.exec_flags = base
    return g.arrays, f


@pytest.mark.parametrize('seed', range(40))
def test_fuzz_gpu_vs_fast(emu, seed):
    case = random_case(seed, ncores=[1, 2, 4, 8][seed % 4])
    mode = _abi.FPROC_MEAS if case['mode'] == 'meas' else _abi.FPROC_LUT
    C = case['ncores']
    groups = [[case['progs'][case['table'][g * C + c]] for c in range(C)] for g in range(case['n_groups'])]
    ps = ProgramSet(groups, cores_per_shot=C)
    cfg = _abi.make_config(C, n_groups=ps.n_groups, max_cycles=6000, event_cap=64, trace_cap=64,
                           meas_cap=16, fproc_mode=mode, meas_latency=1 + seed % 23,
                           sync_latency=1 + seed % 3, sync_mask=(0b0111 if seed % 5 == 0 and C == 4 else 0),
                           seed=seed)
    n_shots = 333 if seed % 2 else 100 * ps.n_groups
    g, f = run_pair(emu, ps, cfg, n_shots, shot0=seed * 1000)
    compare_all(g, f, 'seed {}'.format(seed))


@pytest.mark.parametrize('seed', range(16))
def test_fuzz_straight_programs(emu, seed):
    """pulse / idle / pulse_reset / done / hang programs (straight.hip, and the
    general interpreter's register-free specialisation): register-sourced
    pulse fields read 0, late triggers, the reset-hold double strobe; seeds
    >= 12 with tight cycle / event / measurement caps (max_cycles finishes
    before and at a fetch, dropped events and measurements)"""
    C = [1, 2, 4, 8][seed % 4]
    case = random_case(9000 + seed, ncores=C, mode='meas', allow_late=True, allow_hang=True, straight=True)
    groups = [[case['progs'][case['table'][g * C + c]] for c in range(C)] for g in range(case['n_groups'])]
    ps = ProgramSet(groups, cores_per_shot=C)
    tight = seed >= 12
    cfg = _abi.make_config(C, n_groups=ps.n_groups, max_cycles=150 + 40 * seed if tight else 6000,
                           event_cap=3 if tight else 64, trace_cap=16, meas_cap=1 if tight else 16,
                           meas_latency=1 + seed, seed=seed)
    g, f = run_pair(emu, ps, cfg, 777, shot0=seed * 31)
    compare_all(g, f, 'seed {}'.format(seed))


@pytest.mark.parametrize('seed', range(16))
def test_fuzz_shaped_straight_programs(emu, seed):
    """pulse-only programs sharing one opcode sequence (straight.hip's
    uniform-opcode path) with per-lane parameters, endings, late triggers;
    odd seeds with tight cycle / event / measurement caps"""
    C = [1, 2, 4, 8][seed % 4]
    case = shaped_case(12000 + seed, C, n_groups=1 + seed % 5)
    groups = [[case['progs'][case['table'][g * C + c]] for c in range(C)] for g in range(case['n_groups'])]
    ps = ProgramSet(groups, cores_per_shot=C)
    tight = seed % 2 == 1
    cfg = _abi.make_config(C, n_groups=ps.n_groups, max_cycles=100 + 30 * seed if tight else 6000,
                           event_cap=2 + seed % 3 if tight else 64, trace_cap=4, meas_cap=1 if tight else 16,
                           meas_latency=1 + seed, seed=seed, meas_elem=seed % 4)
    g, f = run_pair(emu, ps, cfg, 1000 + 37 * seed, shot0=seed * 77)
    compare_all(g, f, 'seed {}'.format(seed))


@pytest.mark.parametrize('seed', range(16))
def test_fuzz_linear_programs(emu, seed):
    """branch-free programs with reg_alu / inc_qclk (straight.hip with the
    register file; all 8 ALU ops, register-sourced pulse fields, qclk
    reloads), random per lane (odd seeds) or sharing one opcode sequence (even
    seeds); seeds >= 8 with tight cycle / event / trace / measurement caps"""
    C = [1, 2, 4, 8][seed % 4]
    if seed % 2:
        case = random_case(15000 + seed, ncores=C, mode='meas', allow_late=True, allow_hang=True, linear=True)
    else:
        case = shaped_case(16000 + seed, C, n_groups=1 + seed % 3, linear=True)
    groups = [[case['progs'][case['table'][g * C + c]] for c in range(C)] for g in range(case['n_groups'])]
    ps = ProgramSet(groups, cores_per_shot=C)
    tight = seed >= 8
    cfg = _abi.make_config(C, n_groups=ps.n_groups, max_cycles=120 + 25 * seed if tight else 6000,
                           event_cap=3 if tight else 64, trace_cap=2 if tight else 64,
                           meas_cap=1 if tight else 16, meas_latency=1 + seed, seed=seed, meas_elem=seed % 4)
    g, f = run_pair(emu, ps, cfg, 900 + 41 * seed, shot0=seed * 13)
    compare_all(g, f, 'seed {}'.format(seed))


@pytest.mark.parametrize('seed', range(12))
def test_fuzz_linear_few_registers(emu, seed):
    """branch-free register programs naming 1-4 registers (any indices): the
    macro image renumbers up to 2 of them to VGPR slots (macro_staged_kernel<2>,
    else the LDS file of macro_staged_kernel<16>);
    many program groups with 5-16 shots each so a wave stages several
    programs, traces on (register addresses map back), registers out;
    against oracle_fast and every execution variant (macro_kernel included)"""
    import random
    rr = random.Random(seed)
    C = [1, 2, 4][seed % 3]
    regs = rr.sample(range(16), 1 + seed % 4)
    case = random_case(17000 + seed, ncores=C, mode='meas', allow_late=seed % 2 == 1, allow_hang=True,
                       n_groups=9 + seed, linear=True, regs=regs)
    groups = [[case['progs'][case['table'][g * C + c]] for c in range(C)] for g in range(case['n_groups'])]
    ps = ProgramSet(groups, cores_per_shot=C)
    spg = [10, 16, 32, 5][seed % 4]
    order = (seed // 4) % 2
    cfg = _abi.make_config(C, n_groups=ps.n_groups, shots_per_group=spg, max_cycles=6000, event_cap=64,
                           trace_cap=64, meas_cap=16, meas_latency=5, seed=seed, meas_elem=seed % 4,
                           lane_order=order)
    g, f = run_pair(emu, ps, cfg, 64 * 9 + 7 * seed, shot0=seed * 31)
    compare_all(g, f, 'seed {} regs {}'.format(seed, regs))
    # the kernel the run used (capi.cpp): staged when a wave spans <= 8 distinct
    # programs, or <= 12 (MACRO_SLOTS_WIDE) with the 2-register VGPR file
    shots_run = 64 // C if order else min(256 // C, 64)
    cores_w = C if order else 64 // shots_run
    need = (-(-(shots_run - 1) // spg) + 1) * cores_w
    emu.run(3, 0, cfg=cfg)
    got = emu.last_kernel().replace(',addid', '')   # addid: every ALU op of the image is id0 / add
    if need > 12:
        assert got == 'macro_kernel', got
    elif need > 8:
        if len(regs) <= 2:
            assert got == 'macro_staged_kernel<2,12>', got
        else:                   # the wide kernel only with the 2-register file
            assert got in ('macro_staged_kernel<2,12>', 'macro_kernel'), got
    elif len(regs) <= 2:
        assert got == 'macro_staged_kernel<2>', got
    else:                       # <2> when the programs happen to read / write at most 2 of them
        assert got in ('macro_staged_kernel<2>', 'macro_staged_kernel<16>'), got


@pytest.mark.parametrize('C', [1, 2, 4, 8, 16, 32, 64])
def test_fuzz_all_group_sizes(emu, C):
    case = random_case(500 + C, ncores=C, mode='meas', allow_late=True, allow_hang=True)
    groups = [[case['progs'][case['table'][g * C + c]] for c in range(C)] for g in range(case['n_groups'])]
    ps = ProgramSet(groups, cores_per_shot=C)
    cfg = _abi.make_config(C, n_groups=ps.n_groups, max_cycles=5000, event_cap=48, trace_cap=48,
                           meas_cap=16, meas_latency=7, seed=C)
    g, f = run_pair(emu, ps, cfg, 4096 // C + 3)
    if C > 12:
        f.pop('hist', None)
    compare_all(g, f, 'C={}'.format(C))


def test_config1_golden_program(emu, golden_dir):
    """the reference's own machine-code golden (test_linear_compile_globalasm core 0)"""
    import json
    import os
    with open(os.path.join(golden_dir, 'cmd_buf_golden.json')) as fh:
        gold = json.load(fh)
    ps = ProgramSet([{0: bytes.fromhex(gold['cores']['0']['cmd_buf'])}])
    cfg = _abi.make_config(1, max_cycles=10000, event_cap=8, trace_cap=8, meas_cap=4)
    g, f = run_pair(emu, ps, cfg, 10000)
    compare_all(g, f)
    s = _abi.unpack_summary(g['summary'])
    assert (s['status'] == _abi.ST_DONE).all()
    assert (s['n_events'] == 4).all()            # pulse_reset + 3 strobes
    ev = g['events'][:, 0]
    assert [int(e[0]) for e in ev[:4]] == [0, 8, 24, 324]     # reset @0; cstrobe at cmd_time + 3 = qclk T + 2
    assert [int(e[1]) >> 28 for e in ev[:4]] == [1, 0, 0, 0]  # pulse_reset, then three strobes


@pytest.mark.parametrize('name', ['test_fproc_hold', 'test_hw_virtualz_out', 'test_linear_compile_out',
                                  'test_multirst_cfg', 'test_multirst_fproc_res_cfg', 'test_pulse_compile_out',
                                  'test_simple_loop'])
def test_restated_assembler_goldens(emu, name):
    """the reference's compiler golden programs, assembled by this framework's
    API-compatible GlobalAssembler restatement (byte-identical to the reference's, see
    tests/test_assembler.py), run on the GPU against oracle_fast"""
    from distributed_processor_amd import hwconfig
    from tests.test_assembler import assemble
    ps = ProgramSet([assemble(name, hwconfig.DDSElementConfig)])
    cfg = _abi.make_config(ps.cores_per_shot, max_cycles=20000, event_cap=32, trace_cap=32, meas_cap=8,
                           p1=0.5, seed=len(name))
    g, f = run_pair(emu, ps, cfg, 3000, shot0=11)
    compare_all(g, f, name)
    st = _abi.by_shot(_abi.unpack_summary(g['summary'])['status'], ps.cores_per_shot).T     # [shot, core]
    # two goldens never finish by construction: in test_multirst_cfg core Q1
    # waits (jump_fproc func_id 0) on a measurement it never makes; in
    # test_simple_loop the loop register is never incremented
    expect = {'test_multirst_cfg': [_abi.ST_DONE, _abi.ST_MAX_CYCLES],
              'test_simple_loop': [_abi.ST_MAX_CYCLES, _abi.ST_DONE]}.get(name, [_abi.ST_DONE] * ps.cores_per_shot)
    assert (st == np.array(expect)).all()


def test_config1_dds_element(emu):
    ps = ProgramSet(workloads.config1_linear())
    cfg = _abi.make_config(1, max_cycles=10000, event_cap=8, trace_cap=8, meas_cap=4)
    g, f = run_pair(emu, ps, cfg, 50000, shot0=123)
    compare_all(g, f)


def test_config2_ramsey(emu):
    ps = ProgramSet(workloads.config2_ramsey(n_cores=8, n_points=100))
    cfg = _abi.make_config(8, n_groups=100, max_cycles=20000, event_cap=8, trace_cap=4, meas_cap=4)
    g, f = run_pair(emu, ps, cfg, 3000)
    compare_all(g, f)
    assert (_abi.unpack_summary(g['summary'])['status'] == _abi.ST_DONE).all()


def test_config3_active_reset(emu):
    ps = ProgramSet(workloads.config3_active_reset(8))
    cfg = _abi.make_config(8, max_cycles=50000, event_cap=16, trace_cap=16, meas_cap=4,
                           meas_latency=workloads.CONFIG3_MEAS_LATENCY, p1=0.5)
    g, f = run_pair(emu, ps, cfg, 4000, shot0=10 ** 9)
    compare_all(g, f)
    s = _abi.unpack_summary(g['summary'])
    assert (s['status'] == _abi.ST_DONE).all()
    # the conditional X180 ran exactly for first outcomes of 1
    flip = (s['meas_bits'] & 1).astype(bool)
    assert (s['n_events'][flip] == s['n_events'][~flip].min() + 2).all()
    assert 0.45 < flip.mean() < 0.55


def test_config3_active_reset_readout_model(emu):
    """config 3 with meas_model READOUT: reset branches follow the discriminated
    readout (state + noise) instead of the state; GPU = oracle_fast bit for bit"""
    ps = ProgramSet(workloads.config3_active_reset(8))
    cfg = _abi.make_config(8, max_cycles=50000, event_cap=16, trace_cap=16, meas_cap=4,
                           meas_latency=workloads.CONFIG3_MEAS_LATENCY, p1=0.2,
                           readout=dict(sep=30000, sigma=0.6, thr=2000))
    g, f = run_pair(emu, ps, cfg, 4000, shot0=7 * 10 ** 8)
    compare_all(g, f)
    s = _abi.unpack_summary(g['summary'])
    assert (s['status'] == _abi.ST_DONE).all()


@pytest.mark.parametrize('seed', range(12))
def test_fuzz_readout_model(emu, seed):
    """fuzzed programs (fproc branches on readout outcomes, meas and LUT modes)
    under meas_model READOUT, on both interpreter kernels"""
    C = [1, 2, 4, 8][seed % 4]
    case = random_case(5000 + seed, ncores=C, mode=['meas', 'lut'][seed % 2], straight=seed % 3 == 2)
    mode = _abi.FPROC_MEAS if case['mode'] == 'meas' else _abi.FPROC_LUT
    groups = [[case['progs'][case['table'][g * C + c]] for c in range(C)] for g in range(case['n_groups'])]
    ps = ProgramSet(groups, cores_per_shot=C)
    cfg = _abi.make_config(C, n_groups=ps.n_groups, max_cycles=6000, event_cap=64, trace_cap=64, meas_cap=16,
                           fproc_mode=mode, meas_latency=1 + seed % 13, seed=seed, p1=0.4,
                           readout=dict(sep=[25000, -8000, 60000][seed % 3], sigma=[0.7, 1.5, 0.2][seed % 3],
                                        thr=[0, -1500, 900][seed % 3], win=[0, 40, 900, 4095][seed % 4]))
    g, f = run_pair(emu, ps, cfg, 257, shot0=seed * 977)
    compare_all(g, f, 'readout seed {}'.format(seed))


def test_config4_rb(emu):
    ps = ProgramSet(workloads.config4_rb(n_seq=24, depth=40))
    cfg = _abi.make_config(2, n_groups=24, shots_per_group=5, max_cycles=200000, event_cap=160,
                           trace_cap=256, meas_cap=4)
    g, f = run_pair(emu, ps, cfg, 24 * 5)
    compare_all(g, f)


@pytest.mark.parametrize('n_cores,order', [(2, 'core'), (2, 'shot'), (4, 'core')])
def test_config4_rb2q(emu, n_cores, order):
    """two-qubit Clifford RB programs (config 4's generator, CNOTs and
    recovery Cliffords), every output against oracle_fast in both lane orders
    and with 4 cores (two pairs)"""
    ps = ProgramSet(workloads.config4_rb2q(n_seq=24, depth=30, n_cores=n_cores))
    cfg = _abi.make_config(n_cores, n_groups=24, shots_per_group=5, max_cycles=400000, event_cap=300,
                           trace_cap=600, meas_cap=4, seed=3, p1=0.3,
                           lane_order=_abi.LANES_SHOT_MAJOR if order == 'shot' else _abi.LANES_CORE_MAJOR)
    g, f = run_pair(emu, ps, cfg, 24 * 5)
    compare_all(g, f, 'rb2q C {} {}'.format(n_cores, order))


@pytest.mark.parametrize('mode', ['meas', 'lut'])
def test_lut_and_meas_fuzz_many_shots(emu, mode):
    for seed in range(6):
        case = random_case(7000 + seed, ncores=4, mode=mode, allow_late=False, allow_hang=False)
        groups = [[case['progs'][case['table'][g * 4 + c]] for c in range(4)] for g in range(case['n_groups'])]
        ps = ProgramSet(groups, cores_per_shot=4)
        cfg = _abi.make_config(4, n_groups=ps.n_groups, max_cycles=8000, event_cap=64, trace_cap=64,
                               meas_cap=16, fproc_mode=_abi.FPROC_LUT if mode == 'lut' else _abi.FPROC_MEAS,
                               meas_latency=3 + seed, seed=seed)
        g, f = run_pair(emu, ps, cfg, 2048)
        compare_all(g, f, 'seed {}'.format(seed))


# ---------------------------------------------------------------- full-size properties
def test_ramsey_full_size_sharding_invariant(emu):
    """config 2 at 10^6 shots: per-shard results equal the single run (RNG keyed
    by global shot index), histogram totals, and per-group determinism."""
    ps = ProgramSet(workloads.config2_ramsey(n_cores=8, n_points=100))
    emu.load(ps)
    cfg = _abi.make_config(8, n_groups=100, max_cycles=20000, event_cap=8, meas_cap=2)
    N = 10 ** 6
    full = emu.run(N, 0, cfg=cfg, outputs=('summary', 'hist'))
    assert int(full.arrays['hist'].sum()) == N
    assert (full.summary['status'] == _abi.ST_DONE).all()
    half = [emu.run(N // 2, s, cfg=cfg, outputs=('summary', 'hist')) for s in (0, N // 2)]
    joined = np.concatenate([_abi.by_shot(h.arrays['summary'], 8) for h in half], axis=1)   # [core, shot, 8]
    assert np.array_equal(joined, _abi.by_shot(full.arrays['summary'], 8))
    assert np.array_equal(half[0].arrays['hist'] + half[1].arrays['hist'], full.arrays['hist'])
    t_end = _abi.by_shot(full.summary['t_end'], 8).T                                       # [shot, core]
    grp = np.arange(N) % 100
    for k in (0, 37, 99):
        rows = t_end[grp == k]
        assert (rows == rows[0]).all()
    # P(1) = 0.5 per core: each histogram bin near uniform over 256 keys
    h = full.arrays['hist'].sum(axis=0)
    assert abs(h.mean() - N / 256) < 1e-9 and h.min() > 0.8 * N / 256
