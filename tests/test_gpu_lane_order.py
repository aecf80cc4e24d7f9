"""Shot-major lanes (dpemu_config.lane_order = DPEMU_LANES_SHOT_MAJOR) on the
GPU: every kernel -- straight (pulse-only), macro (branch-free with
registers), branch (jumps, fproc, sync), the general interpreter (meas_lut
back end, DPEMU_X_GENERAL) -- against oracle_fast in the same lane order,
bit for bit on every output and in every execution variant, and the same
run in core-major order permuted into shot-major."""

import numpy as np
import pytest

import oracle
from distributed_processor_amd import _abi, workloads
from distributed_processor_amd.emulator import Emulator, ProgramSet
from tests.progfuzz import random_case, shaped_case
from tests.test_gpu_parity import ALL_OUT, compare_all, run_pair

pytestmark = pytest.mark.gpu

SM = _abi.LANES_SHOT_MAJOR


@pytest.fixture(scope='module')
def emu():
    e = Emulator(0)
    yield e
    e.close()


def to_shot_major(arrays, C, n_shots):
    """core-major output arrays permuted into shot-major lane order"""
    perm = (np.arange(n_shots)[:, None] + np.arange(C)[None, :] * n_shots).reshape(-1)   # new lane -> old lane
    out = {}
    for k, v in arrays.items():
        v = np.asarray(v)
        out[k] = v if k == 'hist' else (v[perm] if k == 'summary' else v[:, perm])
    return out


def check(emu, ps, cfg_kw, n_shots, shot0, C):
    cfg = _abi.make_config(C, n_groups=ps.n_groups, lane_order=SM, **cfg_kw)
    g, f = run_pair(emu, ps, cfg, n_shots, shot0)
    compare_all(g, f, 'shot-major')
    core = emu.run(n_shots, shot0, cfg=_abi.make_config(C, n_groups=ps.n_groups, **cfg_kw), outputs=ALL_OUT)
    compare_all(g, to_shot_major(core.arrays, C, n_shots), 'core-major permuted')


@pytest.mark.parametrize('seed', range(8))
def test_general_fuzz(emu, seed):
    """jumps, fproc_meas / fproc_lut, syncs, register traces (branch_kernel,
    interp_kernel for the LUT back end)"""
    C = [1, 2, 4, 8][seed % 4]
    case = random_case(41000 + seed, ncores=C)
    mode = _abi.FPROC_MEAS if case['mode'] == 'meas' else _abi.FPROC_LUT
    groups = [[case['progs'][case['table'][g * C + c]] for c in range(C)] for g in range(case['n_groups'])]
    ps = ProgramSet(groups, cores_per_shot=C)
    check(emu, ps, dict(max_cycles=6000, event_cap=64, trace_cap=64, meas_cap=16, fproc_mode=mode,
                        meas_latency=1 + seed, sync_latency=1 + seed % 3, seed=seed), 333, seed * 1000, C)


@pytest.mark.parametrize('seed', range(6))
def test_straight_and_linear(emu, seed):
    """pulse-only programs (straight_kernel) and branch-free register programs
    (macro_kernel), random and shaped"""
    C = [1, 2, 4, 8][seed % 4]
    if seed % 3 == 0:
        case = random_case(42000 + seed, ncores=C, mode='meas', allow_late=True, allow_hang=True, straight=True)
    elif seed % 3 == 1:
        case = shaped_case(43000 + seed, C, n_groups=1 + seed % 3)
    else:
        case = random_case(44000 + seed, ncores=C, mode='meas', allow_late=True, allow_hang=True, linear=True)
    groups = [[case['progs'][case['table'][g * C + c]] for c in range(C)] for g in range(case['n_groups'])]
    ps = ProgramSet(groups, cores_per_shot=C)
    check(emu, ps, dict(max_cycles=6000, event_cap=64, trace_cap=64, meas_cap=16, meas_latency=1 + seed,
                        seed=seed, meas_elem=seed % 4), 700 + 13 * seed, seed * 17, C)


def test_baseline_workloads(emu):
    """configs 2, 3 and 4 (small) in shot-major order"""
    ps = ProgramSet(workloads.config2_ramsey(8, 100))
    check(emu, ps, dict(max_cycles=20000, event_cap=8, trace_cap=4, meas_cap=4), 3000, 0, 8)
    ps = ProgramSet(workloads.config3_active_reset(8))
    check(emu, ps, dict(max_cycles=50000, event_cap=16, trace_cap=16, meas_cap=4,
                        meas_latency=workloads.CONFIG3_MEAS_LATENCY, p1=0.5), 4000, 10 ** 6, 8)
    ps = workloads.config4_rb_set(64, 40)
    check(emu, ps, dict(shots_per_group=10, max_cycles=1 << 20, event_cap=128, trace_cap=64, meas_cap=2), 640, 0, 2)


def test_lane_order_rejected_when_invalid(emu):
    ps = ProgramSet(workloads.config1_linear())
    emu.load(ps)
    cfg = _abi.make_config(ps.cores_per_shot)
    cfg.lane_order = 2
    from distributed_processor_amd._native import DpemuError
    with pytest.raises(DpemuError):
        emu.run(4, 0, cfg=cfg, outputs=('summary',))


@pytest.mark.parametrize('seed', range(8))
def test_event_rows_under_divergence(emu, seed):
    """branch_kernel holds each lane's newest event records and stores whole
    wave rows: programs whose lanes diverge (jumps on outcomes, syncs, late
    and hung commands) at small and large event caps, both lane orders, bit
    for bit against oracle_fast (the record a lane pushes out early, the
    cap, the final flush)"""
    C = [2, 4, 8, 8][seed % 4]
    case = random_case(47000 + seed, ncores=C, mode='meas')
    groups = [[case['progs'][case['table'][g * C + c]] for c in range(C)] for g in range(case['n_groups'])]
    ps = ProgramSet(groups, cores_per_shot=C)
    for cap in (1, 2, 3, 64):
        for order in (_abi.LANES_CORE_MAJOR, SM):
            cfg = _abi.make_config(C, n_groups=ps.n_groups, max_cycles=6000, event_cap=cap, trace_cap=8, meas_cap=8,
                                   meas_latency=2 + seed, p1=0.3 + 0.05 * seed, seed=seed, lane_order=order)
            g, f = run_pair(emu, ps, cfg, 257, seed * 100)
            compare_all(g, f, 'event_cap {} order {}'.format(cap, order))
