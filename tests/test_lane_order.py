"""dpemu_config.lane_order on the CPU side: oracle_fast in shot-major order is
its core-major output permuted (every array), the host helpers map (shot,
core) to the same lanes the oracle writes, and DDS channel plans follow the
run's order."""

import numpy as np
import pytest

import oracle
from distributed_processor_amd import _abi, workloads
from distributed_processor_amd.dds import ChannelPlan
from distributed_processor_amd.emulator import EmulationResult, ProgramSet
from tests.progfuzz import random_case

OUT = ('summary', 'events', 'trace', 'meas', 'regs', 'hist')


def _pair(ps, C, n, shot0, **kw):
    res = []
    for order in (_abi.LANES_CORE_MAJOR, _abi.LANES_SHOT_MAJOR):
        cfg = _abi.make_config(C, n_groups=ps.n_groups, lane_order=order, **kw)
        res.append(oracle.fast_run(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, shot0, n, want=OUT))
    return res


@pytest.mark.parametrize('seed', range(6))
def test_oracle_shot_major_is_permuted_core_major(seed):
    C = [1, 2, 4, 8, 2, 4][seed]
    case = random_case(47000 + seed, ncores=C)
    mode = _abi.FPROC_MEAS if case['mode'] == 'meas' else _abi.FPROC_LUT
    groups = [[case['progs'][case['table'][g * C + c]] for c in range(C)] for g in range(case['n_groups'])]
    ps = ProgramSet(groups, cores_per_shot=C)
    n = 57
    cm, sm = _pair(ps, C, n, 1000 * seed, max_cycles=6000, event_cap=32, trace_cap=32, meas_cap=8,
                   fproc_mode=mode, seed=seed)
    lanes = _abi.lane_index(np.repeat(np.arange(n), C), np.tile(np.arange(C), n), n)   # shot-major -> core-major
    np.testing.assert_array_equal(sm['summary'], cm['summary'][lanes])
    for k in ('events', 'trace', 'meas', 'regs'):
        np.testing.assert_array_equal(sm[k], cm[k][:, lanes])
    np.testing.assert_array_equal(sm['hist'], cm['hist'])
    for order, arr in ((_abi.LANES_CORE_MAJOR, cm), (_abi.LANES_SHOT_MAJOR, sm)):
        np.testing.assert_array_equal(_abi.by_shot(arr['summary'], C, lane_order=order),
                                      _abi.by_shot(cm['summary'], C))


def test_result_lane_and_channel_plan_follow_the_order():
    ps = ProgramSet(workloads.config3_active_reset(8))
    for order in (_abi.LANES_CORE_MAJOR, _abi.LANES_SHOT_MAJOR):
        cfg = _abi.make_config(8, n_groups=ps.n_groups, event_cap=16, meas_cap=4,
                               meas_latency=workloads.CONFIG3_MEAS_LATENCY, lane_order=order)
        arrays = oracle.fast_run(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, 100, 20, want=OUT)
        res = EmulationResult(cfg, 20, 100, arrays)
        for shot, core in ((100, 0), (107, 5), (119, 7)):
            L = res.lane(shot, core)
            want = (shot - 100) * 8 + core if order == _abi.LANES_SHOT_MAJOR else core * 20 + shot - 100
            assert L == want
        plan = ChannelPlan(ps, cfg, 100, 20, [(107, 5, workloads.QDRV)], {workloads.QDRV: (16, 1)})
        assert int(plan.desc[0, 0]) == res.lane(107, 5)


def test_make_config_rejects_unknown_order():
    with pytest.raises(ValueError):
        _abi.make_config(2, lane_order=3)
