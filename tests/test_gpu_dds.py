"""HIP DDS kernel (dpemu_dds, through the C ABI) vs oracle_dds, bit for bit.

The event timelines come from the GPU interpreter (itself bit-exact against
oracle_fast, tests/test_gpu_parity.py); both DDS implementations consume the
same device-resident events, copied to the host for the oracle.
"""

import numpy as np
import pytest

import oracle
from distributed_processor_amd import _abi, workloads
from distributed_processor_amd.dds import ChannelPlan, split_iq
from distributed_processor_amd.emulator import Emulator, ProgramSet, alloc_device_outputs
from distributed_processor_amd._native import DpemuError
from distributed_processor_amd.hwconfig import DDSElementConfig, pack_iq16

pytestmark = pytest.mark.gpu

ELEM_PARAMS = {i: (e['samples_per_clk'], e['interp_ratio']) for i, e in enumerate(workloads.ELEMS)}


@pytest.fixture(scope='module')
def emu():
    e = Emulator(0)
    yield e
    e.close()


def host(t):
    return t.cpu().numpy()


def check_equal(gpu_iq, ref_iq, ctx=''):
    a = np.asarray(gpu_iq).view(np.uint32)
    b = np.asarray(ref_iq).view(np.uint32)
    if not np.array_equal(a, b):
        bad = np.argwhere(a != b)
        ai, aq = split_iq(a[tuple(bad[0])])
        bi, bq = split_iq(b[tuple(bad[0])])
        raise AssertionError('{}: {} mismatching samples, first at {}: gpu ({}, {}) ref ({}, {})'.format(
            ctx, len(bad), bad[0].tolist(), ai, aq, bi, bq))


def run_and_synthesize(emu, ps, cfg, n_shots, channels, n_samples, shot0=0):
    import torch
    emu.load(ps)
    out = alloc_device_outputs(cfg, n_shots, want=('summary', 'ev_main', 'ev_amp'))
    emu.run_device(cfg, n_shots, shot0, out)
    plan = ChannelPlan(ps, cfg, shot0, n_shots, channels, ELEM_PARAMS)
    iq = emu.synthesize(plan, out, n_samples)
    torch.cuda.synchronize()
    ref = oracle.dds(plan.desc, host(out['summary']), host(out['ev_main']), host(out['ev_amp']),
                     plan.env, plan.freq, n_samples, cfg.event_cap)
    return host(iq), ref


def test_config1_all_elements(emu):
    ps = ProgramSet(workloads.config1_linear())
    cfg = _abi.make_config(ps.cores_per_shot, event_cap=8, meas_cap=2)
    ch = [(s, 0, e) for s in range(3) for e in range(3)]
    g, r = run_and_synthesize(emu, ps, cfg, 3, ch, 16 * 1400)
    check_equal(g, r, 'config1')
    assert (g != 0).any()


def test_config2_ramsey_channels(emu):
    ps = ProgramSet(workloads.config2_ramsey(8, 100))
    cfg = _abi.make_config(8, n_groups=ps.n_groups, event_cap=8, meas_cap=2)
    rng = np.random.default_rng(1)
    n_shots = 300
    ch = [(int(s), int(c), int(e)) for s, c, e in zip(rng.integers(0, n_shots, 96), rng.integers(0, 8, 96),
                                                       rng.integers(0, 3, 96))]
    g, r = run_and_synthesize(emu, ps, cfg, n_shots, ch, 16 * 2048)
    check_equal(g, r, 'config2')


def test_config4_rb_virtual_z(emu):
    """RB: phase-register virtual Z, many strobes per lane (compaction over
    several 256-event blocks), pulse_reset at the start"""
    ps = ProgramSet(workloads.config4_rb(n_seq=8, depth=150, seed=3))
    cfg = _abi.make_config(ps.cores_per_shot, n_groups=ps.n_groups, event_cap=1024, meas_cap=4)
    ch = [(s, c, e) for s in range(16) for c in range(ps.cores_per_shot) for e in range(3)]
    g, r = run_and_synthesize(emu, ps, cfg, 16, ch, 16 * 8192)
    check_equal(g, r, 'config4')


def test_synthetic_edges_multi_chunk(emu):
    """spc / interp not powers of two, > one 64K-sample chunk, ragged tail,
    strobes on other elements, resets, overriding strobes, events past the
    end, empty lanes"""
    import torch
    rng = np.random.default_rng(7)
    cap, n_lanes = 40, 5
    summary = np.zeros((n_lanes, 8), np.uint32)
    ev = np.zeros((cap, n_lanes, 4), np.uint32)
    amp = np.zeros((cap, n_lanes), np.uint16)
    env_tab = pack_iq16(np.exp(1j * rng.uniform(0, 2 * np.pi, 4 * 64)) * rng.uniform(0, 1, 4 * 64))
    freq_tab = np.concatenate([DDSElementConfig(samples_per_clk=s).get_freq_buffer([f])
                               for s, f in ((16, 91.7e6), (3, -13.1e6), (5, 250e6), (1, 0.0))])
    for L in range(1, n_lanes):                     # lane 0 stays empty
        n = cap if L == 2 else cap - 3 * L
        t = np.sort(rng.integers(0, 30000, n)).astype(np.uint32)
        kind = (rng.random(n) < 0.15).astype(np.uint32)
        A = rng.integers(0, 60, n)
        Ln = rng.integers(0, 5, n)                  # 0 = CW
        envw = (A | (Ln << 12)).astype(np.uint32)
        cfgw = rng.integers(0, 4, n).astype(np.uint32)
        ev[:n, L, 0] = t
        ev[:n, L, 1] = t
        ev[:n, L, 2] = envw | (cfgw << 24) | (kind << 28)
        ev[:n, L, 3] = rng.integers(0, 1 << 17, n).astype(np.uint32) | (rng.integers(0, 5, n).astype(np.uint32) << 17)
        amp[:n, L] = rng.integers(0, 65536, n)
        summary[L, 2] = n + (5 if L == 2 else 0)    # lane 2 overflowed: count > cap
    ev[cap - 10, 3, :2] = 10 ** 9                   # lane 3's last event is beyond the window
    desc = []
    for L in range(n_lanes):
        for e, (spc, interp) in enumerate(((16, 1), (3, 3), (5, 2), (1, 1))):
            desc.append((L, e, spc, interp, 0, len(env_tab), 0, len(freq_tab) if L != 4 else 20))
    desc = np.array(desc, np.uint32)
    n_samples = 2 * 65536 + 4 * 37
    ref = oracle.dds(desc, summary, ev, amp, env_tab, freq_tab, n_samples, cap)

    dev = {'summary': torch.from_numpy(summary.view(np.int32)).cuda(),
           'ev_main': torch.from_numpy(ev.view(np.int32)).cuda(),
           'ev_amp': torch.from_numpy(amp.view(np.int16)).cuda()}
    plan = ChannelPlan.__new__(ChannelPlan)
    plan.desc, plan.env, plan.freq = desc, env_tab, freq_tab
    plan.n_lanes, plan.event_cap, plan._dev = n_lanes, cap, None
    plan._cols = {f: np.ascontiguousarray(desc[:, i]) for i, f in
                  enumerate(('ch_lane', 'ch_elem', 'spc', 'interp', 'env_off', 'env_len', 'freq_off', 'freq_len'))}
    iq = emu.synthesize(plan, dev, n_samples)
    torch.cuda.synchronize()
    check_equal(host(iq), ref, 'synthetic')
    assert (ref != 0).sum() > 1000


def test_bad_arguments_fail_loudly(emu):
    ps = ProgramSet(workloads.config1_linear())
    cfg = _abi.make_config(ps.cores_per_shot, event_cap=8, meas_cap=2)
    emu.load(ps)
    out = alloc_device_outputs(cfg, 2, want=('summary', 'ev_main', 'ev_amp'))
    emu.run_device(cfg, 2, 0, out)
    plan = ChannelPlan(ps, cfg, 0, 2, [(0, 0, 0)], ELEM_PARAMS)
    with pytest.raises(DpemuError):
        emu.synthesize(plan, out, 1002)               # not a multiple of 4
    plan.desc[0, 2] = 17
    plan._cols['spc'] = np.ascontiguousarray(plan.desc[:, 2])
    with pytest.raises(DpemuError):
        emu.synthesize(plan, out, 1024)               # spc out of range
