"""CPU checks of the DDS restatement (oracle/dds_ref.c) and the host plan.

The reference has no signal generator (the DSP is external QubiC gateware,
README.md:3), so DDS sample parity is pinned by oracle_dds alone ("parity
unpinned" against the reference).  These tests pin the
oracle's fixed point against a float model of the same spec within the
stated quantisation tolerance, and check the event-selection rules
(element filter, latest strobe wins, pulse end, CW, pulse_reset phase
reference) exactly.
"""

import numpy as np
import pytest

import oracle
from distributed_processor_amd import _abi, workloads
from distributed_processor_amd.dds import ChannelPlan, split_iq
from distributed_processor_amd.emulator import ProgramSet
from distributed_processor_amd.hwconfig import DDSElementConfig, pack_iq16

# |fixed - float| bound in LSB of a full-scale 16-bit output: carrier phase
# truncated to 4096 table entries (<= 2*pi/4096 * 32767 ~ 50 LSB) plus Q15
# rounding of the env and rotation words and the three products.
FLOAT_TOL_LSB = 64


def events(lane_events, event_cap=16):
    """host event arrays in dpemu_run layout for one lane per list entry;
    each event: dict(t, kind=0, cfg=elem, env=word, phase, freq, amp)"""
    n_lanes = len(lane_events)
    summary = np.zeros((n_lanes, 8), np.uint32)
    ev = np.zeros((event_cap, n_lanes, 4), np.uint32)
    for L, evs in enumerate(lane_events):
        summary[L, 2] = len(evs)
        for k, e in enumerate(evs[:event_cap]):
            ev[k, L] = (e['t'], (e.get('env', 0) & 0xFFFFFF) | (e.get('cfg', 0) << 24) | (e.get('kind', 0) << 28),
                        (e.get('phase', 0) & 0x1FFFF) | (e.get('freq', 0) << 17), e.get('amp', 0) & 0xFFFF)
    return summary, ev


def s16(x):
    x &= 0xFFFF
    return x - 0x10000 if x & 0x8000 else x


def float_model(j, spc, interp, st_t, t_ref, env_iq, A, L, f0_word, phase17, rot_words, amp):
    n, k = j // spc, j % spc
    es = (j - st_t * spc) // interp if L else 0
    if L and es >= 4 * L:
        return 0j
    w = int(env_iq[4 * A + es])
    e = complex(s16(w >> 16), s16(w)) / 32768.0
    theta = 2 * np.pi * (((f0_word * (n - t_ref)) % 2 ** 32) / 2 ** 32 + phase17 / 2 ** 17)
    c = np.exp(1j * theta)
    if k:
        r = int(rot_words[k])
        c *= complex(s16(r >> 16), s16(r)) / 32768.0
    return e * c * amp / 65536.0 * 32768.0


def test_sin_lut_matches_library():
    from distributed_processor_amd._native import load_library
    L = load_library()
    lib_lut = np.zeros(4096, np.int16)
    assert L.dpemu_dds_sin_lut(lib_lut.ctypes.data) == 0
    ref = oracle.dds_sin_lut()
    np.testing.assert_array_equal(lib_lut, ref)
    x = np.round(32767 * np.sin(2 * np.pi * np.arange(4096) / 4096)).astype(np.int16)
    assert np.abs(ref.astype(int) - x).max() <= 1


@pytest.mark.parametrize('spc,interp', [(16, 1), (16, 16), (4, 4), (1, 1), (3, 2)])
def test_oracle_vs_float_model(spc, interp):
    el = DDSElementConfig(samples_per_clk=spc, interp_ratio=interp)
    env = {'env_func': 'gaussian', 'paradict': {'sigmas': 3, 'twidth': 40e-9}}
    env_buf = el.get_env_buffer(env)
    f = 137.3e6
    freq_buf = el.get_freq_buffer([None, f])
    L = len(env_buf) // 4
    st = dict(t=7, cfg=1, env=el.get_env_word(0, len(env_buf)), phase=12345, freq=1, amp=50000)
    summary, ev = events([[dict(t=2, kind=1), st]])
    n_samples = 4 * ((st['t'] + 40) * spc // 4)
    desc = np.array([[0, 1, spc, interp, 0, len(env_buf), 0, len(freq_buf)]], np.uint32)
    iq = oracle.dds(desc, summary, ev, env_buf, freq_buf, n_samples, 16)
    I, Q = split_iq(iq[0])
    got = I.astype(float) + 1j * Q.astype(float)
    want = np.array([float_model(j, spc, interp, 7, 2, env_buf, 0, L, int(freq_buf[16]), 12345,
                                 freq_buf[16:32], 50000) if j >= 7 * spc else 0j for j in range(n_samples)])
    assert np.all(got[:7 * spc] == 0)
    err = np.abs(got - want)
    assert err.max() <= FLOAT_TOL_LSB, err.max()
    assert np.abs(got).max() > 1000        # the pulse is there


def test_selection_rules():
    """element filter, later strobe wins, pulse end, CW, reset re-references phase"""
    spc, interp = 4, 1
    el = DDSElementConfig(samples_per_clk=spc, interp_ratio=interp)
    env_buf = np.concatenate([pack_iq16(np.full(8, 0.5)), pack_iq16(np.full(4, 0.9j))])
    freq_buf = el.get_freq_buffer([0.0])
    sq = el.get_env_word(0, 8)                    # 8 samples = 2 cycles at spc 4
    cw = el.get_cw_env_word(8)
    evs = [dict(t=3, cfg=0, env=sq, amp=65535),
           dict(t=4, cfg=1, env=sq, amp=65535),     # other element: ignored
           dict(t=10, cfg=0, env=sq, amp=65535),
           dict(t=11, cfg=0, env=cw, amp=32768),    # overrides the square mid-pulse
           dict(t=20, cfg=0, env=sq, amp=0)]
    summary, ev = events([evs])
    desc = np.array([[0, 0, spc, interp, 0, len(env_buf), 0, len(freq_buf)]], np.uint32)
    iq = oracle.dds(desc, summary, ev, env_buf, freq_buf, 4 * 24, 16)
    I, Q = split_iq(iq[0])
    cyc_I = I.reshape(-1, spc)[:, 0]
    cyc_Q = Q.reshape(-1, spc)[:, 0]
    assert list(cyc_I[:3]) == [0, 0, 0]
    assert cyc_I[3] == cyc_I[4] and 16000 < cyc_I[3] < 16500          # 0.5 * 0.99998
    assert cyc_I[5] == 0 and cyc_I[6] == 0                               # ended after 8 samples
    assert cyc_I[10] > 16000 and cyc_I[11] == 0 and 14000 < cyc_Q[11] < 15000   # CW 0.9j * 0.5
    assert cyc_Q[19] == cyc_Q[11]                                         # CW holds
    assert np.all(I[4 * 20:] == 0) and np.all(Q[4 * 20:] == 0)            # amp 0


def test_pulse_reset_phase_reference():
    spc = 4
    el = DDSElementConfig(samples_per_clk=spc, interp_ratio=1)
    env_buf = pack_iq16(np.ones(4))
    freq_buf = el.get_freq_buffer([10e6])
    cw = el.get_cw_env_word(0)
    base = [dict(t=0, cfg=2, env=cw, amp=65535)]
    s0, e0 = events([base])
    s1, e1 = events([base + [dict(t=50, kind=1)]])
    desc = np.array([[0, 2, spc, 1, 0, len(env_buf), 0, len(freq_buf)]], np.uint32)
    iq0 = oracle.dds(desc, s0, e0, env_buf, freq_buf, 4 * 80, 16)[0]
    iq1 = oracle.dds(desc, s1, e1, env_buf, freq_buf, 4 * 80, 16)[0]
    np.testing.assert_array_equal(iq0[:200], iq1[:200])
    np.testing.assert_array_equal(iq1[200:200 + 4 * 30], iq0[:4 * 30])     # phase restarts at t=50


def test_plan_from_workload_and_oracle_timeline():
    """config1: qdrv X90 at 5, rdrv at 21, rdlo at 321 -> I/Q non-zero exactly there"""
    ps = ProgramSet(workloads.config1_linear())
    cfg = _abi.make_config(ps.cores_per_shot, n_groups=ps.n_groups, event_cap=8, meas_cap=2)
    out = oracle.fast_run(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, 0, 2, 1,
                          want=('summary', 'events'))
    params = {i: (e['samples_per_clk'], e['interp_ratio']) for i, e in enumerate(workloads.ELEMS)}
    plan = ChannelPlan(ps, cfg, 0, 2, [(1, 0, 0), (1, 0, 1), (1, 0, 2)], params)
    assert plan.desc[:, 0].tolist() == [1] * 3               # core 0 of shot 1: lane 0 * 2 + 1
    iq = oracle.dds(plan.desc, out['summary'], out['events'], plan.env, plan.freq,
                    4 * 1400 * 4, 8)
    first = []
    for c in range(3):
        spc = params[c][0]
        I, Q = split_iq(iq[c])
        nz = np.nonzero((I != 0) | (Q != 0))[0]
        first.append(int(nz[0]) // spc if len(nz) else None)
    ev = out['events'][:, 1]
    strobe_t = {int((w[1] >> 24) & 3): int(w[0]) for w in ev[:int(out['summary'][1, 2])]
                if (w[1] >> 28) == 0}
    # envelopes may open with zero samples (the readout's cosine ramp): the
    # first non-zero output lies in the strobe's first few cycles
    for c in range(3):
        assert strobe_t[c] <= first[c] <= strobe_t[c] + 2, (c, first, strobe_t)


def test_plan_rejects_bad_channels():
    ps = ProgramSet(workloads.config1_linear())
    cfg = _abi.make_config(ps.cores_per_shot, event_cap=8)
    with pytest.raises(ValueError):
        ChannelPlan(ps, cfg, 0, 2, [(2, 0, 0)], {0: (16, 1)})
    with pytest.raises(ValueError):
        ChannelPlan(ps, cfg, 0, 2, [(0, 0, 3)], {0: (16, 1)})
