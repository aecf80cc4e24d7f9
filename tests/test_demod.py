"""The readout demodulation model (meas_model DEMOD; include/dpemu.h,
oracle/readout.c) on the CPU oracle: its fixed-point pieces
against float math, the accumulated I/Q against the float sum of the
demodulated return, and the physics it must show -- a rotated LO flips the
assignment, a detuned LO collapses the state separation, the window sets
meas_valid.  Parity unpinned by the reference (it has no readout model:
SURVEY.md §8c); the GPU is held to this oracle bit for bit
(tests/test_gpu_demod.py)."""

import math
import random

import numpy as np
import pytest

import oracle
from distributed_processor_amd import _abi, isa
from tests.progfuzz import pack_programs

TWO_PI = 2 * math.pi
RDRV, RDLO = 1, 2


def test_sin33_accuracy():
    """sin33(x) = sin(2 pi x / 2^33) 2^61 with relative accuracy ~1e-7, also next to every zero"""
    rng = random.Random(1)
    xs = [rng.randrange(-2 ** 40, 2 ** 40) for _ in range(3000)]
    xs += [q * 2 ** 31 + d for q in range(-4, 5) for d in (-3, -1, 0, 1, 2, 7, 1000, -1000, 2 ** 20)]
    for x in xs:
        got = oracle.sin33(x) / 2 ** 61
        k = round(x / 2 ** 31)                     # x = k pi/2 + r exactly: an accurate reference
        th = TWO_PI * (x - k * 2 ** 31) / 2 ** 33
        want = (math.sin(th), math.cos(th), -math.sin(th), -math.cos(th))[k % 4]
        assert abs(got - want) <= 2e-7 * abs(want) + 2 ** -58, x


def test_dirichlet_matches_float():
    rng = random.Random(2)
    cases = [(n, b) for n in (1, 2, 3, 250, 1000, 4096, 32768) for b in
             (0, 1, -1, 7, 2 ** 12, -2 ** 20, 2 ** 26, 2 ** 31 - 1, -2 ** 31, 12345678)]
    cases += [(rng.randint(1, 32768), rng.randrange(-2 ** 31, 2 ** 31)) for _ in range(2000)]
    for n, b in cases:
        got = oracle.dirichlet_q16(n, b & 0xFFFFFFFF) / 65536
        x = math.pi * b / 2 ** 32
        want = n if b == 0 else math.sin(n * x) / math.sin(x)
        assert abs(got - want) <= 2e-6 * n + 3 / 65536, (n, b, got, want)


# ------------------------------------------------------------------ programs
def ro_program(reads, t0=10, done=True):
    """pulse_reset, then per read (rdrv pulse, rdlo pulse `lo_at` later):
    reads = [dict(A, ph_d, fi_d, L_d, ph_lo, fi_lo, L_lo, lo_at, gap)]"""
    words = [isa.pulse_reset()]
    t = t0
    for r in reads:
        words.append(isa.pulse_cmd(freq_word=r.get('fi_d', 0), phase_word=r.get('ph_d', 0), amp_word=r.get('A', 40000),
                                   env_word=r.get('L_d', 250) << 12, cfg_word=RDRV, cmd_time=t))
        words.append(isa.pulse_cmd(freq_word=r.get('fi_lo', 0), phase_word=r.get('ph_lo', 0), amp_word=0xFFFF,
                                   env_word=r.get('L_lo', 250) << 12, cfg_word=RDLO, cmd_time=t + r.get('lo_at', 300)))
        t += r.get('gap', 3000)
    if done:
        words.append(isa.done_cmd())
    return words


def run_oracle(progs, ro_tabs, n_shots, demod, p1=0.5, meas_latency=32, meas_cap=4, seed=0x5EED, shot0=0):
    """progs: one program per core (one group); ro_tabs: per core (drive words, LO words)"""
    C = len(progs)
    words, offs, ni = pack_programs(progs)
    cfg = _abi.make_config(C, max_cycles=1 << 22, event_cap=16, meas_cap=meas_cap, meas_latency=meas_latency,
                           p1=p1, seed=seed, demod=demod)
    w = np.concatenate([np.asarray(t, np.uint32) for pair in ro_tabs for t in pair] or [np.zeros(0, np.uint32)])
    lens = [len(t) for pair in ro_tabs for t in pair]
    offsets = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint32)
    ro = (w, offsets[0::2], np.array(lens[0::2], np.uint32), offsets[1::2], np.array(lens[1::2], np.uint32))
    out = oracle.fast_run(cfg, words, offs, ni, np.arange(C, dtype=np.uint32), shot0, n_shots, ro=ro)
    return cfg, out


def expected_acc(cfg, ev, f_d, f_lo, state):
    """float model of one lane's readouts from its event records: the
    per-clock sum of (amp_eff / 2) e^{i psi_k} over the overlap"""
    res, t_ref, drive = [], 0, None
    for e in ev:
        t, kind, cfg_w = int(e[0]), int(e[1]) >> 28, (int(e[1]) >> 24) & 15
        L = (int(e[1]) >> 12) & 0xFFF
        words = L if L else 4096
        if kind == 1:
            t_ref = t
            continue
        if cfg_w & 3 == cfg.ro_drv_elem:
            drive = (t, words, int(e[2]) & 0x1FFFF, int(e[3]) & 0xFFFF)
        elif cfg_w & 3 == cfg.meas_elem:
            if drive is None:
                res.append(0j)
                continue
            n_lo = words * cfg.ro_cpw
            t_d, wd, ph_d, amp = drive
            r0 = t_d + cfg.ro_delay
            a, end = max(r0, t), min(t + n_lo, r0 + wd * cfg.ro_cpw)
            amp_eff = (amp * cfg.ro_gain[state]) >> 16
            k = np.arange(a, max(a, end), dtype=np.float64)
            psi = (f_d * (k - cfg.ro_delay - t_ref) + ph_d * 2 ** 15 + cfg.ro_theta[state]
                   - f_lo * (k - t_ref) - (int(e[2]) & 0x1FFFF) * 2 ** 15) * TWO_PI / 2 ** 32
            res.append(amp_eff / 2 * np.exp(1j * psi).sum())
    return res


@pytest.mark.parametrize('case', range(8))
def test_acc_matches_float_sum(case):
    """sigma 0: every readout's accumulated {I, Q} equals the float sum of the
    demodulated return within the fixed-point error (~1e-5 of the signal)"""
    rng = random.Random(100 + case)
    f_d = rng.getrandbits(32)
    det = [0, 1, -3, 2 ** 16, 37 * 2 ** 20, rng.getrandbits(32), 2 ** 31, rng.randint(-5000, 5000)][case]
    f_lo = (f_d - det) & 0xFFFFFFFF
    reads = [dict(A=rng.randint(1000, 65535), ph_d=rng.getrandbits(17), ph_lo=rng.getrandbits(17),
                  L_d=rng.choice([0, 1, 7, 250, 1000]), L_lo=rng.choice([1, 25, 250, 4095]),
                  lo_at=rng.choice([3, 5, 300, 900]), gap=rng.choice([20000, 70000])) for _ in range(3)]
    demod = dict(drv_elem=RDRV, cpw=rng.randint(1, 8), delay=rng.choice([0, 3, 300]),
                 theta=(rng.uniform(-4, 4), rng.uniform(-4, 4)), gain=(rng.random(), 1.0))
    for state, p1 in ((0, 0.0), (1, 1.0)):
        cfg, out = run_oracle([ro_program(reads)], [([f_d], [f_lo])], 1, demod, p1=p1)
        ev = out['events'][:int(out['summary'][0, 2]), 0]
        want = expected_acc(cfg, ev, f_d, f_lo, state)
        got = out['acc'][:len(want), 0]
        assert len(want) == 3 and int(out['summary'][0, 5]) == 3
        for (gi, gq), w in zip(got, want):
            tol = 3e-5 * abs(w) + 4                 # c15 / s15 are Q15; D and sin33 ~1e-7 relative
            assert abs(gi - w.real) <= tol and abs(gq - w.imag) <= tol, (case, state, gi, gq, w)


def test_window_sets_meas_valid_in_order():
    """meas_valid = readout strobe + window (L * cpw) + meas_latency, and never
    before the lane's previous result (a short window right after a long one)"""
    reads = [dict(L_lo=1000, lo_at=3, gap=40), dict(L_lo=2, lo_at=3, gap=3000)]
    cfg, out = run_oracle([ro_program(reads)], [([0], [0])], 1, dict(drv_elem=RDRV, cpw=4), meas_latency=32)
    ev = out['events'][:int(out['summary'][0, 2]), 0]
    t_lo = [int(e[0]) for e in ev if (int(e[1]) >> 24) & 3 == RDLO and (int(e[1]) >> 28) == 0]
    tv = [int(x) for x in out['meas'][:2, 0, 0]]
    assert tv[0] == t_lo[0] + 1000 * 4 + 32
    assert t_lo[1] + 2 * 4 + 32 < tv[0] and tv[1] == tv[0] + 1


def test_no_drive_reads_noise_only():
    words = [isa.pulse_reset(), isa.pulse_cmd(freq_word=0, phase_word=0, amp_word=0xFFFF, env_word=250 << 12,
                                              cfg_word=RDLO, cmd_time=10), isa.done_cmd()]
    cfg, out = run_oracle([words], [([5], [5])], 64, dict(drv_elem=RDRV, sigma=0.0))
    assert not out['acc'][0].any()
    cfg, out = run_oracle([words], [([5], [5])], 64, dict(drv_elem=RDRV, sigma=1.0))
    acc = out['acc'][0].astype(np.int64)
    assert np.abs(acc).max() <= 131070 and acc.std() > 10000      # z * 1.0, |z| <= 131070


def _assign(demod, ph_lo=0, f_lo=None, n=4000, sigma=None, p1=0.5):
    f_d = 0x12345678
    f_lo = f_d if f_lo is None else f_lo
    reads = [dict(A=40000, ph_d=0, ph_lo=ph_lo, L_d=250, L_lo=250, lo_at=300)]
    d = dict(demod)
    if sigma is not None:
        d['sigma'] = sigma
    return run_oracle([ro_program(reads)], [([f_d], [f_lo])], n, d, p1=p1)


def _base_demod(axis):
    return dict(drv_elem=RDRV, cpw=4, delay=300, theta=(math.pi, 0.0), gain=(1.0, 1.0), axis=axis, thr=0)


def _signal_axis(f=0x12345678, delay=300, ph_lo=0):
    """the state-1 direction: psi = -F delay + (0 - ph_lo) 2^15 + theta_1 (beta = 0)"""
    return ((-f * delay - ph_lo * 2 ** 15) % 2 ** 32) * TWO_PI / 2 ** 32


def _states(n, p1=0.5, seed=0x5EED):
    thr = _abi.prob_to_threshold(p1)
    return np.array([oracle.lib().oracle_philox_u32(seed, s, 0, 0) < thr for s in range(n)], np.uint32)


def test_pi_rotation_flips_assignment():
    """rotating the rdlo phase word by pi negates the demodulated signal: with
    the discriminator calibrated for phase 0, the assignment flips"""
    ax = _signal_axis()
    n = 3000
    states = _states(n)
    _, tuned = _assign(_base_demod(ax), n=n, sigma=60.0)
    _, flipped = _assign(_base_demod(ax), ph_lo=2 ** 16, n=n, sigma=60.0)
    bt, bf = tuned['meas'][0, :, 1], flipped['meas'][0, :, 1]
    assert (bt == states).mean() > 0.97
    assert (bf == states).mean() < 0.03
    # noise-free: the signal itself is negated (to the last unit)
    _, a = _assign(_base_demod(ax), n=64, sigma=0.0)
    _, b = _assign(_base_demod(ax), ph_lo=2 ** 16, n=64, sigma=0.0)
    assert np.abs(a['acc'][0].astype(np.int64) + b['acc'][0]).max() <= 2
    assert np.abs(a['acc'][0]).min() > 1000000


def test_detuned_lo_collapses_separation():
    """an LO detuned by ~5 MHz (10 turns over the 1000-clock window) averages
    the return out: the state separation collapses and the assignment is chance"""
    ax = _signal_axis()
    det = int(0.01 * 2 ** 32)
    sep = {}
    for name, f_lo in (('tuned', None), ('detuned', (0x12345678 - det) & 0xFFFFFFFF)):
        m = []
        for p1 in (0.0, 1.0):
            _, o = _assign(_base_demod(ax), f_lo=f_lo, n=8, sigma=0.0, p1=p1)
            m.append(o['acc'][0].astype(np.float64).mean(axis=0))
        sep[name] = float(np.hypot(*(m[1] - m[0])))
    assert sep['tuned'] > 1.9e7                       # 2 x 1000 clocks x 39999 / 2 x 0.9...
    assert sep['detuned'] < 0.01 * sep['tuned']
    n = 3000
    states = _states(n)
    _, o = _assign(_base_demod(ax), f_lo=(0x12345678 - det) & 0xFFFFFFFF, n=n, sigma=60.0)
    assert 0.4 < (o['meas'][0, :, 1] == states).mean() < 0.6


def test_outcomes_drive_fproc_branches():
    """DEMOD outcomes feed fproc_meas exactly like the other models (config 3
    with the demodulation model, oracle_fast vs oracle_rtl on the whole shot)"""
    from distributed_processor_amd import workloads
    from distributed_processor_amd.emulator import ProgramSet
    ps = ProgramSet(workloads.config3_active_reset(4))
    cfg = _abi.make_config(4, max_cycles=50000, event_cap=16, trace_cap=16, meas_cap=4, meas_latency=32,
                           demod=workloads.config3_demod(ps))
    ro = ps.readout_freqs(RDRV, RDLO)
    fast = oracle.fast_run(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, 0, 64, ro=ro)
    summ = _abi.unpack_summary(fast['summary'])
    assert (summ['status'] == _abi.ST_DONE).all() and (summ['n_meas'] == 2).all()
    scfg = oracle.shot_cfg_from_config(cfg)
    w, d_off, d_len, l_off, l_len = ro
    for s in range(0, 64, 9):
        progs = [ps.program(0, c) for c in range(4)]
        tabs = [(w[d_off[p]:d_off[p] + d_len[p]], w[l_off[p]:l_off[p] + l_len[p]]) for p in ps.table[:4]]
        ok, lanes = oracle.rtl_run_shot(scfg, progs, s, 20000, 16, 16, 4, ro_tabs=tabs)
        assert ok
        for c in range(4):
            L = c * 64 + s
            assert lanes[c]['n_events'] == summ['n_events'][L]
            np.testing.assert_array_equal(lanes[c]['events'], fast['events'][:lanes[c]['n_events'], L])
            np.testing.assert_array_equal(lanes[c]['meas'], fast['meas'][:2, L])
            np.testing.assert_array_equal(lanes[c]['acc'], fast['acc'][:2, L])
    # the calibrated discriminator tells the prepared states apart
    states = np.array([[oracle.lib().oracle_philox_u32(0x5EED, s, c, 0) < (1 << 31) for s in range(64)]
                       for c in range(4)], np.uint32)
    first = fast['meas'][0, :, 1].reshape(4, 64)
    assert (first == states).mean() > 0.9
