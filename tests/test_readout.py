"""Readout measurement model (meas_model READOUT, include/dpemu.h).

Build-defined, so parity is pinned by this build's own oracle (bit-exact
GPU/oracle_fast/oracle_rtl comparisons live in test_fast_vs_rtl.py and
test_gpu_parity.py).  Here: the model behaves as documented -- assignment
errors follow the discriminator geometry (normal approximation of the
Irwin-Hall(4) noise), the readout amp word scales the separation, and the
STATE model is unchanged by the new fields.
"""

import math

import numpy as np
import pytest

from distributed_processor_amd import _abi, isa
from tests.progfuzz import pack_programs

SIGMA_Z = math.sqrt(4 * (65536 ** 2 - 1) / 12)      # Irwin-Hall(4) of 16-bit uniforms


def readout_program(amp_word, n_reads=2, env_word=0):
    """n_reads readout strobes (cfg 2 = meas_elem) with amp `amp_word`, then done"""
    w = []
    for k in range(n_reads):
        w.append(isa.pulse_i(0, 0, amp_word, env_word, 2, 10 + 20 * k))
    w.append(isa.done_cmd())
    return w


def outcomes(amp_word, p1, readout, n_shots=60000, n_reads=2, seed=11, env_word=0):
    import oracle
    cfg = _abi.make_config(1, event_cap=8, meas_cap=8, p1=p1, readout=readout, seed=seed)
    words, offs, ni = pack_programs([readout_program(amp_word, n_reads, env_word)])
    f = oracle.fast_run(cfg, words, offs, ni, np.zeros(1, np.uint32), 0, n_shots, want=('summary',))
    bits = _abi.unpack_summary(f['summary'])['meas_bits']
    return np.stack([(bits >> k) & 1 for k in range(n_reads)], axis=1)


def phi(x):
    return 0.5 * (1 + math.erf(x / math.sqrt(2)))


@pytest.mark.parametrize('amp,sep,sigma,thr', [(65535, 20000, 1.0, 0), (65535, 20000, 0.5, 5000),
                                               (32768, 40000, 1.0, -3000), (0, 40000, 1.0, 0)])
def test_assignment_errors_follow_the_geometry(amp, sep, sigma, thr):
    s = (sep * amp) >> 16
    sx = SIGMA_Z * sigma
    for p1, state in ((0.0, 0), (1.0, 1)):
        b = outcomes(amp, p1, dict(sep=sep, sigma=sigma, thr=thr))
        mean = (s if state else -s)
        expect = 1 - phi((thr - mean) / sx)                # P(x > thr)
        got = float(b.mean())
        tol = 0.006 + 5 * math.sqrt(expect * (1 - expect) / b.size + 1e-12)
        assert abs(got - expect) < tol, (p1, got, expect)


def test_state_model_unchanged_and_readout_independent_draws():
    st = outcomes(65535, 0.3, None, n_shots=40000)
    assert abs(st.mean() - 0.3) < 0.01
    ro = outcomes(65535, 0.3, dict(sep=200000, sigma=0.05, thr=0), n_shots=40000)
    np.testing.assert_array_equal(st, ro)                    # high SNR: readout = state
    # two readouts of one shot are independent draws of noise and state
    b = outcomes(65535, 0.5, dict(sep=0, sigma=1.0, thr=0), n_shots=40000)
    assert abs(np.corrcoef(b[:, 0], b[:, 1])[0, 1]) < 0.03


@pytest.mark.parametrize('W,win', [(25, 100), (100, 100), (400, 100), (10, 0)])
def test_window_scales_separation(W, win):
    """ro_win: the separation scales by min(W, ro_win) / ro_win, W the readout
    strobe's envelope-length field; ro_win 0 ignores the window"""
    amp, sep, sigma, thr = 65535, 60000, 1.0, 0
    s = (sep * amp) >> 16
    if win:
        s = (s * (min(W, win) * ((1 << 24) // win))) >> 24
    sx = SIGMA_Z * sigma
    for p1, state in ((0.0, 0), (1.0, 1)):
        b = outcomes(amp, p1, dict(sep=sep, sigma=sigma, thr=thr, win=win), env_word=W << 12)
        expect = 1 - phi((thr - (s if state else -s)) / sx)
        got = float(b.mean())
        tol = 0.006 + 5 * math.sqrt(expect * (1 - expect) / b.size + 1e-12)
        assert abs(got - expect) < tol, (W, win, p1, got, expect)


def test_make_config_rejects_bad_readout():
    with pytest.raises(ValueError):
        _abi.make_config(1, readout=dict(sep=2 ** 31, sigma=1.0))
    with pytest.raises(ValueError):
        _abi.make_config(1, readout=dict(sep=1, sigma=1.0, win=4096))
