"""Synthetic workloads of BASELINE.json, built at the assembler level.

The reference compiler cannot run here (it needs the absent ``qubitconfig``
package), so programs are written directly as machine code
with this package's ISA encoder and ``DDSElementConfig`` word conversions,
mirroring what distproc's compiler + assembler emit for the same circuits
(compare python/test/test_outputs/test_linear_compile_out.txt):

* config 1 -- single-core X90 + readout (the reference's golden program)
* config 2 -- 8-core Ramsey sweep, 100 delay points selected by shot
* config 3 -- 8-core active reset: sync, read, hold, jump_fproc on the own
              measurement, conditional X180, sync, read
* config 4 -- 2-qubit randomized benchmarking, depth-D random Clifford
              sequences with virtual-Z phase registers (long programs)

Channel layout per core follows python/test/channel_config.json: element 0
qdrv (16 samples/clk), element 1 rdrv (16/clk, interp 16), element 2 rdlo
(4/clk, interp 4); cfg word = element index, so readouts are cfg & 3 == 2.
"""

from __future__ import annotations

from collections import OrderedDict
from typing import Dict, List, Sequence

import numpy as np

from . import isa
from .hwconfig import DDSElementConfig

ELEMS = (dict(samples_per_clk=16, interp_ratio=1),     # qdrv
         dict(samples_per_clk=16, interp_ratio=16),    # rdrv
         dict(samples_per_clk=4, interp_ratio=4))      # rdlo
QDRV, RDRV, RDLO = 0, 1, 2

X90_ENV = {'env_func': 'DRAG', 'paradict': {'alpha': -0.26, 'sigmas': 3, 'delta': -268e6, 'twidth': 32e-9}}
RDRV_ENV = {'env_func': 'cos_edge_square', 'paradict': {'ramp_fraction': 0.25, 'twidth': 2e-6}}
RDLO_ENV = {'env_func': 'square', 'paradict': {'phase': 0.0, 'amplitude': 1.0, 'twidth': 2e-6}}
X90_CLKS = 16          # 32 ns
READ_CLKS = 1000       # 2 us
RDLO_DELAY = 300       # rdrv -> rdlo, as in test_linear_compile_out.txt (21 -> 321)


class CoreBuilder:
    """Minimal assembler for one core: machine words + env/freq buffers."""

    def __init__(self):
        self.elems = [DDSElementConfig(**e) for e in ELEMS]
        self.words: List[int] = []
        self._envs = [OrderedDict() for _ in ELEMS]
        self._env_words = [dict() for _ in ELEMS]
        self._freqs: List[List[float]] = [[] for _ in ELEMS]
        self._env_len = [0] * len(ELEMS)

    def env_word(self, elem, env) -> int:
        key = repr(env)
        if key not in self._env_words[elem]:
            buf = self.elems[elem].get_env_buffer(env)
            start = self._env_len[elem]
            self._envs[elem][key] = buf
            self._env_words[elem][key] = self.elems[elem].get_env_word(start, len(buf))
            self._env_len[elem] += len(buf)
        return self._env_words[elem][key]

    def freq_addr(self, elem, f) -> int:
        if f not in self._freqs[elem]:
            self._freqs[elem].append(f)
        return self.elems[elem].get_freq_addr(self._freqs[elem].index(f))

    def pulse(self, elem, freq, phase, amp, env, t=None, phase_reg=None, amp_reg=None):
        e = self.elems[elem]
        kw = dict(freq_word=self.freq_addr(elem, freq), env_word=self.env_word(elem, env),
                  cfg_word=e.get_cfg_word(elem, None), cmd_time=t)
        if phase_reg is not None:
            kw['phase_regaddr'] = phase_reg
        else:
            kw['phase_word'] = e.get_phase_word(phase)
        if amp_reg is not None:
            kw['amp_regaddr'] = amp_reg
        else:
            kw['amp_word'] = e.get_amp_word(amp)
        self.words.append(isa.pulse_cmd(**kw))

    def emit(self, word: int):
        self.words.append(int(word))

    def buffers(self):
        env = [np.concatenate(list(d.values())).astype(np.uint32) if d else np.zeros(0, np.uint32)
               for d in self._envs]
        freq = [e.get_freq_buffer(f).astype(np.uint32) if f else np.zeros(0, np.uint32)
                for e, f in zip(self.elems, self._freqs)]
        return env, freq

    def assembled(self):
        env, freq = self.buffers()
        return {'cmd_buf': isa.words_to_bytes(self.words), 'env_buffers': [b.tobytes() for b in env],
                'freq_buffers': [b.tobytes() for b in freq]}


def qubit_params(core):
    """deterministic per-qubit drive/readout parameters (qubitcfg.json-like)"""
    return dict(fq=4.4e9 + 0.1e9 * core, fr=6.5e9 + 0.05e9 * core, ax90=0.12 + 0.05 * (core % 8),
                ar=0.6, rdlo_phase=(0.7 * core) % (2 * np.pi))


def readout(b: CoreBuilder, q, t):
    b.pulse(RDRV, q['fr'], 0.0, q['ar'], RDRV_ENV, t)
    b.pulse(RDLO, q['fr'], q['rdlo_phase'], 1.0, RDLO_ENV, t + RDLO_DELAY)
    return t + RDLO_DELAY + READ_CLKS


# ---------------------------------------------------------------- config 1
def config1_linear(core=0):
    """X90 qdrv @5, read rdrv @21, rdlo @321 (test_linear_compile_out.txt Q0)."""
    q = qubit_params(core)
    b = CoreBuilder()
    b.emit(isa.pulse_reset())
    b.pulse(QDRV, q['fq'], 0.0, q['ax90'], X90_ENV, 5)
    readout(b, q, 21)
    b.emit(isa.done_cmd())
    return {str(core): b.assembled()}


# ---------------------------------------------------------------- config 2
def config2_ramsey(n_cores=8, n_points=100, tau_step=4):
    """Ramsey: X90 @5, X90 @(21 + tau_k), read; tau_k = tau_step * k.
    Returns a list of n_points assembled-program dicts (group k = shot % n_points)."""
    groups = []
    for k in range(n_points):
        tau = tau_step * k
        prog = {}
        for c in range(n_cores):
            q = qubit_params(c)
            b = CoreBuilder()
            b.emit(isa.pulse_reset())
            b.pulse(QDRV, q['fq'], 0.0, q['ax90'], X90_ENV, 5)
            b.pulse(QDRV, q['fq'], 0.0, q['ax90'], X90_ENV, 21 + tau)
            readout(b, q, 37 + tau)
            b.emit(isa.done_cmd())
            prog[str(c)] = b.assembled()
        groups.append(prog)
    return groups


# ---------------------------------------------------------------- config 3
HOLD_CLKS = 64    # hwconfig.FPROC_MEAS_CLKS: idle after the readout window


def config3_active_reset(n_cores=8):
    """sync; read; hold; if (1 == meas) X90 X90; sync; read; done."""
    prog = {}
    for c in range(n_cores):
        q = qubit_params(c)
        b = CoreBuilder()
        b.emit(isa.pulse_reset())
        b.emit(isa.sync(0))
        t_end = readout(b, q, 10)
        t_idle = t_end + HOLD_CLKS
        b.emit(isa.idle(t_idle))
        jf = len(b.words)
        b.emit(0)                                      # jump_fproc placeholder
        b.emit(isa.jump_i(jf + 4))                     # -> second sync
        t1 = t_idle + 3 + 8 + 4                        # decode after jump_fproc (taken) + slack
        b.pulse(QDRV, q['fq'], 0.0, q['ax90'], X90_ENV, t1)
        b.pulse(QDRV, q['fq'], 0.0, q['ax90'], X90_ENV, t1 + X90_CLKS)
        b.words[jf] = isa.alu_cmd('jump_fproc', 'i', 1, 'eq', jump_cmd_ptr=jf + 2, func_id=c)
        b.emit(isa.sync(1))
        readout(b, q, 10)
        b.emit(isa.done_cmd())
        prog[str(c)] = b.assembled()
    return prog


CONFIG3_MEAS_LATENCY = READ_CLKS + 32   # rdlo strobe -> meas_valid, inside the 64-clock hold


# ---------------------------------------------------------------- config 4
# single-qubit Cliffords as X90 / Y90 pulses with virtual Z (phase register);
# index -> (list of ('x'|'y'), z quarter turns applied after)
def _clifford_table():
    seqs = []
    for pre in ([], ['x'], ['y'], ['x', 'x'], ['x', 'y'], ['y', 'x']):
        for z in range(4):
            seqs.append((pre, z))
    return seqs


CLIFFORDS = _clifford_table()    # 24 entries


def config4_rb(n_seq=1000, depth=200, seed=0x5EED, n_cores=2):
    """2-qubit RB-like sequences: per layer each qubit plays a random Clifford
    (<= 2 pulses, virtual Z by reg_alu on its phase register), and with
    probability 1/2 a cross-resonance pulse on core 0.  Slots are fixed-length
    so the cores stay aligned.  Returns n_seq assembled-program dicts."""
    rng = np.random.default_rng(seed)
    quarter = 2 ** 15        # pi/2 in 17-bit phase words
    groups = []
    for s in range(n_seq):
        cliffs = rng.integers(0, 24, size=(depth, n_cores))
        cr = rng.integers(0, 2, size=depth)
        prog = {}
        for c in range(n_cores):
            q = qubit_params(c)
            b = CoreBuilder()
            preg = 1
            b.emit(isa.pulse_reset())
            b.emit(isa.alu_cmd('reg_alu', 'i', 0, 'id0', 0, preg))         # phase reg = 0
            t = 10
            for d in range(depth):
                pre, z = CLIFFORDS[cliffs[d, c]]
                for i, ax in enumerate(pre):
                    b.emit(isa.alu_cmd('reg_alu', 'i', quarter if ax == 'y' else 0, 'add', preg, 2))
                    b.pulse(QDRV, q['fq'], 0.0, q['ax90'], X90_ENV, t + X90_CLKS * i, phase_reg=2)
                if z:
                    b.emit(isa.alu_cmd('reg_alu', 'i', z * quarter, 'add', preg, preg))
                if c == 0 and cr[d]:
                    b.pulse(QDRV, qubit_params(1)['fq'], 0.0, 0.3, X90_ENV, t + 2 * X90_CLKS)
                t += 3 * X90_CLKS + 16
            readout(b, q, t)
            b.emit(isa.done_cmd())
            prog[str(c)] = b.assembled()
        groups.append(prog)
    return groups
