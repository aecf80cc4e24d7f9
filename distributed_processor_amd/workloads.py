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
* config 4 -- two-qubit Clifford randomized benchmarking (config4_rb2q):
              depth-D random elements of the 11,520-element group and the
              recovery Clifford, decomposed into X90 / Y90 / X-90 / Y-90,
              virtual Z on a frame register, and CNOT by cross resonance
              (clifford2q.py); config4_rb is the older RB-SHAPED generator
              (single-qubit Cliffords + random CR pulses, no recovery), kept as
              a source of small divergent register programs for kernel tests
              and as the DDS leg's 8-core timelines

Channel layout per core follows python/test/channel_config.json: element 0
qdrv (16 samples/clk), element 1 rdrv (16/clk, interp 16), element 2 rdlo
(4/clk, interp 4); cfg word = element index, so readouts are cfg & 3 == 2.
"""

from __future__ import annotations

import functools
import os
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

    def pulse(self, elem, freq, phase, amp, env, t=None, phase_reg=None, amp_reg=None, phase_word=None):
        e = self.elems[elem]
        kw = dict(freq_word=self.freq_addr(elem, freq), env_word=self.env_word(elem, env),
                  cfg_word=e.get_cfg_word(elem, None), cmd_time=t)
        if phase_reg is not None:
            kw['phase_regaddr'] = phase_reg
        else:
            kw['phase_word'] = e.get_phase_word(phase) if phase_word is None else int(phase_word)
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


def config3_active_reset(n_cores=8, extra_pulses=0, read_shift=0):
    """sync; read; hold; if (1 == meas) X90 X90; sync; read; done.
    extra_pulses: that many X90s after the second readout (per-command cost probes).
    read_shift: core c conditions on core (c + read_shift) % n_cores's outcome
    (fproc_meas id, hdl/fproc_meas.sv:18-35: a cross-core read, as in
    cocotb/fproc_meas/test_meas.py:62-83); 0 = its own."""
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
        b.words[jf] = isa.alu_cmd('jump_fproc', 'i', 1, 'eq', jump_cmd_ptr=jf + 2,
                                  func_id=(c + read_shift) % n_cores)
        b.emit(isa.sync(1))
        t_x = readout(b, q, 10)
        for k in range(extra_pulses):
            b.pulse(QDRV, q['fq'], 0.0, q['ax90'], X90_ENV, t_x + k * X90_CLKS)
        b.emit(isa.done_cmd())
        prog[str(c)] = b.assembled()
    return prog


CONFIG3_MEAS_LATENCY = READ_CLKS + 32   # rdlo strobe -> meas_valid, inside the 64-clock hold
CONFIG3_DEMOD_LATENCY = 32              # DEMOD: the window (READ_CLKS) comes first, then this


def config3_demod(ps, sigma=220.0, thr=0):
    """The demodulation readout model (meas_model DEMOD, include/dpemu.h) for
    the readouts of ``ps`` (config 1-3 programs: rdrv at t, rdlo RDLO_DELAY
    later, both 2 us = 250 env words of 4 clocks): the ADC return arrives
    RDLO_DELAY clocks after the drive, so the rdlo window integrates all of
    it; the prepared states return with opposite phase (theta = pi, 0); each
    core's discriminator axis is its state-1 direction, computed from the
    drive and LO words of its program (with equal drive and LO frequencies
    the demodulated phase is -F_d * delay + (phase_d - phase_lo) << 15 +
    theta_1, constant over the window).  sigma: the accumulated value's noise
    scale (float, see make_config): the projected noise is 37837 * sigma
    against a +-1.97e7 signal (0.6 amplitude, 1000 clocks), so 220 puts ~1 %
    of the shots on the wrong side.  Returns make_config's ``demod`` dict; meas_latency
    CONFIG3_DEMOD_LATENCY keeps meas_valid where CONFIG3_MEAS_LATENCY put it."""
    import math
    w, d_off, d_len, l_off, l_len = ps.readout_freqs(RDRV, RDLO)
    axes = []
    for c in range(ps.cores_per_shot):
        p_ = int(ps.table[c])
        f_d = int(w[d_off[p_]]) if d_len[p_] else 0
        words = ps.program(0, c)
        ph = {}
        for cmd in words:                     # the phase words of the core's rdrv / rdlo pulses
            v = int(cmd[0]) | (int(cmd[1]) << 32) | (int(cmd[2]) << 64) | (int(cmd[3]) << 96)
            if v >> 124 in (0x8, 0x9) and ((v >> 37) & 0xF) & 3 in (RDRV, RDLO):
                ph.setdefault((v >> 37) & 3, (v >> 71) & 0x1FFFF)
        g = (-f_d * RDLO_DELAY + ((ph.get(RDRV, 0) - ph.get(RDLO, 0)) << 15)) % 2 ** 32
        axes.append(g * 2 * math.pi / 2 ** 32)
    return dict(drv_elem=RDRV, cpw=4, delay=RDLO_DELAY, theta=(math.pi, 0.0), gain=(1.0, 1.0), axis=axes,
                sigma=sigma, thr=thr)


def config3_lut(n_cores=8):
    """Config 3 with the fproc_lut back end (hdl/fproc_lut.sv): sync; read;
    wait for the syndrome LUT (jump_fproc with fproc id 1 != 0:
    core_state_mgr WAIT_LUT, hdl/core_state_mgr.sv:58-69) -- issued right
    after the readout pulses, so every core waits before the measurements
    arrive; the LUT fires once every masked core has measured
    (meas_lut.sv:27-49) -- X90 X90 on the core's LUT bit; sync; read; done.
    Run it with fproc_mode FPROC_LUT, lut_mask = all cores and lut_table =
    config3_lut_table(n_cores), meas_latency CONFIG3_MEAS_LATENCY."""
    prog = {}
    for c in range(n_cores):
        q = qubit_params(c)
        b = CoreBuilder()
        b.emit(isa.pulse_reset())
        b.emit(isa.sync(0))
        t_end = readout(b, q, 10)
        jf = len(b.words)
        b.emit(0)                                      # jump_fproc placeholder (LUT wait)
        b.emit(isa.jump_i(jf + 4))                     # -> second sync
        # the LUT fires at rdlo strobe + meas_latency (<= t_end + 64); decode
        # after a taken jump_fproc 6 later: the X90 pair after that
        t1 = t_end + HOLD_CLKS + 3 + 8 + 4
        b.pulse(QDRV, q['fq'], 0.0, q['ax90'], X90_ENV, t1)
        b.pulse(QDRV, q['fq'], 0.0, q['ax90'], X90_ENV, t1 + X90_CLKS)
        b.words[jf] = isa.alu_cmd('jump_fproc', 'i', 1, 'eq', jump_cmd_ptr=jf + 2, func_id=1)
        b.emit(isa.sync(1))
        readout(b, q, 10)
        b.emit(isa.done_cmd())
        prog[str(c)] = b.assembled()
    return prog


def config3_lut_table(n_cores=8):
    """syndrome table of config3_lut: address a = the cores' outcomes (bit c
    = core c); core c's correction bit = a_c XOR a_(c+1 mod n) -- the
    neighbour-parity syndrome of a repetition code -- so a core flips when
    its outcome differs from its neighbour's.  256 entries (meas_lut
    addresses are 8 bits wide, include/dpemu.h lut_table)"""
    n = int(n_cores)
    full = (1 << n) - 1
    table = []
    for a in range(256):
        a &= full
        rot = ((a >> 1) | ((a & 1) << (n - 1))) & full
        table.append(a ^ rot)
    return table


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
RB_QUARTER = 2 ** 15               # pi/2 in 17-bit phase words
RB_LAYER_CLKS = 3 * X90_CLKS + 16  # fixed layer length: the cores stay aligned
RB_T0 = 10                         # first layer's cmd_time
RB_PREG, RB_TREG = 1, 2            # virtual-Z phase register, per-pulse phase register


def _mix64(x):
    """splitmix64 finaliser on uint64 arrays (wrapping arithmetic)"""
    with np.errstate(over='ignore'):
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def rb_draws(seqs, depth, n_cores, seed=0x5EED):
    """The random content of RB sequences ``seqs`` (global indices): Clifford
    indices [len(seqs), depth, n_cores] in [0, 24) and cross-resonance bits
    [len(seqs), depth].  Counter-based -- a hash of (seed, sequence, layer,
    slot) -- so sequence s is the same whatever the table size or shard, and
    the whole table is generated vectorised."""
    if depth >= 1 << 16 or n_cores >= 255:
        raise ValueError('depth < 65536 and n_cores < 255')
    s = np.asarray(seqs, np.uint64).reshape(-1, 1, 1)
    d = np.arange(depth, dtype=np.uint64).reshape(1, -1, 1)
    j = np.arange(n_cores + 1, dtype=np.uint64).reshape(1, 1, -1)
    with np.errstate(over='ignore'):
        key = np.uint64((int(seed) * 0x9E3779B97F4A7C15) & (2 ** 64 - 1)) + ((s << np.uint64(24)) | (d << np.uint64(8)) | j)
    h = _mix64(key)
    cliffs = (h[:, :, :n_cores] % np.uint64(24)).astype(np.int64)
    cr = ((h[:, :, n_cores] >> np.uint64(32)) & np.uint64(1)).astype(np.int64)
    return cliffs, cr


def _rb_builder(c):
    """CoreBuilder with core c's RB tables registered in a fixed order, so every
    sequence of a core shares one env / freq buffer set"""
    b = CoreBuilder()
    b.env_word(QDRV, X90_ENV)
    b.freq_addr(QDRV, qubit_params(c)['fq'])
    if c == 0:
        b.freq_addr(QDRV, qubit_params(1)['fq'])   # cross-resonance drive
    return b


def config4_rb(n_seq=1000, depth=200, seed=0x5EED, n_cores=2, first=0):
    """RB-SHAPED 2-qubit sequences (the program shape of BASELINE configs[3],
    not its full circuit): per layer each qubit plays a random single-qubit
    Clifford (<= 2 X90 pulses on X or Y, virtual Z by reg_alu on its phase
    register), and with probability 1/2 a cross-resonance pulse on core 0;
    then one readout per core.  There is no CNOT decomposition of two-qubit
    Cliffords and no recovery Clifford (SURVEY.md §8(d)4 asks for both), so
    the sequences do not return the qubits to |00>: what the emulator's
    throughput depends on -- depth-200 programs of ~740 commands, ~7
    different programs per wave, register phase updates, data-dependent
    pulse counts -- is kept, the circuit's meaning is not.  Layers are
    fixed-length so the cores stay aligned.  Returns n_seq assembled-program
    dicts for global sequences [first, first + n_seq) -- the per-command
    reference for :func:`config4_rb_set`, which builds the same machine code
    vectorised."""
    cliffs, cr = rb_draws(np.arange(first, first + n_seq), depth, n_cores, seed)
    groups = []
    for s in range(n_seq):
        prog = {}
        for c in range(n_cores):
            q = qubit_params(c)
            b = _rb_builder(c)
            b.emit(isa.pulse_reset())
            b.emit(isa.alu_cmd('reg_alu', 'i', 0, 'id0', 0, RB_PREG))         # phase reg = 0
            t = RB_T0
            for d in range(depth):
                pre, z = CLIFFORDS[cliffs[s, d, c]]
                for i, ax in enumerate(pre):
                    b.emit(isa.alu_cmd('reg_alu', 'i', RB_QUARTER if ax == 'y' else 0, 'add', RB_PREG, RB_TREG))
                    b.pulse(QDRV, q['fq'], 0.0, q['ax90'], X90_ENV, t + X90_CLKS * i, phase_reg=RB_TREG)
                if z:
                    b.emit(isa.alu_cmd('reg_alu', 'i', z * RB_QUARTER, 'add', RB_PREG, RB_PREG))
                if c == 0 and cr[s, d]:
                    b.pulse(QDRV, qubit_params(1)['fq'], 0.0, 0.3, X90_ENV, t + 2 * X90_CLKS)
                t += RB_LAYER_CLKS
            readout(b, q, t)
            b.emit(isa.done_cmd())
            prog[str(c)] = b.assembled()
        groups.append(prog)
    return groups


# per-layer command slots of config4_rb: (pre-rotation ALU, X90) x 2, virtual Z, CR
_RB_PRE_AX = np.array([[-1, -1], [0, -1], [1, -1], [0, 0], [0, 1], [1, 0]])   # CLIFFORDS pre lists, 0 = x, 1 = y
(_T_RESET, _T_INIT, _T_ALU_X, _T_ALU_Y, _T_PULSE, _T_Z1, _T_Z2, _T_Z3, _T_CR, _T_RDRV, _T_RDLO,
 _T_DONE) = range(12)


def _rb_templates(c):
    """core c's command templates (cmd_time 0) and its env / freq buffers"""
    q = qubit_params(c)
    b = _rb_builder(c)
    b.emit(isa.pulse_reset())
    b.emit(isa.alu_cmd('reg_alu', 'i', 0, 'id0', 0, RB_PREG))
    b.emit(isa.alu_cmd('reg_alu', 'i', 0, 'add', RB_PREG, RB_TREG))
    b.emit(isa.alu_cmd('reg_alu', 'i', RB_QUARTER, 'add', RB_PREG, RB_TREG))
    b.pulse(QDRV, q['fq'], 0.0, q['ax90'], X90_ENV, 0, phase_reg=RB_TREG)
    for z in (1, 2, 3):
        b.emit(isa.alu_cmd('reg_alu', 'i', z * RB_QUARTER, 'add', RB_PREG, RB_PREG))
    if c == 0:
        b.pulse(QDRV, qubit_params(1)['fq'], 0.0, 0.3, X90_ENV, 0)
    else:
        b.emit(isa.done_cmd())                          # (no CR on other cores: never used)
    b.pulse(RDRV, q['fr'], 0.0, q['ar'], RDRV_ENV, 0)
    b.pulse(RDLO, q['fr'], q['rdlo_phase'], 1.0, RDLO_ENV, 0)
    b.emit(isa.done_cmd())
    return isa.words_to_u32(b.words), b.buffers()


def rb_core_words(cliffs_c, cr, c, depth):
    """Machine code of core c for a batch of sequences, vectorised: (words
    (n, 4) u32 of all programs back to back, n_instr per sequence).
    cliffs_c: [n_seq, depth] Clifford indices, cr: [n_seq, depth] CR bits."""
    tmpl, _ = _rb_templates(c)
    n = cliffs_c.shape[0]
    pre = _RB_PRE_AX[cliffs_c // 4]                     # [n, depth, 2]
    z = cliffs_c % 4
    t = (RB_T0 + RB_LAYER_CLKS * np.arange(depth, dtype=np.int64))[None, :]
    tid = np.full((n, depth, 6), -1, np.int8)
    tt = np.zeros((n, depth, 6), np.uint32)
    for i in (0, 1):
        has = pre[:, :, i] >= 0
        tid[:, :, 2 * i] = np.where(has, np.where(pre[:, :, i] == 1, _T_ALU_Y, _T_ALU_X), -1)
        tid[:, :, 2 * i + 1] = np.where(has, _T_PULSE, -1)
        tt[:, :, 2 * i + 1] = t + X90_CLKS * i
    tid[:, :, 4] = np.where(z > 0, _T_Z1 + z - 1, -1)
    if c == 0:
        tid[:, :, 5] = np.where(cr > 0, _T_CR, -1)
        tt[:, :, 5] = t + 2 * X90_CLKS
    t_ro = RB_T0 + RB_LAYER_CLKS * depth
    head = np.broadcast_to(np.array([_T_RESET, _T_INIT], np.int8), (n, 2))
    tail = np.broadcast_to(np.array([_T_RDRV, _T_RDLO, _T_DONE], np.int8), (n, 3))
    tid = np.concatenate([head, tid.reshape(n, -1), tail], axis=1)
    tt = np.concatenate([np.zeros((n, 2), np.uint32), tt.reshape(n, -1),
                         np.broadcast_to(np.array([t_ro, t_ro + RDLO_DELAY, 0], np.uint32), (n, 3))], axis=1)
    keep = tid >= 0
    n_instr = keep.sum(axis=1).astype(np.uint32)
    words = tmpl[tid[keep].astype(np.int64)]            # program after program (row-major)
    ts = tt[keep]
    words[:, 0] |= ts << np.uint32(5)                   # cmd_time = cmd[36:5] (template field 0)
    words[:, 1] |= ts >> np.uint32(27)
    return words, n_instr


class _SharedBuffers:
    """ProgramSet.buffers for tables shared by every group: (g, c) -> core c's"""

    def __init__(self, per_core):
        self._per_core = per_core

    def get(self, key, default=None):
        return self._per_core.get(key[1], default)

    def __getitem__(self, key):
        return self._per_core[key[1]]


def config4_rb_set(n_seq=100000, depth=200, seed=0x5EED, n_cores=2, chunk=8192):
    """Config 4 at its stated size as a ProgramSet, generated vectorised:
    group g = RB sequence g, program of (g, c) = c * n_seq + g (core-major
    blocks).  Machine code identical to ``config4_rb`` (tests/test_workloads.py)."""
    from .emulator import ProgramSet
    C_ = 1
    while C_ < n_cores:
        C_ <<= 1
    from concurrent.futures import ThreadPoolExecutor
    starts = list(range(0, n_seq, chunk))

    def one(s0):                                        # numpy releases the GIL in the bulk ops
        cl, cr = rb_draws(np.arange(s0, min(s0 + chunk, n_seq)), depth, n_cores, seed)
        return [rb_core_words(cl[:, :, c], cr, c, depth) for c in range(n_cores)]
    with ThreadPoolExecutor(max(1, min(8, len(starts), os.cpu_count() or 1))) as pool:
        parts = list(pool.map(one, starts))
    # core-major: every sequence of core 0, then of core 1, ...
    blocks = [parts[i][c] for c in range(n_cores) for i in range(len(starts))]
    n_instr = np.concatenate([b[1] for b in blocks])
    words = np.concatenate([b[0] for b in blocks]) if blocks else np.zeros((1, 4), np.uint32)
    del parts, blocks
    offsets = np.zeros(len(n_instr), np.uint64)
    np.cumsum(n_instr[:-1], out=offsets[1:])
    if offsets[-1] + n_instr[-1] >= 2 ** 32:
        raise ValueError('program set exceeds 2^32 commands')
    table = np.zeros((n_seq, C_), np.uint32)
    empty = len(n_instr)
    for c in range(C_):
        table[:, c] = c * n_seq + np.arange(n_seq) if c < n_cores else empty
    if C_ > n_cores:                                    # unused cores: one empty program
        n_instr = np.append(n_instr, np.uint32(0))
        offsets = np.append(offsets, np.uint64(len(words)))
    bufs = {c: _rb_templates(c)[1] for c in range(n_cores)}
    return ProgramSet.from_arrays(words, offsets.astype(np.uint32), n_instr, table.reshape(-1), n_seq, C_,
                                  buffers=_SharedBuffers(bufs))


# ------------------------------------------------ config 4: two-qubit Clifford RB
# random two-qubit Cliffords of depth D, each sequence closed
# by its recovery Clifford, decomposed into X90 / Y90 / X-90 / Y-90 pulses,
# virtual Z (reg_alu on the frame register) and CNOT (a cross-resonance ZX90
# on the control's drive at the target's frequency, S-dagger on the control,
# X-90 on the target); the group, its decompositions and the native-operation
# conventions are in clifford2q.py.  Cores (2p, 2p + 1) are qubit pair p
# (control, target); every pair runs its own sequence (simultaneous RB).
# Every element is a run of fixed-length stages -- C1 (x) C1 layers and CNOTs
# alternating -- on a schedule both cores of the pair share, so the CR pulse
# and the target's X-90 line up.
RB2_STAGE_CLKS = 2 * X90_CLKS + 8   # a C1 layer (<= 2 pulses per qubit) or a CNOT (CR, then the target's X-90)
RB2_T0 = 10
RB2_CR_AMP = 0.3
# machine-command templates of one core (rb2q_templates): index -> command
(_R2_RESET, _R2_INIT) = range(2)
_R2_AXIS = 2            # + a: TREG = PREG + a quarter turns
_R2_PULSE = 6           # X90-envelope pulse, phase from TREG
_R2_Z = 6               # + k (k = 1..3): PREG += k quarter turns
_R2_CR = 10             # + ph: cross-resonance pulse at immediate phase ph quarter turns (control cores)
(_R2_RDRV, _R2_RDLO, _R2_DONE) = (14, 15, 16)
_R2_MAXC = 26           # commands of one element on one core, at most (4 C1 layers of 5, 3 CNOTs of 2)


def rb2q_draws(seqs, depth, n_pairs, seed=0x5EED):
    """Two-qubit Clifford indices [len(seqs), n_pairs, depth + 1] of RB
    sequences ``seqs`` (global indices): depth counter-based random elements
    (a hash of (seed, sequence, layer, pair), as rb_draws) and, last, the
    recovery element that returns the pair to the identity."""
    from . import clifford2q
    if depth >= 1 << 16 or n_pairs >= 255:
        raise ValueError('depth < 65536 and fewer than 255 pairs')
    s = np.asarray(seqs, np.uint64).reshape(-1, 1, 1)
    d = np.arange(depth, dtype=np.uint64).reshape(1, 1, -1)
    j = np.arange(n_pairs, dtype=np.uint64).reshape(1, -1, 1)
    with np.errstate(over='ignore'):
        key = (np.uint64((int(seed) * 0xD1B54A32D192ED03) & (2 ** 64 - 1))
               + ((s << np.uint64(24)) | (d << np.uint64(8)) | j))
    el = (_mix64(key) % np.uint64(clifford2q.N_C2)).astype(np.int64)
    tab = clifford2q.table()
    u = np.broadcast_to(np.eye(4, dtype=np.complex128), el.shape[:2] + (4, 4)).copy()
    for k in range(depth):
        u = np.matmul(tab.u[el[:, :, k]], u)
    rec = tab.index(np.conj(np.swapaxes(u, -1, -2))).reshape(el.shape[:2])
    return np.concatenate([el, rec[:, :, None]], axis=2)


def _rb2q_role_cmds(layers, control):
    """(template, stage, clock offset in the stage, target-frame quarter turns
    before it) of one element's commands on the control or target core, and
    the element's stage count and net target-frame turns"""
    from . import clifford2q
    cmds, f_t = [], 0
    for st, (i0, i1) in enumerate(layers):
        if st:                                          # a CNOT before every layer but the first
            if control:
                cmds += [(_R2_CR, 2 * st - 1, 0, f_t), (_R2_Z + 1, 2 * st - 1, 0, 0)]
            else:
                cmds += [(_R2_AXIS + 2, 2 * st - 1, 0, 0), (_R2_PULSE, 2 * st - 1, X90_CLKS, 0)]
        pre, k = clifford2q.c1_ops(i0 if control else i1)
        for n_, a in enumerate(pre):
            cmds += [(_R2_AXIS + a, 2 * st, 0, 0), (_R2_PULSE, 2 * st, X90_CLKS * n_, 0)]
        if k:
            cmds.append((_R2_Z + k, 2 * st, 0, 0))
        f_t = (f_t + clifford2q.c1_ops(i1)[1]) % 4
    return cmds, 2 * len(layers) - 1, f_t


@functools.lru_cache(maxsize=1)
def _rb2q_tables():
    """per element and role: template ids [N_C2, _R2_MAXC] (-1 = none), clock
    offsets (-1: untimed), CR target-frame offsets; stages, net target-frame
    turns and command counts"""
    from . import clifford2q
    tab = clifford2q.table()
    ids = np.full((2, clifford2q.N_C2, _R2_MAXC), -1, np.int8)
    dt = np.zeros((2, clifford2q.N_C2, _R2_MAXC), np.int32)
    crf = np.zeros((clifford2q.N_C2, _R2_MAXC), np.int8)
    stages = np.zeros(clifford2q.N_C2, np.int64)
    f_t = np.zeros(clifford2q.N_C2, np.int64)
    ncmd = np.zeros((2, clifford2q.N_C2), np.int64)
    for e, layers in enumerate(tab.layers):
        for role in (0, 1):
            cmds, stages[e], f = _rb2q_role_cmds(layers, role == 0)
            ncmd[role, e] = len(cmds)
            for i, (tid, st, off, fr) in enumerate(cmds):
                ids[role, e, i] = tid
                dt[role, e, i] = st * RB2_STAGE_CLKS + off if tid in (_R2_PULSE, _R2_CR) else -1
                if role == 0:
                    crf[e, i] = fr
            f_t[e] = f
    return ids, dt, crf, stages, f_t, ncmd


def _rb2q_builder(c, n_cores):
    """CoreBuilder with core c's RB tables registered in a fixed order"""
    b = CoreBuilder()
    b.env_word(QDRV, X90_ENV)
    b.freq_addr(QDRV, qubit_params(c)['fq'])
    if c % 2 == 0 and c + 1 < n_cores:
        b.freq_addr(QDRV, qubit_params(c + 1)['fq'])   # cross-resonance drive at the target's frequency
    return b


def config4_rb2q(n_seq=1000, depth=200, seed=0x5EED, n_cores=2, first=0):
    """Two-qubit Clifford RB (BASELINE configs[3]): per qubit
    pair (cores 2p, 2p + 1) ``depth`` random two-qubit Cliffords and the
    recovery Clifford, each decomposed as clifford2q describes, then one
    readout per core.  The physical pulse sequence is the identity up to a Z
    rotation per qubit (tests/test_rb2q.py).  Returns n_seq assembled-program
    dicts for global sequences [first, first + n_seq) -- the per-command
    reference for :func:`config4_rb2q_set`, which builds the same machine code
    vectorised."""
    from . import clifford2q
    if n_cores % 2:
        raise ValueError('config4_rb2q runs qubit pairs: n_cores must be even')
    el = rb2q_draws(np.arange(first, first + n_seq), depth, n_cores // 2, seed)
    tab = clifford2q.table()
    groups = []
    for s in range(n_seq):
        prog = {}
        for c in range(n_cores):
            q, control = qubit_params(c), c % 2 == 0
            f_tgt = qubit_params(c + 1)['fq'] if control else None
            b = _rb2q_builder(c, n_cores)
            b.emit(isa.pulse_reset())
            b.emit(isa.alu_cmd('reg_alu', 'i', 0, 'id0', 0, RB_PREG))
            t0, f_t = RB2_T0, 0                            # element start, target frame (quarter turns)
            for e in el[s, c // 2]:
                cmds, n_st, df = _rb2q_role_cmds(tab.layers[e], control)
                for tid, st, off, fr in cmds:
                    t = t0 + st * RB2_STAGE_CLKS + off
                    if tid == _R2_CR:
                        b.pulse(QDRV, f_tgt, 0.0, RB2_CR_AMP, X90_ENV, t,
                                phase_word=((f_t + fr) % 4) * RB_QUARTER)
                    elif tid == _R2_PULSE:
                        b.pulse(QDRV, q['fq'], 0.0, q['ax90'], X90_ENV, t, phase_reg=RB_TREG)
                    elif tid >= _R2_Z + 1:
                        b.emit(isa.alu_cmd('reg_alu', 'i', (tid - _R2_Z) * RB_QUARTER, 'add', RB_PREG, RB_PREG))
                    else:
                        b.emit(isa.alu_cmd('reg_alu', 'i', (tid - _R2_AXIS) * RB_QUARTER, 'add', RB_PREG, RB_TREG))
                t0 += n_st * RB2_STAGE_CLKS
                f_t = (f_t + df) % 4
            readout(b, q, t0)
            b.emit(isa.done_cmd())
            prog[str(c)] = b.assembled()
        groups.append(prog)
    return groups


@functools.lru_cache(maxsize=64)
def _rb2q_templates(c, n_cores):
    """core c's command templates (cmd_time 0), indexed by the _R2_* ids, and its env / freq buffers"""
    q, control = qubit_params(c), c % 2 == 0
    b = _rb2q_builder(c, n_cores)
    b.emit(isa.pulse_reset())
    b.emit(isa.alu_cmd('reg_alu', 'i', 0, 'id0', 0, RB_PREG))
    for a in range(4):
        b.emit(isa.alu_cmd('reg_alu', 'i', a * RB_QUARTER, 'add', RB_PREG, RB_TREG))
    b.pulse(QDRV, q['fq'], 0.0, q['ax90'], X90_ENV, 0, phase_reg=RB_TREG)
    for k in (1, 2, 3):
        b.emit(isa.alu_cmd('reg_alu', 'i', k * RB_QUARTER, 'add', RB_PREG, RB_PREG))
    for ph in range(4):
        if control:
            b.pulse(QDRV, qubit_params(c + 1)['fq'], 0.0, RB2_CR_AMP, X90_ENV, 0, phase_word=ph * RB_QUARTER)
        else:
            b.emit(isa.done_cmd())                      # (no CR on target cores: never used)
    b.pulse(RDRV, q['fr'], 0.0, q['ar'], RDRV_ENV, 0)
    b.pulse(RDLO, q['fr'], q['rdlo_phase'], 1.0, RDLO_ENV, 0)
    b.emit(isa.done_cmd())
    return isa.words_to_u32(b.words), b.buffers()


def rb2q_core_words(el_p, c, n_cores):
    """Machine code of core c for a batch of sequences of its pair, vectorised:
    (words (n, 4) u32 of all programs back to back, n_instr per sequence).
    el_p: [n_seq, depth + 1] element indices (rb2q_draws)."""
    ids_t, dt_t, crf_t, stages_t, ft_t, ncmd_t = _rb2q_tables()
    role = c % 2
    tmpl, _ = _rb2q_templates(c, n_cores)
    n, L = el_p.shape
    st = stages_t[el_p]
    start = RB2_T0 + RB2_STAGE_CLKS * (np.cumsum(st, axis=1) - st)            # [n, L] element start cycles
    cnt = ncmd_t[role][el_p]                                                  # [n, L] commands per element
    # one entry per command of the body, sequence after sequence: its element and index in it
    e_flat = np.repeat(el_p.ravel(), cnt.ravel())
    first = np.repeat(np.cumsum(cnt.ravel()) - cnt.ravel(), cnt.ravel())
    j = np.arange(len(e_flat)) - first
    ids = ids_t[role][e_flat, j].astype(np.int64)
    dt = dt_t[role][e_flat, j]
    tt = np.where(dt >= 0, np.repeat(start.ravel(), cnt.ravel()) + dt, 0)
    if role == 0:
        f_t = ft_t[el_p]
        f_entry = (np.cumsum(f_t, axis=1) - f_t) % 4
        ids = np.where(ids == _R2_CR, _R2_CR + (np.repeat(f_entry.ravel(), cnt.ravel()) + crf_t[e_flat, j]) % 4, ids)
    body = cnt.sum(axis=1)                                                    # [n]
    n_instr = (body + 5).astype(np.uint32)                                    # + reset, init, rdrv, rdlo, done
    t_ro = RB2_T0 + RB2_STAGE_CLKS * st.sum(axis=1)
    # assemble: head (2), body, tail (3) per sequence
    out_ids = np.empty(int(n_instr.sum()), np.int64)
    out_t = np.zeros(len(out_ids), np.int64)
    seq_start = np.cumsum(n_instr.astype(np.int64)) - n_instr
    pos = np.repeat(seq_start + 2 - np.cumsum(body) + body, body) + np.arange(len(ids))
    out_ids[pos] = ids
    out_t[pos] = tt
    for k, (tid, tv) in enumerate(((_R2_RESET, 0), (_R2_INIT, 0))):
        out_ids[seq_start + k] = tid
    tail0 = seq_start + 2 + body
    out_ids[tail0], out_t[tail0] = _R2_RDRV, t_ro
    out_ids[tail0 + 1], out_t[tail0 + 1] = _R2_RDLO, t_ro + RDLO_DELAY
    out_ids[tail0 + 2] = _R2_DONE
    words = tmpl[out_ids]
    ts = out_t.astype(np.uint32)
    words[:, 0] |= ts << np.uint32(5)                   # cmd_time = cmd[36:5] (template field 0)
    words[:, 1] |= ts >> np.uint32(27)
    return words, n_instr


def config4_rb2q_set(n_seq=100000, depth=200, seed=0x5EED, n_cores=2, chunk=4096):
    """Config 4 at its stated size as a ProgramSet, generated vectorised:
    group g = RB sequence g, program of (g, c) = c * n_seq + g (core-major
    blocks).  Machine code identical to ``config4_rb2q`` (tests/test_rb2q.py)."""
    from .emulator import ProgramSet
    if n_cores % 2:
        raise ValueError('config4_rb2q runs qubit pairs: n_cores must be even')
    C_ = 1
    while C_ < n_cores:
        C_ <<= 1
    _rb2q_tables()                                      # (built once, before the threads)
    from concurrent.futures import ThreadPoolExecutor
    starts = list(range(0, n_seq, chunk))

    def one(s0):                                        # numpy releases the GIL in the bulk ops
        el = rb2q_draws(np.arange(s0, min(s0 + chunk, n_seq)), depth, n_cores // 2, seed)
        return [rb2q_core_words(el[:, c // 2], c, n_cores) for c in range(n_cores)]
    with ThreadPoolExecutor(max(1, min(8, len(starts), os.cpu_count() or 1))) as pool:
        parts = list(pool.map(one, starts))
    blocks = [parts[i][c] for c in range(n_cores) for i in range(len(starts))]
    n_instr = np.concatenate([b[1] for b in blocks])
    words = np.concatenate([b[0] for b in blocks]) if blocks else np.zeros((1, 4), np.uint32)
    del parts, blocks
    offsets = np.zeros(len(n_instr), np.uint64)
    np.cumsum(n_instr[:-1], out=offsets[1:])
    if offsets[-1] + n_instr[-1] >= 2 ** 32:
        raise ValueError('program set exceeds 2^32 commands')
    table = np.zeros((n_seq, C_), np.uint32)
    empty = len(n_instr)
    for c in range(C_):
        table[:, c] = c * n_seq + np.arange(n_seq) if c < n_cores else empty
    if C_ > n_cores:
        n_instr = np.append(n_instr, np.uint32(0))
        offsets = np.append(offsets, np.uint64(len(words)))
    bufs = {c: _rb2q_templates(c, n_cores)[1] for c in range(n_cores)}
    return ProgramSet.from_arrays(words, offsets.astype(np.uint32), n_instr, table.reshape(-1), n_seq, C_,
                                  buffers=_SharedBuffers(bufs))
