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
* config 4 -- RB-shaped 2-qubit sequences: depth-D random single-qubit
              Cliffords + cross-resonance pulses with virtual-Z phase
              registers (long programs; no CNOT decomposition or recovery
              Clifford, see config4_rb)

Channel layout per core follows python/test/channel_config.json: element 0
qdrv (16 samples/clk), element 1 rdrv (16/clk, interp 16), element 2 rdlo
(4/clk, interp 4); cfg word = element index, so readouts are cfg & 3 == 2.
"""

from __future__ import annotations

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
