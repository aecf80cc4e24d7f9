"""Hardware configuration plugins (mirror of ``python/distproc/hwconfig.py``).

* ``ElementConfig`` -- the plugin ABC the assembler calls to turn physical
  freq/phase/amp/envelope values into hardware words and buffers
  (reference ``hwconfig.py:12-67``; call sites ``assembler.py:359-380,484-488,514``).
* ``FPGAConfig`` / ``FPROCChannel`` / ``ChannelConfig`` / ``load_channel_configs``
  -- same names, fields and defaults as ``hwconfig.py:69-160``.
* ``DDSElementConfig`` -- a concrete element whose words and buffers are the
  ones this framework's DDS kernel consumes (build-defined; the reference's
  concrete element lives in the absent ``qubic`` package, so its numeric
  conversions are *parity unpinned*).  Buffer formats follow
  ``asmparse.py:46-86``: env sample = I16 (high half) | Q16 (low half);
  freq entry = 16 x u32 = [f/f_clk * 2^32, 15 per-sub-sample rotations
  packed I16|Q16].  The env I/Q order resolves SURVEY.md Appendix A #4 in
  favour of the decoder (``asmparse.envparse``).
"""

from __future__ import annotations

import json
import math
from abc import ABC, abstractmethod
from typing import Dict, Optional

import numpy as np

FPROC_MEAS_CLKS = 64     # hwconfig.py:9
N_CORES = 8              # hwconfig.py:10


class ElementConfig(ABC):
    def __init__(self, fpga_clk_period, samples_per_clk):
        self.fpga_clk_period = fpga_clk_period
        self.samples_per_clk = samples_per_clk

    @property
    def sample_period(self):
        return self.fpga_clk_period / self.samples_per_clk

    @property
    def sample_freq(self):
        return 1 / self.sample_period

    @property
    def fpga_clk_freq(self):
        return 1 / self.fpga_clk_period

    @abstractmethod
    def get_phase_word(self, phase): ...

    @abstractmethod
    def length_nclks(self, tlength): ...

    @abstractmethod
    def get_env_word(self, env_start_ind, env_length): ...

    @abstractmethod
    def get_cw_env_word(self, env_start_ind): ...

    @abstractmethod
    def get_env_buffer(self, env): ...

    @abstractmethod
    def get_freq_buffer(self, freqs): ...

    @abstractmethod
    def get_freq_addr(self, freq_ind): ...

    @abstractmethod
    def get_cfg_word(self, elem_ind, mode_bits): ...

    @abstractmethod
    def get_amp_word(self, amplitude): ...


class FPROCChannel:
    """FPROC channel description (hwconfig.py:69-98)."""

    def __init__(self, id, hold_after_chans=None, hold_nclks=0):
        self.id = id
        self.hold_after_chans = list(hold_after_chans or [])
        self.hold_nclks = hold_nclks

    def __repr__(self):
        return 'FPROCChannel(id={!r}, hold_after_chans={!r}, hold_nclks={!r})'.format(
            self.id, self.hold_after_chans, self.hold_nclks)


class FPGAConfig:
    """Scheduler clock/latency constants (hwconfig.py:100-119).

    The defaults are the reference's.  The cycle-exact latencies measured from
    the RTL differ: ALU 4, jump_cond 6 (> the 5 assumed here),
    jump_fproc 8, pulse 3 -- see ``EXACT_LATENCIES``.
    """

    def __init__(self, fpga_clk_period=2.e-9, alu_instr_clks=5, jump_cond_clks=5,
                 jump_fproc_clks=8, pulse_regwrite_clks=3, pulse_load_clks=3):
        self.fpga_clk_period = fpga_clk_period
        self.alu_instr_clks = alu_instr_clks
        self.jump_cond_clks = jump_cond_clks
        self.jump_fproc_clks = jump_fproc_clks
        self.pulse_regwrite_clks = pulse_regwrite_clks
        self.pulse_load_clks = pulse_load_clks
        self.fproc_channels = {
            'Q{}.meas'.format(i): FPROCChannel(id=('Q{}.rdlo'.format(i), 'core_ind'),
                                               hold_after_chans=['Q{}.rdlo'.format(i)],
                                               hold_nclks=FPROC_MEAS_CLKS)
            for i in range(N_CORES)}

    @property
    def fpga_clk_freq(self):
        return 1 / self.fpga_clk_period

    @classmethod
    def rtl_exact(cls, fpga_clk_period=2.e-9, pulse_regwrite_clks=3):
        """the scheduler constants set to the RTL's decode-to-decode cycle
        counts (``EXACT_LATENCIES``): schedules made with it never put a pulse
        before the core can issue it (``tests/test_schedule.py``)"""
        return cls(fpga_clk_period=fpga_clk_period, pulse_regwrite_clks=pulse_regwrite_clks,
                   **{k: EXACT_LATENCIES[k] for k in ('alu_instr_clks', 'jump_cond_clks', 'jump_fproc_clks',
                                                       'pulse_load_clks')})


# Decode-to-decode cycle counts of the RTL (ctrl.v).
EXACT_LATENCIES = {'alu_instr_clks': 4, 'jump_cond_clks': 6, 'jump_fproc_clks': 8,
                   'alu_fproc_clks': 6, 'jump_i_clks': 4, 'pulse_load_clks': 3}


class ChannelConfig:
    """One DAC/ADC channel of a core (hwconfig.py:121-140)."""

    def __init__(self, core_ind, elem_ind, elem_params, env_mem_name, freq_mem_name,
                 acc_mem_name):
        self.core_ind = core_ind
        self.elem_ind = elem_ind
        self.elem_params = elem_params
        self._env_mem_name = env_mem_name
        self._freq_mem_name = freq_mem_name
        self._acc_mem_name = acc_mem_name

    @property
    def env_mem_name(self):
        return self._env_mem_name.format(core_ind=self.core_ind)

    @property
    def freq_mem_name(self):
        return self._freq_mem_name.format(core_ind=self.core_ind)

    @property
    def acc_mem_name(self):
        return self._acc_mem_name.format(core_ind=self.core_ind)


def load_channel_configs(config_dict):
    """dict or JSON path -> {channel name: ChannelConfig, 'fpga_clk_freq': float}."""
    if isinstance(config_dict, str):
        with open(config_dict) as f:
            config_dict = json.load(f)
    assert 'fpga_clk_freq' in config_dict.keys()
    out = {}
    for key, value in config_dict.items():
        out[key] = ChannelConfig(**value) if isinstance(value, dict) else value
    return out


# ---------------------------------------------------------------------------
# Envelope shapes (build-defined; the reference's live in absent qubic)
# ---------------------------------------------------------------------------
def _env_times(n):
    return (np.arange(n) + 0.5) / n


def env_square(n, amplitude=1.0, phase=0.0, **_):
    return np.full(n, amplitude * np.exp(1j * phase), dtype=complex)


def env_cos_edge_square(n, ramp_fraction=0.25, **_):
    x = _env_times(n)
    out = np.ones(n)
    r = max(ramp_fraction, 1e-12)
    lo = x < r
    hi = x > 1 - r
    out[lo] = 0.5 * (1 - np.cos(np.pi * x[lo] / r))
    out[hi] = 0.5 * (1 - np.cos(np.pi * (1 - x[hi]) / r))
    return out.astype(complex)


def env_gaussian(n, sigmas=3, **_):
    x = _env_times(n) - 0.5
    sig = 1.0 / (2 * sigmas)
    return np.exp(-0.5 * (x / sig) ** 2).astype(complex)


def env_drag(n, alpha=0.0, sigmas=3, delta=-268e6, twidth=32e-9, **_):
    x = _env_times(n) - 0.5
    sig = 1.0 / (2 * sigmas)
    g = np.exp(-0.5 * (x / sig) ** 2)
    dg = -x / sig ** 2 * g / twidth            # d/dt, t in seconds
    env = g + 1j * alpha * dg / (2 * np.pi * delta)
    peak = np.max(np.abs(env))
    return env / peak if peak > 1 else env


ENV_FUNCS = {'square': env_square, 'cos_edge_square': env_cos_edge_square,
             'gaussian': env_gaussian, 'DRAG': env_drag}


def pack_iq16(z: np.ndarray) -> np.ndarray:
    """complex in [-1, 1] -> u32 words, I16 in the high half, Q16 in the low half."""
    i = np.clip(np.round(np.real(z) * 32767), -32768, 32767).astype(np.int64) & 0xFFFF
    q = np.clip(np.round(np.imag(z) * 32767), -32768, 32767).astype(np.int64) & 0xFFFF
    return ((i << 16) | q).astype(np.uint32)


class DDSElementConfig(ElementConfig):
    """Concrete element matching the DDS kernel's word/buffer conventions.

    * phase word: 17 bits, phase / 2pi * 2^17 (pinned by test_pulse_reg.py:31)
    * amp word: 16 bits, amp * (2^16 - 1)   (pinned by test_pulse_reg.py:32)
    * env word: start[11:0] | length[23:12], both in 4-sample words
      (asmparse.py:40-41; assembler.py:472-476); length 0 = CW
    * freq addr: index into this element's freq buffer (9 bits)
    * cfg word: element index (as the reference test stubs do)
    """

    def __init__(self, samples_per_clk=16, interp_ratio=1, fpga_clk_period=2.e-9):
        super().__init__(fpga_clk_period, samples_per_clk)
        self.interp_ratio = interp_ratio

    @property
    def env_sample_period(self):
        return self.fpga_clk_period * self.interp_ratio / self.samples_per_clk

    def get_phase_word(self, phase):
        # truncation, as test_pulse_reg.py:31 computes the word
        return int(phase / (2 * np.pi) * 2 ** 17) % 2 ** 17

    def get_amp_word(self, amplitude):
        # truncation, as test_pulse_reg.py:32 computes the word
        return int(min(max(amplitude, 0.0), 1.0) * (2 ** 16 - 1))

    def length_nclks(self, tlength):
        return int(np.ceil(tlength / self.fpga_clk_period))

    def get_env_word(self, env_start_ind, env_length):
        assert env_start_ind % 4 == 0 and env_length % 4 == 0
        return ((env_start_ind // 4) & 0xFFF) | (((env_length // 4) & 0xFFF) << 12)

    def get_cw_env_word(self, env_start_ind, env_length=None):
        return (env_start_ind // 4) & 0xFFF

    def env_samples(self, env) -> np.ndarray:
        if isinstance(env, str) and env == 'cw':
            return np.ones(1, dtype=complex)
        if isinstance(env, dict):
            par = dict(env['paradict'])
            n = max(1, int(round(par.get('twidth', 32e-9) / self.env_sample_period)))
            return ENV_FUNCS[env['env_func']](n, **par)
        return np.asarray(env, dtype=complex)

    def get_env_buffer(self, env):
        z = self.env_samples(env)
        pad = (-len(z)) % 4
        if pad:
            z = np.concatenate([z, np.zeros(pad, dtype=complex)])
        return pack_iq16(z)

    def get_freq_buffer(self, freqs):
        out = []
        for f in freqs:
            if f is None:
                out.append(np.zeros(16, dtype=np.uint32))
                continue
            word0 = int(round(f / self.fpga_clk_freq * 2 ** 32)) % 2 ** 32
            k = np.arange(1, 16)
            rot = np.exp(2j * np.pi * f * k * self.sample_period)
            out.append(np.concatenate([np.array([word0], dtype=np.uint32), pack_iq16(rot)]))
        return np.concatenate(out) if out else np.zeros(0, dtype=np.uint32)

    def get_freq_addr(self, freq_ind):
        return int(freq_ind)

    def get_cfg_word(self, elem_ind, mode_bits):
        return int(elem_ind) & 0xF
