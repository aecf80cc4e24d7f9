"""The API-compatible assembler restatement (distributed_processor_amd.assembler) vs the reference
GlobalAssembler, byte for byte.

Inputs: the reference's compiler golden programs (python/test/test_outputs/*.txt,
copied as data by tests/golden/make_asm_inputs.py) and its channel_config.json.
Expected outputs: tests/golden/asm_programs.json, produced by running the
reference GlobalAssembler on the same inputs (tests/golden/make_golden.py) with
(a) the zero-word stub element of the reference's test_compiler.py:18-47 and
(b) this framework's DDSElementConfig.  Programs the reference assembler
rejects must be rejected here too.  CPU only.
"""

import json
import os
import warnings

import numpy as np
import pytest

from distributed_processor_amd import assembler as am
from distributed_processor_amd import hwconfig as hw
from distributed_processor_amd import isa

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')

with open(os.path.join(GOLDEN, 'asm_inputs.json')) as f:
    INPUTS = json.load(f)['programs']
with open(os.path.join(GOLDEN, 'asm_programs.json')) as f:
    EXPECTED = json.load(f)['programs']


def dec(v):
    if isinstance(v, dict):
        if '__tuple__' in v:
            return tuple(dec(x) for x in v['__tuple__'])
        if '__ndarray__' in v:
            vals = v['__ndarray__']
            return np.array([complex(a, b) for a, b in vals]) if v['complex'] else np.array(vals)
        return {k: dec(x) for k, x in v.items()}
    if isinstance(v, list):
        return [dec(x) for x in v]
    return v


class ZeroElementConfig(hw.ElementConfig):
    """The zero-word element stub of the reference's test_compiler.py:18-47."""

    def __init__(self, samples_per_clk, interp_ratio):
        super().__init__(2.e-9, samples_per_clk)

    def get_phase_word(self, phase):
        return 0

    def get_env_word(self, env_start_ind, env_length):
        return 0

    def get_cw_env_word(self, env_start_ind, env_length=None):
        return 0

    def get_env_buffer(self, env_samples):
        return np.zeros(10)

    def get_freq_buffer(self, freqs):
        return np.zeros(10)

    def get_freq_addr(self, freq_ind):
        return 0

    def get_amp_word(self, amplitude):
        return 0

    def length_nclks(self, tlength):
        return int(np.ceil(tlength / self.fpga_clk_period))

    def get_cfg_word(self, elem_ind, mode_bits):
        return elem_ind


class Compiled:
    """CompiledProgram's attribute surface the assembler reads (compiler.py:338-366)."""

    def __init__(self, program):
        self.program = program
        self.proc_groups = list(program.keys())
        self.fpga_config = None


def program(name):
    return {tuple(g['group']): dec(g['statements']) for g in INPUTS[name]}


def channels():
    return hw.load_channel_configs(os.path.join(GOLDEN, 'channel_config.json'))


def assemble(name, elem_cls):
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        return am.GlobalAssembler(Compiled(program(name)), channels(), elem_cls).get_assembled_program()


def words(buf):
    return isa.bytes_to_words(buf)


@pytest.mark.parametrize('name', sorted(INPUTS))
def test_matches_reference_assembler(name):
    exp = EXPECTED[name]
    if 'reference_error' in exp:
        with pytest.raises(Exception):
            assemble(name, ZeroElementConfig)
        return
    for key, cls in (('zero_elem', ZeroElementConfig), ('dds_elem', hw.DDSElementConfig)):
        if key not in exp:
            continue
        got = assemble(name, cls)
        assert sorted(got) == sorted(exp[key]), (key, sorted(got))
        for core, want in exp[key].items():
            g = got[core]
            assert g['cmd_buf'].hex() == want['cmd_buf'], (name, key, core, 'cmd_buf')
            assert [b.hex() for b in g['env_buffers']] == want['env_buffers'], (name, key, core, 'env')
            assert [b.hex() for b in g['freq_buffers']] == want['freq_buffers'], (name, key, core, 'freq')


def test_every_golden_covered():
    assert sorted(INPUTS) == sorted(EXPECTED)
    assert sum('dds_elem' in v for v in EXPECTED.values()) >= 6


def test_assembled_programs_load():
    """the DDS-element output is a ProgramSet input: whole commands, whole u32
    buffer words, every command of a known opcode class"""
    from distributed_processor_amd.emulator import ProgramSet
    for name, exp in EXPECTED.items():
        if 'dds_elem' not in exp:
            continue
        asm = assemble(name, hw.DDSElementConfig)
        ps = ProgramSet([asm])
        assert ps.n_groups == 1 and ps.cores_per_shot >= 1
        for core in asm.values():
            assert len(core['cmd_buf']) % 16 == 0
            for b in core['env_buffers'] + core['freq_buffers']:
                assert len(b) % 4 == 0
            for w in words(core['cmd_buf']):
                assert isa.decode(w)['op4'] in isa.OP_NAMES


def test_sync_statement():
    """the added sync op encodes command_gen.sync(barrier_id)"""
    a = am.SingleCoreAssembler([hw.DDSElementConfig()])
    a.from_list([{'op': 'phase_reset'}, {'op': 'sync', 'barrier_id': 5}, {'op': 'done_stb'}])
    buf, _, _ = a.get_compiled_program()
    assert words(buf) == [isa.pulse_reset(), isa.sync(5), isa.done_cmd()]


def test_register_pulses_split_and_typed_immediates():
    """register-sourced freq + phase + amp split into three pulse commands; an
    immediate written to a phase / amp register is converted to its word"""
    e = hw.DDSElementConfig()
    a = am.SingleCoreAssembler([e])
    a.declare_reg('f', ('int',))
    a.declare_reg('ph', ('phase', 0))
    a.declare_reg('am', ('amp', 0))
    a.add_reg_write('ph', np.pi / 2)
    a.add_reg_write('am', 0.5)
    a.add_pulse('f', 'ph', 'am', 100, 'cw', 0)
    buf, env, freq = a.get_compiled_program()
    w = words(buf)
    assert len(w) == 5
    assert w[0] == isa.alu_cmd('reg_alu', 'i', e.get_phase_word(np.pi / 2), 'id0', 1, 1)
    assert w[1] == isa.alu_cmd('reg_alu', 'i', e.get_amp_word(0.5), 'id0', 2, 2)
    assert w[2] == isa.pulse_cmd(freq_regaddr=0, cfg_word=0)
    assert w[3] == isa.pulse_cmd(amp_regaddr=2, cfg_word=0)
    assert w[4] == isa.pulse_cmd(phase_regaddr=1, env_word=e.get_cw_env_word(0), cmd_time=100, cfg_word=0)


def test_duplicate_register_and_phase_amp_quirks_warn():
    """reference behaviours kept for parity are announced"""
    a = am.SingleCoreAssembler([hw.DDSElementConfig()])
    a.declare_reg('x')
    with pytest.warns(UserWarning):
        a.declare_reg('x')
    assert a._regs['x']['index'] == 1
    a.declare_reg('ph', ('phase', 0))
    a.declare_reg('am', ('amp', 0))
    with pytest.warns(UserWarning):
        a.add_pulse(5e9, 'ph', 'am', 10, 'cw', 0)
    assert a._program[0] == {'op': 'pulse', 'freq': 'ph'}
