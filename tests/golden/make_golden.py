"""Generate golden fixtures from the reference Python ISA encoder and assembler.

Run in the build container (where /root/reference exists):

    python tests/golden/make_golden.py

It imports ``distproc.command_gen`` and ``distproc.assembler`` from
``/root/reference/python`` -- the only place the reference code is executed --
and writes *data only* (hex words / buffers) next to this script:

* ``isa_kat.json``       -- encoder known-answer words for seeded random
                            arguments of every command_gen entry point
* ``asm_programs.json``  -- the compiler golden programs of
                            ``python/test/test_outputs/*.txt`` run through the
                            reference ``GlobalAssembler`` with (a) the zero
                            stub element of ``test_compiler.py:18-47`` and (b)
                            this framework's ``DDSElementConfig``
* ``cmd_buf_golden.json``-- the reference's one machine-code golden
                            (``test_linear_compile_globalasm.txt``), as hex

Nothing from the reference is copied into the repo: the fixtures are the
reference's outputs on the stated inputs.
"""

import ast
import json
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_PY = '/root/reference/python'
REF_OUT = os.path.join(REF_PY, 'test', 'test_outputs')

sys.path.insert(0, REPO)
sys.path.insert(0, REF_PY)

import distproc.command_gen as cg  # noqa: E402  (reference encoder)
import distproc.assembler as am    # noqa: E402  (reference assembler)
import distproc.hwconfig as rhw    # noqa: E402

from distributed_processor_amd.hwconfig import DDSElementConfig  # noqa: E402


def kat_cases(rng):
    cases = []

    def add(fn, *args, **kwargs):
        word = getattr(cg, fn)(*args, **kwargs)
        cases.append({'fn': fn, 'args': list(args), 'kwargs': kwargs, 'word': '{:032x}'.format(word)})

    s32 = lambda: rng.randint(-2 ** 31, 2 ** 31 - 1)
    r4 = lambda: rng.randint(0, 15)
    for _ in range(40):
        add('pulse_i', rng.randint(0, 511), rng.randint(0, 2 ** 17 - 1), rng.randint(0, 2 ** 16 - 1),
            rng.randint(0, 2 ** 24 - 1), rng.randint(0, 15), rng.randint(0, 2 ** 32 - 1))
    for which in ('freq', 'phase', 'amp', 'env'):
        for _ in range(8):
            kw = {'freq_word': rng.randint(0, 511), 'phase_word': rng.randint(0, 2 ** 17 - 1),
                  'amp_word': rng.randint(0, 2 ** 16 - 1), 'env_word': rng.randint(0, 2 ** 24 - 1),
                  'cfg_word': rng.randint(0, 15)}
            del kw[which + '_word']
            kw[which + '_regaddr'] = r4()
            if rng.random() < 0.5:
                kw['cmd_time'] = rng.randint(0, 2 ** 32 - 1)
            add('pulse_cmd', **kw)
    for _ in range(8):
        add('pulse_cmd', freq_word=rng.randint(0, 511), cfg_word=rng.randint(0, 15))
    for op in ('id0', 'add', 'sub', 'eq', 'le', 'ge', 'id1', 'zero'):
        for _ in range(3):
            add('alu_cmd', 'reg_alu', 'i', s32(), op, r4(), r4())
            add('alu_cmd', 'reg_alu', 'r', r4(), op, r4(), r4())
            add('alu_cmd', 'jump_cond', 'i', s32(), op, r4(), jump_cmd_ptr=rng.randint(0, 2 ** 16 - 1))
            add('alu_cmd', 'jump_cond', 'r', r4(), op, r4(), jump_cmd_ptr=rng.randint(0, 2 ** 16 - 1))
            add('alu_cmd', 'alu_fproc', 'i', s32(), op, write_reg_addr=r4(), func_id=rng.randint(0, 255))
            add('alu_cmd', 'alu_fproc', 'r', r4(), op, write_reg_addr=r4(), func_id=rng.randint(0, 255))
            add('alu_cmd', 'jump_fproc', 'i', s32(), op, jump_cmd_ptr=rng.randint(0, 2 ** 16 - 1),
                func_id=rng.randint(0, 255))
            add('alu_cmd', 'jump_fproc', 'r', r4(), op, jump_cmd_ptr=rng.randint(0, 2 ** 16 - 1),
                func_id=rng.randint(0, 255))
            add('reg_alu_i', s32(), op, r4(), r4())
            add('reg_alu', r4(), op, r4(), r4())
            add('alu_fproc', rng.randint(0, 255), r4(), op, r4())
            add('jump_fproc', rng.randint(0, 255), r4(), op, rng.randint(0, 255))
            add('jump_fproc_i', rng.randint(0, 255), rng.randint(0, 2 ** 31 - 1), op, rng.randint(0, 255))
    for op in ('eq', 'le', 'ge'):
        for _ in range(3):
            add('jump_cond_i', s32(), op, r4(), rng.randint(0, 255))
            add('jump_cond', r4(), op, r4(), rng.randint(0, 255))
    for _ in range(6):
        add('alu_cmd', 'inc_qclk', 'i', s32())
        add('alu_cmd', 'inc_qclk', 'r', r4())
        add('inc_qclk_i', s32())
        add('inc_qclk', r4())
        add('read_fproc', rng.randint(0, 255), r4())
        add('jump_i', rng.randint(0, 2 ** 16 - 1))
        add('idle', rng.randint(0, 2 ** 32 - 1))
        add('sync', rng.randint(0, 255))
    add('done_cmd')
    add('pulse_reset')
    tc = []
    for v in [0, 1, -1, 2 ** 31 - 1, -2 ** 31] + [s32() for _ in range(20)]:
        tc.append({'value': v, 'tc': int(cg.twos_complement(v))})
    return cases, tc


class ZeroElementConfig(rhw.ElementConfig):
    """Behaviour of the ElementConfigTest stub in test_compiler.py:18-47."""

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


class _Compiled:
    """Minimal stand-in for CompiledProgram's attribute surface
    (compiler.py:338-366): program dict, proc_groups, fpga_config."""

    def __init__(self, program):
        self.program = program
        self.proc_groups = list(program.keys())
        self.fpga_config = None


def load_program_txt(path):
    with open(path) as f:
        txt = f.read().strip()
    if 'array(' in txt:
        return eval(txt, {'array': np.array, '__builtins__': {}})   # test_pulse_compile_out.txt
    return ast.literal_eval(txt)


def assemble(program, elem_cls):
    chans = rhw.load_channel_configs(os.path.join(REF_PY, 'test', 'channel_config.json'))
    ga = am.GlobalAssembler(_Compiled(program), chans, elem_cls)
    out = ga.get_assembled_program()
    res = {}
    for core, d in sorted(out.items()):
        res[core] = {'cmd_buf': d['cmd_buf'].hex(),
                     'env_buffers': [bytes(b).hex() for b in d['env_buffers']],
                     'freq_buffers': [bytes(b).hex() for b in d['freq_buffers']]}
    return res


def main():
    rng = random.Random(0x5EED)
    cases, tc = kat_cases(rng)
    with open(os.path.join(HERE, 'isa_kat.json'), 'w') as f:
        json.dump({'source': 'distproc.command_gen (reference @ /root/reference)',
                   'cases': cases, 'twos_complement': tc}, f, indent=0)

    progs = {}
    for fname in sorted(os.listdir(REF_OUT)):
        if not fname.endswith('.txt') or 'globalasm' in fname:
            continue
        prog = load_program_txt(os.path.join(REF_OUT, fname))
        try:
            entry = {'zero_elem': assemble(prog, ZeroElementConfig)}
        except Exception as e:  # the reference assembler rejects this compiler output
            progs[fname[:-4]] = {'reference_error': repr(e)}
            continue
        try:
            entry['dds_elem'] = assemble(prog, DDSElementConfig)
        except Exception as e:  # a program the concrete element cannot express
            entry['dds_elem_error'] = repr(e)
        progs[fname[:-4]] = entry
    with open(os.path.join(HERE, 'asm_programs.json'), 'w') as f:
        json.dump({'source': 'distproc.assembler.GlobalAssembler on python/test/test_outputs/*.txt',
                   'programs': progs}, f, indent=0)

    golden = load_program_txt(os.path.join(REF_OUT, 'test_linear_compile_globalasm.txt'))
    with open(os.path.join(HERE, 'cmd_buf_golden.json'), 'w') as f:
        json.dump({'source': 'python/test/test_outputs/test_linear_compile_globalasm.txt',
                   'cores': {k: {'cmd_buf': v['cmd_buf'].hex(),
                                 'env_buffers': [b.hex() for b in v['env_buffers']],
                                 'freq_buffers': [b.hex() for b in v['freq_buffers']]}
                             for k, v in golden.items()}}, f, indent=0)
    print('wrote', len(cases), 'KAT words,', len(progs), 'assembled programs')


if __name__ == '__main__':
    main()
