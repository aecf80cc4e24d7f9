"""API-compatible restatement of the distproc assembler: assembly-level
program dicts -> machine code.

The API surface, statement handling and error messages are the reference's
(``python/distproc/assembler.py``), kept on purpose for drop-in and
bug-for-bug parity; it is therefore a restatement
that follows the reference's method structure, not a clean-room design:

* ``SingleCoreAssembler(elem_cfgs)`` (``:62-541``) -- build one core's program
  from a list of statement dicts (``from_list``) or ``add_*`` calls;
  ``get_compiled_program()`` returns ``(cmd_buf, env_buffers, freq_buffers)``:
  the u128 little-endian command bytes and, per element, the env and freq
  buffers as packed u32 bytes.
* ``GlobalAssembler(compiled_program, channel_configs, elementconfig_class)``
  (``:543-641``) -- one ``SingleCoreAssembler`` per proc group;
  ``get_assembled_program()`` returns ``{core: {'cmd_buf', 'env_buffers',
  'freq_buffers'}}``, the dict ``emulator.ProgramSet`` consumes.

Statement formats are the ones documented at ``assembler.py:1-46``; numeric
conversions (freq / phase / amp / envelope -> words and buffers) go through
the ``ElementConfig`` plugin (``hwconfig.py``), as in the reference.  Parity:
``tests/test_assembler.py`` reproduces, byte for byte, the reference
``GlobalAssembler``'s output on every compiler golden program of
``python/test/test_outputs`` (``tests/golden/asm_programs.json``), with both a
zero-word stub element and ``DDSElementConfig``.

Reference behaviours kept for drop-in parity --
each one also warns, so it is not silent:

* re-declaring a register name allocates a new index (the reference's
  duplicate check tests the literal key ``'name'``, ``assembler.py:202``);
* a pulse with register-sourced phase AND amp and an immediate freq emits a
  leading write whose *freq* field takes the phase register
  (``assembler.py:330``);
* adjacent ``jump_label`` statements are merged by the reference's in-place
  scan, which skips the statement after each merged label
  (``assembler.py:592-612``); this is restated with the same iteration.

Addition: a ``sync`` statement (``{'op': 'sync', 'barrier_id': id}``), the
barrier the compiler documents (``compiler.py:78-82``) and the ISA encodes
(``command_gen.sync``) but the reference assembler does not accept.
"""

from __future__ import annotations

import copy
import json
import warnings
from collections import OrderedDict
from typing import Dict, List, Optional, Union

import numpy as np

from . import isa

ENV_BITS = 16
N_MAX_REGS = 16

ALU_CLASS = ('reg_alu', 'jump_cond', 'alu_fproc', 'jump_fproc', 'inc_qclk')


def _env_key(env) -> str:
    """identity of an envelope for de-duplication within an element: the raw
    sample bytes of an array, the sorted-key JSON of a function dict"""
    if isinstance(env, np.ndarray):
        return 'nd:' + env.data.tobytes().hex()
    if isinstance(env, dict):
        return 'fn:' + json.dumps(env, sort_keys=True)
    raise Exception('{} not supported!'.format(type(env)))


class SingleCoreAssembler:
    """One proc core: statements -> (cmd_buf, env_buffers, freq_buffers)."""

    def __init__(self, elem_cfgs):
        self._elem_cfgs = list(elem_cfgs)
        self.n_element = len(self._elem_cfgs)
        self._env_dicts = [OrderedDict() for _ in range(self.n_element)]   # env key -> envelope
        self._freq_lists: List[list] = [[] for _ in range(self.n_element)]
        self._program: List[dict] = []
        self._regs: Dict[str, dict] = {}

    # ---------------------------------------------------------------- input
    def from_list(self, cmd_list):
        """Append the statements of an assembly-level list (assembler.py:1-46).
        A ``jump_label`` statement labels the statement after it (and, as in
        the reference, writes that label into ``cmd_list``)."""
        handlers = {
            'reg_write': self.add_reg_write, 'phase_reset': self.add_phase_reset,
            'done_stb': self.add_done_stb, 'declare_freq': self.add_freq,
            'declare_reg': self.declare_reg, 'inc_qclk': self.add_inc_qclk, 'idle': self.add_idle,
            'jump_i': self.add_jump_i, 'sync': self.add_sync,
        }
        for i, cmd in enumerate(cmd_list):
            op = cmd['op']
            args = {k: v for k, v in cmd.items() if k != 'op'}
            if op == 'pulse':
                if sum(isinstance(cmd[k], str) for k in ('freq', 'amp', 'phase')) > 1:
                    warnings.warn('{} will be split into multiple instructions, which may cause timing '
                                  'problems'.format(cmd))
                self.add_pulse(**args)
            elif op in ('reg_alu', 'jump_cond', 'alu_fproc', 'jump_fproc'):
                self.add_alu_cmd(op, **args)
            elif op == 'jump_label':
                cmd_list[i + 1]['label'] = args['dest_label']
            elif op in handlers:
                handlers[op](**args)
            else:
                raise Exception('{} not supported!'.format(cmd))

    def _append(self, cmd: dict, label=None):
        if label is not None:
            cmd['label'] = label
        self._program.append(cmd)

    def add_jump_i(self, jump_label, label=None):
        self._append({'op': 'jump_i', 'jump_label': jump_label}, label)

    def add_idle(self, end_time, label=None):
        self._append({'op': 'idle', 'end_time': end_time}, label)

    def add_sync(self, barrier_id=0, label=None):
        """SYNC barrier (ctrl.v SYNC_WAIT; command_gen.sync)."""
        self._append({'op': 'sync', 'barrier_id': int(barrier_id)}, label)

    def add_alu_cmd(self, op: str, in0: Union[int, str], alu_op: str, in1_reg: Optional[str] = None,
                    out_reg: Optional[str] = None, jump_label: Optional[str] = None,
                    func_id=None, label: Optional[str] = None):
        """reg_alu / jump_cond / alu_fproc / jump_fproc / inc_qclk with the
        reference's operand and register-type checks (assembler.py:135-175)."""
        assert op in ALU_CLASS
        regs = self._regs
        if in1_reg is not None:
            assert in1_reg in regs
        if isinstance(in0, str):
            assert in0 in regs
        cmd = {'op': op, 'in0': in0, 'alu_op': alu_op}
        # second ALU input: a register for reg_alu / jump_cond only
        if op in ('reg_alu', 'jump_cond'):
            assert in1_reg is not None and func_id is None
            if isinstance(in0, str):
                assert regs[in0]['dtype'] == regs[in1_reg]['dtype']
            cmd['in1_reg'] = in1_reg
        else:
            assert in1_reg is None
        # destination register: reg_alu / alu_fproc only
        if op in ('reg_alu', 'alu_fproc'):
            assert out_reg is not None
            if isinstance(in0, str):
                assert regs[in0]['dtype'] == regs[out_reg]['dtype']
            if in1_reg is not None:
                assert regs[in1_reg]['dtype'] == regs[out_reg]['dtype']
            cmd['out_reg'] = out_reg
        else:
            assert out_reg is None
        if op in ('jump_cond', 'jump_fproc'):
            assert jump_label is not None
            cmd['jump_label'] = jump_label
        if op in ('alu_fproc', 'jump_fproc'):
            cmd['func_id'] = func_id              # None: fproc id 0
        else:
            assert func_id is None
        self._append(cmd, label)

    def add_env(self, name, env, elem_ind):
        if np.any(np.abs(env) > 1):
            raise Exception('env mag must be < 1')
        self._env_dicts[elem_ind][name] = env

    def add_freq(self, freq, elem_ind, freq_ind=None):
        """Declare a carrier frequency of an element; freq_ind pins its slot."""
        fl = self._freq_lists[elem_ind]
        if freq_ind is None:
            fl.append(freq)
        elif freq_ind >= len(fl):
            # the reference pads with range(len - freq_ind), i.e. never, then appends
            fl.extend([None] * max(0, len(fl) - freq_ind))
            fl.append(freq)
        else:
            if fl[freq_ind] is None:
                raise ValueError('ind {} is already occupied!'.format(freq_ind))
            fl[freq_ind] = freq

    def declare_reg(self, name, dtype=('int',)):
        """Named register at the next free index (dtype ('int',), ('phase', e)
        or ('amp', e))."""
        if self._regs:
            if name in self._regs:
                warnings.warn('register {!r} declared again: it gets a new index (reference '
                              'behaviour, assembler.py:202)'.format(name))
            top = max(r['index'] for r in self._regs.values())
            if top >= N_MAX_REGS - 1:
                raise Exception('cannot add any more regs, limit of {} reached'.format(N_MAX_REGS))
            index = top + 1
        else:
            index = 0
        self._regs[name] = {'index': index, 'dtype': dtype}

    def add_reg_write(self, name, value, dtype=None, label=None):
        """reg[name] = value (declares name if needed): an id0 reg_alu."""
        if name not in self._regs:
            self.declare_reg(name, ('int',) if dtype is None else dtype)
        elif dtype is not None:
            assert dtype == self._regs[name]['dtype']
        self.add_reg_alu(value, 'id0', name, name, label)

    def add_reg_alu(self, in0, alu_op, in1_reg, out_reg, label=None):
        self.add_alu_cmd('reg_alu', in0, alu_op, in1_reg, out_reg, label=label)

    def add_phase_reset(self, label=None):
        self._append({'op': 'pulse_reset'}, label)

    def add_done_stb(self, label=None):
        self._append({'op': 'done_stb'}, label)

    def add_jump_cond(self, in0, alu_op, in1_reg, jump_label, label=None):
        self.add_alu_cmd('jump_cond', in0, alu_op, in1_reg, jump_label=jump_label, label=label)

    def add_inc_qclk(self, in0, label=None):
        self.add_alu_cmd('inc_qclk', in0, 'add', label=label)

    def add_jump_fproc(self, in0, alu_op, jump_label, func_id=None, label=None):
        self.add_alu_cmd('jump_fproc', in0, alu_op, jump_label=jump_label, func_id=func_id, label=label)

    def _register_env(self, env, elem_ind) -> str:
        envs = self._env_dicts[elem_ind]
        if isinstance(env, np.ndarray):
            if np.any((np.abs(np.real(env)) > 1) | (np.abs(np.imag(env)) > 1)):
                raise Exception('env must be < 1')
            key = _env_key(env)
            envs.setdefault(key, env)
        elif isinstance(env, dict):
            key = _env_key(env)
            envs.setdefault(key, env)
        elif isinstance(env, str):
            key = env
            if key not in envs:
                if key != 'cw':
                    raise Exception('Envelope not found: {}'.format(key))
                envs[key] = 'cw'
        else:
            raise Exception('env must be string, dict, or np array')
        return key

    def add_pulse(self, freq, phase, amp, start_time, env, elem_ind, label=None, tag=None):
        """Pulse on element elem_ind at start_time (clocks).  freq (Hz) /
        phase (rad) / amp (<= 1) are immediates or named registers; env is a
        sample array, an envelope-function dict or a named envelope ('cw').
        The pulse register file takes one register source per command, so
        several register-sourced fields become several commands."""
        key = self._register_env(env, elem_ind)
        regs = self._regs
        if isinstance(freq, str):
            assert freq in regs and regs[freq]['dtype'] == ('int',)
        elif freq not in self._freq_lists[elem_ind]:
            self.add_freq(freq, elem_ind)
        if isinstance(amp, str):
            assert amp in regs and regs[amp]['dtype'] == ('amp', elem_ind)
        if isinstance(phase, str):
            assert phase in regs and regs[phase]['dtype'] == ('phase', elem_ind)

        f_reg, p_reg, a_reg = isinstance(freq, str), isinstance(phase, str), isinstance(amp, str)
        trig = {'op': 'pulse', 'start_time': start_time, 'env': key, 'elem': elem_ind}
        if f_reg and p_reg and a_reg:
            self._program.append({'op': 'pulse', 'freq': freq, 'elem': elem_ind})
            self._program.append({'op': 'pulse', 'amp': amp, 'elem': elem_ind})
            cmd = dict(trig, phase=phase)
        elif f_reg and (p_reg or a_reg):
            self._program.append({'op': 'pulse', 'freq': freq, 'elem': elem_ind})
            cmd = dict(trig, phase=phase, amp=amp)
        elif p_reg and a_reg:
            warnings.warn('pulse with register phase and amp: the leading write carries the phase '
                          'register in its freq field (reference behaviour, assembler.py:330)')
            self._program.append({'op': 'pulse', 'freq': phase})
            cmd = dict(trig, freq=freq, amp=amp)
        else:
            cmd = dict(trig, freq=freq, phase=phase, amp=amp)
        self._append(cmd, label)

    # ---------------------------------------------------------------- output
    def _labels(self) -> Dict[str, int]:
        out = {}
        for addr, cmd in enumerate(self._program):
            if 'label' in cmd:
                if cmd['label'] in out:
                    raise Exception('label already in use!')
                out[cmd['label']] = addr
        return out

    def _env_buffer(self, e):
        """(u32 samples, env word per key) of element e, envelopes in declaration order"""
        cfg = self._elem_cfgs[e]
        words, parts, at = {}, [], 0
        for key, env in self._env_dicts[e].items():
            buf = cfg.get_env_buffer(env)
            words[key] = cfg.get_cw_env_word(at) if key == 'cw' else cfg.get_env_word(at, len(buf))
            at += len(buf)
            parts.append(np.asarray(buf))
        raw = np.concatenate(parts) if parts else np.empty(0)
        return np.array(raw.astype(int), dtype=np.uint32), words

    def _freq_buffer(self, e):
        fl = self._freq_lists[e]
        buf = self._elem_cfgs[e].get_freq_buffer(fl)
        return np.array(buf, dtype=np.uint32), {f: fl.index(f) for f in fl}

    def _pulse_word(self, cmd, env_words, freq_inds) -> int:
        args = {}
        e = cmd.get('elem')
        cfg = self._elem_cfgs[e] if e is not None else None
        for field, conv in (('freq', None), ('phase', 'get_phase_word'), ('amp', 'get_amp_word')):
            if field not in cmd:
                continue
            v = cmd[field]
            if isinstance(v, str):
                args[field + '_regaddr'] = self._regs[v]['index']
            elif field == 'freq':
                args['freq_word'] = cfg.get_freq_addr(freq_inds[e][v])
            else:
                args[field + '_word'] = getattr(cfg, conv)(v)
        if 'env' in cmd:
            args['env_word'] = env_words[e][cmd['env']]
        if 'start_time' in cmd:
            args['cmd_time'] = cmd['start_time']
        if e is not None:
            args['cfg_word'] = cfg.get_cfg_word(e, None)
        return isa.pulse_cmd(**args)

    def _alu_word(self, cmd, labels) -> int:
        in0 = cmd['in0']
        if isinstance(in0, str):
            in0, src = self._regs[in0]['index'], 'r'
        else:
            src = 'i'
            # an immediate meant for a typed register is converted to its word
            typed = cmd.get('out_reg', cmd.get('in1_reg'))
            if typed is not None:
                dtype = self._regs[typed]['dtype']
                if dtype[0] == 'phase':
                    in0 = self._elem_cfgs[dtype[1]].get_phase_word(cmd['in0'])
                elif dtype[0] == 'amp':
                    in0 = self._elem_cfgs[dtype[1]].get_amp_word(cmd['in0'])
        reg = lambda k: self._regs[cmd[k]]['index'] if k in cmd else None
        target = labels[cmd['jump_label']] if 'jump_label' in cmd else None
        return isa.alu_cmd(cmd['op'], src, in0, cmd.get('alu_op'), reg('in1_reg'), reg('out_reg'), target,
                           cmd.get('func_id'))

    def get_compiled_program(self):
        """-> (cmd_buf bytes, [env buffer bytes per element], [freq buffer bytes per element])"""
        envs = [self._env_buffer(e) for e in range(self.n_element)]
        freqs = [self._freq_buffer(e) for e in range(self.n_element)]
        env_words = [w for _, w in envs]
        freq_inds = [m for _, m in freqs]
        labels = self._labels()
        words = []
        for cmd in self._program:
            op = cmd['op']
            if op == 'pulse':
                words.append(self._pulse_word(cmd, env_words, freq_inds))
            elif op in ALU_CLASS:
                words.append(self._alu_word(cmd, labels))
            elif op == 'jump_i':
                words.append(isa.jump_i(labels[cmd['jump_label']]))
            elif op == 'pulse_reset':
                words.append(isa.pulse_reset())
            elif op == 'idle':
                words.append(isa.idle(cmd['end_time']))
            elif op == 'done_stb':
                words.append(isa.done_cmd())
            elif op == 'sync':
                words.append(isa.sync(cmd['barrier_id']))
            else:
                raise Exception('{} not supported'.format(op))
        cmd_buf = b''.join(int(w).to_bytes(16, 'little') for w in words)
        return cmd_buf, [b.tobytes() for b, _ in envs], [b.tobytes() for b, _ in freqs]

    def get_sim_program(self):
        """the statement list with envelope keys replaced by the envelopes"""
        out = []
        for cmd in self._program:
            cmd = copy.deepcopy(cmd)
            if cmd['op'] == 'pulse' and 'env' in cmd:
                cmd['env'] = self._env_dicts[cmd['elem']][cmd['env']]
            out.append(cmd)
        return out


class GlobalAssembler:
    """A compiled program (``.program`` {proc group: statements}, ``.proc_groups``,
    ``.fpga_config``) -> per-core machine code (assembler.py:543-641)."""

    def __init__(self, compiled_program, channel_configs, elementconfig_class):
        self.assemblers: Dict[str, SingleCoreAssembler] = {}
        self.channel_configs = channel_configs
        compiled_program = copy.deepcopy(compiled_program)
        fc = getattr(compiled_program, 'fpga_config', None)
        if fc is not None and int(np.round(channel_configs['fpga_clk_freq'])) != int(np.round(fc.fpga_clk_freq)):
            raise Exception('Program target clock {} Hz does not match HW clock {}'.format(
                fc.fpga_clk_freq, channel_configs['fpga_clk_freq']))
        for group in compiled_program.proc_groups:
            core = str(channel_configs[group[0]].core_ind)
            elems = {}
            for chan in group:
                cc = channel_configs[chan]
                assert cc.core_ind == int(core)
                elems[cc.elem_ind] = elementconfig_class(**cc.elem_params)
            # element indices of a core must be 0, 1, ..., n - 1
            assert sorted(elems) == list(range(len(elems)))
            self.assemblers[core] = SingleCoreAssembler([elems[i] for i in sorted(elems)])
            statements = compiled_program.program[group]
            self._resolve_dest_fproc_chans(statements)
            self._resolve_duplicate_jump_labels(statements)
            self.assemblers[core].from_list(statements)

    def _resolve_dest_fproc_chans(self, statements):
        """pulse 'dest' channel -> 'elem_ind'; fproc func_id: int as is, (channel,
        attribute) tuple -> that ChannelConfig attribute, str -> channel_configs[str]"""
        for st in statements:
            if st['op'] == 'pulse':
                st['elem_ind'] = self.channel_configs[st.pop('dest')].elem_ind
            elif st['op'] in ('alu_fproc', 'jump_fproc'):
                fid = st['func_id']
                if isinstance(fid, tuple):
                    st['func_id'] = getattr(self.channel_configs[fid[0]], fid[1])
                elif isinstance(fid, str):
                    st['func_id'] = self.channel_configs[fid]
                else:
                    assert isinstance(fid, int)

    @staticmethod
    def _resolve_duplicate_jump_labels(statements):
        """Merge runs of jump_label statements into the first label of the run,
        retargeting jumps.  Restates the reference's in-place scan (indices over
        the original length while popping), including the statement it skips
        after each removal."""
        merged = {}
        run_label = None
        for i in range(len(statements) - 1):
            st = statements[i]
            if st['op'] == 'jump_label':
                if run_label is None:
                    run_label = st['dest_label']
                else:
                    merged[st['dest_label']] = run_label
                    statements.pop(i)
            else:
                run_label = None
        if merged:
            for st in statements:
                if st.get('jump_label') in merged:
                    st['jump_label'] = merged[st['jump_label']]

    def get_assembled_program(self):
        """{core index str: {'cmd_buf': bytes, 'env_buffers': [bytes], 'freq_buffers': [bytes]}}"""
        out = {}
        for core, asm in self.assemblers.items():
            cmd_buf, env_raw, freq_raw = asm.get_compiled_program()
            out[core] = {'cmd_buf': cmd_buf, 'env_buffers': env_raw, 'freq_buffers': freq_raw}
        return out
