"""Clean-room restatement of the distproc compiler's scheduling stage
(upstream of the emulated path and optional).

What it restates, with the reference lines it follows:

* ``CoreScoper`` -- channel -> proc-core grouping (``ir/ir.py:324-368``);
  ``QubitScoper`` -- qubit -> channel scope (``ir/ir.py:284-313``).
* ``Schedule`` -- assigns every pulse a ``start_time`` in FPGA clocks,
  resolves ``hold`` into ``idle``, removes ``barrier`` / ``delay``, and
  measures loop bodies (``ir/passes.py:596-742``).
* ``LintSchedule`` -- rejects user schedules whose pulses or idles start
  before the core can issue them (``ir/passes.py:745-822``).
* A straight-line gate-level front end: ``resolve_gates``
  (``ir/passes.py:287-357``), ``resolve_virtual_z`` (``:439-491``),
  ``resolve_freqs`` (``:493-515``) and ``compile_blocks``
  (``compiler.py:227-331``), so a QubiC-circuit list such as
  ``[{'name': 'X90', 'qubit': ['Q0']}, {'name': 'read', 'qubit': ['Q0']}]``
  becomes the ``{proc group: [statements]}`` dict ``assembler.GlobalAssembler``
  consumes -- without the reference's ``qubic`` / ``parse`` / ``networkx``
  dependencies, none of which is in this image.

The IR here is deliberately small: a program is an ordered dict of basic
blocks ``{name: {'instructions': [Instr], 'scope': set(dest)}}`` plus CFG
edges and a loop table (``ScheduleIR``).  ``Instr`` carries the reference
instruction's name and fields (``ir/instructions.py``) as attributes.
Scheduling is exactly the reference's arithmetic, including its quirks:
a ``hold`` whose target is already passed is dropped (``>=``,
``passes.py:714``), and a loop-control block's end time is the loop's start
time (``:641-649``).

* A control-flow front end, ``compile_circuit``: ``flatten``
  (FlattenProgram, ``ir/passes.py:62-124``), ``make_basic_blocks``
  (``:135-178``), ``scope_blocks`` (ScopeProgram, ``:207-234``),
  ``generate_cfg`` (``:368-388``), ``resolve_virtual_z_cfg`` (``:439-491``)
  and ``resolve_fproc_channels`` (hold insertion, ``:532-552``) for
  ``branch_fproc`` / ``branch_var`` / ``loop`` circuits, with ``declare``,
  ``set_var``, ``alu``, ``read_fproc`` / ``alu_fproc`` compiled as in
  ``compiler.py:283-320``, variable registration (``:253-283``) and
  hardware virtual z (``bind_phase``, ResolveHWVirtualZ ``:405-437``) and
  RescopeVars (``:563-593``).  Addition: a ``sync`` statement
  (``{'name': 'sync', 'scope': [...], 'barrier_id': id}``, the barrier
  ``compiler.py:78-82`` documents), scheduled as a qclk restart of its scope
  (build-defined) and compiled to the assembler's ``sync``.

Parity: ``tests/test_schedule.py`` reproduces the reference's scheduling
asserts (``python/test/test_compiler.py:75-98``), its user-schedule lint
verdicts (``:561-606``) and, end to end through ``assembler.py``, all nine
compiler goldens of ``python/test/test_outputs`` (linear, pulse,
multirst_cfg, multirst_fproc_res_cfg, fproc_hold, simple_loop,
compound_loop, nested_loop, hw_virtualz): the compiled statements field by
field, and the assembled bytes exactly (or the reference's rejection).
"""

from __future__ import annotations

import ast
import copy
import math
import re
from collections import OrderedDict
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

from .hwconfig import FPGAConfig

START_NCLKS = 5                      # passes.py:613, :753
DEFAULT_PROC_GROUPING = [('{qubit}.qdrv', '{qubit}.rdrv', '{qubit}.rdlo')]
DEFAULT_QUBIT_GROUPING = ('{qubit}.qdrv', '{qubit}.rdrv', '{qubit}.rdlo')


class Instr:
    """One IR instruction: ``name`` plus the reference instruction's fields."""

    def __init__(self, name: str, **fields):
        self.name = name
        self.__dict__.update(fields)

    def __getattr__(self, item):          # absent optional fields read as None
        if item.startswith('__'):
            raise AttributeError(item)
        return None

    def __repr__(self):
        body = ', '.join('{}={!r}'.format(k, v) for k, v in self.__dict__.items()
                         if k != 'name' and k != 'env')
        return '{}({})'.format(self.name, body)


def instr(d) -> Instr:
    """dict (``{'name': ..., field: ...}``) or Instr -> Instr; ``scope`` becomes a set"""
    if isinstance(d, Instr):
        return d
    d = dict(d)
    name = d.pop('name')
    if name == 'sync':
        # the documented form {'name': 'sync', 'barrier_id': id, 'qubits': [...]}
        # (compiler.py:78-82): qubits / qubit name the scope; none = the whole program
        q = d.pop('qubits', None)
        q = d.pop('qubit', None) if q is None else q
        if d.get('scope') is None and q is not None:
            d['scope'] = [q] if isinstance(q, str) else list(q)
    if 'scope' in d and d['scope'] is not None:
        d['scope'] = set(d['scope'])
    if name == 'pulse' and 'scope' not in d:
        d['scope'] = {d['dest']}
    return Instr(name, **d)


# ---------------------------------------------------------------- scopers
def _pattern_regex(pattern: str):
    """'{qubit}.qdrv' -> regex with named groups (the subset of ``parse`` the
    groupings use: whole-string match, ``{name}`` fields)"""
    out, pos = '', 0
    for m in re.finditer(r'\{(\w+)\}', pattern):
        out += re.escape(pattern[pos:m.start()]) + '(?P<{}>.+?)'.format(m.group(1))
        pos = m.end()
    return re.compile(out + re.escape(pattern[pos:]) + r'\Z')


class CoreScoper:
    """dest channel -> proc-core tuple (``ir/ir.py:324-368``)."""

    def __init__(self, dest_channels: Iterable[str], proc_grouping=DEFAULT_PROC_GROUPING):
        self.proc_groupings: Dict[str, Tuple[str, ...]] = {}
        for dest in dest_channels:
            for group in proc_grouping:
                for pattern in group:
                    m = _pattern_regex(pattern).match(dest)
                    if m is not None:
                        self.proc_groupings[dest] = tuple(p.format(**m.groupdict()) for p in group)
        self.proc_groupings_flat = set(self.proc_groupings.values())

    def get_groups_bydest(self, dests) -> set:
        return {self.proc_groupings[d] for d in dests}


class QubitScoper:
    """qubit -> its channels (``ir/ir.py:284-313``)."""

    def __init__(self, mapping=DEFAULT_QUBIT_GROUPING):
        self._mapping = mapping

    def get_scope(self, qubits) -> set:
        """a qubit name maps to all its channels; a channel name to itself"""
        if isinstance(qubits, str):
            qubits = [qubits]
        out = set()
        for q in qubits:
            if any(_pattern_regex(m).match(q) for m in self._mapping):
                out.add(q)
            else:
                out |= {m.format(qubit=q) for m in self._mapping}
        return out


# ---------------------------------------------------------------- program
class ScheduleIR:
    """Basic blocks + CFG + loops: the parts of ``IRProgram`` (``ir/ir.py:50-272``)
    the scheduling passes read and write."""

    def __init__(self, blocks: Dict[str, Sequence], edges: Sequence[Tuple[str, str]] = (),
                 scope: Optional[Iterable[str]] = None):
        self.blocks: 'OrderedDict[str, dict]' = OrderedDict()
        for name, instrs in blocks.items():
            il = [instr(i) for i in instrs]
            bscope = set()
            for i in il:
                if i.scope:
                    bscope |= set(i.scope)
                if i.name == 'pulse':
                    bscope.add(i.dest)
            self.blocks[name] = {'instructions': il, 'scope': bscope}
        self.edges = [tuple(e) for e in edges]
        for a, b in self.edges:
            if a not in self.blocks or b not in self.blocks:
                raise ValueError('CFG edge {}->{} names an unknown block'.format(a, b))
        self.scope = set(scope) if scope is not None else \
            set().union(*(b['scope'] for b in self.blocks.values())) if self.blocks else set()
        self.loops: Dict[str, dict] = {}
        self.freqs: Dict[str, float] = {}
        self.fpga_config = None

    def predecessors(self, node):
        return [a for a, b in self.edges if b == node]

    def topological_order(self) -> List[str]:
        """Kahn's algorithm, ties broken by block order (any topological order
        gives the same schedule: a block reads only its predecessors)."""
        indeg = {n: 0 for n in self.blocks}
        for _, b in self.edges:
            indeg[b] += 1
        order, ready = [], [n for n in self.blocks if indeg[n] == 0]
        while ready:
            n = ready.pop(0)
            order.append(n)
            for a, b in self.edges:
                if a == n:
                    indeg[b] -= 1
                    if indeg[b] == 0:
                        ready.append(b)
            ready.sort(key=list(self.blocks).index)
        if len(order) != len(self.blocks):
            raise ValueError('control-flow graph has a cycle: loops are expressed as '
                             'a *_loopctrl block ending in a loopctrl jump_cond, not a back edge')
        return order

    def register_loop(self, name, scope, start_time, delta_t=None):
        self.loops[name] = {'scope': set(scope), 'start_time': start_time, 'delta_t': delta_t}


def _nclks(length_secs, fpga_config) -> int:
    return int(np.ceil(length_secs / fpga_config.fpga_clk_period))


def _is_loopctrl_end(instrs) -> bool:
    return bool(instrs) and instrs[-1].name == 'jump_cond' and instrs[-1].jump_type == 'loopctrl'


# ---------------------------------------------------------------- Schedule
class Schedule:
    """``ir/passes.py:596-742``: pulse start times, hold -> idle, loop delta_t."""

    def __init__(self, fpga_config: FPGAConfig, proc_grouping=DEFAULT_PROC_GROUPING):
        self._fpga_config = fpga_config
        self._start_nclks = START_NCLKS
        self._proc_grouping = proc_grouping

    def run_pass(self, prog: ScheduleIR):
        self._core_scoper = CoreScoper(prog.scope, self._proc_grouping)
        for node in prog.topological_order():
            block = prog.blocks[node]
            cur_t = {d: self._start_nclks for d in prog.scope}
            last_end = {g: self._start_nclks for g in self._core_scoper.get_groups_bydest(block['scope'])}
            for pred in prog.predecessors(node):                     # :624-630
                pb = prog.blocks[pred]
                for d in cur_t:
                    if d in pb['scope']:
                        cur_t[d] = max(cur_t[d], pb['block_end_t'][d])
                for g in last_end:
                    if g in pb['last_instr_end_t']:
                        last_end[g] = max(last_end[g], pb['last_instr_end_t'][g])

            if node.split('_')[-1] == 'loopctrl':                    # :634-636, :741-742
                prog.register_loop(node, block['scope'], max(cur_t.values()))

            self._schedule_block(block['instructions'], cur_t, last_end)

            if _is_loopctrl_end(block['instructions']):              # :641-649
                loop = prog.loops[block['instructions'][-1].jump_label]
                block['block_end_t'] = {d: loop['start_time'] for d in block['scope']}
                block['last_instr_end_t'] = {g: loop['start_time']
                                             for g in self._core_scoper.get_groups_bydest(block['scope'])}
                loop['delta_t'] = max(max(last_end.values()), max(cur_t.values())) - loop['start_time']
            else:
                block['block_end_t'] = dict(cur_t)
                block['last_instr_end_t'] = last_end
        prog.fpga_config = self._fpga_config

    def _schedule_block(self, instructions: List[Instr], cur_t, last_end):
        cfg, grp_of = self._fpga_config, self._core_scoper.proc_groupings
        groups = self._core_scoper.get_groups_bydest
        cost = {'alu': cfg.alu_instr_clks, 'set_var': cfg.alu_instr_clks,
                'rc_alu': getattr(cfg, 'rc_alu_clks', cfg.alu_instr_clks),
                'jump_fproc': cfg.jump_fproc_clks, 'read_fproc': cfg.jump_fproc_clks,
                'alu_fproc': cfg.jump_fproc_clks, 'jump_i': cfg.jump_cond_clks,
                'jump_cond': cfg.jump_cond_clks, 'loop_end': cfg.alu_instr_clks}
        i = 0
        while i < len(instructions):
            ins = instructions[i]
            if ins.name == 'pulse':                                  # :662-668
                g = grp_of[ins.dest]
                ins.start_time = max(last_end[g], cur_t[ins.dest])
                last_end[g] = ins.start_time + cfg.pulse_load_clks
                cur_t[ins.dest] = ins.start_time + _nclks(ins.twidth, cfg)
            elif ins.name == 'barrier':                              # :670-677
                t = max(max(cur_t[d] for d in ins.scope),
                        max(last_end[grp_of[d]] for d in ins.scope))
                for d in ins.scope:
                    cur_t[d] = t
                instructions.pop(i)
                continue
            elif ins.name == 'delay':                                # :679-683
                for d in ins.scope:
                    cur_t[d] += _nclks(ins.t, cfg)
                instructions.pop(i)
                continue
            elif ins.name in cost:                                   # :685-707
                for g in groups(ins.scope):
                    last_end[g] += cost[ins.name]
            elif ins.name == 'hold':                                 # :709-724
                idle_end = max(cur_t[d] for d in ins.ref_chans) + ins.nclks
                idle_scope = set()
                for g in groups(ins.scope):
                    if last_end[g] < idle_end:
                        idle_scope |= set(g)
                        last_end[g] = idle_end + cfg.pulse_load_clks
                if idle_scope:
                    instructions[i] = Instr('idle', end_time=idle_end, scope=idle_scope)
                else:
                    instructions.pop(i)
                    continue
            elif ins.name == 'sync':
                # build-defined (the reference schedules no sync): qclk restarts
                # at the barrier (hdl: qclk(S+2) = 0), so the scope's channel
                # and core clocks restart like after reset
                for d in ins.scope:
                    cur_t[d] = self._start_nclks
                for g in groups(ins.scope):
                    last_end[g] = self._start_nclks
            elif ins.name == 'latch_rc_cycle':                       # :726-730
                t = max(last_end[g] for g in groups(ins.scope))
                ins.t = t
                for g in groups(ins.scope):
                    last_end[g] = t + cfg.pulse_load_clks
            elif ins.name == 'gate':
                raise Exception('Must resolve gates first!')
            i += 1


class LintSchedule:
    """``ir/passes.py:745-822``: raise if a scheduled pulse / idle is early."""

    def __init__(self, fpga_config: FPGAConfig, proc_grouping=DEFAULT_PROC_GROUPING):
        self._fpga_config = fpga_config
        self._proc_grouping = proc_grouping

    def run_pass(self, prog: ScheduleIR):
        self._core_scoper = CoreScoper(prog.scope, self._proc_grouping)
        for node in prog.topological_order():
            block = prog.blocks[node]
            last_end = {g: START_NCLKS for g in self._core_scoper.get_groups_bydest(block['scope'])}
            for pred in prog.predecessors(node):
                pl = prog.blocks[pred]['last_instr_end_t']
                for g in last_end:
                    if g in pl:
                        last_end[g] = max(last_end[g], pl[g])
            self._lint_block(block['instructions'], last_end)
            if _is_loopctrl_end(block['instructions']):
                t0 = prog.loops[block['instructions'][-1].jump_label]['start_time']
                block['last_instr_end_t'] = {g: t0 for g in self._core_scoper.get_groups_bydest(block['scope'])}
            else:
                block['last_instr_end_t'] = last_end
        prog.fpga_config = self._fpga_config

    def _lint_block(self, instructions, last_end):
        cfg, grp_of = self._fpga_config, self._core_scoper.proc_groupings
        cost = {'alu': cfg.alu_instr_clks, 'set_var': cfg.alu_instr_clks,
                'jump_fproc': cfg.jump_fproc_clks, 'read_fproc': cfg.jump_fproc_clks,
                'alu_fproc': cfg.jump_fproc_clks, 'jump_i': cfg.jump_cond_clks,
                'jump_cond': cfg.jump_cond_clks, 'loop_end': cfg.alu_instr_clks}
        for i, ins in enumerate(instructions):
            if ins.name == 'pulse':
                g = grp_of[ins.dest]
                if ins.start_time < last_end[g]:
                    raise Exception('instruction {}: {}; start time too early; must be >= {}'
                                    .format(i, ins, last_end[g]))
                last_end[g] = ins.start_time + cfg.pulse_load_clks
            elif ins.name in cost:
                for g in self._core_scoper.get_groups_bydest(ins.scope):
                    last_end[g] += cost[ins.name]
            elif ins.name == 'sync':
                for g in self._core_scoper.get_groups_bydest(ins.scope):
                    last_end[g] = START_NCLKS
            elif ins.name == 'idle':
                for g in self._core_scoper.get_groups_bydest(ins.scope):
                    if ins.end_time < last_end[g]:
                        raise Exception('instruction {}: {}; end time too early; must be >= {}'
                                        .format(i, ins, last_end[g]))
                    last_end[g] = ins.end_time + cfg.pulse_load_clks
            elif ins.name == 'gate':
                raise Exception('Must resolve gates first!')


# ---------------------------------------------------------------- front end
_SAFE_NAMES = {'pi': math.pi}
_BINOPS = {ast.Add: lambda a, b: a + b, ast.Sub: lambda a, b: a - b,
           ast.Mult: lambda a, b: a * b, ast.Div: lambda a, b: a / b}


def _num(v):
    """qubitcfg numeric field: a number or an expression such as
    ``'numpy.pi/2.0'`` / ``'np.pi/2'`` (arithmetic on constants and pi only)"""
    if not isinstance(v, str):
        return v

    def ev(n):
        if isinstance(n, ast.Expression):
            return ev(n.body)
        if isinstance(n, ast.Constant) and isinstance(n.value, (int, float)):
            return n.value
        if isinstance(n, ast.Attribute) and n.attr in _SAFE_NAMES and \
                isinstance(n.value, ast.Name) and n.value.id in ('np', 'numpy', 'math'):
            return _SAFE_NAMES[n.attr]
        if isinstance(n, ast.UnaryOp) and isinstance(n.op, ast.USub):
            return -ev(n.operand)
        if isinstance(n, ast.BinOp) and type(n.op) in _BINOPS:
            return _BINOPS[type(n.op)](ev(n.left), ev(n.right))
        raise ValueError('unsupported numeric expression {!r}'.format(v))

    return ev(ast.parse(v, mode='eval'))


class GateTable:
    """The ``Qubits`` / ``Gates`` sections of a qubitcfg.json (the QChip input
    of ``ResolveGates``): named frequencies and gate -> pulse lists."""

    def __init__(self, qubitcfg: dict):
        self.freqs = {'{}.{}'.format(q, k): float(v)
                      for q, d in qubitcfg.get('Qubits', {}).items() for k, v in d.items()}
        self.gates = qubitcfg['Gates']

    def pulses(self, gate_name: str) -> List[dict]:
        if gate_name not in self.gates:
            raise KeyError('gate {} not in the gate table'.format(gate_name))
        return self.gates[gate_name]


def resolve_gates(program: Sequence[dict], table: GateTable,
                  qubit_grouping=DEFAULT_QUBIT_GROUPING) -> List[Instr]:
    """Straight-line QubiC circuit -> IR (``ir/passes.py:287-357``): each gate
    becomes Barrier(qubit scope), then per gate pulse an optional Delay(t0)
    and a Pulse, or a VirtualZ.  ``pulse`` / ``virtual_z`` / ``barrier`` /
    ``delay`` / ``hold`` statements pass through as IR instructions."""
    scoper = QubitScoper(qubit_grouping)
    out: List[Instr] = []
    for st in program:
        if isinstance(st, Instr):                # flattened control flow / scoped IR
            if st.name != 'gate':
                out.append(st)
                continue
            st = {'name': st.gate, 'qubit': st.qubit}
        name = st['name']
        if name in ('pulse',):
            d = dict(st)
            d['phase'] = _num(d['phase'])
            out.append(instr(d))
        elif name in ('virtual_z', 'virtualz'):
            q = st['qubit'][0] if isinstance(st['qubit'], (list, tuple)) else st['qubit']
            out.append(Instr('virtual_z', freq=st.get('freq', '{}.freq'.format(q)), phase=_num(st['phase']),
                             scope=scoper.get_scope(st['qubit'])))
        elif name in ('barrier', 'delay'):
            scope = scoper.get_scope(st['scope']) if 'scope' in st else scoper.get_scope(st['qubit'])
            out.append(Instr(name, scope=scope, **({'t': st['t']} if name == 'delay' else {})))
        elif name in ('branch_fproc', 'branch_var', 'loop', 'jump_fproc', 'jump_cond'):
            raise NotImplementedError('control flow: use compile_circuit (flatten -> basic blocks)')
        else:
            qubits = st['qubit'] if isinstance(st['qubit'], (list, tuple)) else [st['qubit']]
            out.append(Instr('barrier', scope=scoper.get_scope(qubits)))
            for p in table.pulses(''.join(qubits) + name):
                if 'gate' in p:
                    if p['gate'] != 'virtualz':
                        raise NotImplementedError('gate {} references gate {}: nested gate '
                                                  'dereferencing is not restated'.format(name, p['gate']))
                    out.append(Instr('virtual_z', freq=p['freq'], phase=_num(p['phase']), scope=set()))
                    continue
                if p.get('t0', 0) != 0:
                    out.append(Instr('delay', t=p['t0'], scope={p['dest']}))
                out.append(Instr('pulse', freq=p['freq'], phase=_num(p['phase']), amp=p['amp'],
                                 env=copy.deepcopy(p['env']), twidth=p['twidth'], dest=p['dest'],
                                 scope={p['dest']}))
    return out


def resolve_virtual_z(instructions: List[Instr]) -> List[Instr]:
    """``ir/passes.py:439-491`` on one block: accumulate virtual-z phase per
    frequency, add it to later pulses on that frequency, drop the VirtualZs."""
    acc: Dict[object, float] = {}
    out = []
    for ins in instructions:
        if ins.name == 'pulse':
            if ins.freq in acc:
                ins.phase += acc[ins.freq]
            out.append(ins)
        elif ins.name == 'virtual_z':
            acc[ins.freq] = acc.get(ins.freq, 0) + ins.phase
        else:
            out.append(ins)
    return out


def resolve_freqs(instructions: List[Instr], table: GateTable) -> List[Instr]:
    """``ir/passes.py:493-515``: named frequencies -> Hz."""
    for ins in instructions:
        if ins.name == 'pulse' and isinstance(ins.freq, str):
            ins.freq = table.freqs[ins.freq]
    return instructions


def compile_blocks(prog: ScheduleIR, proc_grouping=DEFAULT_PROC_GROUPING) -> Dict[tuple, List[dict]]:
    """``compiler.py:227-331`` for the instructions a scheduled straight-line /
    block program holds: ``{proc group: [phase_reset, ..., done_stb]}``."""
    scoper = CoreScoper(prog.scope, proc_grouping)
    progs = {g: [{'op': 'phase_reset'}] for g in scoper.proc_groupings_flat}
    for block in prog.blocks.values():
        for ins in block['instructions']:
            if ins.name == 'pulse':
                env = ins.env
                if isinstance(env, (list, tuple)) and env and isinstance(env[0], dict):
                    env = env[0]
                if isinstance(env, dict):
                    if 'twidth' not in env['paradict']:
                        env = copy.deepcopy(env)
                        env['paradict']['twidth'] = ins.twidth
                    elif env['paradict']['twidth'] != ins.twidth:
                        raise Exception('Pulse twidth differs from envelope!')
                st = {'op': 'pulse', 'freq': ins.freq, 'phase': ins.phase, 'amp': ins.amp,
                      'env': env, 'start_time': ins.start_time, 'dest': ins.dest}
                if ins.tag is not None:
                    st['tag'] = ins.tag
                progs[scoper.proc_groupings[ins.dest]].append(st)
            elif ins.name == 'idle':
                for g in scoper.get_groups_bydest(ins.scope):
                    progs[g].append({'op': 'idle', 'end_time': ins.end_time})
            elif ins.name == 'jump_label':
                for g in scoper.get_groups_bydest(ins.scope):
                    progs[g].append({'op': 'jump_label', 'dest_label': ins.label})
            elif ins.name == 'jump_i':
                for g in scoper.get_groups_bydest(ins.scope):
                    progs[g].append({'op': 'jump_i', 'jump_label': ins.jump_label})
            elif ins.name == 'jump_fproc':
                for g in scoper.get_groups_bydest(ins.scope):
                    progs[g].append({'op': 'jump_fproc', 'in0': ins.cond_lhs, 'alu_op': ins.alu_cond,
                                     'jump_label': ins.jump_label, 'func_id': ins.func_id})
            elif ins.name == 'loop_end':
                for g in scoper.get_groups_bydest(ins.scope):
                    progs[g].append({'op': 'inc_qclk', 'in0': -prog.loops[ins.loop_label]['delta_t']})
            elif ins.name == 'sync':          # the barrier compiler.py:78-82 documents
                for g in scoper.get_groups_bydest(ins.scope):
                    progs[g].append({'op': 'sync', 'barrier_id': ins.barrier_id or 0})
            elif ins.name == 'declare':                              # compiler.py:283-287
                dtype = (ins.dtype, 0) if ins.dtype in ('phase', 'amp') else ins.dtype
                for g in scoper.get_groups_bydest(ins.scope):
                    progs[g].append({'op': 'declare_reg', 'name': ins.var, 'dtype': dtype})
            elif ins.name == 'alu':
                for g in scoper.get_groups_bydest(ins.scope):
                    progs[g].append({'op': 'reg_alu', 'in0': ins.lhs, 'in1_reg': ins.rhs,
                                     'alu_op': ins.op, 'out_reg': ins.out})
            elif ins.name == 'set_var':
                for g in scoper.get_groups_bydest(ins.scope):
                    progs[g].append({'op': 'reg_alu', 'in0': ins.value, 'in1_reg': ins.var,
                                     'alu_op': 'id0', 'out_reg': ins.var})
            elif ins.name == 'read_fproc':
                for g in scoper.get_groups_bydest(ins.scope):
                    progs[g].append({'op': 'alu_fproc', 'in0': 0, 'alu_op': 'id1',
                                     'func_id': ins.func_id, 'out_reg': ins.var})
            elif ins.name == 'alu_fproc':
                for g in scoper.get_groups_bydest(ins.scope):
                    progs[g].append({'op': 'alu_fproc', 'in0': ins.lhs, 'alu_op': ins.op,
                                     'func_id': ins.func_id, 'out_reg': ins.out})
            elif ins.name == 'jump_cond':
                for g in scoper.get_groups_bydest(ins.scope):
                    progs[g].append({'op': 'jump_cond', 'in0': ins.cond_lhs, 'alu_op': ins.alu_cond,
                                     'jump_label': ins.jump_label, 'in1_reg': ins.cond_rhs})
            else:
                raise Exception('{} not yet implemented'.format(ins.name))
    for g in progs:
        progs[g].append({'op': 'done_stb'})
    return progs


def sync_mask(program: Dict[tuple, List[dict]], core_order: Sequence[tuple]) -> int:
    """the dpemu_config.sync_mask a compiled program implies: bit c set for
    the proc group at index c of ``core_order`` (the emulator's core order)
    when its program holds a sync.  A sync over a subset of cores needs this
    mask -- the default mask is every core, and a core that never syncs would
    leave the barrier waiting (ST_DEADLOCK)."""
    mask = 0
    for c, g in enumerate(core_order):
        if any(st.get('op') == 'sync' for st in program.get(g, ())):
            mask |= 1 << c
    return mask


class CompiledProgram:
    """The attribute surface ``GlobalAssembler`` reads (``compiler.py:338-366``)."""

    def __init__(self, program: Dict[tuple, List[dict]], fpga_config=None):
        self.program = program
        self.proc_groups = list(program.keys())
        self.fpga_config = fpga_config


def compile_straight(program: Sequence[dict], table: GateTable, fpga_config: FPGAConfig,
                     schedule: bool = True, proc_grouping=DEFAULT_PROC_GROUPING,
                     qubit_grouping=DEFAULT_QUBIT_GROUPING) -> CompiledProgram:
    """Gate-level straight-line circuit -> CompiledProgram: ResolveGates ->
    ResolveVirtualZ -> ResolveFreqs -> Schedule (or LintSchedule when the
    user gave every ``start_time``, ``compiler.py:168-172``) -> compile."""
    instrs = resolve_freqs(resolve_virtual_z(resolve_gates(program, table, qubit_grouping)), table)
    prog = ScheduleIR({'block_0': instrs})
    (Schedule if schedule else LintSchedule)(fpga_config, proc_grouping).run_pass(prog)
    out = CompiledProgram(compile_blocks(prog, proc_grouping), fpga_config)
    out.ir = prog
    return out


# ---------------------------------------------------------------- control flow
# circuit statements that are already IR instructions (ir/instructions.py)
_IR_STATEMENTS = ('sync', 'declare', 'bind_phase', 'set_var', 'alu', 'read_fproc', 'alu_fproc', 'hold', 'idle', 'jump_label',
                  'jump_i', 'jump_cond', 'jump_fproc')

def flatten(program: Sequence, label_prefix: str = '') -> List[Instr]:
    """``ir/passes.py:62-124``: ``branch_fproc`` / ``branch_var`` / ``loop``
    -> jumps and labels (false block inline, true block after it; an empty
    true block jumps straight to the end label).  Gates become ``gate``
    instructions for ``resolve_gates``."""
    out: List[Instr] = []
    branchind = 0
    for st in program:
        st = copy.deepcopy(st)
        name = st['name'] if isinstance(st, dict) else st.name
        if name in ('branch_fproc', 'branch_var'):
            true_b = flatten(st['true'], 'true_' + label_prefix)
            false_b = flatten(st['false'], 'false_' + label_prefix)
            lbl_false = '{}false_{}'.format(label_prefix, branchind)
            lbl_end = '{}end_{}'.format(label_prefix, branchind)
            lbl_true = '{}true_{}'.format(label_prefix, branchind) if true_b else lbl_end
            if name == 'branch_fproc':
                out.append(Instr('jump_fproc', alu_cond=st['alu_cond'], cond_lhs=st['cond_lhs'],
                                 func_id=st['func_id'], scope=st['scope'], jump_label=lbl_true))
            else:
                out.append(Instr('jump_cond', alu_cond=st['alu_cond'], cond_lhs=st['cond_lhs'],
                                 cond_rhs=st['cond_rhs'], scope=st['scope'], jump_label=lbl_true))
            out.append(Instr('jump_label', label=lbl_false, scope=st['scope']))
            out += false_b
            out.append(Instr('jump_i', jump_label=lbl_end, scope=st['scope']))
            if true_b:
                out.append(Instr('jump_label', label=lbl_true, scope=st['scope']))
                out += true_b
            out.append(Instr('jump_label', label=lbl_end, scope=st['scope']))
            branchind += 1
        elif name == 'loop':
            body = flatten(st['body'], 'loop_body_' + label_prefix)
            lbl = '{}loop_{}_loopctrl'.format(label_prefix, branchind)
            out.append(Instr('jump_label', label=lbl, scope=st['scope']))
            out.append(Instr('barrier', qubit=st['scope']))
            out += body
            out.append(Instr('loop_end', loop_label=lbl, scope=st['scope']))
            out.append(Instr('jump_cond', cond_lhs=st['cond_lhs'], cond_rhs=st['cond_rhs'],
                             alu_cond=st['alu_cond'], jump_label=lbl, scope=st['scope'], jump_type='loopctrl'))
            branchind += 1
        elif isinstance(st, Instr):
            out.append(st)
        elif name in _IR_STATEMENTS:
            out.append(instr(st))
        elif name == 'pulse':
            d = dict(st)
            d['phase'] = _num(d['phase'])
            out.append(instr(d))
        elif name in ('virtual_z', 'virtualz', 'barrier', 'delay'):
            d = dict(st)
            if name in ('virtual_z', 'virtualz'):
                q = d['qubit'][0] if isinstance(d['qubit'], (list, tuple)) else d['qubit']
                out.append(Instr('virtual_z', freq=d.get('freq', '{}.freq'.format(q)), phase=_num(d['phase']),
                                 qubit=d['qubit']))
            else:
                out.append(Instr(name, scope=d.get('scope'), qubit=d.get('qubit'),
                                 **({'t': d['t']} if name == 'delay' else {})))
        else:
            out.append(Instr('gate', gate=name, qubit=st['qubit']))
    return out


def make_basic_blocks(flat: Sequence[Instr]) -> 'OrderedDict[str, List[Instr]]':
    """``ir/passes.py:135-178``: split at jumps (each jump is its own
    ``<block>_ctrl`` / ``<loop label>_ctrl`` block) and labels (a label starts
    a block named after it).  Blocks come back in the reference's source
    order (``blocknames_by_ind``: by ``ind``, ties in first-insertion order);
    empty blocks are dropped."""
    nodes: 'OrderedDict[str, list]' = OrderedDict([('block_0', [None, 0])])

    def add(name, instrs, ind):
        if name in nodes:
            nodes[name][0], nodes[name][1] = instrs, ind
        else:
            nodes[name] = [instrs, ind]

    cur_name, cur, blockname_ind, block_ind = 'block_0', [], 1, 0
    for st in flat:
        if st.name in ('jump_fproc', 'jump_cond', 'jump_i'):
            add(cur_name, cur, block_ind)
            block_ind += 1
            if st.jump_label.split('_')[-1] == 'loopctrl':
                ctrl = '{}_ctrl'.format(st.jump_label)
            else:
                ctrl = '{}_ctrl'.format(cur_name)
            add(ctrl, [st], block_ind)
            block_ind += 1
            cur_name, cur = 'block_{}'.format(blockname_ind), []
            blockname_ind += 1
        elif st.name == 'jump_label':
            add(cur_name, cur, block_ind)
            cur, cur_name = [st], st.label
        elif st.name in ('branch_fproc', 'branch_var', 'loop'):
            raise Exception('{}: must flatten all control flow before forming blocks'.format(st))
        else:
            cur.append(st)
    add(cur_name, cur, block_ind)
    order = sorted((n for n in nodes if nodes[n][0]), key=lambda n: nodes[n][1])
    return OrderedDict((n, nodes[n][0]) for n in order)


def scope_blocks(blocks, qubit_grouping=DEFAULT_QUBIT_GROUPING) -> Dict[str, set]:
    """``ir/passes.py:207-234`` (ScopeProgram): instruction scopes (qubits ->
    channels), block scopes, and unscoped barrier / delay / idle (and sync, an
    addition) -> the whole program's scope."""
    scoper = QubitScoper(qubit_grouping)
    scopes = {}
    for name, instrs in blocks.items():
        scope = set()
        for ins in instrs:
            if ins.scope is not None:
                ins.scope = scoper.get_scope(ins.scope)
                scope |= ins.scope
            elif ins.qubit is not None:
                ins.scope = scoper.get_scope(ins.qubit)
                scope |= ins.scope
            elif ins.dest is not None:
                scope |= scoper.get_scope(ins.dest)
        scopes[name] = scope
    everything = set().union(*scopes.values()) if scopes else set()
    for instrs in blocks.values():
        for ins in instrs:
            if ins.name in ('barrier', 'delay', 'idle', 'sync') and ins.scope is None:
                ins.scope = set(everything)
    return scopes


def generate_cfg(blocks, scopes) -> List[Tuple[str, str]]:
    """``ir/passes.py:368-388``: per channel, an edge from the last block
    that touched it; conditional jumps add an edge to their target (loop
    control jumps do not, keeping the graph a DAG); ``jump_i`` adds its target
    and ends the fall-through."""
    edges: List[Tuple[str, str]] = []

    def edge(a, b):
        if (a, b) not in edges:
            edges.append((a, b))

    last = {d: None for d in set().union(*scopes.values())} if scopes else {}
    for name, instrs in blocks.items():
        for d in scopes[name]:
            if last[d] is not None:
                edge(last[d], name)
        tail = instrs[-1]
        if tail.name in ('jump_fproc', 'jump_cond'):
            if tail.jump_type != 'loopctrl':
                edge(name, tail.jump_label)
            for d in scopes[name]:
                last[d] = name
        elif tail.name == 'jump_i':
            edge(name, tail.jump_label)
            for d in scopes[name]:
                last[d] = None
        else:
            for d in scopes[name]:
                last[d] = name
    return edges


def resolve_virtual_z_cfg(prog: ScheduleIR):
    """``ir/passes.py:439-491``: virtual-z phases accumulate along the CFG;
    predecessors must agree on every frequency's phase."""
    for node in prog.topological_order():
        acc: Dict[object, float] = {}
        for pred in prog.predecessors(node):
            for f, ph in prog.blocks[pred]['ending_zphases'].items():
                if f in acc and acc[f] != ph:
                    raise ValueError('Phase mismatch in {} at {} predecessor {} ({} rad)'.format(f, node, pred, ph))
                acc[f] = ph
        block = prog.blocks[node]
        kept = []
        for ins in block['instructions']:
            if ins.name == 'pulse':
                if ins.freq in acc:
                    ins.phase += acc[ins.freq]
                kept.append(ins)
            elif ins.name == 'virtual_z':
                acc[ins.freq] = acc.get(ins.freq, 0) + ins.phase
            else:
                kept.append(ins)
        block['instructions'] = kept
        block['ending_zphases'] = acc


def register_vars(blocks) -> Dict[str, dict]:
    """``ir/passes.py:253-283`` (the variable half of RegisterVarsAndFreqs):
    declared variables with their scope, and register instructions scoped by
    the variables they touch"""
    vars_: Dict[str, dict] = {}
    for instrs in blocks.values():
        for ins in instrs:
            if ins.name == 'declare':
                if ins.scope is None:
                    ins.scope = set()
                # the variable shares the declare's scope set, as register_var does (ir.py)
                vars_[ins.var] = {'scope': ins.scope, 'dtype': ins.dtype}
            elif ins.name == 'alu':
                ins.scope = vars_[ins.rhs]['scope'] | (vars_[ins.lhs]['scope'] if isinstance(ins.lhs, str) else set())
                if not vars_[ins.out]['scope'] <= ins.scope:
                    raise AssertionError('alu output {} is scoped wider than its inputs'.format(ins.out))
            elif ins.name in ('set_var', 'read_fproc'):
                ins.scope = vars_[ins.var]['scope']
            elif ins.name == 'alu_fproc' and isinstance(ins.lhs, str):
                ins.scope = set(vars_[ins.rhs]['scope'])
    return vars_


def resolve_hw_virtual_z(prog: ScheduleIR, vars_: Dict[str, dict]):
    """``ir/passes.py:405-437``: ``bind_phase`` binds a frequency's phase to
    a register (initialised by a set_var 0); virtual z on a bound frequency
    becomes an ``alu add`` on that register, and pulses on it take the
    register as their phase."""
    bound: Dict[object, str] = {}
    for node in prog.topological_order():
        il = prog.blocks[node]['instructions']
        for i, ins in enumerate(il):
            if ins.name == 'bind_phase':
                bound[ins.freq] = ins.var
                il[i] = Instr('set_var', value=0, var=ins.var, scope=set(vars_[ins.var]['scope']))
            elif ins.name == 'virtual_z' and ins.freq in bound:
                var = bound[ins.freq]
                if ins.scope is not None and not set(ins.scope) <= vars_[var]['scope']:
                    raise AssertionError('virtual z on {} outside the scope of {}'.format(ins.freq, var))
                il[i] = Instr('alu', op='add', lhs=ins.phase, rhs=var, out=var, scope=set(vars_[var]['scope']))
            elif ins.name == 'pulse' and ins.freq in bound:
                ins.phase = bound[ins.freq]
            elif ins.name == 'gate':
                raise Exception('All Gate instructions must be resolved before running this pass!')


def rescope_vars(prog: ScheduleIR, vars_: Dict[str, dict]):
    """``ir/passes.py:563-593`` (RescopeVars): a variable used as a pulse
    phase on a channel outside its scope, or in a conditional jump scoped
    wider than it, widens its scope; the declare / set_var / alu
    instructions of that block are rescoped to the variable's scope."""
    for node in prog.topological_order():
        il = prog.blocks[node]['instructions']
        rescope = False
        for ins in il:
            if ins.name == 'pulse':
                if isinstance(ins.phase, str) and ins.phase in vars_ and ins.dest not in vars_[ins.phase]['scope']:
                    rescope = True
                    vars_[ins.phase]['scope'].add(ins.dest)
            elif ins.name in ('jump_cond', 'jump_fproc'):
                sides = [ins.cond_lhs] + ([ins.cond_rhs] if ins.name == 'jump_cond' else [])
                for v in sides:
                    if isinstance(v, str) and v in vars_ and not set(ins.scope) <= vars_[v]['scope']:
                        vars_[v]['scope'] = vars_[v]['scope'] | set(ins.scope)
                        rescope = True
        if rescope:
            for ins in il:
                if ins.name in ('declare', 'set_var'):
                    ins.scope = vars_[ins.var]['scope']
                elif ins.name in ('alu', 'rc_alu'):
                    ins.scope = vars_[ins.out]['scope']


def resolve_fproc_channels(prog: ScheduleIR, fpga_config: FPGAConfig):
    """``ir/passes.py:532-552``: a named fproc channel (``'Q0.meas'``) puts a
    ``hold`` (``hold_nclks`` after its ``hold_after_chans``) before the
    instruction that reads it, and lowers ``func_id`` to the channel id."""
    for node in prog.topological_order():
        il = prog.blocks[node]['instructions']
        i = 0
        while i < len(il):
            ins = il[i]
            if ins.name in ('read_fproc', 'jump_fproc', 'alu_fproc'):
                if ins.func_id in fpga_config.fproc_channels:
                    ch = fpga_config.fproc_channels[ins.func_id]
                    il.insert(i, Instr('hold', nclks=ch.hold_nclks, ref_chans=list(ch.hold_after_chans),
                                       scope=set(ins.scope)))
                    i += 1
                    ins.func_id = ch.id
                elif not isinstance(ins.func_id, int):
                    raise AssertionError('func_id {!r} is neither a named fproc channel nor an int'
                                         .format(ins.func_id))
            i += 1


def compile_circuit(program: Sequence, table: GateTable, fpga_config: FPGAConfig, schedule: bool = True,
                    proc_grouping=DEFAULT_PROC_GROUPING,
                    qubit_grouping=DEFAULT_QUBIT_GROUPING) -> CompiledProgram:
    """QubiC circuit with control flow (``branch_fproc`` / ``branch_var`` /
    ``loop``) -> CompiledProgram, in
    the reference's pass order (``compiler.py:149-174``): FlattenProgram,
    MakeBasicBlocks, ScopeProgram, ResolveGates, GenerateCFG, ResolveVirtualZ,
    ResolveHWVirtualZ, ResolveFreqs, ResolveFPROCChannels, RescopeVars,
    Schedule (or LintSchedule), compile."""
    blocks = make_basic_blocks(flatten(program))
    scopes = scope_blocks(blocks, qubit_grouping)
    vars_ = register_vars(blocks)
    edges = generate_cfg(blocks, scopes)
    prog = ScheduleIR(OrderedDict((n, resolve_gates(il, table, qubit_grouping)) for n, il in blocks.items()),
                      edges)
    for n, s in scopes.items():
        prog.blocks[n]['scope'] = s
    prog.scope = set().union(*scopes.values()) if scopes else set()
    resolve_hw_virtual_z(prog, vars_)
    resolve_virtual_z_cfg(prog)
    for b in prog.blocks.values():
        resolve_freqs(b['instructions'], table)
    resolve_fproc_channels(prog, fpga_config)
    rescope_vars(prog, vars_)
    (Schedule if schedule else LintSchedule)(fpga_config, proc_grouping).run_pass(prog)
    out = CompiledProgram(compile_blocks(prog, proc_grouping), fpga_config)
    out.ir = prog
    return out
