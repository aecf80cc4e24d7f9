"""Scheduling restatement (distributed_processor_amd.schedule) vs the reference.

Pinned by:
* the scheduling asserts of the reference's ``test_compiler.py:75-98``
  (``test_basic_schedule``) and its user-schedule lint verdicts (``:561-606``);
* the compiler goldens ``test_linear_compile_out`` / ``test_pulse_compile_out``
  (``test_compiler.py:100-122, 330-352``): gate-level program -> schedule ->
  compile reproduces the golden pulse statements, and -> assemble reproduces
  the reference GlobalAssembler's bytes (``tests/golden/asm_programs.json``);
* a property: every straight-line schedule, assembled to machine code, runs
  without a late pulse on the RTL latencies -- checked by the machine-code
  linter, by ``oracle_fast`` and (``-m gpu``) by the emulator on cuda:0.
The gate table is the Q0/Q1 part of the reference's ``qubitcfg.json``
(``tests/golden/qchip_q01.json``, made by ``make_qchip_subset.py``).
Control-flow cases (branch merge, loop ``delta_t``, hold -> idle) are
hand-computed from ``ir/passes.py:616-735``: parity unpinned by a reference
output, as the reference compiler is not importable here.
"""

import json
import math
import os
import warnings

import numpy as np
import pytest

from distributed_processor_amd import _abi, hwconfig as hw, isa, lint
from distributed_processor_amd import assembler as am
from distributed_processor_amd import schedule as sc

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')
with open(os.path.join(GOLDEN, 'qchip_q01.json')) as f:
    TABLE = sc.GateTable(json.load(f))
# the fpga_config of test_compiler.py:77-81 (pulse_load_clks default 3)
TEST_FPGA = hw.FPGAConfig(alu_instr_clks=2, fpga_clk_period=2.e-9, jump_cond_clks=3, jump_fproc_clks=4,
                          pulse_regwrite_clks=1)


def golden_inputs(name):
    from tests.test_assembler import program
    return program(name)


def pulse_times(prog):
    return [i.start_time for i in prog.blocks['block_0']['instructions'] if i.name == 'pulse']


def scheduled_block(program, cfg=TEST_FPGA):
    instrs = sc.resolve_freqs(sc.resolve_virtual_z(sc.resolve_gates(program, TABLE)), TABLE)
    prog = sc.ScheduleIR({'block_0': instrs})
    sc.Schedule(cfg).run_pass(prog)
    return prog


def test_basic_schedule():
    """test_compiler.py:75-98"""
    program = [{'name': 'X90', 'qubit': ['Q0']}, {'name': 'X90', 'qubit': ['Q1']},
               {'name': 'X90Z90', 'qubit': ['Q0']}, {'name': 'X90', 'qubit': ['Q0']},
               {'name': 'X90', 'qubit': ['Q1']}, {'name': 'read', 'qubit': ['Q0']}]
    assert pulse_times(scheduled_block(program))[:6] == [5, 5, 21, 37, 13, 53]


def env_equal(a, b):
    if isinstance(a, np.ndarray) or isinstance(b, np.ndarray):
        return np.array_equal(np.asarray(a), np.asarray(b))
    return a == b


PULSE_PROGRAM = [{'name': 'X90', 'qubit': ['Q0']}, {'name': 'X90', 'qubit': ['Q1']},
                 {'name': 'X90Z90', 'qubit': ['Q0']}, {'name': 'X90', 'qubit': ['Q0']},
                 {'name': 'X90', 'qubit': ['Q1']},
                 {'name': 'pulse', 'phase': np.pi / 2, 'freq': 'Q0.freq', 'env': np.ones(100),
                  'twidth': 24.e-9, 'amp': 0.5, 'dest': 'Q0.qdrv'},
                 {'name': 'read', 'qubit': ['Q0']}]
LINEAR_PROGRAM = [{'name': 'X90', 'qubit': ['Q0']}, {'name': 'X90', 'qubit': ['Q1']},
                  {'name': 'read', 'qubit': ['Q0']}]

def two_resets(func0, func1):
    return [{'name': 'X90', 'qubit': ['Q0']},
            {'name': 'branch_fproc', 'alu_cond': 'eq', 'cond_lhs': 1, 'func_id': func0,
             'true': [], 'false': [{'name': 'X90', 'qubit': ['Q0']}], 'scope': ['Q0']},
            {'name': 'branch_fproc', 'alu_cond': 'eq', 'cond_lhs': 1, 'func_id': func1,
             'true': [], 'false': [{'name': 'X90', 'qubit': ['Q1']}], 'scope': ['Q1']},
            {'name': 'X90', 'qubit': ['Q1']}]


# golden name -> (program, fpga_config, compile function); programs from
# test_compiler.py:330-352 (linear), :100-122 (pulse), :224-255 (multirst_cfg),
# :257-291 (multirst_fproc_res_cfg), :293-330 (fproc_hold)
GOLDEN_CASES = {
    'test_linear_compile_out': (LINEAR_PROGRAM, TEST_FPGA, sc.compile_straight),
    'test_pulse_compile_out': (PULSE_PROGRAM, TEST_FPGA, sc.compile_straight),
    'test_multirst_cfg': (two_resets(1, 0), TEST_FPGA, sc.compile_circuit),
    'test_multirst_fproc_res_cfg': (two_resets('Q0.meas', 'Q1.meas'), hw.FPGAConfig(), sc.compile_circuit),
    'test_fproc_hold': ([{'name': 'X90', 'qubit': ['Q0']}, {'name': 'read', 'qubit': ['Q0']},
                         {'name': 'X90', 'qubit': ['Q0']}, {'name': 'read', 'qubit': ['Q1']}]
                        + two_resets('Q0.meas', 'Q1.meas')[1:], hw.FPGAConfig(), sc.compile_circuit),
}


LOOP_FPGA = hw.FPGAConfig(alu_instr_clks=2, fpga_clk_period=2.e-9, jump_cond_clks=3, jump_fproc_clks=4,
                          pulse_load_clks=4, pulse_regwrite_clks=1)       # test_compiler.py:418-423
PREAMBLE = [{'name': 'X90', 'qubit': ['Q0']}, {'name': 'read', 'qubit': ['Q0']}, {'name': 'X90', 'qubit': ['Q1']}]
X90X90_Q0 = [{'name': 'X90', 'qubit': ['Q0']}, {'name': 'X90', 'qubit': ['Q0']}]


def loop(var, body, scope):
    return {'name': 'loop', 'cond_lhs': 10, 'cond_rhs': var, 'alu_cond': 'ge', 'scope': scope, 'body': body}


def declare(var):
    return {'name': 'declare', 'var': var, 'dtype': 'int', 'scope': ['Q0']}


TAIL = [{'name': 'CR', 'qubit': ['Q1', 'Q0']}, {'name': 'X90', 'qubit': ['Q1']}]
# test_compiler.py:376-414 (simple), :416-455 (compound), :457-516 (nested)
GOLDEN_CASES['test_simple_loop'] = (
    PREAMBLE + [{'name': 'Z90', 'qubit': ['Q0']}, {'name': 'X90', 'qubit': ['Q0']}, declare('loopind'),
                loop('loopind', X90X90_Q0, ['Q0']), {'name': 'read', 'qubit': ['Q0']},
                {'name': 'X90', 'qubit': ['Q1']}], TEST_FPGA, sc.compile_circuit)
GOLDEN_CASES['test_compound_loop'] = (
    PREAMBLE + [declare('loopind'), loop('loopind', X90X90_Q0, ['Q0', 'Q1'])] + TAIL, LOOP_FPGA,
    sc.compile_circuit)
GOLDEN_CASES['test_nested_loop'] = (
    PREAMBLE + [declare('loopind'), declare('loopind2'),
                loop('loopind', X90X90_Q0 + [loop('loopind2', [{'name': 'X90', 'qubit': ['Q1']},
                                                              {'name': 'read', 'qubit': ['Q0']}],
                                                   ['Q0', 'Q1'])], ['Q0', 'Q1'])] + TAIL, LOOP_FPGA,
    sc.compile_circuit)

# test_compiler.py:518-559: a phase register bound to Q0.freq (hardware virtual z)
GOLDEN_CASES['test_hw_virtualz_out'] = (
    [{'name': 'declare', 'var': 'q0_phase', 'scope': ['Q0'], 'dtype': 'phase'},
     {'name': 'bind_phase', 'var': 'q0_phase', 'freq': 'Q0.freq'},
     {'name': 'X90', 'qubit': ['Q0']}, {'name': 'X90', 'qubit': ['Q1']},
     {'name': 'virtual_z', 'qubit': 'Q0', 'phase': np.pi / 2},
     {'name': 'X90', 'qubit': ['Q0']}, {'name': 'read', 'qubit': ['Q0']}], TEST_FPGA, sc.compile_circuit)


def test_every_compiler_golden_covered():
    with open(os.path.join(GOLDEN, 'asm_inputs.json')) as f:
        assert sorted(json.load(f)['programs']) == sorted(GOLDEN_CASES)


def compile_case(name):
    prog, cfg, fn = GOLDEN_CASES[name]
    return fn(prog, TABLE, cfg)


@pytest.mark.parametrize('name', sorted(GOLDEN_CASES))
def test_compile_matches_golden_statements(name):
    """the compiled per-core statements equal the golden's, field by field"""
    got = compile_case(name).program
    want = golden_inputs(name)
    assert sorted(got) == sorted(want)
    for grp, stmts in want.items():
        g = got[grp]
        assert [s['op'] for s in g] == [s['op'] for s in stmts], grp
        for a, b in zip(g, stmts):
            assert sorted(a) == sorted(b), (a, b)
            for k in b:
                if k == 'env':
                    assert env_equal(a[k], b[k]), (grp, k)
                elif isinstance(b[k], float):
                    assert math.isclose(a[k], b[k], rel_tol=0, abs_tol=1e-12), (grp, k, a[k], b[k])
                else:
                    assert a[k] == b[k], (grp, k, a[k], b[k])


def test_straight_and_circuit_front_ends_agree():
    """compile_circuit on a branch-free program = compile_straight"""
    for prog in (LINEAR_PROGRAM, PULSE_PROGRAM):
        a = sc.compile_straight(prog, TABLE, TEST_FPGA).program
        b = sc.compile_circuit(prog, TABLE, TEST_FPGA).program
        assert sorted(a) == sorted(b)
        for g in a:
            assert [(s['op'], s.get('start_time')) for s in a[g]] == [(s['op'], s.get('start_time')) for s in b[g]]


def test_fproc_res_lints_clean():
    """test_compiler.py:270-272: LintSchedule accepts the scheduled program"""
    blocks = sc.make_basic_blocks(sc.flatten(two_resets('Q0.meas', 'Q1.meas')))
    assert list(blocks) == ['block_0', 'block_0_ctrl', 'false_0', 'false_0_ctrl', 'end_0', 'end_0_ctrl',
                            'false_1', 'false_1_ctrl', 'end_1']
    compiled = sc.compile_circuit(two_resets('Q0.meas', 'Q1.meas'), TABLE, hw.FPGAConfig())
    sc.LintSchedule(hw.FPGAConfig()).run_pass(compiled.ir)
    with pytest.raises(Exception, match='too early'):      # the RTL needs more than 1 clk per jump
        sc.LintSchedule(hw.FPGAConfig(jump_fproc_clks=30)).run_pass(compiled.ir)


def assemble(compiled):
    chans = hw.load_channel_configs(os.path.join(GOLDEN, 'channel_config.json'))
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        return am.GlobalAssembler(compiled, chans, hw.DDSElementConfig).get_assembled_program()


@pytest.mark.parametrize('func_ids', [(1, 0), ('Q0.meas', 'Q1.meas')])
def test_branch_schedules_vs_rtl_latencies(func_ids):
    """a schedule made with jump_fproc_clks = 4 (test_compiler.py's
    fpga_config) puts a pulse behind a jump_fproc earlier than the RTL can
    decode it (8 clks): oracle_fast flags DPEMU_F_LATE and the machine-code
    linter says ``late``.  With the reference's default FPGAConfig and with
    the RTL's exact latencies no lane is late."""
    from tests.test_lint import oracle_flags
    exact = hw.FPGAConfig.rtl_exact()
    assert (exact.jump_cond_clks, exact.jump_fproc_clks, exact.alu_instr_clks) == (6, 8, 4)
    for cfg, want_late in ((TEST_FPGA, True), (hw.FPGAConfig(), False), (exact, False)):
        asm = assemble(sc.compile_circuit(two_resets(*func_ids), TABLE, cfg))
        late = []
        for core in sorted(asm):
            words = isa.bytes_to_words(asm[core]['cmd_buf'])
            flag = bool(oracle_flags([words])[0] & _abi.F_LATE)
            assert flag == lint.lint_program(words).late, (cfg.jump_fproc_clks, core)
            late.append(flag)
        assert any(late) == want_late, (cfg.jump_fproc_clks, late)


@pytest.mark.parametrize('name', sorted(GOLDEN_CASES))
def test_schedule_compile_assemble_bytes(name):
    """gate program -> schedule -> compile -> assemble is byte-identical to the
    reference GlobalAssembler on the golden (DDSElementConfig)"""
    with open(os.path.join(GOLDEN, 'asm_programs.json')) as f:
        exp = json.load(f)['programs'][name]
    compiled = compile_case(name)
    chans = hw.load_channel_configs(os.path.join(GOLDEN, 'channel_config.json'))
    if 'reference_error' in exp:          # the reference GlobalAssembler raised on it (AssertionError)
        with pytest.raises(Exception), warnings.catch_warnings():
            warnings.simplefilter('ignore')
            am.GlobalAssembler(compiled, chans, hw.DDSElementConfig).get_assembled_program()
        return
    exp = exp['dds_elem']
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        got = am.GlobalAssembler(compiled, chans, hw.DDSElementConfig).get_assembled_program()
    assert sorted(got) == sorted(exp)
    for core, want in exp.items():
        assert got[core]['cmd_buf'].hex() == want['cmd_buf'], core
        assert [b.hex() for b in got[core]['env_buffers']] == want['env_buffers'], core
        assert [b.hex() for b in got[core]['freq_buffers']] == want['freq_buffers'], core


def user_pulses(times):
    dests = ['Q0.qdrv', 'Q0.rdrv', 'Q0.qdrv', 'Q1.qdrv']
    freqs = ['Q0.freq', 'Q0.freq', 'Q0.freq', 1234234]
    return [{'name': 'pulse', 'phase': 'np.pi/2', 'freq': f, 'env': np.ones(100), 'twidth': 24.e-9,
             'amp': 0.5, 'dest': d, 'start_time': t} for d, f, t in zip(dests, freqs, times)]


def test_user_schedule_lint():
    """test_compiler.py:561-606: schedule=False runs LintSchedule instead"""
    prog = sc.compile_straight(user_pulses([5, 8, 11, 5]), TABLE, TEST_FPGA, schedule=False).program
    q0 = prog[('Q0.qdrv', 'Q0.rdrv', 'Q0.rdlo')]
    assert [s['start_time'] for s in q0 if s['op'] == 'pulse'] == [5, 8, 11]
    with pytest.raises(Exception, match='start time too early'):
        sc.compile_straight(user_pulses([5, 6, 11, 5]), TABLE, TEST_FPGA, schedule=False)


def test_hold_becomes_idle():
    """passes.py:709-724: hold(64 after rdlo) -> idle at rdlo end + 64; the next
    gate's barrier waits for idle end + pulse_load_clks"""
    cfg = hw.FPGAConfig()
    instrs = sc.resolve_gates([{'name': 'read', 'qubit': ['Q0']}], TABLE)
    instrs.append(sc.Instr('hold', nclks=64, ref_chans=['Q0.rdlo'],
                           scope={'Q0.qdrv', 'Q0.rdrv', 'Q0.rdlo'}))
    instrs += sc.resolve_gates([{'name': 'X90', 'qubit': ['Q0']}], TABLE)
    prog = sc.ScheduleIR({'block_0': sc.resolve_freqs(instrs, TABLE)})
    sc.Schedule(cfg).run_pass(prog)
    il = prog.blocks['block_0']['instructions']
    assert [i.name for i in il] == ['pulse', 'pulse', 'idle', 'pulse']
    assert [il[0].start_time, il[1].start_time] == [5, 305]
    assert il[2].end_time == 305 + 1000 + 64
    assert il[3].start_time == 305 + 1000 + 64 + 3
    # a hold whose target already passed is dropped (passes.py:714, >=)
    instrs = [sc.Instr('pulse', dest='Q0.qdrv', twidth=2e-9, freq=1e9, phase=0, amp=1, env=None),
              sc.Instr('hold', nclks=0, ref_chans=['Q0.qdrv'], scope={'Q0.qdrv'})]
    prog = sc.ScheduleIR({'block_0': instrs})
    sc.Schedule(cfg).run_pass(prog)
    assert [i.name for i in prog.blocks['block_0']['instructions']] == ['pulse']


def P(dest, tw, **kw):
    return sc.Instr('pulse', dest=dest, twidth=tw * 2e-9, freq=1e9, phase=0.0, amp=1.0, env=None, **kw)


def test_branch_merge_and_loop():
    """passes.py:616-653 on a hand-built CFG: a merge block starts after the
    later predecessor; a *_loopctrl block registers the loop start, its
    loopctrl jump_cond sets delta_t and resets the end time to the loop start"""
    cfg = hw.FPGAConfig()
    Q0 = {'Q0.qdrv', 'Q0.rdrv', 'Q0.rdlo'}
    blocks = {
        'block_0': [P('Q0.qdrv', 10), sc.Instr('jump_fproc', scope=Q0, cond_lhs=1, alu_cond='eq',
                                                 jump_label='true_0', func_id=0)],
        'false_0': [P('Q0.qdrv', 20), sc.Instr('jump_i', scope=Q0, jump_label='end_0')],
        'true_0': [P('Q0.qdrv', 4)],
        'end_0': [sc.Instr('barrier', scope=Q0), P('Q0.rdrv', 7)],
        'body_loopctrl': [P('Q0.qdrv', 6), sc.Instr('alu', scope=Q0),
                          sc.Instr('jump_cond', scope=Q0, jump_type='loopctrl', jump_label='body_loopctrl')],
        'post_0': [P('Q0.qdrv', 1)],
    }
    edges = [('block_0', 'false_0'), ('block_0', 'true_0'), ('false_0', 'end_0'), ('true_0', 'end_0'),
             ('end_0', 'body_loopctrl'), ('body_loopctrl', 'post_0')]
    prog = sc.ScheduleIR(blocks, edges)
    sc.Schedule(cfg).run_pass(prog)
    t = {n: [i.start_time for i in b['instructions'] if i.name == 'pulse'] for n, b in prog.blocks.items()}
    # block_0: pulse @5 (qdrv busy to 15); jump_fproc: last_end 8 + 8 = 16
    assert t['block_0'] == [5]
    assert t['false_0'] == [16] and t['true_0'] == [16]
    # false_0 ends: qdrv 36, last_end 19 + 5 = 24; true_0: qdrv 20, last_end 19
    assert t['end_0'] == [36]                   # barrier: max over Q0 channel times of both branches
    loop = prog.loops['body_loopctrl']
    assert loop['start_time'] == 36 + 7         # rdrv busy until 43
    assert t['body_loopctrl'] == [39]           # qdrv free at 36, core at 36 + 3
    # body: qdrv to 45; last_end 42 + 5 (alu) + 5 (jump_cond) = 52 -> delta_t 52 - 43
    assert loop['delta_t'] == 9
    assert t['post_0'] == [43]                  # loopctrl block ends at the loop start
    # LintSchedule accepts its own output
    sc.LintSchedule(cfg).run_pass(prog)


def test_cfg_errors():
    with pytest.raises(ValueError, match='unknown block'):
        sc.ScheduleIR({'a': []}, [('a', 'b')])
    with pytest.raises(ValueError, match='cycle'):
        sc.ScheduleIR({'a': [P('Q0.qdrv', 1)], 'b': [P('Q0.qdrv', 1)]},
                      [('a', 'b'), ('b', 'a')]).topological_order()
    with pytest.raises(NotImplementedError):
        sc.resolve_gates([{'name': 'Y-90', 'qubit': ['Q1']}], TABLE)
    with pytest.raises(Exception, match='resolve gates'):
        sc.Schedule(hw.FPGAConfig()).run_pass(sc.ScheduleIR({'b': [sc.Instr('gate', scope=set())]}))


def test_core_scoper_patterns():
    s = sc.CoreScoper(['Q0.qdrv', 'Q12.rdlo', 'C0.x'], [('{qubit}.qdrv', '{qubit}.rdrv', '{qubit}.rdlo')])
    assert s.proc_groupings == {'Q0.qdrv': ('Q0.qdrv', 'Q0.rdrv', 'Q0.rdlo'),
                                'Q12.rdlo': ('Q12.qdrv', 'Q12.rdrv', 'Q12.rdlo')}
    assert sc._num('numpy.pi/2.0') == math.pi / 2 and sc._num('-np.pi*3') == -3 * math.pi
    with pytest.raises(ValueError):
        sc._num('__import__("os")')


GATES = {'Q0': ['X90', 'X90Z90', 'Z90', 'read', 'X90_ef', 'rabi'], 'Q1': ['X90', 'read', 'X90_ef', 'rabi']}


def random_program(rng, n):
    prog = []
    for _ in range(n):
        r = rng.random()
        q = ['Q0', 'Q1'][rng.integers(2)]
        if r < 0.1:
            prog.append({'name': 'delay', 't': float(rng.integers(1, 200)) * 2e-9, 'qubit': [q]})
        elif r < 0.15:
            prog.append({'name': 'barrier', 'qubit': ['Q0', 'Q1']})
        elif r < 0.3:
            prog.append({'name': 'pulse', 'phase': float(rng.random()), 'freq': q + '.freq',
                         'env': {'env_func': 'square', 'paradict': {'phase': 0.0, 'amplitude': 1.0}},
                         'twidth': float(rng.integers(1, 40)) * 2e-9, 'amp': 0.5,
                         'dest': q + ['.qdrv', '.rdrv'][rng.integers(2)]})
        else:
            prog.append({'name': GATES[q][rng.integers(len(GATES[q]))], 'qubit': [q]})
    return prog


def assembled_cases(n_cases=24, seed=7):
    rng = np.random.default_rng(seed)
    chans = hw.load_channel_configs(os.path.join(GOLDEN, 'channel_config.json'))
    for k in range(n_cases):
        cfg = hw.FPGAConfig() if k % 2 else TEST_FPGA
        compiled = sc.compile_straight(random_program(rng, int(rng.integers(3, 25))), TABLE, cfg)
        with warnings.catch_warnings():
            warnings.simplefilter('ignore')
            asm = am.GlobalAssembler(compiled, chans, hw.DDSElementConfig).get_assembled_program()
        yield k, compiled, asm


def pulse_counts(compiled, asm, chans):
    """pulse statements per assembled core key (the phase_reset adds one event)"""
    core_of = {str(chans[g[0]].core_ind): g for g in compiled.program}
    return [sum(st['op'] == 'pulse' for st in compiled.program[core_of[c]]) for c in sorted(asm)]


def test_schedules_are_never_late_cpu():
    """every pulse of a scheduled straight-line program is issued on time by
    the RTL: the exact linter verdict and oracle_fast agree (no DPEMU_F_LATE,
    every core done, one event per pulse plus the phase_reset)"""
    import oracle
    from tests.progfuzz import pack_programs
    from tests.test_lint import MAX_CYCLES
    chans = hw.load_channel_configs(os.path.join(GOLDEN, 'channel_config.json'))
    n = 0
    for k, compiled, asm in assembled_cases():
        progs = [isa.bytes_to_words(asm[c]['cmd_buf']) for c in sorted(asm)]
        for c, words in zip(sorted(asm), progs):
            rep = lint.lint_program(words)
            assert rep.exact and not rep.late, (k, c, [str(f) for f in rep.findings])
        C = len(progs)
        cfg = _abi.make_config(C, max_cycles=MAX_CYCLES, event_cap=64, trace_cap=16, meas_cap=16, seed=k)
        words, offs, ni = pack_programs(progs)
        f = oracle.fast_run(cfg, words, offs, ni, np.arange(C, dtype=np.uint32), 0, 1, want=('summary',))
        summ = _abi.unpack_summary(f['summary'])
        assert not (summ['flags'] & _abi.F_LATE).any(), k
        assert (summ['status'] == _abi.ST_DONE).all(), k
        assert summ['n_events'].tolist() == [p + 1 for p in pulse_counts(compiled, asm, chans)], k
        n += C
    assert n >= 24


@pytest.mark.gpu
def test_schedules_are_never_late_gpu():
    """the same property with the emulator on cuda:0 executing the programs"""
    from distributed_processor_amd.emulator import Emulator, ProgramSet
    from tests.test_lint import MAX_CYCLES
    chans = hw.load_channel_configs(os.path.join(GOLDEN, 'channel_config.json'))
    with Emulator(0) as emu:
        for k, compiled, asm in assembled_cases():
            progs = [isa.bytes_to_words(asm[c]['cmd_buf']) for c in sorted(asm)]
            C = len(progs)
            emu.load(ProgramSet([progs], cores_per_shot=C))
            cfg = _abi.make_config(C, max_cycles=MAX_CYCLES, event_cap=64, trace_cap=16, meas_cap=16, seed=k)
            s = emu.run(1, 0, cfg=cfg, outputs=('summary',)).arrays['summary']
            summ = _abi.unpack_summary(np.asarray(s).view(np.uint32))
            assert not (summ['flags'] & _abi.F_LATE).any(), k
            assert (summ['status'] == _abi.ST_DONE).all(), k
            assert summ['n_events'].tolist() == [p + 1 for p in pulse_counts(compiled, asm, chans)], k
        # branch programs: the GPU's F_LATE verdict per core = oracle_fast's
        from tests.test_lint import oracle_flags
        for cfg in (TEST_FPGA, hw.FPGAConfig()):
            for func_ids in ((1, 0), ('Q0.meas', 'Q1.meas')):
                asm = assemble(sc.compile_circuit(two_resets(*func_ids), TABLE, cfg))
                for core in sorted(asm):
                    words = isa.bytes_to_words(asm[core]['cmd_buf'])
                    emu.load(ProgramSet([[words]], cores_per_shot=1))
                    rc = _abi.make_config(1, max_cycles=MAX_CYCLES, event_cap=64, trace_cap=16, meas_cap=16,
                                          seed=0)
                    s = emu.run(1, 0, cfg=rc, outputs=('summary',)).arrays['summary']
                    flags = _abi.unpack_summary(np.asarray(s).view(np.uint32))['flags']
                    assert (flags & _abi.F_LATE).tolist() == (oracle_flags([words]) & _abi.F_LATE).tolist(), \
                        (cfg.jump_fproc_clks, func_ids, core)


def test_rescope_vars_widens_phase_register():
    """passes.py:563-593 (hand-derived): a phase register declared on Q0 but
    bound to Q1.freq is used by a Q1 pulse, so its declare / set_var are
    rescoped to Q1's core too and the pulse waits for the set_var there"""
    prog = [{'name': 'declare', 'var': 'q_phase', 'scope': ['Q0'], 'dtype': 'phase'},
            {'name': 'bind_phase', 'var': 'q_phase', 'freq': 'Q1.freq'},
            {'name': 'X90', 'qubit': ['Q1']}]
    got = sc.compile_circuit(prog, TABLE, TEST_FPGA).program
    q0, q1 = got[('Q0.qdrv', 'Q0.rdrv', 'Q0.rdlo')], got[('Q1.qdrv', 'Q1.rdrv', 'Q1.rdlo')]
    assert [s['op'] for s in q0] == ['phase_reset', 'declare_reg', 'reg_alu', 'done_stb']
    assert [s['op'] for s in q1] == ['phase_reset', 'declare_reg', 'reg_alu', 'pulse', 'done_stb']
    assert q1[3]['phase'] == 'q_phase' and q1[3]['start_time'] == 5 + TEST_FPGA.alu_instr_clks


def random_circuit(rng, decls, depth=0):
    """gates, fproc branches on the cores' own measurements and counted loops
    (a loop register incremented in the body, so every shot terminates).
    Declarations go to ``decls`` (the program head): as in the reference
    assembler, a jump label cannot land on a declare_reg."""
    prog = []
    for _ in range(int(rng.integers(2, 7))):
        q = ['Q0', 'Q1'][rng.integers(2)]
        r = rng.random()
        if r < 0.2 and depth < 2:
            prog.append({'name': 'read', 'qubit': [q]})
            prog.append({'name': 'branch_fproc', 'alu_cond': 'eq', 'cond_lhs': int(rng.integers(2)),
                         'func_id': q + '.meas', 'scope': [q],
                         'true': random_circuit(rng, decls, depth + 1) if rng.random() < 0.5 else [],
                         'false': [{'name': 'X90', 'qubit': [q]}]})
        elif r < 0.3 and depth < 2:
            var = 'i{}'.format(len(decls))
            decls.append({'name': 'declare', 'var': var, 'dtype': 'int', 'scope': ['Q0', 'Q1']})
            # scoped explicitly: the block's scope comes from ScopeProgram, which
            # runs before variables are registered (passes.py:207-223, 278-279)
            prog.append({'name': 'set_var', 'var': var, 'value': 0, 'scope': ['Q0', 'Q1']})
            body = [{'name': 'X90', 'qubit': [q]},
                    {'name': 'alu', 'op': 'add', 'lhs': 1, 'rhs': var, 'out': var}]
            prog.append({'name': 'loop', 'cond_lhs': int(rng.integers(1, 4)), 'cond_rhs': var, 'alu_cond': 'ge',
                         'scope': ['Q0', 'Q1'], 'body': body})
        else:
            gates = GATES[q] if depth == 0 else [g for g in GATES[q] if 'Z' not in g]
            prog.append({'name': gates[rng.integers(len(gates))], 'qubit': [q]})
    return prog


def test_conditional_virtual_z_is_rejected():
    """passes.py:459-467: branches that leave a frequency at different
    virtual-z phases cannot merge (software z needs one phase per point; a
    branch that never touched the frequency does not conflict)"""
    circ = [{'name': 'Z90', 'qubit': ['Q0']}, {'name': 'read', 'qubit': ['Q0']},
            {'name': 'branch_fproc', 'alu_cond': 'eq', 'cond_lhs': 1, 'func_id': 'Q0.meas', 'scope': ['Q0'],
             'true': [{'name': 'Z90', 'qubit': ['Q0']}], 'false': [{'name': 'X90', 'qubit': ['Q0']}]},
            {'name': 'X90', 'qubit': ['Q0']}]
    with pytest.raises(ValueError, match='Phase mismatch'):
        sc.compile_circuit(circ, TABLE, hw.FPGAConfig())


def compiled_circuits(n_cases=12, seed=11):
    rng = np.random.default_rng(seed)
    for k in range(n_cases):
        decls = []
        body = random_circuit(rng, decls)
        circ = decls + body + [{'name': 'read', 'qubit': ['Q0']}, {'name': 'read', 'qubit': ['Q1']}]
        yield k, circ, assemble(sc.compile_circuit(circ, TABLE, hw.FPGAConfig()))


def circuit_config(C, k):
    return _abi.make_config(C, max_cycles=1 << 20, event_cap=96, trace_cap=64, meas_cap=16, p1=0.5, seed=k)


def test_compiled_circuits_run_on_oracle():
    """circuit -> compile_circuit -> assemble -> oracle_fast: every lane of
    every shot finishes, with at least the two closing readouts measured"""
    import oracle
    from distributed_processor_amd.emulator import ProgramSet
    for k, circ, asm in compiled_circuits():
        ps = ProgramSet([asm])
        cfg = circuit_config(ps.cores_per_shot, k)
        f = oracle.fast_run(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, 0, 64, want=('summary',))
        s = _abi.unpack_summary(f['summary'])
        assert (s['status'] == _abi.ST_DONE).all(), (k, circ)
        assert (s['n_meas'] >= 1).all(), k


@pytest.mark.gpu
def test_compiled_circuits_gpu_vs_oracle():
    """the same compiled circuits (branches on measurements, counted loops) on
    cuda:0, bit-exact against oracle_fast on every output"""
    from distributed_processor_amd.emulator import Emulator, ProgramSet
    from tests.test_gpu_parity import compare_all, run_pair
    with Emulator(0) as emu:
        for k, circ, asm in compiled_circuits():
            ps = ProgramSet([asm])
            g, f = run_pair(emu, ps, circuit_config(ps.cores_per_shot, k), 2000, shot0=97 * k)
            compare_all(g, f, 'circuit {}'.format(k))
            assert (_abi.unpack_summary(g['summary'])['status'] == _abi.ST_DONE).all(), k


def sync_circuits(n_cases=10, seed=23):
    """random circuits cut into segments by whole-circuit syncs, scheduled with
    the RTL's latencies"""
    rng = np.random.default_rng(seed)
    for k in range(n_cases):
        decls, body = [], []
        for j in range(int(rng.integers(2, 4))):
            body += random_circuit(rng, decls)
            body.append({'name': 'sync', 'scope': ['Q0', 'Q1'], 'barrier_id': j})
        circ = decls + body + [{'name': 'read', 'qubit': ['Q0']}, {'name': 'read', 'qubit': ['Q1']}]
        yield k, circ, assemble(sc.compile_circuit(circ, TABLE, hw.FPGAConfig.rtl_exact()))


def test_sync_statement_schedules_from_the_barrier():
    """build-defined sync scheduling: qclk restarts at the barrier, so the
    first pulse after it is placed as after reset; compiled to the assembler's
    sync statement on every core of its scope"""
    circ = [{'name': 'read', 'qubit': ['Q0']}, {'name': 'sync', 'scope': ['Q0', 'Q1'], 'barrier_id': 3},
            {'name': 'X90', 'qubit': ['Q0']}, {'name': 'X90', 'qubit': ['Q1']}]
    prog = sc.compile_circuit(circ, TABLE, hw.FPGAConfig()).program
    for g, st in prog.items():
        ops = [s['op'] for s in st]
        assert {'op': 'sync', 'barrier_id': 3} in st, g
        after = [s for s in st[ops.index('sync'):] if s['op'] == 'pulse']
        assert after and after[0]['start_time'] == sc.START_NCLKS, (g, after)


def test_sync_circuits_never_late_cpu():
    """circuits with syncs, branches and loops scheduled with FPGAConfig.rtl_exact():
    every shot finishes and no pulse is late on oracle_fast"""
    import oracle
    from distributed_processor_amd.emulator import ProgramSet
    for k, circ, asm in sync_circuits():
        ps = ProgramSet([asm])
        cfg = circuit_config(ps.cores_per_shot, k)
        f = oracle.fast_run(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, 0, 64, want=('summary',))
        s = _abi.unpack_summary(f['summary'])
        assert (s['status'] == _abi.ST_DONE).all(), (k, circ)
        assert not (s['flags'] & _abi.F_LATE).any(), (k, circ)


def test_sync_over_a_subset_of_cores():
    """a sync scoped to a subset of the cores (the 'qubits' spelling of its
    scope) lands only on those cores; an unscoped sync lands on every core.
    The subset sync needs the sync_mask sc.sync_mask derives: with the
    default all-cores mask the core that never syncs leaves the barrier
    waiting (ST_DEADLOCK); with the derived mask every lane finishes"""
    import oracle
    from distributed_processor_amd.emulator import ProgramSet
    chans = hw.load_channel_configs(os.path.join(GOLDEN, 'channel_config.json'))
    circ = [{'name': 'X90', 'qubit': ['Q0']}, {'name': 'X90', 'qubit': ['Q1']},
            {'name': 'sync', 'barrier_id': 1, 'qubits': ['Q0']},
            {'name': 'read', 'qubit': ['Q0']}, {'name': 'read', 'qubit': ['Q1']}]
    compiled = sc.compile_circuit(circ, TABLE, hw.FPGAConfig.rtl_exact())
    order = sorted(compiled.program, key=lambda g: chans[g[0]].core_ind)
    has_sync = [any(s['op'] == 'sync' for s in compiled.program[g]) for g in order]
    assert has_sync == [True, False]
    assert sc.sync_mask(compiled.program, order) == 0b01

    unscoped = sc.compile_circuit(circ[:2] + [{'name': 'sync', 'barrier_id': 2}] + circ[3:], TABLE,
                                  hw.FPGAConfig.rtl_exact())
    assert all(any(s['op'] == 'sync' for s in st) for st in unscoped.program.values())
    assert sc.sync_mask(unscoped.program, order) == 0b11

    ps = ProgramSet([assemble(compiled)])
    for mask, status in ((0, _abi.ST_DEADLOCK), (sc.sync_mask(compiled.program, order), _abi.ST_DONE)):
        cfg = _abi.make_config(2, max_cycles=1 << 16, event_cap=16, meas_cap=4, sync_mask=mask, seed=1)
        f = oracle.fast_run(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, 0, 16, want=('summary',))
        s = _abi.unpack_summary(f['summary'])
        assert (s['status'][:16] == status).all(), (mask, s['status'])
        assert (s['status'][16:] == _abi.ST_DONE).all(), mask


@pytest.mark.gpu
def test_sync_circuits_gpu_vs_oracle():
    from distributed_processor_amd.emulator import Emulator, ProgramSet
    from tests.test_gpu_parity import compare_all, run_pair
    with Emulator(0) as emu:
        for k, circ, asm in sync_circuits():
            ps = ProgramSet([asm])
            g, f = run_pair(emu, ps, circuit_config(ps.cores_per_shot, k), 1500, shot0=31 * k)
            compare_all(g, f, 'sync circuit {}'.format(k))
            s = _abi.unpack_summary(g['summary'])
            assert (s['status'] == _abi.ST_DONE).all() and not (s['flags'] & _abi.F_LATE).any(), k
