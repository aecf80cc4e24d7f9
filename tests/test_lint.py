"""Late-pulse linter (distributed_processor_amd/lint.py) against execution.

For programs whose qclk intervals are points (branch-free, no fproc, no
register-sourced inc_qclk) the linter is exact: a lane's ``DPEMU_F_LATE``
is set iff the linter finds a reachable ``late`` command, and the reset-hold
double strobe iff it finds ``double_strobe``.  For every other program it
must be sound: no ``late`` / ``may_be_late`` finding => no late flag.  The
CPU tests execute with ``oracle_fast``; the GPU test with the emulator.
"""

import numpy as np
import pytest

from distributed_processor_amd import _abi, hwconfig, isa, lint
from tests.progfuzz import pack_programs, random_case, shaped_case

MAX_CYCLES = 1 << 30           # every non-late wait of the fuzzed programs fits


def group_programs(case):
    C = case['ncores']
    return [[case['progs'][case['table'][g * C + c]] for c in range(C)] for g in range(case['n_groups'])]


def oracle_flags(progs, seed=0):
    import oracle
    C = len(progs)
    cfg = _abi.make_config(C, max_cycles=MAX_CYCLES, event_cap=64, trace_cap=16, meas_cap=16, seed=seed)
    words, offs, ni = pack_programs(progs)
    f = oracle.fast_run(cfg, words, offs, ni, np.arange(C, dtype=np.uint32), 0, 1, want=('summary',))
    return _abi.unpack_summary(f['summary'])['flags']


def check(progs, flags, ctx):
    n_exact = 0
    for c, p in enumerate(progs):
        rep = lint.lint_program(p)
        late = bool(flags[c] & _abi.F_LATE)
        if rep.exact:
            n_exact += 1
            assert rep.late == late, '{} core {}: lint {} vs F_LATE {}\n{}'.format(
                ctx, c, [str(f) for f in rep.findings], late, '\n'.join(isa.disasm(w) for w in p))
            dbl = any(f.kind == 'double_strobe' for f in rep.findings)
            assert dbl == bool(flags[c] & _abi.F_DOUBLE_STROBE), ctx
        elif late:
            assert rep.may_be_late, '{} core {}: late lane without a finding'.format(ctx, c)
    return n_exact


@pytest.mark.parametrize('kind', ['straight', 'linear', 'shaped', 'any'])
def test_lint_matches_oracle_fast(kind):
    n_exact = n_late = 0
    for seed in range(120):
        if kind == 'shaped':
            case = shaped_case(500 + seed, ncores=2, n_groups=2, allow_late=True, linear=seed % 2 == 1)
        else:
            case = random_case(700 + seed, allow_late=True, allow_hang=True, straight=kind == 'straight',
                               linear=kind == 'linear')
        for g, progs in enumerate(group_programs(case)):
            if kind == 'any' and case['ncores'] > 1:
                progs = progs[:1]                   # sync needs partners; a lone core is checked for soundness
            flags = oracle_flags(progs, seed)
            n_exact += check(progs, flags, '{} seed {} group {}'.format(kind, seed, g))
            n_late += int((flags & _abi.F_LATE).any())
    if kind != 'any':
        assert n_exact > 50 and n_late > 5, (n_exact, n_late)


def test_lint_known_programs():
    prog = [isa.pulse_i(1, 2, 3, 4, 0, 10), isa.pulse_i(1, 2, 3, 4, 0, 12), isa.done_cmd()]
    rep = lint.lint_program(prog)
    assert rep.late and rep.exact                          # 10 + 3 > 12
    assert rep.qclk[1] == (13, 13) and rep.slack[0] == 10 and rep.slack[1] == -1
    ok = [isa.pulse_i(1, 2, 3, 4, 0, 10), isa.pulse_i(1, 2, 3, 4, 0, 13), isa.done_cmd()]
    assert not lint.lint_program(ok).late and lint.lint_program(ok).min_slack == 0
    # reset hold: trigger at T = 0 first strobes twice; the next decode sees qclk 2
    rep = lint.lint_program([isa.pulse_i(0, 0, 0, 0, 0, 0), isa.pulse_i(0, 0, 0, 0, 0, 2), isa.done_cmd()])
    assert [f.kind for f in rep.findings] == ['double_strobe'] and not rep.late
    # a loop that rewinds qclk with inc_qclk converges to a point; without it the trigger goes late
    loop = [isa.reg_alu_i(3, 'id0', 0, 1),                              # r1 = 3
            isa.pulse_i(0, 0, 0, 0, 0, 20),                              # 1: trig @ 20
            isa.inc_qclk_i(-20),                                         # 2: qclk -= 20
            isa.reg_alu_i(-1, 'add', 1, 1),                              # 3: r1 -= 1
            isa.jump_cond_i(0, 'le', 1, 1),                              # 4: 0 < r1: back to 1
            isa.done_cmd()]
    rep = lint.lint_program(loop)
    assert not rep.may_be_late, [str(f) for f in rep.findings]
    assert rep.qclk[1] == (3, 17)                   # first entry 3; back edge 23 - 20 + 4 + 4 + 6 = 17
    assert not oracle_flags([loop])[0] & _abi.F_LATE
    noloop = loop[:2] + [isa.reg_alu_i(0, 'id0', 0, 2)] + loop[3:]
    rep = lint.lint_program(noloop)                 # late from the second iteration on
    assert rep.may_be_late and rep.qclk[1] == (3, 37) and oracle_flags([noloop])[0] & _abi.F_LATE
    # fproc waits have no upper bound
    f = [isa.jump_fproc_i(0, 1, 'eq', 2), isa.pulse_i(0, 0, 0, 0, 0, 100), isa.done_cmd()]
    rep = lint.lint_program(f)
    assert not rep.exact and rep.may_be_late and not rep.late


def test_lint_assembled_goldens(golden_dir):
    """the reference's compiler goldens as machine code, against their
    execution by oracle_fast (fproc_meas: responses at the earliest, D+2):
    a ``late`` verdict must come with DPEMU_F_LATE, and a lane without any
    late / may_be_late finding must run without it.  One golden IS late on the
    RTL: test_multirst_cfg core 1 puts a pulse at cmd_time 9 right behind a
    jump_fproc decoded at qclk 2, whose next decode is at qclk >= 10 (the
    compiler's FPGAConfig latencies are not the RTL's)"""
    import json
    import os
    with open(os.path.join(golden_dir, 'asm_programs.json')) as fh:
        progs = json.load(fh)['programs']
    late = []
    for name, ent in progs.items():
        for core, prog in ent.get('dds_elem', {}).items():
            words = isa.bytes_to_words(bytes.fromhex(prog['cmd_buf']))
            rep = lint.lint_program(words)
            flag = bool(oracle_flags([words])[0] & _abi.F_LATE)
            if rep.late:
                assert flag, (name, core)
                late.append((name, core))
            if not rep.may_be_late:
                assert not flag, (name, core)
    assert late == [('test_multirst_cfg', '1')], late


def test_check_fpga_config():
    msgs = lint.check_fpga_config(hwconfig.FPGAConfig())
    assert any(m.startswith('jump_cond_clks = 5 < 6') for m in msgs)
    assert not lint.check_fpga_config(hwconfig.FPGAConfig(jump_cond_clks=6))


@pytest.mark.gpu
def test_lint_matches_gpu_emulator():
    """the same exactness property with the emulator on cuda:0 doing the execution"""
    from distributed_processor_amd.emulator import Emulator, ProgramSet
    n_exact = 0
    with Emulator(0) as emu:
        for seed in range(48):
            case = random_case(900 + seed, allow_late=True, allow_hang=True, straight=seed % 2 == 0,
                               linear=seed % 2 == 1)
            for g, progs in enumerate(group_programs(case)):
                C = len(progs)
                emu.load(ProgramSet([progs], cores_per_shot=C))
                cfg = _abi.make_config(C, max_cycles=MAX_CYCLES, event_cap=64, trace_cap=16, meas_cap=16,
                                       seed=seed)
                s = emu.run(1, 0, cfg=cfg, outputs=('summary',)).arrays['summary']
                flags = _abi.unpack_summary(np.asarray(s).view(np.uint32))['flags']
                n_exact += check(progs, flags, 'gpu seed {} group {}'.format(seed, g))
    assert n_exact > 30
