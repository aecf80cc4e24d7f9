"""Late-pulse linter for assembled distproc machine code, with the RTL's
exact decode-to-decode latencies.

The reference checks schedules at IR level (``LintSchedule``,
``python/distproc/ir/passes.py:745-822``): a pulse's start time must not
precede the end of the previous instruction, with end times advanced by the
``FPGAConfig`` constants (``hwconfig.py:100-119``).  Two things keep that
check approximate: it runs before assembly, and its constants are not the
RTL's -- ``jump_cond_clks`` is 5 where ``ctrl.v`` takes 6 (SURVEY.md
Appendix A #9; :data:`hwconfig.EXACT_LATENCIES`).

This linter runs on what the emulator runs: the u128 command words.  It is a
forward interval analysis over the program's control-flow graph of
qclk(D), the core's timebase at the decode cycle D of every command, using
the latencies of DESIGN.md §2 (``hdl/ctrl.v``):

* pulse write / pulse_reset: D+3; reg_alu / jump_i: D+4; jump_cond: D+6
  (both successors);
* pulse trigger / idle at ``cmd_time`` T: the next decode is at qclk T+3
  whenever it comes; the command is **late** when qclk(D) > T (the core then
  waits for the 32-bit qclk to wrap: the emulator's ``DPEMU_F_LATE``);
* inc_qclk with an immediate operand: qclk(D+4) = alu(imm, qclk(D)) + 4;
  with a register operand the value is unknown;
* alu_fproc / jump_fproc: the response comes at R >= D+2 (later in LUT mode
  or when waiting for a measurement), so qclk(next) >= qclk(D) + 6 / 8 with no
  upper bound;
* sync: qclk is 0 at S+2, so the next decode sees qclk 1 whatever S is;
* the reset hold: qclk(0) = qclk(1) = 0, so a trigger at T = 0 as the first
  command strobes twice (``DPEMU_F_DOUBLE_STROBE``).

Each command gets a verdict: ``late`` (late on every path that reaches it,
taking unbounded fproc waits to end within 2^31 cycles),
``may_be_late`` (late on some path, or the bound is unknown) or ``slack``
(T - the latest qclk(D)).  For a program whose intervals are all points
(no fproc, no register-sourced inc_qclk, no jump_cond), the verdict is exact:
the emulator sets ``DPEMU_F_LATE`` on a lane iff the linter finds a reachable
``late`` command (tests/test_lint.py checks this against ``oracle_fast`` and,
on the GPU, against the emulator itself).

:func:`check_fpga_config` reports where an ``FPGAConfig`` under-estimates the
RTL's latencies, which is how IR-level schedules that pass ``LintSchedule``
can still be late on hardware.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import isa
from .hwconfig import EXACT_LATENCIES

MASK32 = 0xFFFFFFFF
MAX_VISITS = 16        # joins per command before its interval is widened to unknown

Interval = Tuple[Optional[int], Optional[int]]   # (lo, hi) of qclk(D); None = unknown


@dataclass
class Finding:
    index: int                 # command index in the program
    op: str
    kind: str                  # 'late' | 'may_be_late' | 'double_strobe' | 'hang_opcode'
    cmd_time: Optional[int] = None
    qclk_lo: Optional[int] = None
    qclk_hi: Optional[int] = None

    def __str__(self):
        rng = '[{}, {}]'.format(self.qclk_lo, '?' if self.qclk_hi is None else self.qclk_hi)
        t = '' if self.cmd_time is None else ' cmd_time {}'.format(self.cmd_time)
        return 'cmd {} ({}): {}{}; qclk at decode {}'.format(self.index, self.op, self.kind, t, rng)


@dataclass
class LintReport:
    qclk: Dict[int, Interval]                   # qclk(D) interval of every reachable command
    findings: List[Finding] = field(default_factory=list)
    slack: Dict[int, Optional[int]] = field(default_factory=dict)   # trigger / idle: T - max qclk(D)
    exact: bool = True                          # every interval a point: the verdicts are exact

    @property
    def late(self) -> bool:
        return any(f.kind == 'late' for f in self.findings)

    @property
    def may_be_late(self) -> bool:
        return any(f.kind in ('late', 'may_be_late') for f in self.findings)

    @property
    def min_slack(self) -> Optional[int]:
        v = [s for s in self.slack.values() if s is not None]
        return min(v) if v else None


def _alu(op: str, in0: int, in1: int) -> int:
    """hdl/alu.v restated for the immediate inc_qclk forms"""
    a, b = in0 & MASK32, in1 & MASK32
    if op == 'id0':
        return a
    if op == 'add':
        return (a + b) & MASK32
    if op == 'sub':
        return (a - b) & MASK32
    if op == 'id1':
        return b
    if op == 'zero':
        return 0
    sub = (a - b) & MASK32
    sa, sb, ss = a >> 31, b >> 31, sub >> 31
    le = ss ^ ((1 - sa) & sb & ss | sa & (1 - sb) & (1 - ss))
    return {'eq': int(sub == 0), 'le': le, 'ge': 1 - le}[op]


def _late(T: int, q: int) -> bool:
    """the wait from qclk q to T is >= 2^31 cycles (fast_model.c / interp.hip rule)"""
    return ((T - q) & MASK32) >= 0x80000000


def lint_program(words: Sequence[int]) -> LintReport:
    """Interval analysis of one core's program (u128 command words, as
    ``isa`` encodes them or ``GlobalAssembler`` emits them)."""
    n = len(words)
    dec = [isa.decode(w) for w in words]
    # state: qclk(D) as "v" with the reset hold folded in: the first command decodes at
    # D = 0 with v = -1 (qclk(0) = 0) and qclk(D) = max(v, 0) until a reload
    state: Dict[int, Interval] = {0: (-1, -1)}
    visits: Dict[int, int] = {}
    work = [0]

    def succ_state(i: int, iv: Interval) -> List[Tuple[int, Interval]]:
        lo, hi = iv
        d = dec[i] if i < n else {'op': 'done'}
        op = d['op']

        def adv(k, lo=lo, hi=hi):
            return (None if lo is None else lo + k, None if hi is None else hi + k)

        if op in ('done', 'done0', 'hang'):
            return []
        nxt = (i + 1) & 0xFFFF
        if op in ('pulse_write', 'pulse_reset'):
            return [(nxt, adv(3))]
        if op in ('pulse_write_trig', 'idle'):
            T = d['cmd_time']
            if lo == -1 and hi == -1 and T == 0:
                return [(nxt, (2, 2))]              # hold: strobe at t = 2 (and 3); next decode t = 3
            q = (T + 3) & MASK32
            return [(nxt, (q, q))]
        if op == 'reg_alu':
            return [(nxt, adv(EXACT_LATENCIES['alu_instr_clks']))]
        if op == 'jump_i':
            return [(d['target'], adv(EXACT_LATENCIES['jump_i_clks']))]
        if op == 'jump_cond':
            k = EXACT_LATENCIES['jump_cond_clks']
            return [(d['target'], adv(k)), (nxt, adv(k))]
        if op == 'inc_qclk':
            if d['in0_reg'] or lo is None or hi is None or lo != hi:
                return [(nxt, (None, None))]
            q = (_alu(d['alu_op'], d['imm'], max(lo, 0)) + 4) & MASK32
            return [(nxt, (q, q))]
        if op in ('alu_fproc', 'jump_fproc'):
            k = EXACT_LATENCIES['alu_fproc_clks'] if op == 'alu_fproc' else EXACT_LATENCIES['jump_fproc_clks']
            s = (None if lo is None else lo + k, None)
            return [(d['target'], s), (nxt, s)] if op == 'jump_fproc' else [(nxt, s)]
        if op == 'sync':
            return [(nxt, (1, 1))]
        return []

    while work:
        i = work.pop()
        visits[i] = visits.get(i, 0) + 1
        for j, iv in succ_state(i, state[i]):
            if j >= n:                                  # past the program: the zero guard = DONE
                continue
            old = state.get(j)
            if old is None:
                new = iv
            else:
                lo = None if old[0] is None or iv[0] is None else min(old[0], iv[0])
                hi = None if old[1] is None or iv[1] is None else max(old[1], iv[1])
                new = (lo, hi)
                if visits.get(j, 0) >= MAX_VISITS and new != old:
                    new = (None, None)                  # widen: loops whose timing does not converge
            if new != old:
                state[j] = new
                work.append(j)

    rep = LintReport(qclk=dict(sorted(state.items())))
    for i, (lo, hi) in rep.qclk.items():
        d = dec[i]
        op = d['op']
        if lo is None or hi is None or lo != hi:
            rep.exact = False
        if op == 'jump_cond' or op in ('alu_fproc', 'jump_fproc'):
            rep.exact = False
        if op == 'hang':
            rep.findings.append(Finding(i, op, 'hang_opcode'))
            continue
        if op not in ('pulse_write_trig', 'idle'):
            continue
        T = d['cmd_time']
        qlo = None if lo is None else max(lo, 0)
        qhi = None if hi is None else max(hi, 0)
        rep.slack[i] = None if qhi is None else T - qhi
        if lo == -1 and hi == -1:                       # first command, in the reset hold (D = 0)
            if T == 0 and op == 'pulse_write_trig':
                rep.findings.append(Finding(i, op, 'double_strobe', T, 0, 0))
            if T + 1 >= 0x80000000:                     # tT = 1 + T cycles away
                rep.findings.append(Finding(i, op, 'late', T, 0, 0))
            continue
        # late on every path: qclk(D) > T from the lowest bound up (an unknown upper bound
        # comes from fproc waits and register inc_qclk, taken to stay below 2^31 cycles)
        if qlo is not None and _late(T, qlo) and (qhi is None or (_late(T, qhi) and qhi - qlo < 0x80000000)):
            rep.findings.append(Finding(i, op, 'late', T, qlo, qhi))
        elif qlo is None or qhi is None or _late(T, qlo) or _late(T, qhi):
            rep.findings.append(Finding(i, op, 'may_be_late', T, qlo, qhi))
    return rep


def lint_assembled(assembled: dict) -> Dict[str, LintReport]:
    """``GlobalAssembler.get_assembled_program()`` dict -> {core: report}"""
    return {core: lint_program(isa.bytes_to_words(prog['cmd_buf'])) for core, prog in assembled.items()}


def check_fpga_config(fpga_config) -> List[str]:
    """Where ``fpga_config``'s scheduler latencies are shorter than the RTL's:
    an IR schedule built with them can pass ``LintSchedule`` and still
    decode a pulse after its start time on hardware."""
    msgs = []
    for name in ('alu_instr_clks', 'jump_cond_clks', 'jump_fproc_clks', 'pulse_load_clks'):
        have = getattr(fpga_config, name, None)
        need = EXACT_LATENCIES[name]
        if have is not None and have < need:
            msgs.append('{} = {} < {} (RTL decode-to-decode, hdl/ctrl.v)'.format(name, have, need))
    return msgs


def late_lanes(summary: np.ndarray) -> np.ndarray:
    """lanes whose emulation hit a late trigger (``DPEMU_F_LATE``), from the
    emulator's [n_lanes][8] u32 summary"""
    from . import _abi
    s = _abi.unpack_summary(np.asarray(summary).view(np.uint32))
    return np.nonzero(s['flags'] & _abi.F_LATE)[0]
