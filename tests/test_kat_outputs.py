"""The reference's known answers asserted on the emulator's OUTPUTS.

tests/test_rtl_kat.py ports the cocotb testbenches clock for clock onto the
per-clock oracle.  Here the same programs run through the product path --
the HIP kernels via the C ABI (``gpu``, MI355X) -- and through oracle_fast
(``fast``, CPU), and the reference's expected values are checked on what a
run returns: event records (t, env, phase, freq, amp of every cstrobe), the
final register file, the lane summary (qclk at the end, DONE).  Each seeded
test case is one program group, so one launch covers every seed.

Timebase: cycle 0 is the first DECODE; with no qclk reload qclk(t) = t - 1,
so the testbench's "qclk at cstrobe - CSTROBE_DELAY == cmd_time"
(test_proc.py:81-99) is event t - 3 == cmd_time.  Sources:
cocotb/proc/test_proc.py test_pulse_freq_trig (:76), test_pulse_i (:103),
test_regwrite_i (:131), test_reg_i (:185), test_pulse_reg (:246),
test_jump_i (:283), test_jump_i_cond (:304), test_pulse_reset (:541),
test_pulse_sync (:547), test_idle (:605), test_idle_pulse (:622).  The
fproc tests (test_read_fproc, test_jump_fproc_i) drive fproc_data by hand
with arbitrary words; the emulator's fproc returns measurement bits, so they
stay on the per-clock port (tests/test_rtl_kat.py).
"""

import random

import numpy as np
import pytest

import distributed_processor_amd.isa as cg
import oracle
from distributed_processor_amd import _abi
from distributed_processor_amd.emulator import Emulator, ProgramSet, decode_events

SEEDS = range(12)
CSTROBE_DELAY = 2
ENGINES = ['fast', pytest.param('gpu', marks=pytest.mark.gpu)]


_EMU = {}


def run_groups(engine, groups, event_cap=16, **cfg_kw):
    """one single-core program per group, shot g runs group g; returns
    (summary fields, events [n_groups] lists, regs [16, n_groups])"""
    ps = ProgramSet([{'0': list(g)} for g in groups])
    cfg = _abi.make_config(1, n_groups=ps.n_groups, event_cap=event_cap, meas_cap=2, **cfg_kw)
    n = ps.n_groups
    want = ('summary', 'events', 'regs')
    if engine == 'gpu':
        if 'emu' not in _EMU:
            _EMU['emu'] = Emulator(0)
        emu = _EMU['emu']
        emu.load(ps)
        arrays = emu.run(n, 0, cfg=cfg, outputs=want).arrays
    else:
        arrays = oracle.fast_run(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, 0, n, want=want)
    s = _abi.unpack_summary(arrays['summary'])
    ev = [decode_events(arrays['events'][:min(int(s['n_events'][g]), event_cap), g]) for g in range(n)]
    return s, ev, np.asarray(arrays['regs']).view(np.uint32)


def _random_pulse(rng):
    return dict(freq_word=rng.randint(0, 2 ** 9 - 1), phase_word=rng.randint(0, 2 ** 17 - 1),
                env_word=rng.randint(0, 2 ** 24 - 1), amp_word=rng.randint(0, 2 ** 16 - 1),
                cfg_word=rng.randint(0, 2 ** 4 - 1))


def alu_ref(in0, op, in1):
    """test_proc.py:639-653 (signed operands; add / sub through
    twos_complement), ge as the RTL computes it (>=, alu.v:29)"""
    if op in ('add', 'sub'):
        a, b = cg.twos_complement(in0), cg.twos_complement(in1)
        return (b + a) % 2 ** 32 if op == 'add' else (a - b) % 2 ** 32
    return {'ge': int(in0 >= in1), 'le': int(in0 < in1), 'eq': int(in0 == in1),
            'id0': in0 % 2 ** 32, 'id1': in1 % 2 ** 32}[op]


@pytest.mark.parametrize('engine', ENGINES)
def test_pulse_freq_trig(engine):
    times = [3, 6, 11, 15, 18, 22]
    groups, freqs = [], []
    for seed in SEEDS:
        rng = random.Random(seed)
        f = [rng.randint(0, 2 ** 9 - 1) for _ in times]
        freqs.append(f)
        groups.append([(0b10010000 << 120) + ((x + 2 ** 10) << 60) + (t << 5) for x, t in zip(f, times)])
    s, ev, _ = run_groups(engine, groups)
    for g in range(len(groups)):
        assert list(ev[g]['freq']) == freqs[g]
        assert list(ev[g]['t'].astype(np.int64) - 1 - CSTROBE_DELAY) == times
    assert (s['status'] == _abi.ST_DONE).all()


@pytest.mark.parametrize('engine', ENGINES)
def test_pulse_i(engine):
    times = [3, 6, 11, 15, 18, 22]
    groups, want = [], []
    for seed in SEEDS:
        rng = random.Random(seed)
        ps = [_random_pulse(rng) for _ in times]
        want.append(ps)
        groups.append([cg.pulse_i(p['freq_word'], p['phase_word'], p['amp_word'], p['env_word'], p['cfg_word'], t)
                       for p, t in zip(ps, times)])
    _, ev, _ = run_groups(engine, groups)
    for g, ps in enumerate(want):
        assert len(ev[g]) == len(times)
        for p, t, e in zip(ps, times, ev[g]):
            assert (int(e['freq']), int(e['phase']), int(e['env_word'])) == (p['freq_word'], p['phase_word'],
                                                                              p['env_word'])
            assert int(e['t']) - 1 - CSTROBE_DELAY == t


@pytest.mark.parametrize('engine', ENGINES)
def test_regwrite_i(engine):
    groups, want = [], []
    for seed in SEEDS:
        rng = random.Random(seed)
        addr, val = rng.randint(0, 15), rng.randint(0, 2 ** 32 - 1)
        groups.append([(0b00010000 << 120) + (val << 88) + (addr << 80)])
        want.append((addr, val))
    _, _, regs = run_groups(engine, groups)
    for g, (addr, val) in enumerate(want):
        assert int(regs[addr, g]) == val


@pytest.mark.parametrize('engine', ENGINES)
def test_reg_i(engine):
    groups, want = [], []
    for seed in SEEDS:
        rng = random.Random(seed)
        for _ in range(100):
            a0, a1 = rng.randint(0, 15), rng.randint(0, 15)
            reg_val = rng.randint(-2 ** 31, 2 ** 31 - 1)
            ival = rng.randint(-2 ** 31, 2 ** 31 - 1)
            op = rng.choice(['add', 'sub', 'le', 'ge', 'eq'])
            groups.append([cg.alu_cmd('reg_alu', 'i', reg_val, 'id0', 0, a0),
                           cg.alu_cmd('reg_alu', 'i', ival, op, a0, a1)])
            want.append((a1, alu_ref(ival, op, reg_val)))
    _, _, regs = run_groups(engine, groups)
    for g, (a1, v) in enumerate(want):
        assert int(regs[a1, g]) == v, (g, a1, v)


@pytest.mark.parametrize('engine', ENGINES)
def test_pulse_reg(engine):
    times = [9, 15, 18]
    reg_word, reg_addr = 0x000000a3, 2
    groups, want = [], []
    for seed in SEEDS:
        rng = random.Random(seed)
        cmds = [cg.alu_cmd('reg_alu', 'i', reg_word, 'id0', 0, write_reg_addr=reg_addr)]
        w = []
        for i in range(3):
            p = _random_pulse(rng)
            p['cfg_word'] = rng.randint(0, 3)
            kw = dict(p)
            field = ('freq', 'phase', 'env')[i]
            p[field + '_word'] = reg_word
            del kw[field + '_word']
            kw[field + '_regaddr'] = reg_addr
            cmds.append(cg.pulse_cmd(cmd_time=times[i], **kw))
            w.append(p)
        groups.append(cmds)
        want.append(w)
    _, ev, _ = run_groups(engine, groups)
    for g, w in enumerate(want):
        assert len(ev[g]) == 3
        for p, t, e in zip(w, times, ev[g]):
            assert int(e['t']) - 1 - CSTROBE_DELAY == t
            got = dict(freq_word=int(e['freq']), phase_word=int(e['phase']), amp_word=int(e['amp']),
                       env_word=int(e['env_word']), cfg_word=int(e['cfg']))
            assert got == p


@pytest.mark.parametrize('engine', ENGINES)
def test_jump_i_and_cond(engine):
    """the command after jump_i is cmds[jump_addr]; after jump_cond it is
    cmds[jump_addr] iff the ALU condition holds, else cmds[2].  The reference
    fills the memory with random words and reads cmd_buf_out; here every
    address holds a pulse whose amp word is its address, so the first strobe
    names the command executed next"""
    def marked(n):
        return [cg.pulse_i(0, 0, a, 0, 0, 500) for a in range(n)]   # cmd_time 500: after any jump
    groups, want = [], []
    for seed in SEEDS:
        rng = random.Random(seed)
        jump_addr = rng.randint(2, 2 ** 8 - 1)
        cmds = marked(2 ** 8)
        cmds[0] = cg.jump_i(jump_addr)
        groups.append(cmds)
        want.append(jump_addr)
        for _ in range(8):
            jump_addr = rng.randint(3, 2 ** 8 - 1)
            a0 = rng.randint(0, 15)
            reg_val = rng.randint(-2 ** 31, 2 ** 31 - 1)
            ival = rng.choice([reg_val, rng.randint(-2 ** 31, 2 ** 31 - 1)])
            op = rng.choice(['le', 'ge', 'eq'])
            cmds = marked(2 ** 8)
            cmds[0] = cg.alu_cmd('reg_alu', 'i', reg_val, 'id0', 0, a0)
            cmds[1] = cg.alu_cmd('jump_cond', 'i', ival, op, a0, jump_cmd_ptr=jump_addr)
            groups.append(cmds)
            want.append(jump_addr if alu_ref(ival, op, reg_val) else 2)
    _, ev, _ = run_groups(engine, groups, event_cap=4, max_cycles=20000)
    for g, addr in enumerate(want):
        assert int(ev[g][0]['amp']) == addr, (g, addr)


@pytest.mark.parametrize('engine', ENGINES)
def test_pulse_reset_idle_done(engine):
    """pulse_reset strobes pulse_iface.reset (an event of kind 1); idle(100)
    then done ends with qclk past 100; idle then a pulse at 103 strobes once
    with qclk 105 (cmd_time + 2) and its immediates (test_proc.py:541-636)"""
    groups = [[cg.pulse_reset()],
              [cg.idle(100), cg.done_cmd()],
              [cg.idle(100), cg.pulse_i(10, 3, 1, 0, 0, 103), cg.done_cmd()]]
    s, ev, _ = run_groups(engine, groups)
    assert list(ev[0]['kind']) == [_abi.EV_PULSE_RESET]
    assert (s['status'] == _abi.ST_DONE).all()
    assert int(s['qclk_end'][1]) > 100
    assert [(int(e['t']) - 1, int(e['freq']), int(e['phase']), int(e['amp'])) for e in ev[2]] == [(105, 10, 3, 1)]
    assert int(s['qclk_end'][2]) > 105


@pytest.mark.parametrize('engine', ENGINES)
def test_pulse_sync(engine):
    """test_proc.py:547-599: six pulses, a sync, a seventh pulse at cmd_time 4
    -- qclk restarts from 0 at the sync, so the last strobe is at qclk 6
    whenever sync.ready arrives (the testbench drives it by hand, the
    emulator's controller at the last arrival + sync_latency); the register
    trace's qclk-reset record gives the restart cycle"""
    times = [3, 6, 11, 15, 18, 22, 4]
    groups, want = [], []
    for seed in SEEDS:
        rng = random.Random(seed)
        ps = [_random_pulse(rng) for _ in times]
        cmds = [cg.pulse_i(p['freq_word'], p['phase_word'], p['amp_word'], p['env_word'], p['cfg_word'], t)
                for p, t in zip(ps, times)]
        cmds.insert(-1, cg.sync(0))
        groups.append(cmds)
        want.append(ps)
    ps_ = ProgramSet([{'0': list(g)} for g in groups])
    for lat in (1, 17):
        cfg = _abi.make_config(1, n_groups=ps_.n_groups, event_cap=16, trace_cap=4, meas_cap=2, sync_latency=lat)
        want_out = ('summary', 'events', 'trace')
        if engine == 'gpu':
            if 'emu' not in _EMU:
                _EMU['emu'] = Emulator(0)
            _EMU['emu'].load(ps_)
            arrays = _EMU['emu'].run(ps_.n_groups, 0, cfg=cfg, outputs=want_out).arrays
        else:
            arrays = oracle.fast_run(cfg, ps_.words, ps_.offsets, ps_.n_instr, ps_.table, 0, ps_.n_groups,
                                     want=want_out)
        s = _abi.unpack_summary(arrays['summary'])
        tr = np.asarray(arrays['trace']).view(np.uint32)
        for g, ps in enumerate(want):
            ev = decode_events(arrays['events'][:int(s['n_events'][g]), g])
            assert len(ev) == len(times)
            t_rst = [int(r[0]) for r in tr[:int(s['n_trace'][g]), g] if r[1] == _abi.TRACE_QCLK_RST]
            assert len(t_rst) == 1
            qclk = [int(e['t']) - 1 for e in ev[:-1]] + [int(ev[-1]['t']) - t_rst[0]]
            for p, t, e, q in zip(ps, times, ev, qclk):
                assert (int(e['freq']), int(e['phase']), int(e['env_word'])) == (p['freq_word'], p['phase_word'],
                                                                                  p['env_word'])
                assert q - CSTROBE_DELAY == t


def teardown_module(module):
    emu = _EMU.pop('emu', None)
    if emu is not None:
        emu.close()
