"""Config 4 at its stated size on the GPU (BASELINE.json configs[3]):
10^5 distinct two-qubit Clifford RB sequences of depth 200 plus their
recovery Cliffords (workloads.config4_rb2q: about 2.6 * 10^8 commands, a
4.2 GB device-resident program image), 10 shots per sequence = 10^6 shots =
2 * 10^6 (shot, core) lanes in one launch.  (The kernel-edge tests below use
the RB-shaped generator workloads.config4_rb_set: small tables of the same
program class.)

* bit-exact, the WHOLE launch: all 10^6 shots (2 * 10^6 lanes) compared
  with oracle_fast on every output array -- summaries, event records,
  measurements, final registers, the histogram -- in chunks of 50,000 shots
  (device slices to host, the oracle on the same shot range);
* 2,000 shots in 50 windows spread over the whole program table, run as
  small launches with register traces, against oracle_fast;
* full-size properties: every lane DONE, histogram total and per-sequence
  counts, sharding invariance (two half-size launches = the full launch).

Programs are longer than hdl/proc.sv:12's 256-deep cmd_mem, within
sim_modules/toplevel_sim.sv:5's 2^16 (SURVEY.md §7 hard part 6).
"""

import os

import numpy as np
import pytest

import oracle
from distributed_processor_amd import _abi, isa, workloads
from distributed_processor_amd.emulator import Emulator, ProgramSet, alloc_device_outputs

pytestmark = pytest.mark.gpu

N_SEQ, DEPTH, SPG = 100000, 200, 10
N_SHOTS = N_SEQ * SPG
WINDOWS, WIN = 50, 40


@pytest.fixture(scope='module')
def rb():
    import torch
    ps = workloads.config4_rb2q_set(N_SEQ, DEPTH)
    ops = ps.words[:, 3] >> 28
    strobes = np.add.reduceat(((ops == isa.OP_PULSE_TRIG) | (ops == isa.OP_PULSE_RESET)).astype(np.int64),
                              ps.offsets.astype(np.int64))
    alus = np.add.reduceat((ops == isa.OP_REG_ALU).astype(np.int64), ps.offsets.astype(np.int64))
    cfg = _abi.make_config(2, n_groups=N_SEQ, shots_per_group=SPG, max_cycles=1 << 20,
                           event_cap=int(strobes.max()) + 1, trace_cap=int(alus.max()) + 1, meas_cap=2,
                           meas_latency=64, seed=0xC0FFEE, p1=0.5)
    emu = Emulator(0)
    emu.load(ps)
    out = alloc_device_outputs(cfg, N_SHOTS, want=('summary', 'events', 'meas', 'regs', 'hist'))
    for t in out.values():
        t.zero_()                                        # slots past a lane's count stay 0, as in the oracle's
    emu.run_device(cfg, N_SHOTS, 0, out)
    torch.cuda.synchronize()
    yield emu, ps, cfg, out
    del out
    emu.close()
    torch.cuda.empty_cache()


def window_starts():
    return [int(x) for x in np.linspace(0, N_SHOTS - WIN, WINDOWS).astype(np.int64) + np.arange(WINDOWS) % 7]


CHUNK = 50000


def test_full_launch_bit_exact(rb):
    """every lane of the full-size launch against oracle_fast, chunk by chunk"""
    emu, ps, cfg, out = rb
    assert emu.last_kernel().startswith('macro_staged_kernel'), emu.last_kernel()
    threads = int(os.environ.get('OMP_NUM_THREADS', '0') or 0) or min(16, os.cpu_count() or 1)
    want = ('summary', 'events', 'meas', 'regs')
    for w0 in range(0, N_SHOTS, CHUNK):
        n = min(CHUNK, N_SHOTS - w0)
        f = oracle.fast_run(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, w0, n, threads=threads, want=want)
        # core-major lanes: core c's shots [w0, w0 + n) are lanes c * N_SHOTS + [w0, w0 + n), which the
        # chunk's oracle run holds at c * n + [0, n)
        for c in range(2):
            full = slice(c * N_SHOTS + w0, c * N_SHOTS + w0 + n)
            part = slice(c * n, (c + 1) * n)
            got = {'summary': out['summary'][full], 'events': out['events'][:, full],
                   'meas': out['meas'][:, full], 'regs': out['regs'][:, full]}
            ref = {'summary': f['summary'][part], 'events': f['events'][:, part],
                   'meas': f['meas'][:, part], 'regs': f['regs'][:, part]}
            for k in want:
                a = got[k].cpu().numpy().view(ref[k].dtype)
                if not np.array_equal(a, ref[k]):
                    bad = np.argwhere(a != ref[k])
                    raise AssertionError('shots [{}, {}) core {} {}: {} mismatches, first at {}'.format(
                        w0, w0 + n, c, k, len(bad), bad[0].tolist()))
        del f
    # the histogram of the whole launch: one oracle pass, histogram only
    f = oracle.fast_run(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, 0, N_SHOTS, threads=threads,
                        want=('hist',))
    assert np.array_equal(out['hist'].cpu().numpy().view(f['hist'].dtype).reshape(f['hist'].shape), f['hist'])


def test_full_launch_stream_hint_same_bytes(rb):
    """the bench's config-4 launch sets DPEMU_X_STREAM_EVENTS (nontemporal
    event rows): the whole launch's outputs equal the oracle-checked launch
    without it"""
    import torch
    emu, ps, cfg, out = rb
    base = cfg.exec_flags
    cfg.exec_flags = base | _abi.X_STREAM_EVENTS
    out2 = None
    try:
        out2 = alloc_device_outputs(cfg, N_SHOTS, want=('summary', 'events', 'meas', 'regs', 'hist'))
        for t in out2.values():
            t.zero_()
        emu.run_device(cfg, N_SHOTS, 0, out2)
        torch.cuda.synchronize()
        assert emu.last_kernel().startswith('macro_staged_kernel'), emu.last_kernel()
        for k in out2:
            assert torch.equal(out2[k], out[k]), k
    finally:
        cfg.exec_flags = base
        del out2
        torch.cuda.empty_cache()


def test_full_table_windows_with_traces(rb):
    """the same windows as small launches (the small-grid kernel) with every
    output, register traces included"""
    emu, ps, cfg, _ = rb
    outs = ('summary', 'events', 'trace', 'meas', 'regs', 'hist')
    for w0 in window_starts()[::5]:
        g = emu.run(WIN, w0, cfg=cfg, outputs=outs).arrays
        f = oracle.fast_run(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, w0, WIN, want=outs)
        for k in outs:
            assert np.array_equal(g[k], f[k]), 'shots [{}, {}) {}'.format(w0, w0 + WIN, k)


def test_full_size_properties(rb):
    import torch
    emu, ps, cfg, out = rb
    s = _abi.unpack_summary(out['summary'].cpu().numpy().view(np.uint32))
    assert (s['status'] == _abi.ST_DONE).all()
    assert (s['flags'] == 0).all()                       # no late pulse, no overflow
    assert (s['n_events'] <= cfg.event_cap).all()
    hist = out['hist'].cpu().numpy()
    assert hist.sum() == N_SHOTS
    assert (hist.sum(axis=1) == SPG).all()               # every sequence ran its 10 shots
    # per lane: the executed instruction count is the program length
    prog = ps.table.reshape(N_SEQ, 2)[np.arange(N_SHOTS) // SPG]               # [shot, core]
    assert np.array_equal(_abi.by_shot(s['n_instr'], 2).T, ps.n_instr[prog])
    # sharding invariance: two half-size launches reproduce the full launch
    half = N_SHOTS // 2
    for r in range(2):
        o = alloc_device_outputs(cfg, half, want=('summary', 'meas', 'hist'))
        o['meas'].zero_()
        emu.run_device(cfg, half, r * half, o)
        torch.cuda.synchronize()
        for c in range(2):                               # core-major lanes: core c's shots of the half
            full = slice(c * N_SHOTS + r * half, c * N_SHOTS + (r + 1) * half)
            part = slice(c * half, (c + 1) * half)
            assert torch.equal(o['summary'][part], out['summary'][full])
            assert torch.equal(o['meas'][:, part], out['meas'][:, full])
        g0 = r * half // SPG
        assert torch.equal(o['hist'][g0:g0 + half // SPG], out['hist'][g0:g0 + half // SPG])
        assert int(o['hist'].sum()) == half
        del o


@pytest.mark.parametrize('max_cycles', [9, 700, 1501, 4003, 20000])
def test_rb_lean_path_edges(max_cycles):
    """macro_staged_kernel's lean path (MACRO_SIMPLE macros, id0 / add ALU
    image) hands over to the general slots when a lane comes within 8 cycles
    of max_cycles, and on late cmd_times (stops): small RB tables cut at
    several max_cycles, both lane orders, traces off and on (trace forces the
    general path), every output against oracle_fast"""
    ps = workloads.config4_rb_set(96, 40)
    ops = ps.words[:, 3] >> 28
    strobes = np.add.reduceat(((ops == isa.OP_PULSE_TRIG) | (ops == isa.OP_PULSE_RESET)).astype(np.int64),
                              ps.offsets.astype(np.int64))
    from tests.test_gpu_parity import compare_all, run_pair
    with Emulator(0) as emu:
        for order in (_abi.LANES_CORE_MAJOR, _abi.LANES_SHOT_MAJOR):
            for trace_cap in (0, 8):
                cfg = _abi.make_config(2, n_groups=ps.n_groups, shots_per_group=SPG, max_cycles=max_cycles,
                                       event_cap=int(strobes.max()) + 1, trace_cap=trace_cap, meas_cap=2,
                                       meas_latency=64, seed=7, p1=0.5, lane_order=order)
                g, f = run_pair(emu, ps, cfg, 960, 13)
                compare_all(g, f, 'max_cycles {} order {} trace {}'.format(max_cycles, order, trace_cap))
                emu.run(3, 0, cfg=cfg)
                # shot-major waves span 5 sequences x 2 cores > MACRO_SLOTS: the 12-slot staged kernel
                want = 'macro_staged_kernel<2,addid>' if order == _abi.LANES_CORE_MAJOR else \
                    'macro_staged_kernel<2,addid,12>'
                assert emu.last_kernel() == want, emu.last_kernel()


@pytest.mark.parametrize('max_cycles', [1400, 1500, 1560, 1620, 4000])
def test_lean_chunk_after_qclk_wrap(max_cycles):
    """an inc_qclk by a negative value puts qclk just below 2^32, so the next
    pulses' small cmd_times fire only after qclk wraps (~1000 cycles later):
    the lean-chunk bound (macro.hip lean_chunk_ok) must not take those chunks
    as inside max_cycles.  40 reg_alu + pulse macros after the wrap (whole
    16-macro chunks of MACRO_SIMPLE macros), max_cycles inside and past them;
    every output against oracle_fast"""
    from tests.test_gpu_parity import compare_all, run_pair

    def core(w, step):
        words = [isa.pulse_reset(), isa.reg_alu_i(0, 'id0', 0, 1), isa.inc_qclk_i(-w)]
        for k in range(40):
            words.append(isa.reg_alu_i(5, 'add', 1, 1))
            words.append(isa.pulse_i(freq_word=3, phase_word=0, amp_word=100, env_word=1 | (4 << 12),
                                     cfg_word=0, cmd_time=10 + step * k))
        words.append(isa.done_cmd())
        return isa.words_to_bytes(words)
    ps = ProgramSet([{0: core(1000, 20), 1: core(1100, 17)}])
    cfg = _abi.make_config(2, n_groups=1, max_cycles=max_cycles, event_cap=48, trace_cap=0, meas_cap=2,
                           meas_latency=64, seed=7, p1=0.5)
    with Emulator(0) as emu:
        g, f = run_pair(emu, ps, cfg, 256)
        compare_all(g, f, 'qclk wrap, max_cycles {}'.format(max_cycles))
        emu.run(3, 0, cfg=cfg)
        assert emu.last_kernel() == 'macro_staged_kernel<2,addid>', emu.last_kernel()
    status = _abi.unpack_summary(np.asarray(g['summary']).view(np.uint32))['status']
    if max_cycles < 1600:
        assert (status == _abi.ST_MAX_CYCLES).all()


@pytest.mark.parametrize('spg,kernel', [(8, 'macro_staged_kernel<2,addid,12>'), (6, 'macro_staged_kernel<2,addid,12>'),
                                        (4, 'macro_kernel')])
def test_fewer_shots_per_sequence(spg, kernel):
    """RB sequences with 8 / 6 / 4 shots each: a wave of 64 consecutive shots
    spans 9-12 programs (the 12-slot staged kernel) or more (the per-lane
    fetch macro_kernel); every output against oracle_fast"""
    import torch
    n_seq = 3000
    ps = workloads.config4_rb_set(n_seq, 60)
    ops = ps.words[:, 3] >> 28
    strobes = np.add.reduceat(((ops == isa.OP_PULSE_TRIG) | (ops == isa.OP_PULSE_RESET)).astype(np.int64),
                              ps.offsets.astype(np.int64))
    cfg = _abi.make_config(2, n_groups=n_seq, shots_per_group=spg, max_cycles=1 << 20,
                           event_cap=int(strobes.max()) + 1, meas_cap=2, meas_latency=64, seed=0xBEEF, p1=0.5)
    n_shots = n_seq * spg
    emu = Emulator(0)
    try:
        emu.load(ps)
        want = ('summary', 'events', 'meas', 'regs')
        out = alloc_device_outputs(cfg, n_shots, want=want + ('hist',))
        for t in out.values():
            t.zero_()
        emu.run_device(cfg, n_shots, 0, out)
        torch.cuda.synchronize()
        assert emu.last_kernel() == kernel, emu.last_kernel()
        f = oracle.fast_run(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, 0, n_shots, threads=8,
                            want=want + ('hist',))
        for k in want:
            a = out[k].cpu().numpy().view(f[k].dtype)
            assert np.array_equal(a, f[k]), (spg, k, int((a != f[k]).sum()))
        assert np.array_equal(out['hist'].cpu().numpy().view(f['hist'].dtype).reshape(f['hist'].shape), f['hist'])
    finally:
        emu.close()
