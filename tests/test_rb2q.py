"""CPU tests of config 4's two-qubit Clifford RB (SURVEY.md §8(d)4;
distributed_processor_amd/clifford2q.py, workloads.config4_rb2q[_set]).

* the group: 11,520 distinct elements in the classes 576 / 5184 / 5184 / 576
  (0-3 CNOTs), every decomposition's unitary is its element, the native
  CNOT is a CNOT up to phase;
* the machine code: the vectorised generator equals the per-command builder
  (ISA encoder + ElementConfig), sequences depend only on their global index;
* the physics, on the EMULATED pulse stream: oracle_fast runs the programs and
  the qdrv events it emits (phases as the processor resolved them from the
  frame registers and immediates) multiply to a diagonal unitary -- every
  sequence with its recovery Clifford returns |00> to |00>; no pulse is late.
"""

import numpy as np
import pytest

import oracle
from distributed_processor_amd import _abi, clifford2q, isa, workloads
from distributed_processor_amd.emulator import ProgramSet


def test_clifford_group():
    t = clifford2q.table()
    assert len(np.unique(t.key)) == clifford2q.N_C2
    assert np.bincount(t.n_cnot).tolist() == [576, 5184, 5184, 576]
    assert np.allclose(t.u[0], np.eye(4))
    cnot = np.array([[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 0, 1], [0, 0, 1, 0]], complex)
    assert clifford2q.keys(cnot)[0] == clifford2q.keys(clifford2q.CNOT_U)[0]
    c1 = np.stack([clifford2q.c1_u(i) for i in range(24)])
    assert len(np.unique(clifford2q.keys(np.stack([np.kron(u, np.eye(2)) for u in c1])))) == 24
    rng = np.random.default_rng(1)
    for e in rng.integers(0, clifford2q.N_C2, 200):
        u = np.eye(4, dtype=complex)
        for j, (i0, i1) in enumerate(t.layers[e]):
            if j:
                u = clifford2q.CNOT_U @ u
            u = np.kron(clifford2q.c1_u(i0), clifford2q.c1_u(i1)) @ u
        assert len(t.layers[e]) == t.n_cnot[e] + 1
        # equal up to global phase
        k = np.argmax(np.abs(u.ravel()) > 0.1)
        ph = u.ravel()[k] / t.u[e].ravel()[k]
        assert abs(abs(ph) - 1) < 1e-9 and np.allclose(u, ph * t.u[e])
    # index() inverts the table, under a global phase and rounding noise
    idx = rng.integers(0, clifford2q.N_C2, 64)
    assert np.array_equal(t.index(t.u[idx] * np.exp(1j * 0.7) + 1e-12), idx)
    with pytest.raises(ValueError):
        t.index(np.diag(np.exp(1j * np.array([0, 0.1, 0.2, 0.3]))))


def test_recovery_closes_sequences():
    t = clifford2q.table()
    el = workloads.rb2q_draws(np.arange(40), 25, 2)
    assert el.shape == (40, 2, 26)
    for s in range(40):
        for p in range(2):
            u = np.eye(4, dtype=complex)
            for e in el[s, p]:
                u = t.u[e] @ u
            assert clifford2q.keys(u)[0] == t.key[0]
    # draws are counter-based: a sequence does not depend on the batch it is drawn in
    assert np.array_equal(workloads.rb2q_draws(np.arange(5, 40), 25, 2), el[5:])
    # spread: the random layers cover the group (11,520 elements, 40 * 2 * 25 draws)
    assert len(np.unique(el[:, :, :-1])) > 1500


@pytest.mark.parametrize('n_cores,depth,chunk', [(2, 12, 4), (4, 7, 3), (8, 5, 3)])
def test_rb2q_vectorised_matches_builder(n_cores, depth, chunk):
    n_seq = 7
    ref = ProgramSet(workloads.config4_rb2q(n_seq=n_seq, depth=depth, n_cores=n_cores))
    ps = workloads.config4_rb2q_set(n_seq=n_seq, depth=depth, n_cores=n_cores, chunk=chunk)
    assert ps.n_groups == n_seq and ps.cores_per_shot == ref.cores_per_shot
    for g in range(n_seq):
        for c in range(n_cores):
            a, b = ref.program(g, c), ps.program(g, c)
            assert a.shape == b.shape and np.array_equal(a, b), (g, c)
            for x, y in zip(ref.buffers[(g, c)], ps.buffers[(g, c)]):
                assert len(x) == len(y) and all(np.array_equal(u, v) for u, v in zip(x, y))
    whole = workloads.config4_rb2q(n_seq=4, depth=depth, n_cores=n_cores)
    assert workloads.config4_rb2q(n_seq=2, depth=depth, n_cores=n_cores, first=2) == whole[2:]


def emulated_unitaries(ps, n_seq, n_cores, ev_cap):
    """oracle_fast over one shot per sequence; per (sequence, pair) the unitary
    of the qdrv pulses it emitted, in time order"""
    cfg = _abi.make_config(n_cores, n_groups=n_seq, max_cycles=1 << 22, event_cap=ev_cap, meas_cap=2)
    f = oracle.fast_run(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, 0, n_seq, want=('summary', 'events'))
    s = _abi.unpack_summary(f['summary'].view(np.uint32))
    assert (s['status'] == _abi.ST_DONE).all() and (s['flags'] == 0).all()       # nothing late, nothing dropped
    ev = f['events'].view(np.uint32).reshape(ev_cap, -1, 4)
    out = []
    for g in range(n_seq):
        for p in range(n_cores // 2):
            pulses = []
            for q in (0, 1):
                lane = (2 * p + q) * n_seq + g                                 # core-major lanes
                for k in range(int(s['n_events'][lane])):
                    t_, w1, w2, _ = (int(x) for x in ev[k, lane])
                    if (w1 >> 24) & 0xF != workloads.QDRV or w1 >> 28:        # drive triggers only
                        continue
                    phase, freq = w2 & 0x1FFFF, w2 >> 17
                    assert phase % workloads.RB_QUARTER == 0
                    pulses.append((t_, q, freq, phase // workloads.RB_QUARTER))
            u = np.eye(4, dtype=complex)
            for t_, q, freq, a in sorted(pulses, key=lambda x: (x[0], x[1])):
                if q == 0 and freq == 1:
                    g_ = clifford2q.zx90_u(a)                                  # cross resonance
                elif q == 0:
                    g_ = np.kron(clifford2q.pulse_u(a), np.eye(2))
                else:
                    g_ = np.kron(np.eye(2), clifford2q.pulse_u(a))
                u = g_ @ u
            out.append(u)
    return out, s


@pytest.mark.parametrize('n_cores,depth', [(2, 40), (4, 15)])
def test_emulated_pulses_return_to_ground(n_cores, depth):
    n_seq = 16
    ps = workloads.config4_rb2q_set(n_seq=n_seq, depth=depth, n_cores=n_cores)
    us, s = emulated_unitaries(ps, n_seq, n_cores, ev_cap=8 * depth + 16)
    for u in us:
        ph = u[0, 0]
        assert abs(abs(ph) - 1) < 1e-9                                         # |00> -> |00>
        assert np.allclose(u, np.diag(np.diag(u)))                             # only Z rotations left


def test_rb2q_program_shape():
    """depth-200 programs: ~1,300 commands per core (P ~ 10^3),
    2 registers (the VGPR register file), pulses on the stage grid, cores of a
    pair reading out together"""
    ps = workloads.config4_rb2q_set(n_seq=40, depth=200)
    assert 1000 < ps.n_instr.mean() < 1700 and ps.n_instr.max() < 2 ** 16
    for c in (0, 1):
        p = ps.program(3, c)
        ops = p[:, 3] >> 28
        assert ops[0] == isa.OP_PULSE_RESET and ops[-1] == isa.OP_DONE
        trig = p[ops == isa.OP_PULSE_TRIG]
        t = ((trig[:, 0] >> 5) | ((trig[:, 1] & 31) << 27)).astype(np.int64)
        assert (np.diff(t) > 0).all()
        assert np.isin((t[:-2] - workloads.RB2_T0) % workloads.RB2_STAGE_CLKS, (0, workloads.X90_CLKS)).all()
        if c == 0:
            t_ro0 = t[-2]
        else:
            assert t[-2] == t_ro0
    regs = set()
    for w in ps.words[:5000]:
        d = isa.decode(int(w[0]) | (int(w[1]) << 32) | (int(w[2]) << 64) | (int(w[3]) << 96))
        if d['op'] == 'reg_alu':
            regs |= {d['rd']}
    assert regs == {workloads.RB_PREG, workloads.RB_TREG}


def test_rb2q_rtl_matches_fast():
    ps = workloads.config4_rb2q_set(n_seq=6, depth=12)
    cfg = _abi.make_config(2, n_groups=6, shots_per_group=2, event_cap=120, trace_cap=300, meas_cap=2)
    f = oracle.fast_run(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, 3, 12, want=('summary',))
    r, done = oracle.rtl_run_batch(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, 3, 12, 1 << 20, 2)
    assert done == 12
    assert np.array_equal(r, f['summary'])
