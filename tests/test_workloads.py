"""CPU tests of the BASELINE workloads and of the per-clock batch baseline.

* config 4 (RB): the vectorised generator ``config4_rb_set`` emits the same
  machine code and env / freq buffers as the per-command builder
  ``config4_rb`` (which goes through the ISA encoder and ElementConfig), and a
  sequence's content depends only on its global index (sharded generation);
* ``oracle.rtl_run_batch`` (the per-clock model over many shots, the bench's
  Verilator stand-in) agrees with ``oracle.fast_run`` summary for summary on
  configs 1-4.
"""

import numpy as np
import pytest

import oracle
from distributed_processor_amd import _abi, isa, workloads
from distributed_processor_amd.emulator import ProgramSet


@pytest.mark.parametrize('n_cores,depth', [(2, 30), (1, 12), (4, 25)])
def test_rb_vectorised_matches_builder(n_cores, depth):
    ref = ProgramSet(workloads.config4_rb(n_seq=9, depth=depth, n_cores=n_cores))
    ps = workloads.config4_rb_set(n_seq=9, depth=depth, n_cores=n_cores, chunk=4)
    assert ps.n_groups == 9 and ps.cores_per_shot == ref.cores_per_shot
    for g in range(9):
        for c in range(n_cores):
            a, b = ref.program(g, c), ps.program(g, c)
            assert a.shape == b.shape and np.array_equal(a, b), (g, c)
            for x, y in zip(ref.buffers[(g, c)], ps.buffers[(g, c)]):
                assert len(x) == len(y) and all(np.array_equal(u, v) for u, v in zip(x, y))


def test_rb_sequences_are_shard_independent():
    whole = workloads.config4_rb(n_seq=6, depth=20)
    tail = workloads.config4_rb(n_seq=2, depth=20, first=4)
    assert whole[4:] == tail
    c, r = workloads.rb_draws(np.arange(10), 50, 2)
    c2, r2 = workloads.rb_draws(np.arange(5, 10), 50, 2)
    assert np.array_equal(c[5:], c2) and np.array_equal(r[5:], r2)
    assert c.min() >= 0 and c.max() < 24 and set(np.unique(r)) == {0, 1}
    # the draws are spread: every Clifford appears, CR about half the layers
    assert len(np.unique(c)) == 24 and 0.4 < r.mean() < 0.6


def test_rb_program_shape():
    """depth-200 programs: ~740 commands, pulses at the layer grid, done last"""
    ps = workloads.config4_rb_set(n_seq=50, depth=200)
    assert 600 < ps.n_instr.mean() < 900 and ps.n_instr.max() < 2 ** 16
    p = ps.program(3, 0)
    ops = p[:, 3] >> 28
    assert ops[0] == isa.OP_PULSE_RESET and ops[-1] == isa.OP_DONE
    trig = p[ops == isa.OP_PULSE_TRIG]
    t = (trig[:, 0] >> 5) | ((trig[:, 1] & 31) << 27)
    assert (np.diff(t.astype(np.int64)) > 0).all()          # cmd_times increase along the program
    assert t[-1] == workloads.RB_T0 + workloads.RB_LAYER_CLKS * 200 + workloads.RDLO_DELAY


def test_from_arrays_validates():
    w = np.zeros((4, 4), np.uint32)
    with pytest.raises(ValueError):
        ProgramSet.from_arrays(w, [0, 2], [2, 3], [0, 1], 1, 2)      # program 1 runs past the end
    with pytest.raises(ValueError):
        ProgramSet.from_arrays(w, [0], [2], [0, 1], 1, 2)            # table names program 1
    with pytest.raises(ValueError):
        ProgramSet.from_arrays(w, [0], [2], [0, 0, 0], 1, 3)         # C not a power of two


def lut_case():
    ps = ProgramSet(workloads.config3_lut(8))
    cfg = _abi.make_config(8, max_cycles=50000, event_cap=16, trace_cap=16, meas_cap=4, fproc_mode=_abi.FPROC_LUT,
                           meas_latency=workloads.CONFIG3_MEAS_LATENCY, lut_mask=0xFF,
                           lut_table=workloads.config3_lut_table(8), p1=0.5)
    return ps, cfg


def test_config3_lut_syndrome():
    """the syndrome-LUT workload on oracle_fast: every shot DONE, each core
    plays its X90 pair exactly when bit c of lut_table[outcomes] is set"""
    ps, cfg = lut_case()
    n, C = 3000, 8
    f = oracle.fast_run(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, 0, n, want=('summary',))
    s = _abi.unpack_summary(f['summary'])
    assert (s['status'] == _abi.ST_DONE).all() and (s['flags'] == 0).all()
    first = (s['meas_bits'].reshape(C, n) & 1).astype(np.int64)
    a = (first << np.arange(C)[:, None]).sum(0)
    tab = np.array(workloads.config3_lut_table(C))
    flip = (tab[a][None, :] >> np.arange(C)[:, None]) & 1
    np.testing.assert_array_equal(s['n_events'].reshape(C, n), 5 + 2 * flip)
    assert 0.4 < flip.mean() < 0.6


@pytest.mark.parametrize('name', ['config1', 'config2', 'config3', 'config4', 'config3_lut'])
def test_rtl_batch_matches_fast(name):
    if name == 'config1':
        ps = ProgramSet(workloads.config1_linear())
        cfg = _abi.make_config(1, max_cycles=10000, event_cap=8, trace_cap=8, meas_cap=4)
    elif name == 'config2':
        ps = ProgramSet(workloads.config2_ramsey(n_points=10))
        cfg = _abi.make_config(8, n_groups=10, event_cap=8, meas_cap=2)
    elif name == 'config3':
        ps = ProgramSet(workloads.config3_active_reset(8))
        cfg = _abi.make_config(8, max_cycles=50000, event_cap=16, trace_cap=16, meas_cap=4,
                               meas_latency=workloads.CONFIG3_MEAS_LATENCY)
    elif name == 'config3_lut':
        ps, cfg = lut_case()
    else:
        ps = workloads.config4_rb_set(n_seq=12, depth=40)
        cfg = _abi.make_config(2, n_groups=12, shots_per_group=3, event_cap=200, trace_cap=300, meas_cap=2)
    f = oracle.fast_run(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, 7, 36, want=('summary',))
    r, done = oracle.rtl_run_batch(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, 7, 36, 1 << 20, 2)
    assert done == 36
    assert np.array_equal(r, f['summary'])


def test_config3_cross_core_reads_oracle():
    """read_shift: core c's conditional X90 pair follows core (c + 3) % 8's first outcome (oracle_fast)"""
    import oracle
    ps = ProgramSet(workloads.config3_active_reset(8, read_shift=3))
    cfg = _abi.make_config(8, n_groups=ps.n_groups, max_cycles=50000, event_cap=16, meas_cap=4,
                           meas_latency=workloads.CONFIG3_MEAS_LATENCY, seed=11, p1=0.5,
                           lane_order=_abi.LANES_SHOT_MAJOR)
    n = 1000
    f = oracle.fast_run(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, 0, n, want=('summary',))
    s = _abi.unpack_summary(f['summary'].view(np.uint32))
    assert (s['status'] == _abi.ST_DONE).all()
    flip = np.roll((s['meas_bits'] & 1).astype(bool).reshape(n, 8), -3, axis=1)
    ne = s['n_events'].reshape(n, 8)
    assert (ne[flip] == ne[~flip].min() + 2).all() and flip.any() and (~flip).any()
