"""HIP DDS kernel (dpemu_dds, through the C ABI) vs oracle_dds, bit for bit.

The event timelines come from the GPU interpreter (itself bit-exact against
oracle_fast, tests/test_gpu_parity.py); both DDS implementations consume the
same device-resident events, copied to the host for the oracle.  The library
ships one synthesis path (dds_index_kernel + dds_tile_kernel with its quad
sweep and generic per-sample sweep), so these tests cover exactly what ships.
"""

import numpy as np
import pytest

import oracle
from distributed_processor_amd import _abi, workloads
from distributed_processor_amd.dds import ChannelPlan, split_iq
from distributed_processor_amd.emulator import Emulator, ProgramSet, alloc_device_outputs
from distributed_processor_amd._native import DpemuError
from distributed_processor_amd.hwconfig import DDSElementConfig, pack_iq16

pytestmark = pytest.mark.gpu

ELEM_PARAMS = {i: (e['samples_per_clk'], e['interp_ratio']) for i, e in enumerate(workloads.ELEMS)}


@pytest.fixture(scope='module')
def emu():
    e = Emulator(0)
    yield e
    e.close()


def host(t):
    return t.cpu().numpy()


def check_equal(gpu_iq, ref_iq, ctx=''):
    a = np.asarray(gpu_iq).view(np.uint32)
    b = np.asarray(ref_iq).view(np.uint32)
    if not np.array_equal(a, b):
        bad = np.argwhere(a != b)
        ai, aq = split_iq(a[tuple(bad[0])])
        bi, bq = split_iq(b[tuple(bad[0])])
        raise AssertionError('{}: {} mismatching samples, first at {}: gpu ({}, {}) ref ({}, {})'.format(
            ctx, len(bad), bad[0].tolist(), ai, aq, bi, bq))


def run_and_synthesize(emu, ps, cfg, n_shots, channels, n_samples, shot0=0):
    import torch
    emu.load(ps)
    out = alloc_device_outputs(cfg, n_shots, want=('summary', 'events'))
    emu.run_device(cfg, n_shots, shot0, out)
    plan = ChannelPlan(ps, cfg, shot0, n_shots, channels, ELEM_PARAMS)
    iq = emu.synthesize(plan, out, n_samples)
    torch.cuda.synchronize()
    ref = oracle.dds(plan.desc, host(out['summary']), host(out['events']), plan.env, plan.freq, n_samples,
                     cfg.event_cap)
    return host(iq), ref


def test_config1_all_elements(emu):
    ps = ProgramSet(workloads.config1_linear())
    cfg = _abi.make_config(ps.cores_per_shot, event_cap=8, meas_cap=2)
    ch = [(s, 0, e) for s in range(3) for e in range(3)]
    g, r = run_and_synthesize(emu, ps, cfg, 3, ch, 16 * 1400)
    check_equal(g, r, 'config1')
    assert (g != 0).any()


def test_config2_ramsey_channels(emu):
    ps = ProgramSet(workloads.config2_ramsey(8, 100))
    cfg = _abi.make_config(8, n_groups=ps.n_groups, event_cap=8, meas_cap=2)
    rng = np.random.default_rng(1)
    n_shots = 300
    ch = [(int(s), int(c), int(e)) for s, c, e in zip(rng.integers(0, n_shots, 96), rng.integers(0, 8, 96),
                                                       rng.integers(0, 3, 96))]
    g, r = run_and_synthesize(emu, ps, cfg, n_shots, ch, 16 * 2048)
    check_equal(g, r, 'config2')


def test_config4_rb_virtual_z(emu):
    """RB: phase-register virtual Z, many strobes per lane (compaction over
    several 256-event blocks), pulse_reset at the start"""
    ps = ProgramSet(workloads.config4_rb(n_seq=8, depth=150, seed=3))
    cfg = _abi.make_config(ps.cores_per_shot, n_groups=ps.n_groups, event_cap=1024, meas_cap=4)
    ch = [(s, c, e) for s in range(16) for c in range(ps.cores_per_shot) for e in range(3)]
    g, r = run_and_synthesize(emu, ps, cfg, 16, ch, 16 * 8192)
    check_equal(g, r, 'config4')


def test_synthetic_edges_multi_chunk(emu):
    """spc / interp not powers of two, > one 64K-sample chunk, ragged tail,
    strobes on other elements, resets, overriding strobes, events past the
    end, empty lanes"""
    import torch
    rng = np.random.default_rng(7)
    cap, n_lanes = 40, 5
    summary = np.zeros((n_lanes, 8), np.uint32)
    ev = np.zeros((cap, n_lanes, 4), np.uint32)
    env_tab = pack_iq16(np.exp(1j * rng.uniform(0, 2 * np.pi, 4 * 64)) * rng.uniform(0, 1, 4 * 64))
    freq_tab = np.concatenate([DDSElementConfig(samples_per_clk=s).get_freq_buffer([f])
                               for s, f in ((16, 91.7e6), (3, -13.1e6), (5, 250e6), (1, 0.0))])
    for L in range(1, n_lanes):                     # lane 0 stays empty
        n = cap if L == 2 else cap - 3 * L
        t = np.sort(rng.integers(0, 30000, n)).astype(np.uint32)
        kind = (rng.random(n) < 0.15).astype(np.uint32)
        A = rng.integers(0, 60, n)
        Ln = rng.integers(0, 5, n)                  # 0 = CW
        envw = (A | (Ln << 12)).astype(np.uint32)
        cfgw = rng.integers(0, 4, n).astype(np.uint32)
        ev[:n, L, 0] = t
        ev[:n, L, 1] = envw | (cfgw << 24) | (kind << 28)
        ev[:n, L, 2] = rng.integers(0, 1 << 17, n).astype(np.uint32) | (rng.integers(0, 5, n).astype(np.uint32) << 17)
        ev[:n, L, 3] = rng.integers(0, 65536, n)
        summary[L, 2] = n + (5 if L == 2 else 0)    # lane 2 overflowed: count > cap
    ev[cap - 10:, 3, 0] = 10 ** 9                   # lane 3's last events are beyond the window
    desc = []
    for L in range(n_lanes):
        for e, (spc, interp) in enumerate(((16, 1), (3, 3), (5, 2), (1, 1))):
            desc.append((L, e, spc, interp, 0, len(env_tab), 0, len(freq_tab) if L != 4 else 20))
    desc = np.array(desc, np.uint32)
    n_samples = 2 * 65536 + 4 * 37
    ref = oracle.dds(desc, summary, ev, env_tab, freq_tab, n_samples, cap)

    dev = {'summary': torch.from_numpy(summary.view(np.int32)).cuda(),
           'events': torch.from_numpy(ev.view(np.int32)).cuda()}
    plan = ChannelPlan.__new__(ChannelPlan)
    plan.desc, plan.env, plan.freq = desc, env_tab, freq_tab
    plan.n_lanes, plan.event_cap, plan._dev = n_lanes, cap, None
    plan._cols = {f: np.ascontiguousarray(desc[:, i]) for i, f in
                  enumerate(('ch_lane', 'ch_elem', 'spc', 'interp', 'env_off', 'env_len', 'freq_off', 'freq_len'))}
    iq = emu.synthesize(plan, dev, n_samples)
    torch.cuda.synchronize()
    check_equal(host(iq), ref, 'synthetic')
    assert (ref != 0).sum() > 1000


def test_bad_arguments_fail_loudly(emu):
    ps = ProgramSet(workloads.config1_linear())
    cfg = _abi.make_config(ps.cores_per_shot, event_cap=8, meas_cap=2)
    emu.load(ps)
    out = alloc_device_outputs(cfg, 2, want=('summary', 'events'))
    emu.run_device(cfg, 2, 0, out)
    plan = ChannelPlan(ps, cfg, 0, 2, [(0, 0, 0)], ELEM_PARAMS)
    with pytest.raises(DpemuError):
        emu.synthesize(plan, out, 1002)               # not a multiple of 4
    plan.desc[0, 2] = 17
    plan._cols['spc'] = np.ascontiguousarray(plan.desc[:, 2])
    with pytest.raises(DpemuError):
        emu.synthesize(plan, out, 1024)               # spc out of range


def synthetic_timelines(rng, n_lanes, cap, n_cycles, env_len, n_freq):
    """random, time-sorted event arrays: strobes on elements 0-3 (some CW, some
    past the window), pulse_resets (some inside pulses), ragged counts, an
    overflowed lane and an empty lane"""
    summary = np.zeros((n_lanes, 8), np.uint32)
    ev = np.zeros((cap, n_lanes, 4), np.uint32)
    for L in range(1, n_lanes):                     # lane 0 stays empty
        n = cap if L == 2 else cap - 2 * L
        t = np.sort(rng.integers(0, n_cycles, n)).astype(np.uint32)
        t[-2:] = n_cycles + np.array([5, 10 ** 6], np.uint32)      # past the window
        kind = (rng.random(n) < 0.2).astype(np.uint32)
        A = rng.integers(0, env_len // 4 + 2, n)                  # some past the table end
        Ln = rng.integers(0, 6, n)                                # 0 = CW
        envw = (A | (Ln << 12)).astype(np.uint32)
        cfgw = rng.integers(0, 4, n).astype(np.uint32)
        ev[:n, L, 0] = t
        ev[:n, L, 1] = envw | (cfgw << 24) | (kind << 28)
        ev[:n, L, 2] = (rng.integers(0, 1 << 17, n).astype(np.uint32)
                        | (rng.integers(0, n_freq + 1, n).astype(np.uint32) << 17))   # n_freq: no entry
        ev[:n, L, 3] = rng.integers(0, 65536, n)
        summary[L, 2] = n + (7 if L == 2 else 0)    # lane 2 overflowed: count > cap
    return summary, ev


def plan_from(desc, env_tab, freq_tab, n_lanes, cap):
    plan = ChannelPlan.__new__(ChannelPlan)
    plan.desc, plan.env, plan.freq = desc, env_tab, freq_tab
    plan.n_lanes, plan.event_cap, plan._dev = n_lanes, cap, None
    plan._cols = {f: np.ascontiguousarray(desc[:, i]) for i, f in
                  enumerate(('ch_lane', 'ch_elem', 'spc', 'interp', 'env_off', 'env_len', 'freq_off', 'freq_len'))}
    return plan


SWEEP_CASES = {   # (samples per clock, interp) of the four elements
    'spc16': ((16, 1), (16, 3), (16, 16), (16, 2)),
    'spc_mixed': ((16, 1), (8, 3), (4, 16), (16, 2)),
    'spc8': ((8, 1), (16, 3), (8, 16), (8, 2)),
    'interp_4_8_32': ((16, 4), (8, 8), (16, 32), (8, 1)),
    'bad_words': ((16, 1), (16, 4), (8, 16), (16, 2)),
}


@pytest.mark.parametrize('case', list(SWEEP_CASES))
def test_sweep_edges(emu, case):
    """every pulse rule against oracle_dds on both sweeps: CW, pulse end
    inside a thread's samples (odd env lengths), non-power-of-two interp
    (generic sweep), resets inside pulses, odd env / freq offsets, missing
    freq entries, env words past the table, ragged tail, overflowed and empty
    lanes; 'bad_words' puts Q = -32768 into env and rotation words (no Y
    form: the workgroup takes the generic sweep)"""
    import torch
    rng = np.random.default_rng(11)
    cap, n_lanes, n_cycles = 48, 6, 9000
    env_tab = pack_iq16(np.exp(1j * rng.uniform(0, 2 * np.pi, 301)) * rng.uniform(0, 1, 301))
    freq_tab = np.concatenate([np.zeros(3, np.uint32)] + [DDSElementConfig(samples_per_clk=16).get_freq_buffer([f])
                              for f in (91.7e6, -13.1e6, 250e6)])
    if case == 'bad_words':
        env_tab[::37] = (env_tab[::37] & 0xFFFF0000) | 0x8000
        freq_tab[3 + 16 + 5] = (freq_tab[3 + 16 + 5] & 0xFFFF0000) | 0x8000
    summary, ev = synthetic_timelines(rng, n_lanes, cap, n_cycles, 280, 3)
    desc = []
    for L in range(n_lanes):
        for e, (spc, interp) in enumerate(SWEEP_CASES[case]):
            env_off = (0, 1, 5, 2)[e]                       # odd offsets: unaligned env reads
            env_len = (280, 279, 290, 301 - 2)[e]           # not multiples of 4
            desc.append((L, e, spc, interp, env_off, env_len, 3 if e % 2 else 1, len(freq_tab) - 3))
    desc = np.array(desc, np.uint32)
    n_samples = 16 * n_cycles + 4 * 37                   # ragged last tile
    ref = oracle.dds(desc, summary, ev, env_tab, freq_tab, n_samples, cap)
    dev = {'summary': torch.from_numpy(summary.view(np.int32)).cuda(),
           'events': torch.from_numpy(ev.view(np.int32)).cuda()}
    iq = emu.synthesize(plan_from(desc, env_tab, freq_tab, n_lanes, cap), dev, n_samples)
    torch.cuda.synchronize()
    check_equal(host(iq), ref, 'sweep edges ' + case)
    assert (ref != 0).sum() > 10000


def test_config5_slice(emu):
    """the bench's config-5 shape (RB timelines, qdrv + rdrv at 16 samples/clk)
    on a few sequences, full length, against oracle_dds"""
    ps = ProgramSet(workloads.config4_rb(n_seq=4, depth=200, n_cores=8))
    cfg = _abi.make_config(8, n_groups=ps.n_groups, event_cap=512, meas_cap=4)
    ch = [(q, c, e) for q in range(4) for c in range(8) for e in (workloads.QDRV, workloads.RDRV)]
    import torch
    emu.load(ps)
    out = alloc_device_outputs(cfg, 4, want=('summary', 'events'))
    emu.run_device(cfg, 4, 0, out)
    torch.cuda.synchronize()
    n_samples = ((int(out['summary'][:, 0].max().item()) + 8) * 16 + 3) // 4 * 4
    plan = ChannelPlan(ps, cfg, 0, 4, ch, ELEM_PARAMS)
    iq = emu.synthesize(plan, out, n_samples)
    torch.cuda.synchronize()
    ref = oracle.dds(plan.desc, host(out['summary']), host(out['events']), plan.env, plan.freq, n_samples,
                     cfg.event_cap, threads=8)
    check_equal(host(iq), ref, 'config5 slice')


@pytest.mark.parametrize('layout', ['same_element_pairs', 'one_broken_pair'])
def test_channel_pair_detection(emu, layout):
    """the index kernel's pair mode (channels 2i and 2i + 1 on one lane share a
    workgroup; its reset records are written for both): pairs whose two
    channels play the SAME element (with different sample rates), and an
    even channel list in which one pair breaks the shared-lane rule, so the
    host falls back to one workgroup per channel -- both against oracle_dds"""
    import torch
    rng = np.random.default_rng(31 if layout == 'same_element_pairs' else 37)
    cap, n_lanes, n_cycles = 96, 6, 1500
    env_tab = pack_iq16(np.exp(1j * rng.uniform(0, 2 * np.pi, 2000)) * rng.uniform(0, 1, 2000))
    freq_tab = np.concatenate([DDSElementConfig(samples_per_clk=16).get_freq_buffer([f])
                               for f in (91.7e6, -13.1e6, 250e6)])
    summary, ev = synthetic_timelines(rng, n_lanes, cap, n_cycles, 2000, 3)
    desc = []
    for L in range(n_lanes):
        e = L % 4
        desc.append((L, e, 16, 1, 0, 2000, 0, len(freq_tab)))
        desc.append((L, e if layout == 'same_element_pairs' else (e + 1) % 4, 8, 4, 0, 2000, 0, len(freq_tab)))
    if layout == 'one_broken_pair':
        desc[7] = (4,) + desc[7][1:]                    # pair 3: lanes 3 and 4 -- not one lane
    desc = np.array(desc, np.uint32)
    n_samples = 16 * n_cycles + 4 * 5
    ref = oracle.dds(desc, summary, ev, env_tab, freq_tab, n_samples, cap)
    dev = {'summary': torch.from_numpy(summary.view(np.int32)).cuda(),
           'events': torch.from_numpy(ev.view(np.int32)).cuda()}
    iq = emu.synthesize(plan_from(desc, env_tab, freq_tab, n_lanes, cap), dev, n_samples)
    torch.cuda.synchronize()
    check_equal(host(iq), ref, layout)
    assert (ref != 0).sum() > 5000


def test_global_record_fallback(emu):
    """a staged 32-KiB envelope leaves room for only DDS_REC_LDS_MIN records in
    a tile workgroup's LDS: stripes with denser windows read their strobes and
    resets from the global index, the sparse lanes of the same launch stage
    them; both against oracle_dds"""
    import torch
    rng = np.random.default_rng(23)
    cap, n_lanes, n_cycles = 320, 5, 2500
    env_tab = pack_iq16(np.exp(1j * rng.uniform(0, 2 * np.pi, 4000)) * rng.uniform(0, 1, 4000))
    freq_tab = np.concatenate([DDSElementConfig(samples_per_clk=16).get_freq_buffer([f])
                               for f in (91.7e6, -13.1e6, 250e6)])
    summary, ev = synthetic_timelines(rng, n_lanes, cap, n_cycles, 4000, 3)
    summary[4, 2] = 20                                     # a sparse lane: its stripes fit in LDS
    desc = []
    for L in range(n_lanes):
        for e, (spc, interp) in enumerate(((16, 1), (16, 4), (8, 1), (16, 3))):
            desc.append((L, e, spc, interp, 0, 4000, 0, len(freq_tab)))
    desc = np.array(desc, np.uint32)
    n_samples = 16 * n_cycles + 4 * 5
    ref = oracle.dds(desc, summary, ev, env_tab, freq_tab, n_samples, cap)
    dev = {'summary': torch.from_numpy(summary.view(np.int32)).cuda(),
           'events': torch.from_numpy(ev.view(np.int32)).cuda()}
    iq = emu.synthesize(plan_from(desc, env_tab, freq_tab, n_lanes, cap), dev, n_samples)
    torch.cuda.synchronize()
    check_equal(host(iq), ref, 'global record fallback')
    assert (ref != 0).sum() > 10000


@pytest.mark.parametrize('cap', [600, 720, 1024])
def test_dense_channels_staged(emu, cap):
    """event caps past what the 20-KiB workgroup budget holds (the two-qubit
    RB drive channels: 560-720 strobes): with a small envelope every record
    is staged under the dense budget with 24 tiles per stripe, up to the
    largest cap (DDS_MAX_EVENTS); against oracle_dds.  (A budget the records
    exceed even then: test_global_record_fallback.)"""
    import torch
    rng = np.random.default_rng(cap)
    n_lanes, n_cycles = 6, 40000
    env_tab = pack_iq16(np.exp(1j * rng.uniform(0, 2 * np.pi, 64)) * rng.uniform(0, 1, 64))
    freq_tab = np.concatenate([DDSElementConfig(samples_per_clk=16).get_freq_buffer([f])
                               for f in (91.7e6, -13.1e6, 250e6)])
    summary, ev = synthetic_timelines(rng, n_lanes, cap, n_cycles, 64, 3)
    desc = np.array([(L, e, 16, 1 + 3 * (e & 1), 0, 64, 0, len(freq_tab)) for L in range(n_lanes) for e in range(4)],
                    np.uint32)
    n_samples = 16 * n_cycles + 4 * 7
    ref = oracle.dds(desc, summary, ev, env_tab, freq_tab, n_samples, cap)
    dev = {'summary': torch.from_numpy(summary.view(np.int32)).cuda(),
           'events': torch.from_numpy(ev.view(np.int32)).cuda()}
    iq = emu.synthesize(plan_from(desc, env_tab, freq_tab, n_lanes, cap), dev, n_samples)
    torch.cuda.synchronize()
    check_equal(host(iq), ref, 'dense channels cap {}'.format(cap))
    assert (ref != 0).sum() > 100000


def test_dense_tile_raw_event_lookup(emu):
    """a 32-KiB envelope leaves the multi-pass kernel room for only
    DDS_REC_MIN (64) records of each kind; lanes with 150 strobes and 120
    resets packed into one 1,024-sample tile (repeated times: hand-built
    events, not dpemu_run's) make that tile look its records up in the raw
    events, next to tiles swept from staged records; against oracle_dds"""
    import torch
    rng = np.random.default_rng(29)
    cap, n_lanes, n_cycles = 400, 3, 1200
    env_tab = pack_iq16(np.exp(1j * rng.uniform(0, 2 * np.pi, 4000)) * rng.uniform(0, 1, 4000))
    freq_tab = np.concatenate([DDSElementConfig(samples_per_clk=16).get_freq_buffer([f])
                               for f in (91.7e6, -13.1e6, 250e6)])
    summary, ev = synthetic_timelines(rng, n_lanes, cap, n_cycles, 4000, 3)
    for L in (1, 2):
        # 270 events between cycles 300 and 340 (tile 4 at 16 samples / clk
        # holds cycles 256..319, tile 5 320..383), the rest spread after them
        n = 270
        t = np.sort(np.concatenate([300 + rng.integers(0, 20, 150), 320 + rng.integers(0, 20, 120)])).astype(np.uint32)
        kind = np.zeros(n, np.uint32)
        kind[rng.permutation(n)[:120]] = 1
        ev[:n, L, 0] = t
        ev[:n, L, 1] = (ev[:n, L, 1] & ~np.uint32(0xF3000000)) | (kind << 28)   # element 0 strobes / resets
        rest = np.sort(rng.integers(400, n_cycles, cap - n)).astype(np.uint32)
        ev[n:, L, 0] = rest
        summary[L, 2] = cap
    desc = []
    for L in range(n_lanes):
        for e, (spc, interp) in enumerate(((16, 1), (16, 4), (8, 1), (16, 3))):
            desc.append((L, e, spc, interp, 0, 4000, 0, len(freq_tab)))
    desc = np.array(desc, np.uint32)
    n_samples = 16 * n_cycles + 4 * 5
    ref = oracle.dds(desc, summary, ev, env_tab, freq_tab, n_samples, cap)
    dev = {'summary': torch.from_numpy(summary.view(np.int32)).cuda(),
           'events': torch.from_numpy(ev.view(np.int32)).cuda()}
    iq = emu.synthesize(plan_from(desc, env_tab, freq_tab, n_lanes, cap), dev, n_samples)
    torch.cuda.synchronize()
    check_equal(host(iq), ref, 'dense tile')
    assert (ref[4 * 1:4 * 3, 16 * 300:16 * 340] != 0).sum() > 1000


@pytest.mark.parametrize('depth', [2, 8])
def test_synthesis_pipeline_batches(emu, depth):
    """dds.SynthesisPipeline (`depth` contexts / streams, batch k + 1's index
    beside batch k's tiles, the bench's config-5 step at depth 8): twelve
    batches of different RB timelines, each batch's I/Q read on its returned
    stream while later batches run, every one bit for bit equal to oracle_dds"""
    import torch
    from distributed_processor_amd.dds import SynthesisPipeline
    ps = ProgramSet(workloads.config4_rb(n_seq=16, depth=12, n_cores=2))
    emu.load(ps)
    cfg = _abi.make_config(2, n_groups=ps.n_groups, max_cycles=1 << 20, event_cap=128, meas_cap=4,
                           meas_latency=64, seed=0x5EED)
    batches = []
    for b in range(12):                                 # batch b: sequences [b, b + 3) of the table
        out = alloc_device_outputs(cfg, 3, want=('summary', 'events'))
        emu.run_device(cfg, 3, b, out)
        chans = [(b + q, c, e) for q in range(3) for c in range(2) for e in (workloads.QDRV, workloads.RDRV)]
        batches.append((out, ChannelPlan(ps, cfg, b, 3, chans, ELEM_PARAMS)))
    torch.cuda.synchronize()
    n_samples = 4096
    pipe = SynthesisPipeline(0, depth=depth)
    try:
        got = []
        for out, plan in batches:
            iq, s = pipe.synthesize(plan, out, n_samples)
            with torch.cuda.stream(s):                   # consume on the batch's stream
                got.append(iq.clone())
        pipe.drain()
        assert pipe.k == 12
        for b, ((out, plan), g) in enumerate(zip(batches, got)):
            ref = oracle.dds(plan.desc, host(out['summary']), host(out['events']), plan.env, plan.freq, n_samples,
                             cfg.event_cap)
            check_equal(host(g), ref, 'batch {}'.format(b))
    finally:
        pipe.close()
    with pytest.raises(ValueError):
        SynthesisPipeline(0, depth=0)
