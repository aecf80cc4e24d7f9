"""sharding.HistogramPipeline on CUDA tensors with the real kernel (bench.py's
batch loop): every batch's histogram must be that batch alone, whatever the
asynchronous exchange and the buffer reuse overlap."""

import numpy as np
import pytest

import oracle
from distributed_processor_amd import _abi, sharding, workloads
from distributed_processor_amd.emulator import Emulator, ProgramSet, alloc_device_outputs

pytestmark = pytest.mark.gpu


def test_pipeline_zero_ahead_elementwise():
    import torch
    h = torch.zeros(4, dtype=torch.int64, device='cuda')
    pipe = sharding.HistogramPipeline(h)
    n = len(pipe.bufs)
    for b in range(7):
        pipe.step(lambda t, b=b: t.add_(b + 1))
    pipe.drain()
    assert pipe.result().tolist() == [7] * 4
    assert pipe.bufs[(7 - 2) % n].tolist() == [6] * 4


def test_pipeline_with_interpreter_batches():
    import torch
    ps = ProgramSet(workloads.config2_ramsey(n_cores=8, n_points=100))
    cfg = _abi.make_config(8, n_groups=ps.n_groups, max_cycles=1 << 20, event_cap=8, meas_cap=2,
                           meas_latency=64, seed=0x5EED, p1=0.5)
    n, batches = 20000, 6
    with Emulator(0) as emu:
        emu.load(ps)
        out = alloc_device_outputs(cfg, n, want=('summary', 'hist'))
        pipe = sharding.HistogramPipeline(out['hist'])
        for b in range(batches):
            def launch(h, b=b):
                out['hist'] = h
                emu.run_device(cfg, n, b * n, out)
            pipe.step(launch)
        pipe.drain()
        torch.cuda.synchronize()
        got = [pipe.bufs[(batches - 1 - j) % len(pipe.bufs)].cpu().numpy() for j in (1, 0)]
    for j, b in enumerate((batches - 2, batches - 1)):
        ref = oracle.fast_run(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, b * n, n, want=('hist',))['hist']
        np.testing.assert_array_equal(got[j], ref.astype(np.int64))


@pytest.mark.parametrize('flags', [_abi.X_HIST_REPL, _abi.X_HIST_DIRECT])
def test_hist_assign_and_replica_rezero(flags):
    """hist_assign = 1 writes the run's histogram over whatever the buffer
    held; accumulate runs after it add exactly one run each (the replicas the
    reduce kernel read are zero again); both histogram strategies"""
    import torch
    ps = ProgramSet(workloads.config2_ramsey(n_cores=8, n_points=100))
    kw = dict(n_groups=ps.n_groups, max_cycles=1 << 20, event_cap=8, meas_cap=2, meas_latency=64, seed=0x5EED,
              p1=0.5, exec_flags=flags)
    add, assign = _abi.make_config(8, **kw), _abi.make_config(8, hist_assign=True, **kw)
    n = 30000
    ref = [oracle.fast_run(add, ps.words, ps.offsets, ps.n_instr, ps.table, s, n, want=('hist',))['hist'].astype(np.int64)
           for s in (0, n)]
    with Emulator(0) as emu:
        emu.load(ps)
        out = alloc_device_outputs(add, n, want=('hist',))
        out['hist'].fill_(12345)
        emu.run_device(assign, n, 0, out)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(out['hist'].cpu().numpy(), ref[0])
        emu.run_device(add, n, n, out)
        emu.run_device(add, n, 0, out)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(out['hist'].cpu().numpy(), 2 * ref[0] + ref[1])
        emu.run_device(assign, n, n, out)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(out['hist'].cpu().numpy(), ref[1])


def test_pipeline_without_zeroing_on_assign():
    """bench.py's pipeline: no zeroing launch, every batch's histogram is that
    batch alone because each run assigns it"""
    import torch
    ps = ProgramSet(workloads.config2_ramsey(n_cores=8, n_points=100))
    cfg = _abi.make_config(8, n_groups=ps.n_groups, max_cycles=1 << 20, event_cap=8, meas_cap=2,
                           meas_latency=64, seed=0x5EED, p1=0.5, hist_assign=True)
    n, batches = 20000, 5
    with Emulator(0) as emu:
        emu.load(ps)
        out = alloc_device_outputs(cfg, n, want=('summary', 'hist'))
        pipe = sharding.HistogramPipeline(out['hist'], zero=False)
        for b in range(batches):
            def launch(h, b=b):
                out['hist'] = h
                emu.run_device(cfg, n, b * n, out)
            pipe.step(launch)
        pipe.drain()
        torch.cuda.synchronize()
        got = pipe.result().cpu().numpy()
    ref = oracle.fast_run(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, (batches - 1) * n, n, want=('hist',))['hist']
    np.testing.assert_array_equal(got, ref.astype(np.int64))


def _kernel_cases():
    """one workload per kernel: straight (config 2), macro (config 4),
    branch (config 3), the general interpreter (config 3, DPEMU_X_GENERAL)"""
    c3 = dict(max_cycles=50000, event_cap=16, meas_cap=4, meas_latency=workloads.CONFIG3_MEAS_LATENCY, p1=0.5)
    return {
        'straight': (ProgramSet(workloads.config2_ramsey(8, 100)), dict(max_cycles=1 << 20, event_cap=8, meas_cap=2)),
        'macro': (workloads.config4_rb_set(64, 40), dict(shots_per_group=10, max_cycles=1 << 20, event_cap=128,
                                                         meas_cap=2)),
        'branch': (ProgramSet(workloads.config3_active_reset(8)), c3),
        'interp': (ProgramSet(workloads.config3_active_reset(8)), dict(c3, exec_flags=_abi.X_GENERAL)),
    }


@pytest.mark.parametrize('kernel', ['straight', 'macro', 'branch', 'interp'])
@pytest.mark.parametrize('hist_flags', [_abi.X_HIST_DIRECT, _abi.X_HIST_REPL])
def test_hist_next_cleared_by_every_kernel(kernel, hist_flags):
    """dpemu_outputs.hist_next: the run zeroes it whatever it held (every
    kernel, both histogram strategies, a grid smaller than the buffer) and
    its own histogram is unchanged"""
    import torch
    ps, kw = _kernel_cases()[kernel]
    kw = dict(kw)
    kw['exec_flags'] = kw.get('exec_flags', 0) | hist_flags
    C = ps.cores_per_shot
    cfg = _abi.make_config(C, n_groups=ps.n_groups, seed=0x5EED, **kw)
    with Emulator(0) as emu:
        emu.load(ps)
        for n in (3, 2000):
            out = alloc_device_outputs(cfg, n, want=('summary', 'events', 'meas', 'hist', 'hist_next'))
            out['hist_next'].fill_(0x5A5A5A5A)
            emu.run_device(cfg, n, 7, out)
            torch.cuda.synchronize()
            assert not out['hist_next'].any(), (kernel, n)
            ref = oracle.fast_run(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, 7, n, want=('hist',))['hist']
            np.testing.assert_array_equal(out['hist'].cpu().numpy(), ref.astype(np.int64))


def test_hist_next_contract_edges():
    """an empty run still clears hist_next; an overlapping hist_next and a
    host run with one are rejected"""
    import ctypes as C
    import torch
    from distributed_processor_amd._native import DpemuError
    ps = ProgramSet(workloads.config2_ramsey(8, 100))
    cfg = _abi.make_config(8, n_groups=ps.n_groups, event_cap=8, meas_cap=2)
    with Emulator(0) as emu:
        emu.load(ps)
        out = alloc_device_outputs(cfg, 0, want=('hist', 'hist_next'))
        out['hist_next'].fill_(9)
        emu.run_device(cfg, 0, 0, out)
        torch.cuda.synchronize()
        assert not out['hist_next'].any()
        big = torch.zeros((2,) + tuple(out['hist'].shape), dtype=torch.int64, device='cuda')
        flat = big.view(-1)
        half = out['hist'].numel() // 2
        with pytest.raises(DpemuError):
            emu.run_device(cfg, 10, 0, {'hist': big[0], 'hist_next': flat[half:half + out['hist'].numel()]
                                        .view(out['hist'].shape)})
        host = _abi.alloc_host_outputs(cfg, 4, ('summary', 'hist'))
        o = _abi.outputs_struct(host)
        nxt = np.zeros_like(host['hist'])
        o.hist_next = nxt.ctypes.data
        rc = emu._L.dpemu_run_host(emu._h, C.addressof(cfg), 0, 4, C.addressof(o))
        assert rc != 0


@pytest.mark.parametrize('hist_flags', [_abi.X_HIST_DIRECT, _abi.X_HIST_REPL])
def test_pipeline_clear_next_batches(hist_flags):
    """bench.py's config-2 loop: three buffers, each run accumulating into
    the buffer the previous run's kernel zeroed -- no zeroing launch -- and
    every batch's histogram that batch alone"""
    import torch
    ps = ProgramSet(workloads.config2_ramsey(n_cores=8, n_points=100))
    cfg = _abi.make_config(8, n_groups=ps.n_groups, max_cycles=1 << 20, event_cap=8, meas_cap=2,
                           meas_latency=64, seed=0x5EED, p1=0.5, exec_flags=hist_flags,
                           lane_order=_abi.LANES_SHOT_MAJOR)
    n, batches = 20000, 7
    with Emulator(0) as emu:
        emu.load(ps)
        out = alloc_device_outputs(cfg, n, want=('summary', 'hist'))
        out['hist'].fill_(77)                               # the pipeline zeroes batch 0's buffer
        pipe = sharding.HistogramPipeline(out['hist'], zero=False, clear_next=True)
        for b in range(batches):
            def launch(h, h_next, b=b):
                out['hist'], out['hist_next'] = h, h_next
                emu.run_device(cfg, n, b * n, out)
            pipe.step(launch)
        pipe.drain()
        torch.cuda.synchronize()
        got = [pipe.bufs[(batches - 1 - j) % 3].cpu().numpy() for j in (1, 0)]
        assert not pipe.bufs[batches % 3].any()            # the last run cleared the next batch's buffer
    for j, b in enumerate((batches - 2, batches - 1)):
        ref = oracle.fast_run(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, b * n, n, want=('hist',))['hist']
        np.testing.assert_array_equal(got[j], ref.astype(np.int64))


def test_empty_run_ordered_across_streams():
    """an empty run's hist_next clear is in call order like any other call
    (include/dpemu.h): a 10^6-shot run accumulating into H on one stream,
    then an empty run on another stream naming H as hist_next, must leave H
    zero -- the clear waits for the earlier run's counts"""
    import torch
    ps = ProgramSet(workloads.config2_ramsey(8, 100))
    cfg = _abi.make_config(8, n_groups=ps.n_groups, max_cycles=1 << 20, event_cap=8, meas_cap=2, seed=0x5EED, p1=0.5)
    a, b = torch.cuda.Stream(), torch.cuda.Stream()
    with Emulator(0) as emu:
        emu.load(ps)
        out = alloc_device_outputs(cfg, 10 ** 6, want=('summary', 'events', 'meas', 'hist'))
        H = out['hist']
        for _ in range(3):
            emu.run_device(cfg, 10 ** 6, 0, out, a)
            emu.run_device(cfg, 0, 0, {'hist_next': H}, b)
            torch.cuda.synchronize()
            assert not H.any()


@pytest.mark.parametrize('short', [0, 1, 3])
def test_load_programs_bounds_in_commands(short):
    """dpemu_load_programs' n_cmds counts 16-byte commands: a caller passing
    fewer commands than a program spans (e.g. the u32 count / 4 off by a
    few, or a truncated buffer) gets DPEMU_E_INVALID, never a read past it"""
    import ctypes as C
    ps = ProgramSet(workloads.config2_ramsey(8, 4))
    need = int((ps.offsets.astype(np.int64) + ps.n_instr).max())
    with Emulator(0) as emu:
        L = emu._L
        n = need - short
        rc = L.dpemu_load_programs(emu._h, ps.words.ctypes.data, n, ps.offsets.ctypes.data, ps.n_instr.ctypes.data,
                                   ps.n_programs, ps.table.ctypes.data, ps.n_groups, ps.cores_per_shot)
        assert (rc == 0) == (short == 0), (short, rc)
        if rc:
            assert rc == -22 and b'run past' in L.dpemu_last_error(emu._h)


@pytest.mark.parametrize('depth', [1, 2, 3])
def test_run_pipeline_batches_in_flight(depth):
    """emulator.RunPipeline (bench.py's config-4 step: batches on `depth`
    contexts and streams) with the histogram exchange pipeline: each batch's
    outputs, read on its own stream before the slot is reused, and its
    histogram equal oracle_fast over that batch's shots"""
    import torch
    from distributed_processor_amd.emulator import RunPipeline
    ps = workloads.config4_rb_set(24, 20)
    cfg = _abi.make_config(2, n_groups=ps.n_groups, shots_per_group=3, max_cycles=1 << 20, event_cap=80,
                           meas_cap=2, meas_latency=64, seed=0x5EED, p1=0.5)
    n, batches = 30, 7
    want = ('summary', 'events', 'meas', 'hist')
    with Emulator(0) as emu:
        emu.load(ps)
        rp = RunPipeline(ps, cfg, n, want=want, depth=depth, first=emu)
        hp = sharding.HistogramPipeline(rp.outputs[0]['hist'], n_buffers=max(2, depth))
        got = []
        try:
            for b in range(batches):
                with torch.cuda.stream(rp.streams[rp.k % depth]):
                    h = hp.step(lambda t, b=b: rp.launch(cfg, n, b * n, hist=t))
                    out = rp.outputs[(rp.k - 1) % depth]
                    got.append({k: (h if k == 'hist' else out[k]).clone() for k in want})
            hp.drain()
            rp.drain()
            assert rp.k == batches
        finally:
            rp.close()
    for b, g in enumerate(got):
        ref = oracle.fast_run(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, b * n, n, want=want)
        s = _abi.unpack_summary(ref['summary'])
        # the records a batch wrote (slots past a lane's count keep an earlier
        # batch's records: the output contract leaves them undefined)
        valid = {'events': np.minimum(s['n_events'], cfg.event_cap), 'meas': np.minimum(s['n_meas'], cfg.meas_cap)}
        for k in want:
            a = g[k].cpu().numpy().view(ref[k].dtype).reshape(ref[k].shape)
            r = ref[k]
            if k in valid:
                m = np.arange(r.shape[0])[:, None] < valid[k][None, :]
                a, r = a[m], r[m]
            assert np.array_equal(a, r), 'depth {} batch {}: {} differs'.format(depth, b, k)
