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
