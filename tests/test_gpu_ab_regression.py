"""Regression case for the round-2 hipErrorIllegalAddress seen during a
same-process A/B of config 2 in shot-major lane order.

The shape of that run: scripts/ab.py's `ramsey` workload (8-core Ramsey, 100
delay points, 10^6 shots, event_cap 8, meas_cap 2) with
DPEMU_LANES_SHOT_MAJOR, two libdpemu.so builds loaded into one process (two
contexts), one shared set of device output buffers, runs interleaved A B B A
with the histogram zeroed between them and kernel timing on.  Here both
"builds" are copies of the in-tree library at different paths, so each has its
own code objects and context, exactly as in the A/B; every output of every
run must equal oracle_fast over the same 10^6 shots, and the library must
reject a config whose lane order it does not know.
"""

import os
import shutil

import numpy as np
import pytest

import oracle
from distributed_processor_amd import _abi, _native, workloads
from distributed_processor_amd.emulator import Emulator, ProgramSet, alloc_device_outputs

pytestmark = pytest.mark.gpu

THREADS = int(os.environ.get('OMP_NUM_THREADS', '0') or 0) or min(16, os.cpu_count() or 1)
WANT = ('summary', 'events', 'meas', 'hist')


def test_two_libraries_shot_major_ramsey(tmp_path):
    import torch
    lib_b = str(tmp_path / 'libdpemu_b.so')
    shutil.copy(_native.LIB_PATH, lib_b)
    ps = ProgramSet(workloads.config2_ramsey(n_cores=8, n_points=100))
    cfg = _abi.make_config(8, n_groups=100, max_cycles=1 << 20, event_cap=8, meas_cap=2, seed=0x5EED,
                           lane_order=_abi.LANES_SHOT_MAJOR)
    n = 10 ** 6
    emus = [Emulator(0), Emulator(0, lib_path=lib_b)]
    try:
        for e in emus:
            e.load(ps)
        out = alloc_device_outputs(cfg, n, want=WANT)
        for t in out.values():
            t.zero_()
        ref = oracle.fast_run(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, 0, n, threads=THREADS, want=WANT)
        for i in (0, 1, 1, 0):
            for flags in (0, _abi.X_PROG_MAJOR):
                cfg.exec_flags = flags
                emus[i].kernel_timing(True)
                for _ in range(2):
                    out['hist'].zero_()
                    emus[i].run_device(cfg, n, 0, out)
                torch.cuda.synchronize()
                assert len(emus[i].kernel_times()) == 2
                emus[i].kernel_timing(False)
                assert emus[i].last_kernel().startswith('straight_kernel'), emus[i].last_kernel()
                for k in WANT:
                    a = out[k].cpu().numpy().view(ref[k].dtype).reshape(ref[k].shape)
                    assert np.array_equal(a, ref[k]), 'library {} flags {:#x}: {} differs'.format(i, flags, k)
    finally:
        for e in emus:
            e.close()
