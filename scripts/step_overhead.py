"""Diagnostic: where the config-2 bench step's time beyond the kernel goes.
Interleaved variants of the bench step (hist zero + interpreter launch):
kernel timing on / off, and (diagnostic only, not a valid step) no zeroing.

    python scripts/step_overhead.py [steps] [rounds]
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from distributed_processor_amd import _abi  # noqa: E402
from distributed_processor_amd.emulator import Emulator, alloc_device_outputs  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    ps = bench.build_workload()
    emu = Emulator(0)
    emu.load(ps)
    n = 10 ** 6
    cfg = _abi.make_config(8, n_groups=ps.n_groups, shots_per_group=1, max_cycles=1 << 20, event_cap=8,
                           trace_cap=0, meas_cap=2, meas_latency=64, seed=0x5EED, p1=0.5)
    out = alloc_device_outputs(cfg, n, want=('summary', 'ev_main', 'ev_amp', 'meas', 'hist'))
    stream = torch.cuda.current_stream()

    def run(timing, zero):
        emu.kernel_timing(timing)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            if zero:
                out['hist'].zero_()
            emu.run_device(cfg, n, 0, out, stream)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps * 1e3
        emu.kernel_timing(False)
        kt = emu.kernel_times()
        return dt, (float(np.mean(kt)) if len(kt) else None)

    for _ in range(5):
        run(False, True)
    res = {}
    for r in range(rounds):
        for name, timing, zero in (('timing_on', True, True), ('timing_off', False, True),
                                   ('timing_off_nozero_diag', False, False)):
            res.setdefault(name, []).append(run(timing, zero))
    print(json.dumps(res))


if __name__ == '__main__':
    main()
