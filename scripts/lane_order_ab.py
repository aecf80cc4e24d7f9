"""Kernel time of configs 2, 3 and 4 in core-major and in shot-major lane
order (dpemu_config.lane_order), same library, interleaved, median of the
library's HIP-event pairs around the kernel.  One JSON line."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from distributed_processor_amd import _abi, workloads
    from distributed_processor_amd.emulator import Emulator, ProgramSet, alloc_device_outputs
    work = {
        'ramsey': (lambda: ProgramSet(workloads.config2_ramsey(8, 100)), 8, 10 ** 6,
                   dict(max_cycles=1 << 20, event_cap=8, meas_cap=2, meas_latency=64, p1=0.5)),
        'active_reset': (lambda: ProgramSet(workloads.config3_active_reset(8)), 8, 1250000,
                         dict(max_cycles=50000, event_cap=16, meas_cap=4, meas_latency=workloads.CONFIG3_MEAS_LATENCY,
                              p1=0.5)),
        'rb': (lambda: workloads.config4_rb_set(100000, 200), 2, 10 ** 6,
               dict(shots_per_group=10, max_cycles=1 << 20, event_cap=434, meas_cap=2)),
    }
    only = sys.argv[1:] or list(work)
    res = {}
    with Emulator(0) as emu:
        for name in only:
            mk, C, n, kw = work[name]
            ps = mk()
            emu.load(ps)
            cfgs = {o: _abi.make_config(C, n_groups=ps.n_groups, seed=0x5EED, hist_assign=True, lane_order=o, **kw)
                    for o in (_abi.LANES_CORE_MAJOR, _abi.LANES_SHOT_MAJOR)}
            out = alloc_device_outputs(cfgs[0], n, want=('summary', 'events', 'meas', 'hist'))
            times = {o: [] for o in cfgs}
            steps = 3 if name == 'rb' else 10
            for rep in range(4):
                for o, cfg in cfgs.items():
                    for _ in range(2):
                        emu.run_device(cfg, n, 0, out)
                    torch.cuda.synchronize()
                    emu.kernel_times()
                    emu.kernel_timing(True)
                    for _ in range(steps):
                        emu.run_device(cfg, n, 0, out)
                    torch.cuda.synchronize()
                    kt = emu.kernel_times()
                    emu.kernel_timing(False)
                    if rep:
                        times[o] += kt
            res[name] = {'core_major_ms': float(np.median(times[0])), 'shot_major_ms': float(np.median(times[1])),
                         'kernel': emu.last_kernel()}
            del out
            torch.cuda.empty_cache()
    print(json.dumps(res))


if __name__ == '__main__':
    main()
