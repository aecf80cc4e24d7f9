"""Where config 3's kernel time goes: the production branch_kernel timed
(HIP events around the kernel, library side) with fewer outputs requested --
all of them, without event records, without events and measurements -- so
the store-side share of a launch shows beside the compute.  One JSON line.
    python scripts/ar_probe.py [lib.so] [--shot-major]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from distributed_processor_amd import _abi, workloads
    from distributed_processor_amd.emulator import Emulator, ProgramSet, alloc_device_outputs
    ps = ProgramSet(workloads.config3_active_reset(8))
    order = _abi.LANES_SHOT_MAJOR if '--shot-major' in sys.argv else _abi.LANES_CORE_MAJOR
    cfg = _abi.make_config(8, n_groups=ps.n_groups, max_cycles=50000, event_cap=16, trace_cap=0, meas_cap=4,
                           meas_latency=workloads.CONFIG3_MEAS_LATENCY, seed=0x5EED, p1=0.5, hist_assign=True,
                           lane_order=order)
    n = 1250000
    res = {}
    args = [a for a in sys.argv[1:] if not a.startswith('--')]
    lib = args[0] if args else None
    with Emulator(0, lib_path=lib) if lib else Emulator(0) as emu:
        emu.load(ps)
        full = alloc_device_outputs(cfg, n, want=('summary', 'events', 'meas', 'hist'))
        sets = {'all': ('summary', 'events', 'meas', 'hist'), 'no_events': ('summary', 'meas', 'hist'),
                'summary_hist': ('summary', 'hist'), 'hist_only': ('hist',)}
        for rep in range(3):
            for name, want in sets.items():
                out = {k: full[k] for k in want}
                for _ in range(30):
                    emu.run_device(cfg, n, 0, out)
                torch.cuda.synchronize()
                emu.kernel_times()
                emu.kernel_timing(True)
                for _ in range(20):
                    emu.run_device(cfg, n, 0, out)
                torch.cuda.synchronize()
                kt = emu.kernel_times()
                emu.kernel_timing(False)
                if rep:
                    res.setdefault(name, []).append(float(np.median(kt)))
        res = {k: float(np.median(v)) for k, v in res.items()}
        res['kernel'] = emu.last_kernel()
        res['lane_order'] = 'shot_major' if order else 'core_major'
    print(json.dumps(res))


if __name__ == '__main__':
    main()
