"""Run one interpreter workload a few times (profiling driver).
usage: python scripts/prof_interp.py [config2|config3|config4] [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_processor_amd import _abi, workloads  # noqa: E402
from distributed_processor_amd.emulator import Emulator, ProgramSet, alloc_device_outputs  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else 'config2'
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
OUT = ('summary', 'ev_main', 'ev_amp', 'meas', 'hist')
if which == 'config2':
    ps, n = ProgramSet(workloads.config2_ramsey(8, 100)), 10 ** 6
    cfg = _abi.make_config(8, n_groups=100, event_cap=8, meas_cap=2)
elif which == 'config3':
    ps, n = ProgramSet(workloads.config3_active_reset(8)), 10 ** 6
    cfg = _abi.make_config(8, meas_latency=workloads.CONFIG3_MEAS_LATENCY, max_cycles=1 << 16, event_cap=16,
                           meas_cap=4)
else:
    ps, n = ProgramSet(workloads.config4_rb(n_seq=1000, depth=200, n_cores=2)), 10 ** 5
    cfg = _abi.make_config(2, n_groups=1000, shots_per_group=100, event_cap=512, meas_cap=4)
emu = Emulator(0)
emu.load(ps)
out = alloc_device_outputs(cfg, n, OUT)
for _ in range(reps):
    emu.run_device(cfg, n, 0, out)
torch.cuda.synchronize()
print('ok', which, n)
