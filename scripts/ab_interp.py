"""Interleaved A/B timing of interpreter variants in ONE process (guide §5.4 rule 24).
usage: python scripts/ab_interp.py [rounds] [steps]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_processor_amd import _abi, workloads  # noqa: E402
from distributed_processor_amd.emulator import Emulator, ProgramSet, alloc_device_outputs  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
N = 10 ** 6
ramsey = ProgramSet(workloads.config2_ramsey(8, 100))
lin = ProgramSet(workloads.config1_linear())
rst = ProgramSet(workloads.config3_active_reset(8))
OUT = ('summary', 'ev_main', 'ev_amp', 'meas', 'hist')
variants = {
    'ramsey': (ramsey, dict(n_groups=100), OUT),
    'ramsey_nohist': (ramsey, dict(n_groups=100), OUT[:-1]),
    'ramsey_summary_only': (ramsey, dict(n_groups=100), ('summary',)),
    'config1_linear_8e6': (lin, dict(), OUT),
    'config3_reset': (rst, dict(meas_latency=workloads.CONFIG3_MEAS_LATENCY, max_cycles=1 << 16, event_cap=16,
                                meas_cap=4), OUT),
}
emu = Emulator(0)
stream = torch.cuda.current_stream()
times = {k: [] for k in variants}
for r in range(rounds):
    for k, (ps, kw, want) in variants.items():
        emu.load(ps)
        kw = dict(kw)
        kw.setdefault('max_cycles', 1 << 20)
        kw.setdefault('event_cap', 8)
        kw.setdefault('meas_cap', 2)
        cfg = _abi.make_config(ps.cores_per_shot, **kw)
        n = N * 8 // ps.cores_per_shot                  # 8e6 lanes in every variant
        out = alloc_device_outputs(cfg, n, want)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        for a, b in ev:
            a.record(stream)
            emu.run_device(cfg, n, 0, out, stream)
            b.record(stream)
        torch.cuda.synchronize()
        times[k] += [a.elapsed_time(b) for a, b in ev]
        del out
res = {k: {'median_ms': round(float(np.median(v)), 4), 'min_ms': round(float(np.min(v)), 4)}
       for k, v in times.items()}
print(json.dumps(res, indent=1))
