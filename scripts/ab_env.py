"""Interleaved A/B of environment knobs (DPEMU_FETCH_BATCH, DPEMU_LINEAR, ...)
read at each launch, in ONE process, checking identical outputs.
usage: python scripts/ab_env.py [rounds] [steps]"""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from distributed_processor_amd import _abi, workloads  # noqa: E402
from distributed_processor_amd.emulator import Emulator, ProgramSet, alloc_device_outputs  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
OUT = ('summary', 'ev_main', 'ev_amp', 'meas', 'hist')
KNOBS = {'auto': {}, 'fb4': {'DPEMU_FETCH_BATCH': '4'}, 'fb1': {'DPEMU_FETCH_BATCH': '1'},
         'general': {'DPEMU_LINEAR': '0'}, 'linear': {'DPEMU_LINEAR': '1'},
         'sum_lane': {'DPEMU_SUMMARY_WAVE': '0'}, 'general_sum_lane': {'DPEMU_LINEAR': '0', 'DPEMU_SUMMARY_WAVE': '0'}}
ramsey = ProgramSet(workloads.config2_ramsey(8, 100))
rb = ProgramSet(workloads.config4_rb(n_seq=1000, depth=200, n_cores=2))
cases = {
    'ramsey': (ramsey, 10 ** 6, dict(n_groups=100), OUT, ('auto', 'sum_lane')),
    'ramsey_summary_only': (ramsey, 10 ** 6, dict(n_groups=100), ('summary',), ('auto', 'sum_lane')),
    'config3_reset': (ProgramSet(workloads.config3_active_reset(8)), 10 ** 6,
                      dict(meas_latency=workloads.CONFIG3_MEAS_LATENCY, max_cycles=1 << 16, event_cap=16,
                           meas_cap=4), OUT, ('auto', 'sum_lane')),

}
emu = Emulator(0)
stream = torch.cuda.current_stream()
times = {}
for r in range(rounds):
    for c, (ps, n, kw, want, knobs) in cases.items():
        emu.load(ps)
        ref = None
        k = dict(kw)
        k.setdefault('max_cycles', 1 << 20)
        k.setdefault('event_cap', 8)
        k.setdefault('meas_cap', 2)
        cfg = _abi.make_config(ps.cores_per_shot, **k)
        for kn in knobs:
            for var in ('DPEMU_FETCH_BATCH', 'DPEMU_LINEAR', 'DPEMU_SUMMARY_WAVE'):
                os.environ.pop(var, None)
            os.environ.update(KNOBS[kn])
            out = alloc_device_outputs(cfg, n, want)
            for v in out.values():
                v.zero_()
            emu.run_device(cfg, n, 0, out, stream)
            torch.cuda.synchronize()
            got = {kk: v.cpu() for kk, v in out.items()}
            if ref is None:
                ref = got
            for kk in got:
                assert torch.equal(ref[kk], got[kk]), '{}: {} {} differs'.format(c, kn, kk)
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
            for a, b in ev:
                a.record(stream)
                emu.run_device(cfg, n, 0, out, stream)
                b.record(stream)
            torch.cuda.synchronize()
            times.setdefault((c, kn), []).extend(a.elapsed_time(b) for a, b in ev)
            del out
res = {'{}/{}'.format(c, f): round(float(np.median(v)), 4) for (c, f), v in times.items()}
print(json.dumps(res, indent=1))
