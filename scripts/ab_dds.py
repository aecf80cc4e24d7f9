"""Interleaved A/B of the DDS paths on the config-5 workload, in ONE process,
next to a pure streaming-store reference (torch fill of the same output
buffer) that measures the achievable HBM write bandwidth.
usage: python scripts/ab_dds.py [rounds] [steps] [n_seq] [elements: 01 = qdrv + rdrv, 0, 1]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_processor_amd import _abi, workloads  # noqa: E402
from distributed_processor_amd.dds import ChannelPlan  # noqa: E402
from distributed_processor_amd.emulator import Emulator, ProgramSet, alloc_device_outputs  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
n_seq = int(sys.argv[3]) if len(sys.argv) > 3 else 128
elems = tuple(int(c) for c in (sys.argv[4] if len(sys.argv) > 4 else '01'))

ps = ProgramSet(workloads.config4_rb(n_seq=n_seq, depth=200, n_cores=8))
ctx = {}
VARIANTS = [  # name, env knobs (read once, at dpemu_create)
    ('lean4_c16k', {}),
    ('lean4_c16k_b', {}),
]
KNOBS = ('DPEMU_DDS_CYC', 'DPEMU_DDS_SPT', 'DPEMU_DDS_YFORM', 'DPEMU_DDS_INDEX', 'DPEMU_DDS_SEG', 'DPEMU_DDS_SEG_CHUNK', 'DPEMU_DDS_SEG_PER_CU', 'DPEMU_DDS_PROBE', 'DPEMU_DDS_ROWS', 'DPEMU_DDS_CHUNK')
for name, knobs in VARIANTS:
    for k in KNOBS:
        os.environ.pop(k, None)
    os.environ.update(knobs)
    ctx[name] = Emulator(0)
for k in KNOBS:
    os.environ.pop(k, None)
emu = ctx[VARIANTS[0][0]]
emu.load(ps)
cfg = _abi.make_config(8, n_groups=ps.n_groups, event_cap=512, meas_cap=4)
ev = alloc_device_outputs(cfg, n_seq, want=('summary', 'ev_main', 'ev_amp'))
emu.run_device(cfg, n_seq, 0, ev)
torch.cuda.synchronize()
t_end = int(ev['summary'][:, 0].max().item())
n_samples = ((t_end + 8) * 16 + 3) // 4 * 4
params = {i: (e['samples_per_clk'], e['interp_ratio']) for i, e in enumerate(workloads.ELEMS)}
plan = ChannelPlan(ps, cfg, 0, n_seq, [(q, c, e) for q in range(n_seq) for c in range(8) for e in elems], params)
iq = torch.empty((plan.n_channels, n_samples), dtype=torch.int32, device='cuda')
ref = None
stream = torch.cuda.current_stream()
variants = {k: (lambda e=e: e.synthesize(plan, ev, n_samples, iq, stream)) for k, e in ctx.items()}
variants['store_only_fill'] = lambda: iq.fill_(0x01020304)
times = {k: [] for k in variants}
for r in range(rounds):
    for k, fn in variants.items():
        fn()
        torch.cuda.synchronize()
        if not k.startswith(('store_only', 'probe')):
            h = iq[::97].cpu()
            if ref is None:
                ref = h
            assert torch.equal(ref, h), 'variant {} differs'.format(k)
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        for a, b in evs:
            a.record(stream)
            fn()
            b.record(stream)
        torch.cuda.synchronize()
        times[k] += [a.elapsed_time(b) for a, b in evs]
nbytes = plan.n_channels * n_samples * 4
res = {k: {'median_ms': round(float(np.median(v)), 4), 'GB/s': round(nbytes / (float(np.median(v)) * 1e-3) / 1e9, 1)}
       for k, v in times.items()}
res['bytes'] = nbytes
print(json.dumps(res, indent=1))
