"""Run the config-5 DDS synthesis a few times (profiling driver).
usage: python scripts/prof_dds.py [reps] [n_seq] [n_samples or 0=full] [elements: 01, 0, 1]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_processor_amd import _abi, workloads  # noqa: E402
from distributed_processor_amd.dds import ChannelPlan  # noqa: E402
from distributed_processor_amd.emulator import Emulator, ProgramSet, alloc_device_outputs  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
n_seq = int(sys.argv[2]) if len(sys.argv) > 2 else 128
n_samp = int(sys.argv[3]) if len(sys.argv) > 3 else 0
elems = tuple(int(c) for c in (sys.argv[4] if len(sys.argv) > 4 else '01'))
ps = ProgramSet(workloads.config4_rb(n_seq=n_seq, depth=200, n_cores=8))
emu = Emulator(0)
emu.load(ps)
cfg = _abi.make_config(8, n_groups=ps.n_groups, event_cap=512, meas_cap=4)
ev = alloc_device_outputs(cfg, n_seq, want=('summary', 'ev_main', 'ev_amp'))
emu.run_device(cfg, n_seq, 0, ev)
torch.cuda.synchronize()
t_end = int(ev['summary'][:, 0].max().item())
n_samples = n_samp or ((t_end + 8) * 16 + 3) // 4 * 4
params = {i: (e['samples_per_clk'], e['interp_ratio']) for i, e in enumerate(workloads.ELEMS)}
plan = ChannelPlan(ps, cfg, 0, n_seq, [(q, c, e) for q in range(n_seq) for c in range(8) for e in elems], params)
iq = torch.empty((plan.n_channels, n_samples), dtype=torch.int32, device='cuda')
s = torch.cuda.current_stream()
for _ in range(reps):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    emu.synthesize(plan, ev, n_samples, iq, s)
    b.record(s)
    torch.cuda.synchronize()
    print('dds {} ch x {} samples: {:.4f} ms'.format(plan.n_channels, n_samples, a.elapsed_time(b)), flush=True)
