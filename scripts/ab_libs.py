"""Interleaved A/B of two libdpemu builds (the in-tree one and
distributed_processor_amd/libdpemu_ab.so) on the interpreter workloads, in ONE
process, checking that both produce identical summaries.
usage: python scripts/ab_libs.py [rounds] [steps]"""
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
ramsey = ProgramSet(workloads.config2_ramsey(8, 100))
rb = ProgramSet(workloads.config4_rb(n_seq=1000, depth=200, n_cores=2))
rst = ProgramSet(workloads.config3_active_reset(8))
cases = {
    'ramsey': (ramsey, 10 ** 6, dict(n_groups=100), OUT),
    'ramsey_progmajor': (ramsey, 10 ** 6, dict(n_groups=100, exec_flags=_abi.X_PROG_MAJOR), OUT),
    'ramsey_summary_only': (ramsey, 10 ** 6, dict(n_groups=100), ('summary',)),
    'config3_reset': (rst, 10 ** 6, dict(meas_latency=workloads.CONFIG3_MEAS_LATENCY, max_cycles=1 << 16,
                                         event_cap=16, meas_cap=4), OUT),
    'config4_rb_2core': (rb, 10 ** 5, dict(n_groups=1000, shots_per_group=100, event_cap=512, meas_cap=4), OUT),
    'config4_rb_summary': (rb, 10 ** 5, dict(n_groups=1000, shots_per_group=100, event_cap=512, meas_cap=4),
                           ('summary',)),
    'config4_rb_1e6': (rb, 10 ** 6, dict(n_groups=1000, shots_per_group=1000, event_cap=512, meas_cap=4),
                       ('summary', 'meas', 'hist')),
}
libs = {'new': Emulator(0), 'old': Emulator(0, lib_path=os.path.join(REPO, 'distributed_processor_amd',
                                                                     'libdpemu_ab.so'))}
stream = torch.cuda.current_stream()
times = {(c, l): [] for c in cases for l in libs}
for r in range(rounds):
    for c, (ps, n, kw, want) in cases.items():
        kw = dict(kw)
        kw.setdefault('max_cycles', 1 << 20)
        kw.setdefault('event_cap', 8)
        kw.setdefault('meas_cap', 2)
        cfg = _abi.make_config(ps.cores_per_shot, **kw)
        out = alloc_device_outputs(cfg, n, want)
        ref = None
        for name, emu in libs.items():
            emu.load(ps)
            emu.run_device(cfg, n, 0, out, stream)
            torch.cuda.synchronize()
            s = out['summary'][::977].cpu()
            if ref is None:
                ref = s
            assert torch.equal(ref, s), '{}: {} differs'.format(c, name)
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
            for a, b in ev:
                a.record(stream)
                emu.run_device(cfg, n, 0, out, stream)
                b.record(stream)
            torch.cuda.synchronize()
            times[(c, name)] += [a.elapsed_time(b) for a, b in ev]
        del out
res = {'{}/{}'.format(c, l): round(float(np.median(v)), 4) for (c, l), v in times.items()}
print(json.dumps(res, indent=1))
