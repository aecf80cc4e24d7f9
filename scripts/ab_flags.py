"""Interleaved A/B of DPEMU_X_* execution flags on the interpreter workloads,
in ONE process, checking that every flag set produces identical outputs.
usage: python scripts/ab_flags.py [rounds] [steps]"""
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
X = _abi
FLAGS = {'default': 0, 'gm': X.X_GROUP_MAJOR, 'gm_lds': X.X_GROUP_MAJOR | X.X_PROG_LDS,
         'lds': X.X_PROG_LDS, 'progmajor': X.X_PROG_MAJOR, 'general': X.X_GENERAL}
ramsey = ProgramSet(workloads.config2_ramsey(8, 100))
rb = ProgramSet(workloads.config4_rb(n_seq=1000, depth=200, n_cores=2))
rst = ProgramSet(workloads.config3_active_reset(8))
lin = ProgramSet(workloads.config1_linear())
cases = {
    'ramsey': (ramsey, 10 ** 6, dict(n_groups=100), OUT, ('default', 'general', 'progmajor')),
    'ramsey_summary_only': (ramsey, 10 ** 6, dict(n_groups=100), ('summary',), ('default', 'general')),
    'config1_linear_8e6': (lin, 8 * 10 ** 6, dict(), OUT, ('default', 'lds')),
    'config3_reset': (rst, 10 ** 6, dict(meas_latency=workloads.CONFIG3_MEAS_LATENCY, max_cycles=1 << 16,
                                         event_cap=16, meas_cap=4), OUT, ('default', 'lds', 'progmajor')),
    'config4_rb_2core': (rb, 10 ** 5, dict(n_groups=1000, shots_per_group=100, event_cap=512, meas_cap=4), OUT,
                         ('default', 'lds', 'progmajor')),
    'config4_rb_2core_summary': (rb, 10 ** 5, dict(n_groups=1000, shots_per_group=100, event_cap=512, meas_cap=4),
                                 ('summary',), ('default', 'progmajor')),
}
emu = Emulator(0)
stream = torch.cuda.current_stream()
times = {}
for r in range(rounds):
    for c, (ps, n, kw, want, flags) in cases.items():
        emu.load(ps)
        ref = None
        for fl in flags:
            k = dict(kw)
            k.setdefault('max_cycles', 1 << 20)
            k.setdefault('event_cap', 8)
            k.setdefault('meas_cap', 2)
            cfg = _abi.make_config(ps.cores_per_shot, exec_flags=FLAGS[fl], **k)
            out = alloc_device_outputs(cfg, n, want)
            for v in out.values():
                v.zero_()
            emu.run_device(cfg, n, 0, out, stream)
            torch.cuda.synchronize()
            got = {kk: v.cpu() for kk, v in out.items()}
            if ref is None:
                ref = got
            for kk in got:
                assert torch.equal(ref[kk], got[kk]), '{}: {} {} differs'.format(c, fl, kk)
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
            for a, b in ev:
                a.record(stream)
                emu.run_device(cfg, n, 0, out, stream)
                b.record(stream)
            torch.cuda.synchronize()
            times.setdefault((c, fl), []).extend(a.elapsed_time(b) for a, b in ev)
            del out
res = {'{}/{}'.format(c, f): round(float(np.median(v)), 4) for (c, f), v in times.items()}
print(json.dumps(res, indent=1))
