"""Per-wave start / end times of one launch (a probe build: scripts/ab_libs.sh wt
-DDPEMU_PROBE_WAVETIME), to see how full the chip is over a launch -- the
tail after the last wave is dispatched, per-XCD spans, wave durations.

    python scripts/wavetime_probe.py --lib ab_build/libdpemu_wt.so --workload rb
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

TICK_NS = 10.0   # wall_clock64: 100 MHz


def analyse(wt):
    t0, t1, hw, xcc = (wt[:, i].astype(np.int64) for i in range(4))
    live = (t1 != 0)
    t0, t1, hw, xcc = t0[live], t1[live], hw[live], xcc[live]
    base = t0.min()
    t0, t1 = t0 - base, t1 - base
    dur = t1 - t0
    span = int(t1.max())
    ev = np.concatenate([np.stack([t0, np.ones_like(t0)], 1), np.stack([t1, -np.ones_like(t1)], 1)])
    ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
    conc = np.cumsum(ev[:, 1])
    tt = ev[:, 0]
    cmax = int(conc.max())
    dt = np.diff(tt, append=tt[-1])
    area = float((conc * dt).sum())
    last_start = int(t0.max())
    # time in which fewer than 90 % / 50 % of the peak number of waves were resident
    below90 = float(dt[conc < 0.9 * cmax].sum())
    below50 = float(dt[conc < 0.5 * cmax].sum())
    q = lambda a, x: float(np.quantile(a, x)) * TICK_NS / 1e6
    per_xcc = {}
    for x in np.unique(xcc):
        m = xcc == x
        per_xcc[int(x)] = {'waves': int(m.sum()), 'start_ms': float(t0[m].min()) * TICK_NS / 1e6,
                           'end_ms': float(t1[m].max()) * TICK_NS / 1e6}
    ends = np.sort(t1)
    return {
        'waves': int(live.sum()), 'span_ms': span * TICK_NS / 1e6, 'peak_resident_waves': cmax,
        'mean_resident_waves': area / span, 'utilisation': area / (cmax * span),
        'last_dispatch_ms': last_start * TICK_NS / 1e6, 'tail_ms': (span - last_start) * TICK_NS / 1e6,
        'below90_ms': below90 * TICK_NS / 1e6, 'below50_ms': below50 * TICK_NS / 1e6,
        'wave_ms': {'mean': float(dur.mean()) * TICK_NS / 1e6, 'p10': q(dur, 0.1), 'p50': q(dur, 0.5),
                    'p90': q(dur, 0.9), 'max': q(dur, 1.0)},
        'wave_ms_last_10pct_dispatched': float(dur[t0 >= np.quantile(t0, 0.9)].mean()) * TICK_NS / 1e6,
        'wave_ms_first_10pct_dispatched': float(dur[t0 <= np.quantile(t0, 0.1)].mean()) * TICK_NS / 1e6,
        'ends_ms_at_quantiles': {str(x): float(ends[int(x * (len(ends) - 1))]) * TICK_NS / 1e6
                                 for x in (0.5, 0.9, 0.95, 0.99, 1.0)},
        'per_xcc': per_xcc,
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--lib', required=True)
    ap.add_argument('--workload', default='rb')
    ap.add_argument('--runs', type=int, default=3)
    a = ap.parse_args()
    import torch
    from ab import workload
    from distributed_processor_amd.emulator import Emulator, alloc_device_outputs
    lib = os.path.abspath(a.lib)
    ps, cfg, n = workload(a.workload)
    e = Emulator(0, lib_path=lib)
    e.load(ps)
    probe = ctypes.CDLL(lib).dpemu_probe_wavetime
    probe.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    out = alloc_device_outputs(cfg, n, want=('summary', 'events', 'meas', 'hist'))
    res = []
    for r in range(a.runs + 1):
        assert probe(None, 0, 1) == 0
        torch.cuda.synchronize()
        e.kernel_timing(True)
        out['hist'].zero_()
        e.run_device(cfg, n, 0, out)
        torch.cuda.synchronize()
        kt = e.kernel_times()
        e.kernel_timing(False)
        wt = np.zeros((1 << 18, 4), np.uint32)
        assert probe(wt.ctypes.data, wt.nbytes, 0) == 0
        if r:
            d = analyse(wt)
            d['kernel_ms_events'] = float(kt[-1]) if kt else None
            res.append(d)
    print(json.dumps({'workload': a.workload, 'kernel': e.last_kernel(), 'runs': res}))


if __name__ == '__main__':
    main()
