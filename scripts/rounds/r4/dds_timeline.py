"""Workgroup timeline of dds_tile_kernel (diagnostic builds with
-DDDS_PROBE_TIMES, scripts/ab_libs.sh): every workgroup's start / end
(s_memrealtime, 100 MHz), CU and XCD, on the config-5 synthesis.  Reports per
build: kernel span, workgroup durations by channel element, resident
workgroups over time (mean / max, the time below 90 % of the max at the start
and the end = ramp and tail).  One JSON line per library.

    python scripts/dds_timeline.py --libs ab_build/libdpemu_ddsS7t.so,ab_build/libdpemu_ddsX7t.so
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--libs', required=True)
    ap.add_argument('--seqs', type=int, default=128)
    ap.add_argument('--reps', type=int, default=5)
    a = ap.parse_args()
    import torch
    from distributed_processor_amd import _abi, workloads
    from distributed_processor_amd.dds import ChannelPlan
    from distributed_processor_amd.emulator import Emulator, ProgramSet, alloc_device_outputs
    libs = [os.path.abspath(x) for x in a.libs.split(',')]
    emus = [Emulator(0, lib_path=l) for l in libs]
    ps = ProgramSet(workloads.config4_rb(n_seq=a.seqs, depth=200, n_cores=8))
    cfg = _abi.make_config(8, n_groups=ps.n_groups, max_cycles=1 << 20, event_cap=512, meas_cap=4,
                           meas_latency=64, seed=0x5EED)
    emus[0].load(ps)
    ev = alloc_device_outputs(cfg, a.seqs, want=('summary', 'events'))
    emus[0].run_device(cfg, a.seqs, 0, ev)
    torch.cuda.synchronize()
    s = _abi.unpack_summary(ev['summary'].cpu().numpy().view(np.uint32))
    n_samples = ((int(s['t_end'].max()) + 8) * 16 + 3) // 4 * 4
    params = {i: (e['samples_per_clk'], e['interp_ratio']) for i, e in enumerate(workloads.ELEMS)}
    chans = [(q, c, e) for q in range(a.seqs) for c in range(8) for e in (workloads.QDRV, workloads.RDRV)]
    plan = ChannelPlan(ps, cfg, 0, a.seqs, chans, params)
    iq = torch.empty((plan.n_channels, n_samples), dtype=torch.int32, device='cuda')
    elem = plan.desc[:, 1]
    for lib, e in zip(libs, emus):
        L = e._L
        L.dpemu_probe_dds_times.restype = C.c_uint64
        L.dpemu_probe_dds_times.argtypes = [C.c_void_p, C.c_uint64]
        runs = []
        for r in range(a.reps + 1):
            e.synthesize(plan, ev, n_samples, iq)
            torch.cuda.synchronize()
            buf = np.zeros((1 << 20, 3), np.uint64)
            n = int(L.dpemu_probe_dds_times(buf.ctypes.data, buf.shape[0]))
            if r:
                runs.append(buf[:n].copy())
        res = []
        for b in runs:
            b = b[b[:, 1] > 0]                                   # workgroups that ran their sweep
            t0, t1 = b[:, 0].astype(np.int64), b[:, 1].astype(np.int64)
            base = t0.min()
            t0, t1 = (t0 - base) * 10, (t1 - base) * 10            # ns (100 MHz)
            span = int(t1.max())
            ch = (b[:, 2] >> 40).astype(np.int64)
            dur = t1 - t0
            edges = np.arange(0, span + 1000, 1000)               # 1-us bins: resident workgroups
            occ = np.zeros(len(edges))
            for s_, e_ in zip(t0, t1):
                i0, i1 = s_ // 1000, e_ // 1000
                occ[i0:i1 + 1] += 1
            mx = occ.max()
            full = np.nonzero(occ >= 0.9 * mx)[0]
            res.append({'span_ns': span, 'wgs': int(len(b)), 'occ_mean': float(occ.mean()), 'occ_max': float(mx),
                        'ramp_us': float(full[0]) if len(full) else None,
                        'tail_us': float(len(occ) - 1 - full[-1]) if len(full) else None,
                        'dur_us_qdrv': [float(np.percentile(dur[elem[ch] == workloads.QDRV], q)) / 1e3
                                        for q in (10, 50, 90, 99)],
                        'dur_us_rdrv': [float(np.percentile(dur[elem[ch] == workloads.RDRV], q)) / 1e3
                                        for q in (10, 50, 90, 99)],
                        'last_start_us': float(t0.max()) / 1e3})
        med = sorted(res, key=lambda x: x['span_ns'])[len(res) // 2]
        print(json.dumps({'lib': os.path.basename(lib), **med}), flush=True)


if __name__ == '__main__':
    main()
