"""Same-process A/B of libdpemu.so builds (scripts/ab_libs.sh) on one workload.

    python scripts/ab.py --libs ab_build/libdpemu_a.so,ab_build/libdpemu_b.so --workload rb

Every library runs the same launches, interleaved (A B A B ...), with HIP
events around the kernel (dpemu_kernel_times); the outputs of all libraries
must be identical.  Prints one JSON line: median kernel ms per library.
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def workload(name):
    from distributed_processor_amd import _abi, isa, workloads
    from distributed_processor_amd.emulator import ProgramSet
    if name in ('rb', 'rb_sm', 'rb8', 'rb2q'):
        # rb: the RB-shaped programs of rounds 2-6; rb2q: config 4's two-qubit
        # Clifford RB; rb_sm: 10^4 shots (a quick check of a new build); rb8: 8 shots per sequence
        spg = 8 if name == 'rb8' else 10
        gen = workloads.config4_rb2q_set if name == 'rb2q' else workloads.config4_rb_set
        ps = gen(100000 if name != 'rb_sm' else 1000, 200)
        ops = ps.words[:, 3] >> 28
        ev = np.add.reduceat(((ops == isa.OP_PULSE_TRIG) | (ops == isa.OP_PULSE_RESET)).astype(np.int64),
                             ps.offsets.astype(np.int64))
        cfg = _abi.make_config(2, n_groups=ps.n_groups, shots_per_group=spg, max_cycles=1 << 20,
                               event_cap=int(ev.max()) + 1, meas_cap=2, seed=0x5EED)
        return ps, cfg, 10 ** 4 if name == 'rb_sm' else spg * 10 ** 5
    if name == 'config1':   # the reference's golden single-core program, 10^6 shots
        ps = ProgramSet(workloads.config1_linear())
        cfg = _abi.make_config(1, max_cycles=10000, event_cap=8, meas_cap=4, seed=0x5EED)
        return ps, cfg, 10 ** 6
    if name == 'ramsey':
        ps = ProgramSet(workloads.config2_ramsey(n_cores=8, n_points=100))
        cfg = _abi.make_config(8, n_groups=100, max_cycles=1 << 20, event_cap=8, meas_cap=2, seed=0x5EED)
        return ps, cfg, 10 ** 6
    if name in ('ar', 'ar0', 'ar1', 'ar0x32', 'ar_sm'):   # config 3; ar0 / ar1: every outcome 0 / 1 (no divergence)
        ps = ProgramSet(workloads.config3_active_reset(8, extra_pulses=32 if name.endswith('x32') else 0))
        cfg = _abi.make_config(8, max_cycles=50000, event_cap=48, meas_cap=4,
                               meas_latency=workloads.CONFIG3_MEAS_LATENCY, seed=0x5EED,
                               p1={'ar': 0.5, 'ar0': 0.0, 'ar1': 1.0, 'ar0x32': 0.0, 'ar_sm': 0.5}[name],
                               lane_order=_abi.LANES_SHOT_MAJOR if name == 'ar_sm' else _abi.LANES_CORE_MAJOR)
        return ps, cfg, 1250000
    if name == 'demod_sm':   # config 3 with the demodulation readout model, the bench's launch shape
        ps = ProgramSet(workloads.config3_active_reset(8))
        cfg = _abi.make_config(8, max_cycles=50000, event_cap=16, meas_cap=4,
                               meas_latency=workloads.CONFIG3_DEMOD_LATENCY, seed=0x5EED, p1=0.5,
                               lane_order=_abi.LANES_SHOT_MAJOR, demod=workloads.config3_demod(ps))
        return ps, cfg, 1250000
    if name == 'lut_sm':   # config 3 through the fproc_lut back end, the bench's launch shape
        ps = ProgramSet(workloads.config3_lut(8))
        cfg = _abi.make_config(8, max_cycles=50000, event_cap=16, meas_cap=4, fproc_mode=_abi.FPROC_LUT,
                               meas_latency=workloads.CONFIG3_MEAS_LATENCY, lut_mask=0xFF,
                               lut_table=workloads.config3_lut_table(8), seed=0x5EED, p1=0.5,
                               lane_order=_abi.LANES_SHOT_MAJOR)
        return ps, cfg, 1250000
    raise ValueError(name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--libs', required=True)
    ap.add_argument('--workload', default='rb')
    ap.add_argument('--reps', type=int, default=4)
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--no-compare', action='store_true', help='probe builds: outputs may differ')
    ap.add_argument('--flags', default='', help='per-library exec_flags (comma list, e.g. 0,0x40)')
    ap.add_argument('--outputs', default='summary,events,meas,hist', help='outputs the runs write')
    ap.add_argument('--lane-order', type=int, default=None, help='override the workload lane order')
    a = ap.parse_args()
    import torch
    from distributed_processor_amd.emulator import Emulator, alloc_device_outputs
    libs = [os.path.abspath(x) for x in a.libs.split(',')]
    ps, cfg, n = workload(a.workload)
    flags = [int(x, 0) for x in a.flags.split(',')] if a.flags else [cfg.exec_flags] * len(libs)
    emus = [Emulator(0, lib_path=l) for l in libs]
    for e in emus:
        e.load(ps)
    if a.lane_order is not None:
        cfg.lane_order = a.lane_order
    want = tuple(x for x in a.outputs.split(',') if x)
    out = alloc_device_outputs(cfg, n, want=want)   # one buffer set for all
    ref = None
    times = [[] for _ in emus]
    same = True
    for rep in range(a.reps):
        order = range(len(emus)) if rep % 2 == 0 else reversed(range(len(emus)))
        for i in order:
            e = emus[i]
            cfg.exec_flags = flags[i]
            e.kernel_timing(True)
            for _ in range(a.steps):
                if 'hist' in out:
                    out['hist'].zero_()
                e.run_device(cfg, n, 0, out)
            torch.cuda.synchronize()
            kt = e.kernel_times()
            e.kernel_timing(False)
            if rep:
                times[i] += kt
            snap = {k: out[k].clone() for k in ('summary', 'meas', 'hist') if k in out}
            if ref is None:
                ref = snap
            elif not a.no_compare:
                same &= all(torch.equal(ref[k], snap[k]) for k in ref)
    print(json.dumps({'workload': a.workload, 'same_outputs': bool(same), 'kernels': [e.last_kernel() for e in emus],
                      'flags': flags,
                      'median_ms': [float(np.median(t)) for t in times],
                      'min_ms': [float(np.min(t)) for t in times], 'libs': [os.path.basename(l) for l in libs]}))


if __name__ == '__main__':
    main()
