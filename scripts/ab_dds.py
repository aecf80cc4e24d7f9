"""Same-process A/B of libdpemu.so builds (scripts/ab_libs.sh) on the config-5
DDS step: the RB timelines are emulated once (first library), then every
library synthesises them, interleaved (A B A B ...), with HIP events around
the synthesis kernel (dpemu_kernel_times) and a block of whole steps; the I/Q
of all libraries must be identical.  One JSON line.

    python scripts/ab_dds.py --libs ab_build/libdpemu_a.so,ab_build/libdpemu_b.so
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--libs', required=True)
    ap.add_argument('--seqs', type=int, default=128)
    ap.add_argument('--reps', type=int, default=4)
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--align', type=int, default=4, help='round n_samples up to a multiple of this')
    ap.add_argument('--workload', default='rb2q', choices=('rb2q', 'rb'),
                    help='timelines: config 4\'s two-qubit RB on 4 pairs, or the RB-shaped 8-core generator')
    a = ap.parse_args()
    import torch
    from distributed_processor_amd import _abi, workloads
    from distributed_processor_amd.dds import ChannelPlan
    from distributed_processor_amd.emulator import Emulator, ProgramSet, alloc_device_outputs
    libs = [os.path.abspath(x) for x in a.libs.split(',')]
    emus = [Emulator(0, lib_path=l) for l in libs]
    if a.workload == 'rb2q':
        ps = workloads.config4_rb2q_set(a.seqs, 200, n_cores=8)
    else:
        ps = ProgramSet(workloads.config4_rb(n_seq=a.seqs, depth=200, n_cores=8))
    ops = ps.words[:, 3] >> 28
    strobes = np.add.reduceat(((ops == 0x9) | (ops == 0xB)).astype(np.int64), ps.offsets.astype(np.int64))
    cfg = _abi.make_config(8, n_groups=ps.n_groups, max_cycles=1 << 20, event_cap=max(512, int(strobes.max()) + 1),
                           meas_cap=4, meas_latency=64, seed=0x5EED)
    emus[0].load(ps)
    ev = alloc_device_outputs(cfg, a.seqs, want=('summary', 'events'))
    emus[0].run_device(cfg, a.seqs, 0, ev)
    torch.cuda.synchronize()
    s = _abi.unpack_summary(ev['summary'].cpu().numpy().view(np.uint32))
    n_samples = ((int(s['t_end'].max()) + 8) * 16 + a.align - 1) // a.align * a.align
    params = {i: (e['samples_per_clk'], e['interp_ratio']) for i, e in enumerate(workloads.ELEMS)}
    chans = [(q, c, e) for q in range(a.seqs) for c in range(8) for e in (workloads.QDRV, workloads.RDRV)]
    plan = ChannelPlan(ps, cfg, 0, a.seqs, chans, params)
    iq = torch.empty((plan.n_channels, n_samples), dtype=torch.int32, device='cuda')
    ref = None
    same = True
    kern = [[] for _ in emus]
    step = [[] for _ in emus]
    for rep in range(a.reps):
        order = range(len(emus)) if rep % 2 == 0 else reversed(range(len(emus)))
        for i in order:
            e = emus[i]
            e.synthesize(plan, ev, n_samples, iq)
            torch.cuda.synchronize()
            e.kernel_times()
            e.kernel_timing(True)
            for _ in range(a.steps):
                e.synthesize(plan, ev, n_samples, iq)
            torch.cuda.synchronize()
            kt = e.kernel_times()
            e.kernel_timing(False)
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0.record()
            for _ in range(a.steps):
                e.synthesize(plan, ev, n_samples, iq)
            t1.record()
            torch.cuda.synchronize()
            if rep:
                kern[i] += kt
                step[i].append(t0.elapsed_time(t1) / a.steps)
            snap = iq.clone()
            if ref is None:
                ref = snap
            else:
                same &= bool(torch.equal(ref, snap))
    gb = plan.n_channels * n_samples * 4 / 1e9
    fills = []                       # the same buffer written by a fill (hipMemsetAsync): the store ceiling
    for _ in range(a.reps):
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(a.steps):
            iq.fill_(1)
        t1.record()
        torch.cuda.synchronize()
        fills.append(t0.elapsed_time(t1) / a.steps)
    print(json.dumps({'workload': a.workload, 'same_iq': same, 'GB': gb, 'n_samples': n_samples, 'fill_ms': float(np.median(fills)),
                      'kernel_ms': {os.path.basename(l): float(np.median(k)) for l, k in zip(libs, kern)},
                      'kernel_min_ms': {os.path.basename(l): float(np.min(k)) for l, k in zip(libs, kern)},
                      'step_ms': {os.path.basename(l): float(np.median(k)) for l, k in zip(libs, step)}}))


if __name__ == '__main__':
    main()
