"""Batches in flight for the interpreter legs: K launches of a bench workload
(scripts/ab.py's workloads) on one context and stream, against the same
launches spread round-robin over d contexts, each with its own stream and
output set (hist_assign, so no zeroing launch).  Checks every output set
against the single-stream one.  Prints one JSON line: median ms per launch.

    python scripts/pipe_probe.py --workload ramsey --depths 2,4,8
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scripts.ab import workload  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--workload', default='ramsey')
    ap.add_argument('--depths', default='2,4,8')
    ap.add_argument('--steps', type=int, default=40)
    ap.add_argument('--reps', type=int, default=5)
    ap.add_argument('--lane-order', type=int, default=1)
    ap.add_argument('--bench-cfg', action='store_true', help='rb: bench.py leg_rb\'s config (no trace, p1 0.5)')
    ap.add_argument('--accumulate', action='store_true', help='histogram accumulated, not assigned')
    args = ap.parse_args()
    import torch
    from distributed_processor_amd.emulator import Emulator, alloc_device_outputs
    ps, cfg, n = workload(args.workload)
    cfg.lane_order = args.lane_order
    cfg.hist_assign = 0 if args.accumulate else 1
    if args.bench_cfg:
        from distributed_processor_amd import _abi
        cfg = _abi.make_config(2, n_groups=ps.n_groups, shots_per_group=10, max_cycles=1 << 20,
                               event_cap=cfg.event_cap, trace_cap=0, meas_cap=2, meas_latency=64, seed=0x5EED,
                               p1=0.5, hist_assign=not args.accumulate)
    depths = [int(x) for x in args.depths.split(',')]
    dmax = max(depths + [1])
    emus = [Emulator(0) for _ in range(dmax)]
    for e in emus:
        e.load(ps)
    streams = [torch.cuda.Stream() for _ in range(dmax)]
    want = ('summary', 'events', 'meas', 'hist')
    outs = [alloc_device_outputs(cfg, n, want=want) for _ in range(dmax)]

    def run(k, d):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(k):
            j = i % d
            emus[j].run_device(cfg, n, 0, outs[j], streams[j])
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / k * 1e3

    keys = [1] + depths
    for d in keys:
        run(4, d)
    res = {d: [] for d in keys}
    for _ in range(args.reps):
        for d in keys:
            res[d].append(run(args.steps, d))
    same = all(torch.equal(outs[0][k], outs[j][k]) for j in range(1, dmax) for k in want)
    out = {'workload': args.workload, 'trace_cap': int(cfg.trace_cap), 'hist_assign': int(cfg.hist_assign), 'n_shots': n, 'steps': args.steps, 'kernel': emus[0].last_kernel(),
           'same_outputs': bool(same)}
    for d in keys:
        out['depth{}_ms'.format(d)] = float(np.median(res[d]))
    print(json.dumps(out))
    for e in emus:
        e.close()


if __name__ == '__main__':
    main()
