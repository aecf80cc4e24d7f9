"""DDS step with batches in flight: does dds_index_kernel of batch k+1
overlap dds_tile_kernel of batch k when the batches go to separate contexts
on separate streams (each context owns its own event index)?

    python scripts/dds_pipe.py [--seqs 128] [--steps 40] [--reps 5] [--depths 2,3]

Times K steps of the bench's config-5 DDS leg (a) on one context and stream,
(b) through dds.SynthesisPipeline at each depth, and checks that all give the
same I/Q.  Prints one JSON line: median ms/step.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--seqs', type=int, default=128)
    ap.add_argument('--steps', type=int, default=40)
    ap.add_argument('--reps', type=int, default=5)
    ap.add_argument('--depths', default='2')
    args = ap.parse_args()
    import torch
    from distributed_processor_amd import _abi, workloads
    from distributed_processor_amd.dds import ChannelPlan, SynthesisPipeline
    from distributed_processor_amd.emulator import Emulator, ProgramSet, alloc_device_outputs
    ps = ProgramSet(workloads.config4_rb(n_seq=args.seqs, depth=200, n_cores=8))
    emus = [Emulator(0)]
    emus[0].load(ps)
    cfg = _abi.make_config(8, n_groups=ps.n_groups, max_cycles=1 << 20, event_cap=512, meas_cap=4,
                           meas_latency=64, seed=0x5EED)
    n = args.seqs
    ev = alloc_device_outputs(cfg, n, want=('summary', 'events'))
    emus[0].run_device(cfg, n, 0, ev)
    torch.cuda.synchronize()
    s = _abi.unpack_summary(ev['summary'].cpu().numpy().view(np.uint32))
    n_samples = ((int(s['t_end'].max()) + 8) * 16 + 3) // 4 * 4
    params = {i: (e['samples_per_clk'], e['interp_ratio']) for i, e in enumerate(workloads.ELEMS)}
    chans = [(q, c, e) for q in range(n) for c in range(8) for e in (workloads.QDRV, workloads.RDRV)]
    plan = ChannelPlan(ps, cfg, 0, n, chans, params)
    depths = [int(x) for x in args.depths.split(',')]
    pipes = {d: SynthesisPipeline(0, depth=d) for d in depths}
    iq1 = torch.empty((plan.n_channels, n_samples), dtype=torch.int32, device='cuda')

    def run(k, d):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            if d == 1:
                emus[0].synthesize(plan, ev, n_samples, iq1)
            else:
                pipes[d].synthesize(plan, ev, n_samples)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / k * 1e3

    keys = [1] + depths
    for d in keys:
        run(4, d)
    res = {d: [] for d in keys}
    for _ in range(args.reps):
        for d in keys:
            res[d].append(run(args.steps, d))
    same = all(bool(torch.equal(iq1, b)) for d in depths for b in pipes[d].iq if b is not None)
    samples = plan.n_channels * n_samples
    out = {'channels': plan.n_channels, 'samples_per_channel': n_samples, 'steps': args.steps, 'same_iq': same}
    for d in keys:
        name = 'one_stream' if d == 1 else 'depth{}'.format(d)
        out[name + '_ms'] = float(np.median(res[d]))
        out[name + '_frac'] = samples * 4 / (out[name + '_ms'] * 1e-3) / 8e12
        out['all_' + name] = res[d]
    print(json.dumps(out))
    for p in pipes.values():
        p.close()
    for e in emus:
        e.close()


if __name__ == '__main__':
    main()
