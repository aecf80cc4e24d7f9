"""DDS step with two batches in flight: does dds_index_kernel of batch k+1
overlap dds_tile_kernel of batch k when the two batches go to two contexts
on two streams (each context owns its own event index)?

    python scripts/dds_pipe.py [--seqs 128] [--steps 40] [--reps 5]

Times K steps of the bench's config-5 DDS leg (a) on one context and stream,
(b) alternating over two contexts and streams with one I/Q buffer each, and
checks that both give the same I/Q.  Prints one JSON line: median ms/step.
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
    args = ap.parse_args()
    import torch
    from distributed_processor_amd import _abi, workloads
    from distributed_processor_amd.dds import ChannelPlan
    from distributed_processor_amd.emulator import Emulator, ProgramSet, alloc_device_outputs
    ps = ProgramSet(workloads.config4_rb(n_seq=args.seqs, depth=200, n_cores=8))
    emus = [Emulator(0), Emulator(0)]
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
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    iq = [torch.empty((plan.n_channels, n_samples), dtype=torch.int32, device='cuda') for _ in range(2)]

    def run(k, two):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(k):
            j = i & 1 if two else 0
            emus[j].synthesize(plan, ev, n_samples, iq[j], streams[j])
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / k * 1e3

    for two in (False, True):
        run(4, two)
    res = {False: [], True: []}
    for _ in range(args.reps):
        for two in (False, True):
            res[two].append(run(args.steps, two))
    same = bool(torch.equal(iq[0], iq[1]))
    samples = plan.n_channels * n_samples
    out = {'channels': plan.n_channels, 'samples_per_channel': n_samples, 'steps': args.steps,
           'one_stream_ms': float(np.median(res[False])), 'two_streams_ms': float(np.median(res[True])),
           'all_one': res[False], 'all_two': res[True], 'same_iq': same}
    for k in ('one_stream_ms', 'two_streams_ms'):
        out[k.replace('_ms', '_frac')] = samples * 4 / (out[k] * 1e-3) / 8e12
    print(json.dumps(out))
    for e in emus:
        e.close()


if __name__ == '__main__':
    main()
