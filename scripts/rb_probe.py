"""Config 4 at full size: generation / load / kernel times, one JSON line.
    python scripts/rb_probe.py [--seqs 100000] [--spg 10] [--flags 0]"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--seqs', type=int, default=100000)
    ap.add_argument('--spg', type=int, default=10)
    ap.add_argument('--flags', type=int, default=0)
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--outputs', default='summary,events,meas,hist')
    a = ap.parse_args()
    import torch
    from distributed_processor_amd import _abi, isa, workloads
    from distributed_processor_amd.emulator import Emulator, alloc_device_outputs
    t0 = time.perf_counter()
    ps = workloads.config4_rb_set(a.seqs, 200)
    t1 = time.perf_counter()
    ops = ps.words[:, 3] >> 28
    ev = np.add.reduceat(((ops == isa.OP_PULSE_TRIG) | (ops == isa.OP_PULSE_RESET)).astype(np.int64),
                         ps.offsets.astype(np.int64))
    emu = Emulator(0)
    emu.load(ps)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    n = a.seqs * a.spg
    cfg = _abi.make_config(2, n_groups=a.seqs, shots_per_group=a.spg, max_cycles=1 << 20,
                           event_cap=int(ev.max()) + 1, meas_cap=2, seed=0x5EED, exec_flags=a.flags)
    out = alloc_device_outputs(cfg, n, want=tuple(a.outputs.split(',')))
    res = {}
    for rep in range(2):
        emu.kernel_timing(True)
        for _ in range(a.steps):
            emu.run_device(cfg, n, 0, out)
        torch.cuda.synchronize()
        kt = emu.kernel_times()
        emu.kernel_timing(False)
        torch.cuda.synchronize()
        ts = time.perf_counter()
        for _ in range(a.steps):
            emu.run_device(cfg, n, 0, out)
        torch.cuda.synchronize()
        res['step_ms'] = (time.perf_counter() - ts) / a.steps * 1e3
        res['kernel_ms'] = kt
    s = _abi.unpack_summary(out['summary'].cpu().numpy().view(np.uint32))
    lanes = n * 2
    res.update({'gen_s': t1 - t0, 'load_s': t2 - t1, 'kernel': emu.last_kernel(), 'lanes': lanes,
                'commands': int(ps.words.shape[0]), 'all_done': bool((s['status'] == 1).all()),
                'instr_per_lane': float(s['n_instr'].mean()), 'events_per_lane': float(s['n_events'].mean()),
                'event_cap': cfg.event_cap,
                'core_shots_per_s': lanes / (np.median(res['kernel_ms']) * 1e-3),
                'instr_per_s': float(s['n_instr'].astype(np.float64).sum()) / (np.median(res['kernel_ms']) * 1e-3),
                'alg_GBps': (lanes * 32 + float(np.minimum(s['n_events'], cfg.event_cap).sum()) * 16 +
                             float(s['n_meas'].sum()) * 8) / (np.median(res['kernel_ms']) * 1e-3) / 1e9})
    print(json.dumps(res), flush=True)


if __name__ == '__main__':
    main()
