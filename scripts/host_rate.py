"""Host enqueue rate of a bench step (config 1, config 2): the time to
enqueue K steps without waiting, against the GPU time of the same K steps.
A step whose enqueue takes longer than its GPU time is host-bound.

    python scripts/host_rate.py
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from distributed_processor_amd import _abi, workloads
    from distributed_processor_amd.emulator import Emulator, ProgramSet, alloc_device_outputs
    gold = json.load(open(os.path.join(os.path.dirname(__file__), '..', 'tests', 'golden', 'cmd_buf_golden.json')))
    cases = {
        'config1': (ProgramSet([{0: bytes.fromhex(gold['cores']['0']['cmd_buf'])}]),
                    _abi.make_config(1, max_cycles=10000, event_cap=8, meas_cap=4, seed=0x5EED, p1=0.5), 10 ** 6),
        'config2': (ProgramSet(workloads.config2_ramsey(n_cores=8, n_points=100)),
                    _abi.make_config(8, n_groups=100, max_cycles=1 << 20, event_cap=8, meas_cap=2, seed=0x5EED,
                                     p1=0.5, lane_order=_abi.LANES_SHOT_MAJOR), 10 ** 6),
    }
    stream = torch.cuda.current_stream()
    for name, (ps, cfg, n) in cases.items():
        emu = Emulator(0)
        emu.load(ps)
        out = alloc_device_outputs(cfg, n, want=('summary', 'events', 'meas', 'hist'))
        for _ in range(5):
            emu.run_device(cfg, n, 0, out, stream)
        torch.cuda.synchronize()
        K = 200
        t0 = time.perf_counter()
        for _ in range(K):
            emu.run_device(cfg, n, 0, out, stream)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(json.dumps({'case': name, 'enqueue_us_per_step': (t1 - t0) / K * 1e6,
                          'wall_us_per_step': (t2 - t0) / K * 1e6}), flush=True)


if __name__ == '__main__':
    main()
