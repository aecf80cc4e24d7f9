"""Where a config-2 bench step's time goes: host issue time per step (no
synchronisation inside the loop) against the GPU time per step, for the
bench's step and for bare dpemu_run calls.  One JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from distributed_processor_amd import _abi, sharding, workloads
    from distributed_processor_amd.emulator import Emulator, ProgramSet, alloc_device_outputs
    ps = ProgramSet(workloads.config2_ramsey(n_cores=8, n_points=100))
    cfg = _abi.make_config(8, n_groups=ps.n_groups, max_cycles=1 << 20, event_cap=8, trace_cap=0, meas_cap=2,
                           meas_latency=64, seed=0x5EED, p1=0.5, hist_assign=True)
    n, K = 10 ** 6, 50
    res = {}
    with Emulator(0) as emu:
        emu.load(ps)
        out = alloc_device_outputs(cfg, n, want=('summary', 'events', 'meas', 'hist'))
        stream = torch.cuda.current_stream()
        pipe = sharding.HistogramPipeline(out['hist'], zero=False)

        def launch(h):
            out['hist'] = h
            emu.run_device(cfg, n, 0, out, stream)
        variants = [
            ('bench_step_cold', lambda: pipe.step(launch)),
            ('run_device', lambda: emu.run_device(cfg, n, 0, out, stream)),
            ('bench_step', lambda: pipe.step(launch)),
            ('run_device_nohist', lambda: emu.run_device(cfg, n, 0, {k: v for k, v in out.items() if k != 'hist'},
                                                         stream)),
            ('bench_step_again', lambda: pipe.step(launch)),
        ]
        for name, fn in variants:
            for _ in range(5):
                fn()
            pipe.drain()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(K):
                fn()
            t1 = time.perf_counter()
            pipe.drain()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            res[name] = {'issue_ms': (t1 - t0) / K * 1e3, 'wall_ms': (t2 - t0) / K * 1e3}
        # host cost of the Python checks alone
        want = None
        from distributed_processor_amd import emulator as em
        t0 = time.perf_counter()
        for _ in range(K):
            want = em.device_output_specs(cfg, n)
            for k, t in out.items():
                em._check_tensor(k, t, want[k], emu.device)
        res['checks_ms'] = (time.perf_counter() - t0) / K * 1e3
    print(json.dumps(res))


if __name__ == '__main__':
    main()
