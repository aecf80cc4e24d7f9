"""Configs 1-4 on one MI355X beside the CPU restatements:
GPU emulator (HIP events around the interpreter kernel + wall clock of the
step), oracle_fast (event-driven C, OpenMP), and oracle_rtl (per-clock C
model) single-threaded and on a thread pool (ctypes releases the GIL).  CPU
legs run a bounded sample of the same workload (~`CPU_S` seconds each).
One JSON line per config on stdout.  Test infrastructure: the oracle is the
baseline here, never the thing measured on the GPU.

    python scripts/configs_table.py [steps]
"""
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import oracle  # noqa: E402
from distributed_processor_amd import _abi, workloads  # noqa: E402
from distributed_processor_amd.emulator import Emulator, ProgramSet, alloc_device_outputs  # noqa: E402

CPU_S = 4.0
THREADS = min(len(os.sched_getaffinity(0)), 16)
WANT = ('summary', 'ev_main', 'ev_amp', 'meas', 'hist')


def configs():
    yield ('config1_linear_1core', ProgramSet(workloads.config1_linear()),
           dict(cores=1, max_cycles=10000, event_cap=8, meas_cap=4), 10 ** 6,
           'SURVEY config 1: golden linear program, 1 core, 1e6 shots')
    yield ('config2_ramsey_8core_100pt', ProgramSet(workloads.config2_ramsey(n_cores=8, n_points=100)),
           dict(cores=8, n_groups=100, max_cycles=20000, event_cap=8, meas_cap=4), 10 ** 6,
           'SURVEY config 2: 8-core Ramsey, 100 delays by shot, 1e6 shots')
    yield ('config3_active_reset_8core', ProgramSet(workloads.config3_active_reset(8)),
           dict(cores=8, max_cycles=50000, event_cap=16, meas_cap=4, meas_latency=workloads.CONFIG3_MEAS_LATENCY,
                p1=0.5), 1250000, 'SURVEY config 3: 8-core active reset, 1.25e6 shots (1/8 of 1e7)')
    n_seq, spg = 1000, 100
    yield ('config4_rb_2q_depth200', ProgramSet(workloads.config4_rb(n_seq=n_seq, depth=200, n_cores=2)),
           dict(cores=2, n_groups=n_seq, shots_per_group=spg, max_cycles=400000, event_cap=640, meas_cap=4),
           n_seq * spg, 'config 4: 2-qubit RB depth 200, 1000 sequences x 100 shots (SURVEY: 1e5 x 10; '
                        'sequence generation in Python bounds the count)')


def make_cfg(ps, d):
    d = dict(d)
    C = d.pop('cores')
    return _abi.make_config(C, n_groups=d.pop('n_groups', ps.n_groups), trace_cap=0, seed=0x5EED, **d)


def gpu_leg(emu, ps, cfg, n, steps):
    import torch
    emu.load(ps)
    out = alloc_device_outputs(cfg, n, want=WANT)
    stream = torch.cuda.current_stream()
    for _ in range(2):
        out['hist'].zero_()
        emu.run_device(cfg, n, 0, out, stream)
    torch.cuda.synchronize()
    emu.kernel_times()
    emu.kernel_timing(True)
    t0 = time.perf_counter()
    for _ in range(steps):
        out['hist'].zero_()
        emu.run_device(cfg, n, 0, out, stream)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    emu.kernel_timing(False)
    kms = float(np.mean(emu.kernel_times()))
    s = _abi.unpack_summary(out['summary'].cpu().numpy().view(np.uint32))
    done = float((s['status'] == _abi.ST_DONE).mean())
    return {'core_shots_per_s': n * cfg.cores_per_shot / dt, 'ms_per_step': dt * 1e3, 'kernel_ms': kms,
            'kernel': emu.last_kernel(), 'done_fraction': done,
            'instr_per_s': float(s['n_instr'].astype(np.float64).sum()) / dt}


def fast_leg(ps, cfg):
    chunk, done = 5000, 0
    oracle.fast_run(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, 0, 100, THREADS, WANT)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < CPU_S:
        oracle.fast_run(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, done, chunk, THREADS, WANT)
        done += chunk
    dt = time.perf_counter() - t0
    return {'core_shots_per_s': done * cfg.cores_per_shot / dt, 'threads': THREADS, 'shots': done}


def rtl_leg(ps, cfg, threads):
    scfg = oracle.shot_cfg_from_config(cfg)
    C, G, spg = cfg.cores_per_shot, ps.n_groups, cfg.shots_per_group

    def progs(shot):
        g = (shot // spg) % G
        return [ps.words[ps.offsets[p]:ps.offsets[p] + ps.n_instr[p]] for p in ps.table[g * C:(g + 1) * C]]

    def one(shot):
        ok, _ = oracle.rtl_run_shot(scfg, progs(shot), shot, cfg.max_cycles + 16, 64, 1, 8)
        return ok

    t0, done = time.perf_counter(), 0
    with ThreadPoolExecutor(threads) as pool:
        while time.perf_counter() - t0 < CPU_S:
            done += sum(1 for _ in pool.map(one, range(done, done + 4 * threads)))
    dt = time.perf_counter() - t0
    return {'core_shots_per_s': done * C / dt, 'threads': threads, 'shots': done}


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    with Emulator(0) as emu:
        for name, ps, d, n, desc in configs():
            cfg = make_cfg(ps, d)
            row = {'workload': name, 'description': desc, 'gpu_shots': n, 'gpu': gpu_leg(emu, ps, cfg, n, steps),
                   'oracle_fast': fast_leg(ps, cfg), 'oracle_rtl_1t': rtl_leg(ps, cfg, 1),
                   'oracle_rtl_mt': rtl_leg(ps, cfg, THREADS)}
            print(json.dumps(row), flush=True)


if __name__ == '__main__':
    main()
