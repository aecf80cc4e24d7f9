"""Benchmark: batched emulation of assembled distproc machine code on MI355X.

Workload (BASELINE.json configs[1]): 8-core (8-qubit) parallel Ramsey sweep,
100 delay points selected by shot, no branching, 10^6 shots per GPU.  One
step = one pass of the hot path over one batch: the interpreter kernel
emulates every (shot, core) lane cycle-exactly and writes the full pulse-event
timeline, lane summaries, measurement records and the outcome histogram to
HBM; with N > 1 ranks the histograms are all-reduced over RCCL (the path's
only exchange).  Shots shard by global index (weak scaling).

Metric: emulated core-shots/s (whole job).  Also reported: emulated qclk
cycles/s and instructions/s, the interpreter's HBM roofline fraction, and
the CPU baseline (oracle_fast, the event-driven C restatement, on the host
cores; the Verilator/cocotb testbench itself cannot run here or on the box).

    python bench.py --gpus 1 --steps 20 --warmup 3
    torchrun --nproc-per-node N bench.py --gpus N ...
"""

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec


def build_workload(n_points=100, n_cores=8):
    from distributed_processor_amd import workloads
    from distributed_processor_amd.emulator import ProgramSet
    return ProgramSet(workloads.config2_ramsey(n_cores=n_cores, n_points=n_points))


def bytes_per_lane(summary_np, cfg):
    """algorithmic HBM bytes written per lane: 32 B summary + 18 B per event
    (16 B record + 2 B amplitude) + 8 B per measurement record"""
    n_ev = np.minimum(summary_np[:, 2], cfg.event_cap).astype(np.float64)
    n_me = np.minimum(summary_np[:, 5], cfg.meas_cap).astype(np.float64)
    return 32.0 + 18.0 * n_ev + 8.0 * n_me


def cpu_baseline(ps, cfg, target_s=12.0):
    """oracle_fast on the host cores over a bounded sample of the same workload."""
    import oracle
    threads = os.cpu_count() or 1
    try:
        threads = len(os.sched_getaffinity(0))
    except Exception:
        pass
    threads = min(threads, 16)
    chunk = 20000
    want = ('summary', 'ev_main', 'ev_amp', 'meas', 'hist')
    oracle.fast_run(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, 0, 1000, threads, want)  # warm
    done = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < target_s:
        oracle.fast_run(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, done, chunk, threads, want)
        done += chunk
    dt = time.perf_counter() - t0
    return {'value': done * cfg.cores_per_shot / dt, 'unit': 'core-shots/s', 'cores': threads,
            'kind': 'port',
            'sample': '{} shots x {} cores of the same Ramsey workload, oracle_fast (event-driven C '
                      'restatement, OpenMP) in {}-shot chunks, {:.1f} s'.format(done, cfg.cores_per_shot, chunk, dt)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--shots', type=int, default=10 ** 6, help='shots per GPU per step')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-seconds', type=float, default=12.0)
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world > 1:
        dist.init_process_group('nccl')
    torch.cuda.set_device(local)

    from distributed_processor_amd import _abi
    from distributed_processor_amd.emulator import Emulator, alloc_device_outputs

    ps = build_workload()
    emu = Emulator(local)
    emu.load(ps)
    cfg = _abi.make_config(8, n_groups=ps.n_groups, max_cycles=1 << 20, event_cap=8, trace_cap=0,
                           meas_cap=2, meas_latency=64, seed=0x5EED, p1=0.5)
    n = args.shots
    out = alloc_device_outputs(cfg, n, want=('summary', 'ev_main', 'ev_amp', 'meas', 'hist'))
    stream = torch.cuda.current_stream()
    shot0 = rank * n

    def step(ev_pair=None):
        out['hist'].zero_()
        if ev_pair:
            ev_pair[0].record(stream)
        emu.run_device(cfg, n, shot0, out, stream)
        if ev_pair:
            ev_pair[1].record(stream)
        if world > 1:
            dist.all_reduce(out['hist'])

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(events[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device='cuda')
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    kernel_ms = float(np.mean([a.elapsed_time(b) for a, b in events]))

    # accounting from the last step's outputs (identical every step)
    summ = out['summary'].cpu().numpy().view(np.uint32)
    s = _abi.unpack_summary(summ)
    assert (s['status'] == _abi.ST_DONE).all(), 'not every lane reached DONE'
    hist_total = int(out['hist'].sum().item())
    assert hist_total == n * world, hist_total
    lanes = n * cfg.cores_per_shot
    cycles = float(s['t_end'].astype(np.float64).sum())
    instrs = float(s['n_instr'].astype(np.float64).sum())
    alg_bytes = float(bytes_per_lane(summ, cfg).sum())

    total_core_shots = lanes * world * args.steps
    value = total_core_shots / dt
    achieved_gbs = alg_bytes / (kernel_ms * 1e-3) / 1e9

    traffic = None
    pmc = os.path.join(REPO, 'profiles', 'r01_interp_pmc.json')
    if os.path.exists(pmc):
        with open(pmc) as f:
            traffic = json.load(f).get('hbm_bytes_per_launch')

    result = {
        'metric': 'emulated core-shots/s (config 2: 8-core Ramsey, 100 delays, 1e6 shots/GPU)',
        'value': value,
        'unit': 'core-shots/s',
        'n_gpus': world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': dt / args.steps * 1e3,
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': None,
        'dtype': 'u32',
        'data': 'synthetic (assembled Ramsey programs, Philox outcomes p=0.5)',
        'config': {'workload': 'config2_ramsey_8core_100pt', 'shots_per_gpu': n, 'cores_per_shot': 8,
                   'global_shots_per_step': n * world, 'parallelism': 'shots sharded, {} GPU(s)'.format(world)},
        'shots_per_s': value / 8,
        'qclk_cycles_per_s': cycles * world * args.steps / dt,
        'instructions_per_s': instrs * world * args.steps / dt,
        'kernel_ms': kernel_ms,
        'roofline': {'bound': 'hbm', 'achieved': achieved_gbs, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                     'frac': achieved_gbs / HBM_PEAK_GBS, 'traffic': traffic,
                     'bytes_per_launch': alg_bytes,
                     'kernel': 'dpemu::interp_kernel<0>'},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result['cpu_baseline'] = cpu_baseline(ps, cfg, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(result), flush=True)
    emu.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
