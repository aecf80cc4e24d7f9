"""Benchmark: batched emulation of assembled distproc machine code on MI355X.

Workload (BASELINE.json configs[1]): 8-core (8-qubit) parallel Ramsey sweep,
100 delay points selected by shot, no branching, 10^6 shots per GPU.  One
step = one pass of the hot path over one batch: the interpreter kernel
emulates every (shot, core) lane cycle-exactly and writes the full pulse-event
timeline, lane summaries, measurement records and the outcome histogram to
HBM; with N > 1 ranks the histograms are all-reduced over RCCL (the path's
only exchange).  Shots shard by global index (weak scaling).

Active-reset leg (config 3, under "active_reset"): fproc_meas branching and
sync barriers on the general interpreter kernel, 1.25*10^6 shots per GPU.

DDS leg (config 5, reported under "dds" on the same line): the config-4 RB
timelines (8 cores, depth 200) synthesised to int16 I/Q on 16 channels per
sequence at 16 samples/clk; GSamples/s (whole job) and the DDS kernel's HBM
write roofline.

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
PROFILE_TAG = 'r01'            # profiles/<tag>_{interp,dds}_pmc.json: PMC passes of this workload


def build_workload(n_points=100, n_cores=8):
    from distributed_processor_amd import workloads
    from distributed_processor_amd.emulator import ProgramSet
    return ProgramSet(workloads.config2_ramsey(n_cores=n_cores, n_points=n_points))


def kernel_pass(emu, steps, step, drain=None):
    """Run `steps` more steps with the library's HIP events recorded around
    each main kernel launch (dpemu_set_kernel_timing), outside the timed
    region; emu.kernel_times() then holds one duration per launch."""
    import torch
    torch.cuda.synchronize()
    emu.kernel_times()                                # drop earlier records
    emu.kernel_timing(True)
    for _ in range(steps):
        step()
    if drain is not None:
        drain()
    torch.cuda.synchronize()
    emu.kernel_timing(False)


def bytes_per_lane(summary_np, cfg):
    """algorithmic HBM bytes written per lane: 32 B summary + 16 B per event
    record + 8 B per measurement record"""
    n_ev = np.minimum(summary_np[:, 2], cfg.event_cap).astype(np.float64)
    n_me = np.minimum(summary_np[:, 5], cfg.meas_cap).astype(np.float64)
    return 32.0 + 16.0 * n_ev + 8.0 * n_me


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
    want = ('summary', 'events', 'meas', 'hist')
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


def dds_workload(n_seq):
    """config 5: the config-4 RB timelines (8 cores, depth 200) synthesised on
    16 channels per sequence (8 cores x {qdrv, rdrv}) at 16 samples/clk"""
    from distributed_processor_amd import workloads
    from distributed_processor_amd.emulator import ProgramSet
    return ProgramSet(workloads.config4_rb(n_seq=n_seq, depth=200, n_cores=8))


def dds_cpu_baseline(plan, host_ev, n_samples, target_s=8.0):
    """oracle_dds (scalar C restatement, OpenMP over channels) on whole
    channels of the same timelines until ~target_s of CPU work"""
    import oracle
    threads = min(len(os.sched_getaffinity(0)), 16)
    per = max(threads, 16)
    done = 0
    t0 = time.perf_counter()
    i = 0
    while time.perf_counter() - t0 < target_s and i < plan.n_channels:
        d = plan.desc[i:i + per]
        oracle.dds(d, host_ev['summary'], host_ev['events'], plan.env, plan.freq,
                   n_samples, plan.event_cap, threads)
        done += len(d) * n_samples
        i += per
    dt = time.perf_counter() - t0
    return {'value': done / dt / 1e9, 'unit': 'GSamples/s', 'cores': threads, 'kind': 'port',
            'sample': '{} channels x {} samples of the config-5 timelines, oracle_dds (scalar C '
                      'restatement, OpenMP over channels), {:.1f} s'.format(done // n_samples, n_samples, dt)}


def dds_leg(emu, args, world, rank, stream):
    """time K synthesis steps of config 5; returns the 'dds' sub-object"""
    import torch
    import torch.distributed as dist
    from distributed_processor_amd import _abi, sharding, workloads
    from distributed_processor_amd.dds import ChannelPlan
    from distributed_processor_amd.emulator import alloc_device_outputs
    ps = dds_workload(args.dds_seqs)
    emu.load(ps)
    cfg = _abi.make_config(8, n_groups=ps.n_groups, max_cycles=1 << 20, event_cap=512, meas_cap=4,
                           meas_latency=64, seed=0x5EED)
    shot0, n = sharding.weak_shard(args.dds_seqs, rank)
    ev = alloc_device_outputs(cfg, n, want=('summary', 'events'))
    emu.run_device(cfg, n, shot0, ev, stream)
    torch.cuda.synchronize()
    summ = ev['summary'].cpu().numpy().view(np.uint32)
    s = _abi.unpack_summary(summ)
    assert (s['status'] == _abi.ST_DONE).all() and (s['n_events'] <= cfg.event_cap).all()
    n_cyc = int(s['t_end'].max()) + 8
    n_samples = (n_cyc * 16 + 3) // 4 * 4
    params = {i: (e['samples_per_clk'], e['interp_ratio']) for i, e in enumerate(workloads.ELEMS)}
    chans = [(shot0 + q, c, e) for q in range(n) for c in range(8) for e in (workloads.QDRV, workloads.RDRV)]
    plan = ChannelPlan(ps, cfg, shot0, n, chans, params)
    iq = torch.empty((plan.n_channels, n_samples), dtype=torch.int32, device='cuda')
    for _ in range(args.warmup):
        emu.synthesize(plan, ev, n_samples, iq, stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        emu.synthesize(plan, ev, n_samples, iq, stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = sharding.max_over_ranks(time.perf_counter() - t0, device='cuda')
    kernel_pass(emu, args.steps, lambda: emu.synthesize(plan, ev, n_samples, iq, stream))
    kt = emu.kernel_times()
    assert len(kt) == args.steps, kt
    kernel_ms = float(np.mean(kt))                    # HIP events around the DDS kernel, same stream
    samples = plan.n_channels * n_samples
    gbs = samples * 4 / (kernel_ms * 1e-3) / 1e9
    traffic = None
    pmc = os.path.join(REPO, 'profiles', PROFILE_TAG + '_dds_pmc.json')
    if os.path.exists(pmc):
        with open(pmc) as f:
            traffic = json.load(f).get('hbm_bytes_per_launch')
    res = {'metric': 'DDS I/Q GSamples/s (config 5: RB timelines, 16 channels/sequence, 16 samples/clk)',
           'value': samples * world * args.steps / dt / 1e9, 'unit': 'GSamples/s',
           'ms_per_step': dt / args.steps * 1e3, 'kernel_ms': kernel_ms, 'dtype': 'int16 I/Q',
           'step': 'dds_index_kernel (per-channel event index) + dds_chunk_kernel; kernel_ms and the roofline '
                   'hold dds_chunk_kernel alone, value and ms_per_step the whole step',
           'config': {'workload': 'config5_dds_rb8', 'sequences_per_gpu': n, 'channels_per_gpu': plan.n_channels,
                      'samples_per_channel': n_samples, 'rb_depth': 200},
           'roofline': {'bound': 'hbm', 'achieved': gbs, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                        'frac': gbs / HBM_PEAK_GBS, 'traffic': traffic, 'bytes_per_launch': samples * 4,
                        'kernel': 'dpemu::dds_tile_kernel'}}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        host_ev = {k: v.cpu().numpy() for k, v in ev.items()}
        res['cpu_baseline'] = dds_cpu_baseline(plan, host_ev, n_samples, args.cpu_seconds * 2 / 3)
    del iq
    return res


def active_reset_leg(emu, args, world, rank, stream):
    """config 3 (BASELINE configs[2]): 8-core active reset -- readout, fproc_meas
    branch to a conditional X180, sync barriers -- 10^7 shots per step over 8
    GPUs, i.e. 1.25*10^6 shots per GPU (weak).  Runs on the general
    interpreter kernel (fproc + sync).  Returns the 'active_reset' sub-object."""
    import torch
    from distributed_processor_amd import _abi, sharding, workloads
    from distributed_processor_amd.emulator import ProgramSet, alloc_device_outputs
    ps = ProgramSet(workloads.config3_active_reset(8))
    emu.load(ps)
    cfg = _abi.make_config(8, n_groups=ps.n_groups, max_cycles=50000, event_cap=16, trace_cap=0, meas_cap=4,
                           meas_latency=workloads.CONFIG3_MEAS_LATENCY, seed=0x5EED, p1=0.5)
    n_per = args.ar_shots
    out = alloc_device_outputs(cfg, n_per, want=('summary', 'events', 'meas', 'hist'))
    shot0, n = sharding.weak_shard(n_per, rank)

    def step():
        out['hist'].zero_()
        emu.run_device(cfg, n, shot0, out, stream)
        sharding.allreduce_histogram(out['hist'])
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    dt = sharding.max_over_ranks(time.perf_counter() - t0, device='cuda')
    kernel_pass(emu, args.steps, step)
    kt = emu.kernel_times()
    kernel_ms = float(np.mean(kt))
    summ = out['summary'].cpu().numpy().view(np.uint32)
    s = _abi.unpack_summary(summ)
    assert (s['status'] == _abi.ST_DONE).all(), 'config 3: not every lane reached DONE'
    assert int(out['hist'].sum().item()) == n * world
    alg = float(bytes_per_lane(summ, cfg).sum())
    gbs = alg / (kernel_ms * 1e-3) / 1e9
    res = {'metric': 'emulated core-shots/s (config 3: 8-core active reset, fproc_meas branch + sync, '
                     '1.25e6 shots/GPU)',
           'value': n * 8 * world * args.steps / dt, 'unit': 'core-shots/s', 'shots_per_s': n * world * args.steps / dt,
           'ms_per_step': dt / args.steps * 1e3, 'kernel_ms': kernel_ms, 'kernel': 'dpemu::' + emu.last_kernel(),
           'instructions_per_s': float(s['n_instr'].astype(np.float64).sum()) * world * args.steps / dt,
           'config': {'workload': 'config3_active_reset_8core', 'shots_per_gpu': n,
                      'global_shots_per_step': n * world},
           'roofline': {'bound': 'hbm', 'achieved': gbs, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                        'frac': gbs / HBM_PEAK_GBS, 'bytes_per_launch': alg}}
    pmc = os.path.join(REPO, 'profiles', PROFILE_TAG + '_active_reset_pmc.json')
    if os.path.exists(pmc):
        with open(pmc) as f:
            prof = json.load(f)
        res['roofline']['traffic'] = prof.get('hbm_bytes_per_launch')
        res['roofline']['valu'] = {k: prof.get(k) for k in ('valu_insts_per_wave', 'valu_issue_pct',
                                                            'valu_lane_util_pct', 'duration_ns', 'kernel')}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        import oracle
        threads = min(len(os.sched_getaffinity(0)), 16)
        want = ('summary', 'events', 'meas', 'hist')
        done, chunk, t0 = 0, 20000, time.perf_counter()
        while time.perf_counter() - t0 < args.cpu_seconds / 3:
            oracle.fast_run(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, done, chunk, threads, want)
            done += chunk
        dtc = time.perf_counter() - t0
        res['cpu_baseline'] = {'value': done * 8 / dtc, 'unit': 'core-shots/s', 'cores': threads, 'kind': 'port',
                               'sample': '{} shots x 8 cores of config 3, oracle_fast (OpenMP), {:.1f} s'.format(
                                   done, dtc)}
    del out
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--shots', type=int, default=10 ** 6, help='shots per GPU per step')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-seconds', type=float, default=12.0)
    ap.add_argument('--spg', type=int, default=1,
                    help='shots per delay point run back to back (1: delay k = shot mod 100)')
    ap.add_argument('--exec-flags', type=int, default=0, help='DPEMU_X_* execution knobs')
    ap.add_argument('--dds-seqs', type=int, default=128, help='RB sequences per GPU for the DDS leg (config 5)')
    ap.add_argument('--no-dds', action='store_true')
    ap.add_argument('--ar-shots', type=int, default=1250000, help='config-3 shots per GPU per step (0: skip the leg)')
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world > 1:
        # RCCL; DPEMU_BENCH_BACKEND=gloo rehearses the multi-rank path with
        # several ranks on fewer GPUs (never for measurement)
        dist.init_process_group(os.environ.get('DPEMU_BENCH_BACKEND', 'nccl'))
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)

    from distributed_processor_amd import _abi, sharding
    from distributed_processor_amd.emulator import Emulator, alloc_device_outputs

    ps = build_workload()
    emu = Emulator(local)
    emu.load(ps)
    n = args.shots
    spg = args.spg
    cfg = _abi.make_config(8, n_groups=ps.n_groups, shots_per_group=spg, max_cycles=1 << 20, event_cap=8,
                           trace_cap=0, meas_cap=2, meas_latency=64, seed=0x5EED, p1=0.5,
                           exec_flags=args.exec_flags)
    out = alloc_device_outputs(cfg, n, want=('summary', 'events', 'meas', 'hist'))
    stream = torch.cuda.current_stream()
    shot0, n = sharding.weak_shard(n, rank)
    # double-buffered histogram: batch k's all-reduce (the path's only exchange,
    # RCCL) runs on RCCL's stream while batch k+1's kernel runs
    hists = [out['hist'], torch.zeros_like(out['hist'])]
    pending = [None, None]
    n_steps = [0]

    def step():
        b = n_steps[0] % 2
        n_steps[0] += 1
        if pending[b] is not None:
            pending[b].wait()                          # this buffer's previous exchange is done
            pending[b] = None
        out['hist'] = hists[b]
        out['hist'].zero_()
        emu.run_device(cfg, n, shot0, out, stream)
        pending[b] = sharding.allreduce_histogram(out['hist'], async_op=True)

    def drain():
        for b in range(2):
            if pending[b] is not None:
                pending[b].wait()
                pending[b] = None

    for _ in range(args.warmup):
        step()
    drain()
    torch.cuda.synchronize()

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step()
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = sharding.max_over_ranks(time.perf_counter() - t0, device='cuda')
    # the roofline's kernel time: a second pass of the same steps with HIP
    # events recorded around the interpreter kernel, so the event records stay
    # out of the timed region (they cost ~4 % of a step)
    kernel_pass(emu, args.steps, step, drain)
    kt = emu.kernel_times()
    assert len(kt) == args.steps, kt
    kernel_ms = float(np.mean(kt))
    kernel_name = emu.last_kernel()

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

    # rocprofv3 PMC passes of this workload (scripts/gpu_r01.sh -> profiles/): HBM
    # bytes per launch, and the VALU view (instructions per wave, issue share,
    # active lanes per VALU instruction = divergence)
    traffic, valu = None, None
    pmc = os.path.join(REPO, 'profiles', PROFILE_TAG + '_interp_pmc.json')
    if os.path.exists(pmc):
        with open(pmc) as f:
            prof = json.load(f)
        traffic = prof.get('hbm_bytes_per_launch')
        valu = {k: prof.get(k) for k in ('valu_insts_per_wave', 'valu_issue_pct', 'valu_lane_util_pct',
                                         'duration_ns', 'kernel')}
        valu['source'] = os.path.relpath(pmc, REPO)

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
                   'shots_per_delay_point': spg,
                   'global_shots_per_step': n * world, 'parallelism': 'shots sharded, {} GPU(s)'.format(world)},
        'shots_per_s': value / 8,
        'qclk_cycles_per_s': cycles * world * args.steps / dt,
        'instructions_per_s': instrs * world * args.steps / dt,
        'kernel_ms': kernel_ms,
        'roofline': {'bound': 'hbm', 'achieved': achieved_gbs, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                     'frac': achieved_gbs / HBM_PEAK_GBS, 'traffic': traffic,
                     'bytes_per_launch': alg_bytes, 'kernel_ms': kernel_ms,
                     'kernel': 'dpemu::' + kernel_name, 'valu': valu},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result['cpu_baseline'] = cpu_baseline(ps, cfg, args.cpu_seconds)
    if not args.no_dds:
        result['dds'] = dds_leg(emu, args, world, rank, stream)
    if args.ar_shots > 0:
        result['active_reset'] = active_reset_leg(emu, args, world, rank, stream)
    if rank == 0:
        print(json.dumps(result), flush=True)
    emu.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
