"""Benchmark: batched emulation of assembled distproc machine code on MI355X.

One JSON line on rank 0.  The headline (BASELINE.json configs[1]) is config 2:
8-core (8-qubit) parallel Ramsey sweep, 100 delay points selected by shot, no
branching, 10^6 shots per GPU.  One step = one pass of the hot path over one
batch: the interpreter emulates every (shot, core) lane cycle-exactly and
writes the full pulse-event timeline, lane summaries, measurement records and
the outcome histogram to HBM; with N > 1 ranks the histograms are all-reduced
over RCCL (the path's only exchange), overlapped with the next
batch (sharding.HistogramPipeline).  Shots shard by global index (weak
scaling).  After the timed steps a fixed sample of lane timelines is gathered
to every rank (sharding.gather_sample).

Sub-objects on the same line, each with its own roofline and CPU baselines:
  "config1"       config 1: the reference's golden single-core program
                  (test_linear_compile_globalasm core 0) at 10^6 shots, beside
                  oracle_rtl (the per-clock stand-in for the Verilator testbench)
  "dds"           config 5: RB timelines (8 cores, depth 200) synthesised to
                  int16 I/Q on 16 channels per sequence at 16 samples/clk;
                  one synthesis per step on one stream (--dds-depth > 1 also
                  measures batches in flight, dds.SynthesisPipeline)
  "active_reset"  config 3: fproc_meas branching + sync barriers, 1.25*10^6
                  shots per GPU (10^7 over 8 GPUs)
  "lut"           config 3's circuit through the fproc_lut back end: every
                  core waits on a syndrome LUT over the 8 measurements
  "demod"         config 3 with the readout demodulation model (meas_model
                  DEMOD: each rdlo window demodulates its rdrv return into an
                  accumulated I/Q, written per readout, and a per-core
                  discriminator decides the outcome); its cost over the
                  STATE model's leg is on the line ("model_cost")
  "rb"            config 4 at its stated size: 10^5 distinct 2-core depth-200
                  RB sequences x 10 shots per GPU, one batch per step
                  (--rb-depth > 1 also measures batches in flight,
                  emulator.RunPipeline)

CPU baselines (rank 0, one GPU): the reference's Verilator/cocotb testbench
cannot run here or on the box, so each leg reports
oracle_fast (the event-driven C restatement, OpenMP over shots, every core
this process may use) as `cpu_baseline.value`, and oracle_rtl (the per-clock
restatement: one evaluation per clock like Verilator) at 1 thread and at all
cores beside it; each a median of 5 timed runs of a fixed sample after one
warm-up run.

    python bench.py --gpus 1 --steps 20 --warmup 3
    torchrun --nproc-per-node N bench.py --gpus N ...
"""

import argparse
import csv
import glob
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s
PROFILE_TAG = 'r06'            # profiles/<tag>_*: rocprofv3 kernel stats and PMC passes of this bench


def _valu_peak():
    """the measured wave64 integer-VALU issue peak (instructions/s, whole chip)
    and its cycles per instruction: scripts/micro/valu_peak.hip under
    rocprofv3 with SQ_INSTS_VALU + GRBM_GUI_ACTIVE in one pass
    (profiles/r04_valu_peak_pmc.json, scripts/valu_peak_summary.py)"""
    with open(os.path.join(REPO, 'profiles', 'r04_valu_peak_pmc.json')) as f:
        v = json.load(f)
    return v['peak_valu_insts_per_s'], v['peak_cycles_per_inst'], v['peak_variant']


VALU_PEAK, VALU_CPI, VALU_PEAK_VARIANT = _valu_peak()
# where the profile summaries are read from: the committed profiles/, or
# (DPEMU_BENCH_PROFILES) the summaries of a profile pass just taken on the same box
PROFILE_DIR = os.environ.get('DPEMU_BENCH_PROFILES') or os.path.join(REPO, 'profiles')


def _kernel_valu_peaks():
    """each bench kernel's own VALU issue peak: its opcode mix weighted by the
    measured per-opcode issue costs (scripts/kernel_mixes.sh ->
    profiles/<tag>_kernel_valu_peaks.json); {readable name: record}"""
    path = os.path.join(PROFILE_DIR, '{}_kernel_valu_peaks.json'.format(PROFILE_TAG))
    if not os.path.exists(path):
        return {}
    with open(path) as f:
        return {k['name']: k for k in json.load(f)['kernels']}


KERNEL_VALU_PEAKS = _kernel_valu_peaks()


def kernel_key(name):
    """'void dpemu::branch_kernel<11, 8>(dpemu::KParams)' -> 'branch_kernel<11,8>'"""
    n = (name or '').split('(')[0].replace('void ', '').replace('dpemu::', '').replace(' ', '')
    return n


# ---------------------------------------------------------------------------- helpers
def host_cores():
    """threads for the CPU baselines: every core this process may run on
    (sched_getaffinity), within the job's CPU share when the harness sets one
    (OMP_NUM_THREADS); both recorded"""
    aff = len(os.sched_getaffinity(0))
    omp = os.environ.get('OMP_NUM_THREADS')
    use = min(aff, int(omp)) if omp and omp.isdigit() and int(omp) > 0 else aff
    return use, {'nproc': aff, 'os_cpu_count': os.cpu_count(), 'omp_num_threads': omp}


def share_note(threads, info):
    """what the CPU baseline's thread count is a share of (BASELINE.md:46 asks
    for every host core; the harness grants a one-GPU job OMP_NUM_THREADS of
    the machine's nproc, and the baseline stays inside that share)"""
    return ('{} threads = the job\'s CPU share (OMP_NUM_THREADS={}) of the {} CPUs this process sees; any GPU/CPU '
            'ratio taken from `value` compares against {}/{} of the host, not all of it'.format(
                threads, info.get('omp_num_threads'), info.get('nproc'), threads, info.get('nproc')))


def median_rate(run, units_per_n, n0, target_s=0.8, reps=5):
    """one warm-up / calibration run of n0, then `reps` timed runs of a fixed
    n sized to ~target_s each; returns (median units/s, n, [seconds])"""
    t = time.perf_counter()
    run(n0)
    dt = max(time.perf_counter() - t, 1e-4)
    n = max(1, int(n0 * target_s / dt))
    times = []
    for _ in range(reps):
        t = time.perf_counter()
        run(n)
        times.append(time.perf_counter() - t)
    return n * units_per_n / float(np.median(times)), n, times


def cpu_baselines(ps, cfg, horizon, what, all_cores=False, ro=None):
    """oracle_fast (the job's threads) and oracle_rtl (1 thread, the job's
    threads) on the leg's workload.  all_cores: also oracle_fast at one
    thread, and the whole host's rate (BASELINE.md:46 asks for all host
    cores) extrapolated from the job's share -- not run at nproc threads: the
    harness grants a one-GPU job OMP_NUM_THREADS of the host's CPUs and asks
    it to keep its worker pools within that share."""
    import oracle
    threads, info = host_cores()
    C = cfg.cores_per_shot
    want = ('summary', 'events', 'meas', 'hist')
    fast = lambda k: lambda n: oracle.fast_run(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, 0, n, k, want, ro=ro)
    rtl = lambda k: lambda n: oracle.rtl_run_batch(cfg, ps.words, ps.offsets, ps.n_instr, ps.table, 0, n, horizon, k,
                                                   ro=ro)
    f_rate, f_n, f_t = median_rate(fast(threads), C, 2000)
    r1_rate, r1_n, r1_t = median_rate(rtl(1), C, 20)
    ra_rate, ra_n, ra_t = median_rate(rtl(threads), C, 20 * threads)
    res = dict(value=f_rate, unit='core-shots/s', cores=threads, kind='port', **info,
               per_core=f_rate / threads, share_note=share_note(threads, info),
               method='median of 5 timed runs of a fixed sample after one warm-up run',
               sample='{}: {} shots x {} cores per oracle_fast run (event-driven C restatement, OpenMP over '
                      'shots, {} threads)'.format(what, f_n, C, threads),
               oracle_fast={'value': f_rate, 'threads': threads, 'shots_per_run': f_n,
                            'run_s': [round(x, 4) for x in f_t]},
               oracle_rtl={'value_1_thread': r1_rate, 'value_all_cores': ra_rate, 'threads': threads,
                           'shots_per_run': [r1_n, ra_n],
                           'note': 'per-clock restatement of hdl/ (one evaluation per clock, the closest '
                                   'stand-in for the Verilator testbench of cocotb/proc/Makefile:1-14, '
                                   'which cannot run here)'})
    if all_cores:
        f1_rate, f1_n, _ = median_rate(fast(1), C, 200)
        nproc = info['nproc']
        res['oracle_fast']['value_1_thread'] = f1_rate
        eff = f_rate / (f1_rate * threads)
        res['all_cores'] = {
            'value': f_rate * nproc / threads, 'unit': 'core-shots/s', 'threads': nproc, 'kind': 'extrapolated',
            'bound': 'upper', 'scaling_1_to_{}_threads'.format(threads): eff,
            'note': 'an UPPER BOUND on oracle_fast over all {} host CPUs: the measured {}-thread rate scaled '
                    'linearly, although the 1 -> {} thread efficiency measured beside it is only {:.2f}; not run '
                    'at {} threads because the harness grants this job {} of them'.format(
                        nproc, threads, threads, eff, nproc, threads)}
    return res


def pmc(name):
    """per-launch PMC summary of a kernel from profiles/<tag>_<name>_pmc.json (scripts/pmc_summary.py)"""
    path = os.path.join(PROFILE_DIR, '{}_{}_pmc.json'.format(PROFILE_TAG, name))
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f)


def rocprof_avg_ms(kernel_substr):
    """the committed rocprofv3 --stats average of a kernel (profiles/<tag>_*kernel_stats.csv)"""
    for path in sorted(glob.glob(os.path.join(PROFILE_DIR, PROFILE_TAG + '*kernel_stats.csv'))):
        with open(path) as f:
            for r in csv.DictReader(f):
                if kernel_substr in r.get('Name', ''):
                    return float(r['AverageNs']) * 1e-6
    return None


def valu_view(prof, kernel_ms=None, instrs=None):
    """the kernel's VALU roofline beside its HBM one: VALU instructions per
    launch (rocprof SQ_INSTS_VALU) over the kernel time against the measured
    integer-VALU issue peak -- at the bench's HIP-event kernel time (`frac`)
    and at rocprof's trace duration (`frac_rocprof`, = pmc_summary's
    valu_frac_of_measured_peak) -- plus the same-pass PMC ratios"""
    if not prof or not prof.get('SQ_INSTS_VALU'):
        return None
    n = float(prof['SQ_INSTS_VALU'])
    # graded against the measured wave64 integer-VALU issue peak (the fastest
    # add / shift / xor mix, profiles/r04_valu_peak_pmc.json); the kernel's
    # static opcode mix weighted by single-opcode chain costs
    # (profiles/<tag>_kernel_valu_peaks.json) is reported beside it as
    # frac_own_mix -- that table does not predict a mixed kernel's issue rate
    # (DESIGN.md §6), so it is not the grading peak
    own = KERNEL_VALU_PEAKS.get(kernel_key(prof.get('kernel')))
    peak = VALU_PEAK
    v = {'bound': 'valu', 'unit': 'wave64 VALU instr/s', 'peak': peak, 'peak_cycles_per_inst': VALU_CPI,
         'peak_source': 'profiles/r04_valu_peak_pmc.json ({})'.format(VALU_PEAK_VARIANT),
         'valu_insts_per_launch': n}
    if own:
        v['own_mix_peak'] = own['peak_valu_insts_per_s']
    if kernel_ms:
        v['achieved'] = n / (kernel_ms * 1e-3)
        v['frac'] = v['achieved'] / peak
        if own:
            v['frac_own_mix'] = v['achieved'] / own['peak_valu_insts_per_s']
    if prof.get('duration_ns'):
        v['frac_rocprof'] = n / (prof['duration_ns'] * 1e-9) / peak
    if instrs:
        # VALU lane-ops per emulated instruction (the kernel's constant)
        v['valu_ops_per_instruction'] = n * 64 / instrs
    for k in ('valu_insts_per_wave', 'valu_issue_pct', 'valu_lane_util_pct', 'duration_ns',
              'kernel', 'warnings'):
        if prof.get(k) is not None:
            v[k] = prof.get(k)
    return v


def hbm_roofline(alg_bytes, kernel_ms, ms_per_step, kernel, prof, rocprof_key):
    """HBM roofline of a kernel: algorithmic bytes / kernel time.  The kernel
    time is the median HIP-event duration of the launches, capped at the
    step's own time (the event pair cannot make the kernel longer than the
    whole step); the committed rocprofv3 kernel-trace average of this leg's
    launch shape (profiles/<tag>_<leg>_pmc.json duration_ns; else the
    kernel's --stats row) gives a second fraction"""
    k_ms = min(kernel_ms, ms_per_step)
    gbs = alg_bytes / (k_ms * 1e-3) / 1e9
    r = {'bound': 'hbm', 'achieved': gbs, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s', 'frac': gbs / HBM_PEAK_GBS,
         'traffic': prof.get('hbm_bytes_per_launch') if prof else None, 'bytes_per_launch': alg_bytes,
         'kernel_ms': k_ms, 'kernel_ms_events': kernel_ms, 'kernel': kernel}
    rp = (prof['duration_ns'] * 1e-6 if prof.get('duration_ns') else rocprof_avg_ms(rocprof_key)) if prof else None
    if rp:
        r['kernel_ms_rocprof'] = rp
        r['frac_rocprof'] = alg_bytes / (rp * 1e-3) / 1e9 / HBM_PEAK_GBS
    return r


def bytes_per_lane(summary_np, cfg, acc=False):
    """algorithmic HBM bytes written per lane: 32 B summary + 16 B per event
    record + 8 B per measurement record (+ 8 B of accumulated I/Q per
    measurement when the run writes dpemu_outputs.acc)"""
    n_ev = np.minimum(summary_np[:, 2], cfg.event_cap).astype(np.float64)
    n_me = np.minimum(summary_np[:, 5], cfg.meas_cap).astype(np.float64)
    return 32.0 + 16.0 * n_ev + (16.0 if acc else 8.0) * n_me


SETTLE_S = 0.3
LANE_ORDER_NAMES = ('core-major', 'shot-major')   # dpemu_config.lane_order


def settle(step, drain, seconds=SETTLE_S, sync=None, device='cuda'):
    """untimed steps for about `seconds` of wall time: the GPU's clocks ramp
    up under load, and a leg that starts after an idle host-side phase would
    otherwise time its first milliseconds at low clocks (config 2 measured
    0.202 ms per step cold against 0.176-0.179 warm, scripts/step_probe.py).
    Every rank runs the SAME number of steps (a step may enqueue a
    collective): the count comes from 3 timed steps, maxed over ranks."""
    from distributed_processor_amd import sharding
    if sync is None:
        import torch
        sync = torch.cuda.synchronize
    sync()
    t0 = time.perf_counter()
    for _ in range(3):
        step()
    drain()
    sync()
    per = (time.perf_counter() - t0) / 3
    n = int(sharding.max_over_ranks(float(int(seconds / max(per, 1e-6))), device=device))
    for i in range(n):
        step()
        if i % 10 == 9:
            drain()
            sync()
    drain()
    sync()
    return n + 3


def timed(step, drain, steps, warmup, world):
    """clock settle, warm-up, then exactly `steps` steps between barrier +
    synchronize; returns the max over ranks of the wall time"""
    import torch
    from distributed_processor_amd import sharding
    settle(step, drain)
    for _ in range(warmup):
        step()
    drain()
    torch.cuda.synchronize()
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    drain()
    torch.cuda.synchronize()
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    return sharding.max_over_ranks(time.perf_counter() - t0, device='cuda')


def kernel_pass(emu, steps, step, drain):
    """`steps` more steps with the library's HIP events around each main
    kernel launch, outside the timed region; returns their median ms"""
    import torch
    torch.cuda.synchronize()
    emu.kernel_times()
    emu.kernel_timing(True)
    for _ in range(steps):
        step()
    drain()
    torch.cuda.synchronize()
    emu.kernel_timing(False)
    kt = emu.kernel_times()
    assert len(kt) == steps, kt
    return float(np.median(kt))


def block_pass(launch, k):
    """ms per launch of `k` back-to-back launches of one kernel between two
    HIP events on the launch stream (torch's current stream): per-launch event
    pairs add their own overhead to a 0.2-ms kernel, a block of k launches
    only the k - 1 dependent-launch gaps"""
    import torch
    launch()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(k):
        launch()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / k


def interp_kernel_ms(emu, cfg, n, shot0, out, stream, steps, step, drain):
    """the interpreter kernel's time per launch: the median of the library's
    HIP-event pairs around the kernel inside `steps` real steps (the same
    launch as the timed ones; it agrees with rocprofv3's average), beside a
    block of back-to-back launches without the histogram output"""
    nohist = {k: v for k, v in out.items() if k not in ('hist', 'hist_next')}
    ev = kernel_pass(emu, steps, step, drain)
    blk = block_pass(lambda: emu.run_device(cfg, n, shot0, nohist, stream), max(steps, 10))
    return ev, blk


def fill_gbps(device='cuda'):
    """a torch fill of 1 GiB on this box (HIP events): the store rate the
    HBM roofline's 8 TB/s compares against, measured (boxes differ)"""
    import torch
    buf = torch.empty(1 << 28, dtype=torch.int32, device=device)
    for _ in range(3):
        buf.fill_(1)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10):
        buf.fill_(2)
    b.record()
    torch.cuda.synchronize()
    gbs = buf.numel() * 4 * 10 / (a.elapsed_time(b) * 1e-3) / 1e9
    del buf
    return gbs


def _sig(x, n=4):
    return None if x is None else float('{:.{}g}'.format(x, n))


def compact_leg(res):
    """the few numbers of a leg that must survive a truncated record (the
    driver keeps the last 2,000 characters of stdout): value, step and kernel
    ms, the graded roofline's bound and fraction, and for a pipelined leg the
    whole step's fraction / the one-context step"""
    roof = res.get('roofline') or {}
    c = {'value': _sig(res['value']), 'ms_per_step': _sig(res['ms_per_step']),
         'kernel_ms': _sig(roof.get('kernel_ms', res.get('kernel_ms'))), 'bound': roof.get('bound'),
         'frac': _sig(roof.get('frac'), 3)}
    if roof.get('bound') == 'valu' and roof.get('hbm'):
        c['hbm_frac'] = _sig(roof['hbm'].get('frac'), 3)
    if 'step_roofline_frac' in res:
        c['step_frac'] = _sig(res['step_roofline_frac'], 3)
    if 'serial_ms_per_step' in res:
        c['serial_ms'] = _sig(res['serial_ms_per_step'])
    if 'pipelined_ms_per_step' in res:
        c['pipe_ms'] = _sig(res['pipelined_ms_per_step'])
    if 'model_cost' in res:
        c['cost_x'] = _sig(res['model_cost']['kernel_ratio'], 3)
    if 'cpu_baseline' in res:
        c['cpu'] = _sig(res['cpu_baseline']['value'], 3)
        if 'all_cores' in res['cpu_baseline']:
            c['cpu_all'] = _sig(res['cpu_baseline']['all_cores']['value'], 3)
    return c


# ---------------------------------------------------------------------------- legs
def leg_ramsey(emu, args, world, rank, stream):
    """config 2 (the headline line)"""
    import torch
    from distributed_processor_amd import _abi, sharding, workloads
    from distributed_processor_amd.emulator import ProgramSet, alloc_device_outputs
    ps = ProgramSet(workloads.config2_ramsey(n_cores=8, n_points=100))
    emu.load(ps)
    # shot-major lanes: a wave (8 shots x 8 cores) writes each event slot as
    # one 1-KiB run (core-major: two 512-B runs), 0.180 -> 0.159 ms per kernel
    # (scripts/lane_order_ab.py, profiles/r02_lane_order_ab.json)
    cfg = _abi.make_config(8, n_groups=ps.n_groups, max_cycles=1 << 20, event_cap=8, trace_cap=0, meas_cap=2,
                           meas_latency=64, seed=0x5EED, p1=0.5, lane_order=_abi.LANES_SHOT_MAJOR)
    shot0, n = sharding.weak_shard(args.shots, rank)
    out = alloc_device_outputs(cfg, n, want=('summary', 'events', 'meas', 'hist'))
    # direct histogram atomics (100 groups x 256 bins): each run accumulates
    # into a buffer the previous run's kernel zeroed (dpemu_outputs.hist_next)
    # -- no memset launch per step (4.4 us, 2.5 % of a step, with hist_assign)
    pipe = sharding.HistogramPipeline(out['hist'], zero=False, clear_next=True)

    def launch(h, h_next):
        out['hist'], out['hist_next'] = h, h_next
        emu.run_device(cfg, n, shot0, out, stream)
    step = lambda: pipe.step(launch)
    dt = timed(step, pipe.drain, args.steps, args.warmup, world)
    kernel_ms, kernel_ms_blk = interp_kernel_ms(emu, cfg, n, shot0, out, stream, args.steps, step, pipe.drain)
    kernel = emu.last_kernel()
    # accounting from the last step's outputs (identical every step)
    summ = out['summary'].cpu().numpy().view(np.uint32)
    s = _abi.unpack_summary(summ)
    assert (s['status'] == _abi.ST_DONE).all(), 'not every lane reached DONE'
    assert int(pipe.result().sum().item()) == n * world
    # the north star's timeline gather: a fixed sample of lanes (summaries and
    # their event records) from every rank, after the timed region
    lanes = torch.from_numpy(sharding.sample_lanes(n, 8, 16, cfg.lane_order)).to('cuda')
    sample = torch.cat([out['summary'][lanes], out['events'][:, lanes].permute(1, 0, 2).reshape(len(lanes), -1)], 1)
    gathered = sharding.gather_sample(sample)
    assert gathered.shape[0] == world and torch.equal(gathered[rank], sample)
    ms_step = dt / args.steps * 1e3
    alg = float(bytes_per_lane(summ, cfg).sum())
    prof = pmc('ramsey') if args.shots == 10 ** 6 else None         # profiled at the default size only
    roof = hbm_roofline(alg, kernel_ms, ms_step, 'dpemu::' + kernel, prof, 'straight_kernel')
    roof['kernel_ms_block'] = kernel_ms_blk
    roof['valu'] = valu_view(prof, roof['kernel_ms'], float(s['n_instr'].astype(np.float64).sum()))
    res = {'value': n * 8 * world * args.steps / dt, 'ms_per_step': ms_step,
           'shots_per_s': n * world * args.steps / dt,
           'qclk_cycles_per_s': float(s['t_end'].astype(np.float64).sum()) * world * args.steps / dt,
           'instructions_per_s': float(s['n_instr'].astype(np.float64).sum()) * world * args.steps / dt,
           'kernel_ms': kernel_ms, 'roofline': roof,
           'timeline_gather': {'ranks': int(gathered.shape[0]), 'lanes_per_rank': int(len(lanes)),
                               'bytes': int(gathered.numel() * gathered.element_size())},
           'config': {'workload': 'config2_ramsey_8core_100pt', 'shots_per_gpu': n, 'cores_per_shot': 8,
                      'lane_order': LANE_ORDER_NAMES[cfg.lane_order],
                      'global_shots_per_step': n * world, 'parallelism': 'shots sharded, {} GPU(s)'.format(world)}}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res['cpu_baseline'] = cpu_baselines(ps, cfg, 4096, 'config 2 Ramsey', all_cores=True)
    del out
    torch.cuda.empty_cache()
    return res


def leg_config1(emu, args, world, rank, stream):
    """config 1 (BASELINE configs[0]): the reference's own golden machine
    code -- core 0 of python/test/test_outputs/test_linear_compile_globalasm.txt
    (phase reset, X90, readout drive, readout LO, done; the fixture
    tests/golden/cmd_buf_golden.json holds its bytes) -- at 10^6 shots per GPU.
    The reference runs this program on the single-core Verilator/cocotb
    testbench (cocotb/proc/Makefile:1-14), which cannot run here or on the
    box: oracle_rtl, the per-clock restatement of hdl/, is its stand-in in
    cpu_baseline (1 thread and every granted thread), oracle_fast beside it."""
    import torch
    from distributed_processor_amd import _abi, sharding
    from distributed_processor_amd.emulator import ProgramSet, alloc_device_outputs
    with open(os.path.join(REPO, 'tests', 'golden', 'cmd_buf_golden.json')) as f:
        gold = json.load(f)
    ps = ProgramSet([{0: bytes.fromhex(gold['cores']['0']['cmd_buf'])}])
    emu.load(ps)
    cfg = _abi.make_config(1, max_cycles=10000, event_cap=8, trace_cap=0, meas_cap=4, seed=0x5EED, p1=0.5)
    shot0, n = sharding.weak_shard(args.c1_shots, rank)
    out = alloc_device_outputs(cfg, n, want=('summary', 'events', 'meas', 'hist'))
    pipe = sharding.HistogramPipeline(out['hist'], zero=False, clear_next=True)

    def launch(h, h_next):
        out['hist'], out['hist_next'] = h, h_next
        emu.run_device(cfg, n, shot0, out, stream)
    step = lambda: pipe.step(launch)
    dt = timed(step, pipe.drain, args.steps, args.warmup, world)
    kernel_ms, kernel_ms_blk = interp_kernel_ms(emu, cfg, n, shot0, out, stream, args.steps, step, pipe.drain)
    kernel = emu.last_kernel()
    summ = out['summary'].cpu().numpy().view(np.uint32)
    s = _abi.unpack_summary(summ)
    assert (s['status'] == _abi.ST_DONE).all(), 'config 1: not every lane reached DONE'
    assert int(pipe.result().sum().item()) == n * world
    ms_step = dt / args.steps * 1e3
    alg = float(bytes_per_lane(summ, cfg).sum())
    prof = pmc('config1') if args.c1_shots == 10 ** 6 else None
    roof = hbm_roofline(alg, kernel_ms, ms_step, 'dpemu::' + kernel, prof, 'straight_kernel')
    roof['kernel_ms_block'] = kernel_ms_blk
    roof['valu'] = valu_view(prof, roof['kernel_ms'], float(s['n_instr'].astype(np.float64).sum()))
    res = {'metric': 'emulated core-shots/s (config 1: the reference\'s golden single-core program, '
                     'test_linear_compile_globalasm core 0)',
           'value': n * world * args.steps / dt, 'unit': 'core-shots/s', 'ms_per_step': ms_step, 'kernel_ms': kernel_ms,
           'qclk_cycles_per_s': float(s['t_end'].astype(np.float64).sum()) * world * args.steps / dt,
           'instructions_per_s': float(s['n_instr'].astype(np.float64).sum()) * world * args.steps / dt,
           'config': {'workload': 'config1_golden_linear_core0', 'shots_per_gpu': n, 'cores_per_shot': 1,
                      'program': gold['source'] + ' core 0', 'commands': int(ps.words.shape[0])},
           'roofline': roof}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cb = cpu_baselines(ps, cfg, 2048, 'config 1 golden program')
        cb['substitute_for'] = ('the reference\'s single-core Verilator/cocotb testbench (cocotb/proc/Makefile:1-14, '
                                'sim_modules/toplevel_sim.sv), absent from this image: oracle_rtl is the per-clock '
                                'restatement of the same RTL, timed at 1 thread and at every granted thread')
        res['cpu_baseline'] = cb
    del out
    torch.cuda.empty_cache()
    return res


def leg_dds(emu, args, world, rank, stream):
    """config 5: DDS over the config-4 RB timelines, 8 cores x {qdrv, rdrv}
    (--dds-workload rb2q: four qubit pairs of two-qubit Clifford RB, config 4's
    generator; rb: the RB-shaped 8-core timelines of rounds 2-6)"""
    import torch
    from distributed_processor_amd import _abi, isa, sharding, workloads
    from distributed_processor_amd.dds import ChannelPlan, SynthesisPipeline
    from distributed_processor_amd.emulator import ProgramSet, alloc_device_outputs
    if args.dds_workload == 'rb2q':
        ps = workloads.config4_rb2q_set(args.dds_seqs, 200, n_cores=8)
    else:
        ps = ProgramSet(workloads.config4_rb(n_seq=args.dds_seqs, depth=200, n_cores=8))
    emu.load(ps)
    ops = ps.words[:, 3] >> 28
    strobes = np.add.reduceat(((ops == isa.OP_PULSE_TRIG) | (ops == isa.OP_PULSE_RESET)).astype(np.int64),
                              ps.offsets.astype(np.int64))
    cfg = _abi.make_config(8, n_groups=ps.n_groups, max_cycles=1 << 20, event_cap=max(512, int(strobes.max()) + 1),
                           meas_cap=4, meas_latency=64, seed=0x5EED)
    shot0, n = sharding.weak_shard(args.dds_seqs, rank)
    ev = alloc_device_outputs(cfg, n, want=('summary', 'events'))
    emu.run_device(cfg, n, shot0, ev, stream)
    torch.cuda.synchronize()
    s = _abi.unpack_summary(ev['summary'].cpu().numpy().view(np.uint32))
    assert (s['status'] == _abi.ST_DONE).all() and (s['n_events'] <= cfg.event_cap).all()
    n_cyc = int(s['t_end'].max()) + 8
    n_samples = (n_cyc * 16 + 3) // 4 * 4
    params = {i: (e['samples_per_clk'], e['interp_ratio']) for i, e in enumerate(workloads.ELEMS)}
    chans = [(shot0 + q, c, e) for q in range(n) for c in range(8) for e in (workloads.QDRV, workloads.RDRV)]
    plan = ChannelPlan(ps, cfg, shot0, n, chans, params)
    iq = torch.empty((plan.n_channels, n_samples), dtype=torch.int32, device='cuda')
    # a step is one batch's whole synthesis (dds_index_kernel + dds_tile_kernel)
    # on one context and stream, in call order
    serial = lambda: emu.synthesize(plan, ev, n_samples, iq, stream)
    dt_serial = timed(serial, lambda: None, args.steps, args.warmup, world)
    kernel_ms = kernel_pass(emu, args.steps, serial, lambda: None)
    torch.cuda.synchronize()
    dt, mode = dt_serial, 'serial'
    pipe_ms = None
    if args.dds_depth > 1:
        # opt-in: `dds_depth` batches in flight on as many contexts / streams
        # (dds.SynthesisPipeline); the flag, not the faster measurement, picks
        # the reported mode (no best-of-two bias), both on the line
        pipe = SynthesisPipeline(torch.cuda.current_device(), depth=args.dds_depth, streams=args.pipe_streams)
        last = {}

        def step():
            last['iq'] = pipe.synthesize(plan, ev, n_samples)[0]
        dt_pipe = timed(step, pipe.drain, args.steps, args.warmup, world)
        pipe.drain()
        # the pipelined batches and the serial ones must produce the same I/Q
        # (a cross-stream ordering bug would still yield a throughput number)
        assert torch.equal(last['iq'], iq), 'config 5: pipelined and serial I/Q differ'
        pipe.close()
        pipe_ms = dt_pipe / args.steps * 1e3
        dt, mode = dt_pipe, 'pipelined'
    samples = plan.n_channels * n_samples
    ms_step = dt / args.steps * 1e3
    prof = pmc('dds') if args.dds_seqs == 128 else None
    # the tile kernel's own roofline, capped at the one-context step
    roof = hbm_roofline(samples * 4, kernel_ms, dt_serial / args.steps * 1e3, 'dpemu::dds_tile_kernel', prof,
                        'dds_tile_kernel')
    res = {'metric': 'DDS I/Q GSamples/s (config 5: RB timelines, 16 channels/sequence, 16 samples/clk)',
           'value': samples * world * args.steps / dt / 1e9, 'unit': 'GSamples/s', 'ms_per_step': ms_step,
           'kernel_ms': kernel_ms, 'dtype': 'int16 I/Q',
           'step': 'dds_index_kernel (per-channel event index and counts; each tile\'s window found in the '
                   'tile kernel) + dds_tile_kernel per batch on one stream ({}); kernel_ms and the roofline hold '
                   'dds_tile_kernel alone, value and ms_per_step the whole step'.format(
                       'serial' if args.dds_depth <= 1 else
                       '{} batches in flight reported (--dds-depth), the serial step measured beside it'.format(
                           args.dds_depth)),
           'step_mode': mode, 'batches_in_flight': args.dds_depth if mode == 'pipelined' else 1,
           'step_roofline_frac': samples * 4 / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS,
           'serial_ms_per_step': dt_serial / args.steps * 1e3,
           'config': {'workload': 'config5_dds_{}8'.format(args.dds_workload), 'sequences_per_gpu': n,
                      'channels_per_gpu': plan.n_channels,
                      'samples_per_channel': n_samples, 'rb_depth': 200},
           'roofline': roof}
    if pipe_ms is not None:
        res['pipelined_ms_per_step'] = pipe_ms
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        import oracle
        threads, info = host_cores()
        host_ev = {k: v.cpu().numpy() for k, v in ev.items()}

        def run(k):
            oracle.dds(plan.desc[:k], host_ev['summary'], host_ev['events'], plan.env, plan.freq, n_samples,
                       plan.event_cap, threads)
        rate, k, times = median_rate(run, n_samples, max(threads, 16))
        res['cpu_baseline'] = dict(value=rate / 1e9, unit='GSamples/s', cores=threads, kind='port', **info,
                                   per_core=rate / 1e9 / threads, share_note=share_note(threads, info),
                                   method='median of 5 timed runs of a fixed sample after one warm-up run',
                                   sample='{} channels x {} samples of the config-5 timelines per run, oracle_dds '
                                          '(C restatement, OpenMP over channels)'.format(k, n_samples))
    del iq, ev
    torch.cuda.empty_cache()
    return res


def leg_active_reset(emu, args, world, rank, stream, lut=False, demod=False):
    """config 3 (BASELINE configs[2]): 8-core active reset -- readout,
    fproc_meas branch to a conditional X180, sync barriers -- 10^7 shots per
    step over 8 GPUs, i.e. 1.25*10^6 shots per GPU (weak).  lut: the same
    circuit through the fproc_lut back end (workloads.config3_lut: every core
    waits on a syndrome LUT over all 8 measurements, hdl/fproc_lut.sv).
    demod: the same circuit with the readout demodulation model
    (workloads.config3_demod: the rdlo window demodulates the rdrv return,
    the accumulated I/Q of every readout is an output, a per-core
    discriminator decides; meas_valid at the same cycles as the STATE leg)"""
    import torch
    from distributed_processor_amd import _abi, sharding, workloads
    from distributed_processor_amd.emulator import ProgramSet, alloc_device_outputs
    ps = ProgramSet(workloads.config3_lut(8) if lut else workloads.config3_active_reset(8))
    emu.load(ps)
    lut_kw = dict(fproc_mode=_abi.FPROC_LUT, lut_mask=0xFF, lut_table=workloads.config3_lut_table(8)) if lut else {}
    if demod:
        lut_kw = dict(demod=workloads.config3_demod(ps))
    cfg = _abi.make_config(8, n_groups=ps.n_groups, max_cycles=50000, event_cap=16, trace_cap=0, meas_cap=4,
                           meas_latency=workloads.CONFIG3_DEMOD_LATENCY if demod else workloads.CONFIG3_MEAS_LATENCY,
                           seed=0x5EED, p1=0.5, hist_assign=True,
                           lane_order=_abi.LANES_SHOT_MAJOR, **lut_kw)   # whole-line event stores
    shot0, n = sharding.weak_shard(args.ar_shots, rank)
    out = alloc_device_outputs(cfg, n, want=('summary', 'events', 'meas', 'hist') + (('acc',) if demod else ()))
    pipe = sharding.HistogramPipeline(out['hist'], zero=False)     # each run assigns its histogram

    def launch(h):
        out['hist'] = h
        emu.run_device(cfg, n, shot0, out, stream)
    step = lambda: pipe.step(launch)
    dt = timed(step, pipe.drain, args.steps, args.warmup, world)
    kernel = emu.last_kernel()
    kernel_ms, kernel_ms_blk = interp_kernel_ms(emu, cfg, n, shot0, out, stream, args.steps, step, pipe.drain)
    summ = out['summary'].cpu().numpy().view(np.uint32)
    s = _abi.unpack_summary(summ)
    assert (s['status'] == _abi.ST_DONE).all(), 'config 3: not every lane reached DONE'
    assert int(pipe.result().sum().item()) == n * world
    alg = float(bytes_per_lane(summ, cfg, acc=demod).sum())
    pname = 'lut' if lut else 'demod' if demod else 'active_reset'
    prof = pmc(pname) if args.ar_shots == 1250000 else None
    ms_step = dt / args.steps * 1e3
    roof = hbm_roofline(alg, kernel_ms, ms_step, 'dpemu::' + kernel, prof, 'branch_kernel')
    roof['kernel_ms_block'] = kernel_ms_blk
    roof['valu'] = valu_view(prof, roof['kernel_ms'], float(s['n_instr'].astype(np.float64).sum()))
    res = {'metric': ('emulated core-shots/s (config 3 via the fproc_lut back end: syndrome LUT over 8 '
                      'measurements + sync, 1.25e6 shots/GPU)') if lut else
                     ('emulated core-shots/s (config 3 with the readout demodulation model: rdrv return x rdlo '
                      'LO accumulated per readout, per-core discriminator, 1.25e6 shots/GPU)') if demod else
                     ('emulated core-shots/s (config 3: 8-core active reset, fproc_meas branch + sync, '
                      '1.25e6 shots/GPU)'),
           'value': n * 8 * world * args.steps / dt, 'unit': 'core-shots/s', 'shots_per_s': n * world * args.steps / dt,
           'ms_per_step': ms_step, 'kernel_ms': kernel_ms,
           'instructions_per_s': float(s['n_instr'].astype(np.float64).sum()) * world * args.steps / dt,
           'kernel': kernel,
           'config': {'workload': 'config3_lut_8core' if lut else 'config3_demod_8core' if demod else
                      'config3_active_reset_8core', 'shots_per_gpu': n,
                      'global_shots_per_step': n * world,
                      'lane_order': LANE_ORDER_NAMES[cfg.lane_order]},
           'roofline': roof}
    if demod:
        # the first readout's assignment against the prepared state (Philox word 0 of (shot, core, 0))
        import oracle
        st = np.array([[oracle.lib().oracle_philox_u32(0x5EED, int(shot0 + i), c, 0) < (1 << 31)
                        for c in range(8)] for i in range(2048)])
        res['assignment_fidelity'] = float(((s['meas_bits'][:2048 * 8] & 1).reshape(2048, 8) == st).mean())
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res['cpu_baseline'] = cpu_baselines(ps, cfg, 8192, 'config 3 ' + ('syndrome LUT' if lut else
                                                                         'demod readout' if demod else 'active reset'),
                                            ro=ps.readout_freqs(cfg.ro_drv_elem, cfg.meas_elem) if demod else None)
    del out
    torch.cuda.empty_cache()
    return res


def leg_rb(emu, args, world, rank, stream, shaped=False):
    """config 4 at its stated size: 10^5 distinct two-qubit Clifford RB
    sequences of depth 200 plus their recovery Cliffords (workloads.config4_rb2q:
    X90 / Y90 / X-90 / Y-90, virtual Z, CNOT by cross resonance; ~1,300
    commands per core, 2.6*10^8 commands, a 4.2 GB program image), 10 shots
    each = 10^6 shots = 2*10^6 lanes per GPU.  Branch-free programs with
    register commands: macro_staged_kernel.  Divergent: a wave's lanes run ~7
    different programs.  shaped: the RB-SHAPED programs of rounds 2-6
    (workloads.config4_rb_set: single-qubit Cliffords + random CR pulses, no
    recovery; ~740 commands per core), kept on the line as the round-over-round
    comparison for the same kernel (no CPU baseline, no PMC pass).  VALU-bound: the roofline is VALU issue against
    the measured peak, with the VALU ops per emulated instruction and the
    active lanes per VALU instruction (divergence) from the PMC pass."""
    import torch
    from distributed_processor_amd import _abi, isa, sharding, workloads
    from distributed_processor_amd.emulator import RunPipeline, alloc_device_outputs
    t0 = time.perf_counter()
    ps = (workloads.config4_rb_set if shaped else workloads.config4_rb2q_set)(args.rb_seqs, 200)
    gen_s = time.perf_counter() - t0
    emu.load(ps)
    torch.cuda.synchronize()
    load_s = time.perf_counter() - t0 - gen_s
    ops = ps.words[:, 3] >> 28
    strobes = np.add.reduceat(((ops == isa.OP_PULSE_TRIG) | (ops == isa.OP_PULSE_RESET)).astype(np.int64),
                              ps.offsets.astype(np.int64))
    cfg = _abi.make_config(2, n_groups=ps.n_groups, shots_per_group=args.rb_spg, max_cycles=1 << 20,
                           event_cap=int(strobes.max()) + 1, trace_cap=0, meas_cap=2, meas_latency=64,
                           seed=0x5EED, p1=0.5,
                           # the caller's cache hint: event rows nontemporal on the two-qubit RB
                           # programs (-6 to -9 % same-process); it costs the RB-shaped ones +10-13 %
                           # (profiles/r06_stpol_ab.json), which run without it
                           exec_flags=0 if shaped else _abi.X_STREAM_EVENTS)
    shot0, n = sharding.weak_shard(args.rb_seqs * args.rb_spg, rank)
    want = ('summary', 'events', 'meas', 'hist')
    steps = max(1, args.steps)
    # a step is one batch (10^6 shots) on one context, in call order
    out = alloc_device_outputs(cfg, n, want=want)
    pipe = sharding.HistogramPipeline(out['hist'])

    def launch(h):
        out['hist'] = h
        emu.run_device(cfg, n, shot0, out, stream)
    serial = lambda: pipe.step(launch)
    dt_serial = timed(serial, pipe.drain, steps, min(args.warmup, 2), world)
    kernel = emu.last_kernel()
    kernel_ms, kernel_ms_blk = interp_kernel_ms(emu, cfg, n, shot0, out, stream, steps, serial, pipe.drain)
    dt, mode, pipe_ms, s_pipe = dt_serial, 'serial', None, None
    depth = max(1, args.rb_depth)
    if depth > 1:
        # opt-in: `rb_depth` batches in flight on as many contexts / streams
        # (emulator.RunPipeline: the next batch's waves fill the CUs this
        # batch's tail of long sequences leaves idle); the flag picks the
        # reported mode, both on the line
        rp = RunPipeline(ps, cfg, n, want=want, depth=depth, device=torch.cuda.current_device(), first=emu,
                         streams=args.pipe_streams)
        hp = sharding.HistogramPipeline(rp.outputs[0]['hist'], n_buffers=max(2, depth))

        def step():
            with torch.cuda.stream(rp.streams[rp.k % depth]):
                hp.step(lambda h: rp.launch(cfg, n, shot0, hist=h))
        dt_pipe = timed(step, hp.drain, steps, min(args.warmup, 2), world)
        hp.drain()
        rp.drain()
        assert int(hp.result().sum().item()) == n * world
        s_pipe = rp.outputs[(rp.k - 1) % depth]['summary'].cpu().numpy()
        rp.close()
        del rp
        pipe_ms = dt_pipe / steps * 1e3
        dt, mode = dt_pipe, 'pipelined'
    summ = out['summary'].cpu().numpy().view(np.uint32)
    if s_pipe is not None:
        assert np.array_equal(summ, s_pipe.view(np.uint32)), 'config 4: pipelined and serial batches differ'
    s = _abi.unpack_summary(summ)
    assert (s['status'] == _abi.ST_DONE).all(), 'config 4: not every lane reached DONE'
    assert int(pipe.result().sum().item()) == n * world
    instrs = float(s['n_instr'].astype(np.float64).sum())
    ms_step = dt / steps * 1e3
    serial_ms = dt_serial / steps * 1e3
    k_ms = min(kernel_ms, serial_ms)            # (capped at the one-context step: batches in flight overlap)
    prof = pmc('rb') if (args.rb_seqs, args.rb_spg) == (100000, 10) and not shaped else None
    alg = float(bytes_per_lane(summ, cfg).sum())
    hbm = hbm_roofline(alg, kernel_ms, serial_ms, 'dpemu::' + kernel, prof, kernel.split('<')[0])
    hbm['kernel_ms_block'] = kernel_ms_blk
    valu = valu_view(prof, k_ms)
    if valu:
        roof = dict(valu, kernel_ms=k_ms, kernel=hbm['kernel'],
                    valu_ops_per_instruction=valu['valu_insts_per_launch'] * 64 / instrs,
                    active_lanes_per_valu_pct=prof.get('valu_lane_util_pct'), traffic=hbm['traffic'], hbm=hbm)
    else:
        roof = hbm
    res = {'metric': 'emulated core-shots/s (config 4: {}, 1e5 sequences x depth 200, 10 shots each)'.format(
               'RB-shaped programs of rounds 2-6' if shaped else '2-qubit Clifford RB + recovery'),
           'value': n * 2 * world * steps / dt, 'unit': 'core-shots/s', 'shots_per_s': n * world * steps / dt,
           'ms_per_step': ms_step, 'kernel_ms': kernel_ms, 'steps': steps,
           'serial_ms_per_step': dt_serial / steps * 1e3, 'step_mode': mode,
           'batches_in_flight': depth if mode == 'pipelined' else 1,
           'instructions_per_s': instrs * world * steps / dt,
           'qclk_cycles_per_s': float(s['t_end'].astype(np.float64).sum()) * world * steps / dt,
           'config': {'workload': 'config4_{}_2core_1e5seq_depth200'.format('rb_shaped' if shaped else 'rb2q'),
                      'sequences': args.rb_seqs,
                      'lane_order': LANE_ORDER_NAMES[cfg.lane_order], 'exec_flags': hex(cfg.exec_flags),
                      'shots_per_sequence': args.rb_spg, 'shots_per_gpu': n, 'commands': int(ps.words.shape[0]),
                      'program_image_bytes': int(ps.words.nbytes), 'event_cap': cfg.event_cap,
                      'generate_s': gen_s, 'load_s': load_s},
           'roofline': roof}
    if pipe_ms is not None:
        res['pipelined_ms_per_step'] = pipe_ms
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not shaped:
        res['cpu_baseline'] = cpu_baselines(ps, cfg, 1 << 20, 'config 4 RB', all_cores=True)
    del out
    torch.cuda.empty_cache()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--shots', type=int, default=10 ** 6, help='config-2 shots per GPU per step')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--dds-seqs', type=int, default=128, help='RB sequences per GPU for the DDS leg (config 5)')
    ap.add_argument('--dds-depth', type=int, default=1,
                    help='DDS batches in flight (> 1: dds.SynthesisPipeline reported, the serial step measured '
                         'beside it; 1: serial only).  Default 1: on the two-qubit RB timelines two batches in '
                         'flight measured slower than one context (0.846 vs 0.779 ms kernel, r06)')
    ap.add_argument('--dds-workload', default='rb2q', choices=('rb2q', 'rb'),
                    help='config-5 timelines: rb2q = config 4\'s two-qubit Clifford RB on 4 qubit pairs; rb = the '
                         'RB-shaped 8-core generator of rounds 2-6')
    ap.add_argument('--rb-depth', type=int, default=1,
                    help='config-4 batches in flight (opt-in, > 1: emulator.RunPipeline, reported with the serial '
                         'step measured beside it)')
    ap.add_argument('--ar-shots', type=int, default=1250000, help='config-3 shots per GPU per step')
    ap.add_argument('--rb-seqs', type=int, default=100000, help='config-4 RB sequences')
    ap.add_argument('--rb-spg', type=int, default=10, help='config-4 shots per sequence')
    ap.add_argument('--c1-shots', type=int, default=10 ** 6, help='config-1 shots per GPU per step')
    ap.add_argument('--legs', default='config1,dds,active_reset,demod,lut,rb,rb_shaped',
                    help='sub-legs to run (comma list; "" for none)')
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
    # the pipelines' streams, made before any other: each on its own hardware
    # queue where the process has enough (emulator.RunPipeline)
    args.pipe_streams = [torch.cuda.Stream() for _ in range(max(1, args.dds_depth, args.rb_depth))]

    from distributed_processor_amd.emulator import Emulator
    emu = Emulator(local)
    stream = torch.cuda.current_stream()
    main_leg = leg_ramsey(emu, args, world, rank, stream)
    result = {
        'metric': 'emulated core-shots/s (config 2: 8-core Ramsey, 100 delays, 1e6 shots/GPU)',
        'value': main_leg['value'],
        'unit': 'core-shots/s',
        'n_gpus': world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': main_leg['ms_per_step'],
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': None,
        'dtype': 'u32',
        'data': 'synthetic (assembled Ramsey programs, Philox outcomes p=0.5)',
        'config': main_leg['config'],
        'collective_world_size': dist.get_world_size() if dist.is_initialized() else 1,
        'collective_backend': dist.get_backend() if dist.is_initialized() else None,
    }
    for k in ('shots_per_s', 'qclk_cycles_per_s', 'instructions_per_s', 'kernel_ms', 'roofline', 'timeline_gather',
              'cpu_baseline'):
        if k in main_leg:
            result[k] = main_leg[k]
    fns = {'config1': leg_config1, 'dds': leg_dds, 'active_reset': leg_active_reset, 'rb': leg_rb,
           'rb_shaped': lambda *a: leg_rb(*a, shaped=True),
           'lut': lambda *a: leg_active_reset(*a, lut=True), 'demod': lambda *a: leg_active_reset(*a, demod=True)}
    for name in [x for x in args.legs.split(',') if x]:
        result[name] = fns[name](emu, args, world, rank, stream)
    if 'demod' in result and 'active_reset' in result:
        # the demodulation model's own cost: the same circuit, shots and launch
        # shape as the STATE leg, so the kernel-time ratio is the model's price
        a, d = result['active_reset'], result['demod']
        d['model_cost'] = {'kernel_ms_state': a['kernel_ms'], 'kernel_ms_demod': d['kernel_ms'],
                           'kernel_ratio': d['kernel_ms'] / a['kernel_ms'],
                           'step_ratio': d['ms_per_step'] / a['ms_per_step'],
                           'extra_bytes_per_launch': d['roofline']['bytes_per_launch'] -
                           a['roofline']['bytes_per_launch']}
    result['box'] = {'fill_GBps': fill_gbps(), 'device': torch.cuda.get_device_name(local)}
    # LAST on the line: one compact record per leg, so that a reader who keeps
    # only the tail of the line (the driver stores ~8 KB) still has every
    # leg's number and roofline fraction
    result['legs'] = {'config2': compact_leg(main_leg)}
    for name in [x for x in args.legs.split(',') if x]:
        result['legs'][name] = compact_leg(result[name])
    if rank == 0:
        print(json.dumps(result), flush=True)
    emu.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
