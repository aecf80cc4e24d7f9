"""Summarise rocprofv3 kernel-trace + PMC passes of the bench into per-kernel JSON.

usage: python scripts/pmc_summary.py <prof root (e.g. gpurun_out/r01)> <tag> [dest dir] [key=substr|substr[@grid],...]

Reads <root>/prof_trace or <root>/trace (--kernel-trace --stats) and every
other subdirectory's PMC pass (counter_collection.csv), groups dispatches by (kernel, grid size),
keeps each kernel's most frequent shape (the bench's timed launches) and
writes <dest>/<tag>_<kernel>_pmc.json with per-launch means:

* duration_ns     kernel-trace average over those dispatches that overlap no
                  other dispatch (the bench's pipelines run batches
                  concurrently; a kernel sharing the GPU takes longer);
                  dispatches_overlapped counts the ones left out
* write_bytes     WRITE_SIZE x 1024 (exact for 16-B-per-lane streaming stores)
* fetch_bytes     FETCH_SIZE x 1024 x 2: on gfx950 FETCH_SIZE reads 1/2 of a
                  wide coalesced read (MI355X_MICROARCH.md, HBM section)
* hbm_bytes_per_launch = write_bytes + fetch_bytes
* SQ_* / GRBM_* raw means
* VALU ratios, each from counters of the SAME pass and dispatch (prof_cmd.sh
  puts GRBM_GUI_ACTIVE in both SQ passes), then averaged over dispatches:
    valu_issue_pct   SQ_INSTS_VALU x c / 1024 SIMDs / (GRBM_GUI_ACTIVE / 8 XCDs),
                     c = the measured cycles per wave64 integer-VALU
                     instruction at the issue peak (profiles/r04_valu_peak_pmc.json)
    (SQ_ACTIVE_INST_VALU equals SQ_INSTS_VALU on the peak microbenchmark, so
    a 'busy' ratio of it at an assumed 4 cycles per instruction overstates the
    VALU share wherever the kernel issues faster than 4; it is not reported)
    valu_frac_of_measured_peak  SQ_INSTS_VALU / duration / the measured peak
  A ratio above 100 % is reported as measured and flagged in 'warnings'.
* valu_lane_util_pct = SQ_THREAD_CYCLES_VALU / (SQ_ACTIVE_INST_VALU x 64)
"""
import collections
import csv
import glob
import json
import os
import sys

# summary key -> kernel-name substrings, one per bench leg: config 2 runs on
# straight_kernel (pulse-only programs), config 3 on branch_kernel (fproc
# branches, syncs), config 4 on macro_kernel, config 5 on dds_tile_kernel
KERNELS = {'ramsey': ('straight_kernel',), 'active_reset': ('branch_kernel<11,', 'branch_kernel<3,', 'branch_kernel<11>', 'branch_kernel<3>'), 'rb': ('macro_kernel', 'macro_staged_kernel'),
           'dds': ('dds_tile_kernel',), 'dds_index': ('dds_index_kernel',), 'hist_reduce': ('hist_reduce_kernel',),
           'config1': ('straight_kernel',), 'lut': ('branch_kernel<14,', 'branch_kernel<6,', 'branch_kernel<14>', 'branch_kernel<6>'),
           'demod': ('branch_kernel<75,', 'branch_kernel<67,', 'branch_kernel<75>', 'branch_kernel<67>')}
# legs that share a kernel: the leg's launch grid (threads) picks its dispatches
# (config 1: 10^6 single-core lanes; config 2: 10^6 shots x 8 cores)
GRIDS = {'config1': (10 ** 6 + 255) // 256 * 256, 'ramsey': 8 * 10 ** 6}


REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def valu_peak():
    """the measured wave64 integer-VALU issue peak (instructions/s, whole chip)
    and its cycles per instruction per SIMD: scripts/micro/valu_peak.hip under
    rocprofv3, summarised by scripts/valu_peak_summary.py"""
    with open(os.path.join(REPO, 'profiles', 'r04_valu_peak_pmc.json')) as f:
        v = json.load(f)
    return v['peak_valu_insts_per_s'], v['peak_cycles_per_inst']


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def which(name, grid):
    for k, subs in KERNELS.items():
        if any(sub in name for sub in subs) and GRIDS.get(k, grid) == grid:
            return k
    return None


def main():
    root, tag = sys.argv[1], sys.argv[2]
    dest = sys.argv[3] if len(sys.argv) > 3 else root
    if len(sys.argv) > 4:          # kernel keys of this run: key=substr|substr,...
        KERNELS.clear()
        GRIDS.clear()
        for item in sys.argv[4].split(','):
            k, subs = item.split('=')
            if '@' in subs:            # key=substr@grid: only dispatches of that grid size (threads)
                subs, g = subs.split('@')
                GRIDS[k] = int(g)
            KERNELS[k] = tuple(subs.split('|'))
    os.makedirs(dest, exist_ok=True)
    # kernel trace: per (kernel, grid) durations
    dur = collections.defaultdict(list)
    n_over = collections.Counter()
    names = {}
    tdir = 'prof_trace' if os.path.isdir(os.path.join(root, 'prof_trace')) else 'trace'
    spans = []
    for r in rows(os.path.join(root, tdir, '**', '*kernel_trace.csv')):
        grid = int(r['Grid_Size']) if r.get('Grid_Size') else \
            int(r['Grid_Size_X']) * int(r.get('Grid_Size_Y') or 1) * int(r.get('Grid_Size_Z') or 1)
        spans.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), which(r['Kernel_Name'], grid), grid,
                      r['Kernel_Name']))
    spans.sort()
    end_before = -1                                   # latest end of any earlier-starting dispatch
    for i, (t0, t1, k, grid, name) in enumerate(spans):
        alone = end_before <= t0 and (i + 1 == len(spans) or spans[i + 1][0] >= t1)
        end_before = max(end_before, t1)
        if not k:
            continue
        names[(k, grid)] = name
        if alone:
            dur[(k, grid)].append(t1 - t0)
        else:
            n_over[(k, grid)] += 1
    for key in n_over:
        dur.setdefault(key, [])
    shape = {}
    for (k, grid), v in dur.items():
        nk = len(v) + n_over[(k, grid)]
        if k not in shape or nk > len(dur[(k, shape[k])]) + n_over[(k, shape[k])]:
            shape[k] = grid
    peak, cpi = valu_peak()
    # counters: per (kernel, grid) -> {(pass dir, dispatch): {counter: sum}}
    ctr = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
    for d in sorted(glob.glob(os.path.join(root, '*'))):
        if not os.path.isdir(d) or os.path.basename(d) == tdir:
            continue
        for r in rows(os.path.join(d, '**', '*counter_collection.csv')):
            grid = int(r.get('Grid_Size') or 0)
            k = which(r['Kernel_Name'], grid)
            if not k:
                continue
            ctr[(k, grid)][(d, r['Dispatch_Id'])][r['Counter_Name']] += float(r['Counter_Value'])
    for k, grid in shape.items():
        d = dur[(k, grid)]
        res = {'kernel': names[(k, grid)], 'grid_size': grid, 'dispatches_traced': len(d),
               'dispatches_overlapped': n_over[(k, grid)], 'duration_ns': sum(d) / len(d) if d else None}
        disp = ctr.get((k, grid), {})
        names_c = sorted({c for v in disp.values() for c in v})
        for name in names_c:
            vals = [v[name] for v in disp.values() if name in v]
            res[name] = sum(vals) / len(vals)
        # same-pass, same-dispatch VALU ratios
        def ratio(num, scale):
            xs = [v[num] * scale / 1024.0 / (v['GRBM_GUI_ACTIVE'] / 8.0) * 100.0 for v in disp.values()
                  if num in v and v.get('GRBM_GUI_ACTIVE')]
            return sum(xs) / len(xs) if xs else None
        res['valu_peak_insts_per_s'] = peak
        res['valu_peak_cycles_per_inst'] = cpi
        warnings = []
        for key, num, scale in (('valu_issue_pct', 'SQ_INSTS_VALU', cpi),):
            r_ = ratio(num, scale)
            if r_ is not None:
                res[key] = r_
                if r_ > 100.0:
                    warnings.append('{} = {:.1f} % exceeds 100 %: the counter basis does not hold here'.format(key, r_))
        if warnings:
            res['warnings'] = warnings
        if 'WRITE_SIZE' in res:
            res['write_bytes'] = res['WRITE_SIZE'] * 1024
        if 'FETCH_SIZE' in res:
            res['fetch_bytes'] = res['FETCH_SIZE'] * 1024 * 2
        if 'write_bytes' in res and 'fetch_bytes' in res:
            res['hbm_bytes_per_launch'] = res['write_bytes'] + res['fetch_bytes']
            if res.get('duration_ns'):
                res['hbm_GBps_at_traced_duration'] = res['hbm_bytes_per_launch'] / res['duration_ns']
        if 'SQ_THREAD_CYCLES_VALU' in res and 'SQ_ACTIVE_INST_VALU' in res and res['SQ_ACTIVE_INST_VALU']:
            # active lanes per VALU instruction (divergence): thread-cycles / (quad-cycles * 64)
            res['valu_lane_util_pct'] = 100.0 * res['SQ_THREAD_CYCLES_VALU'] / (res['SQ_ACTIVE_INST_VALU'] * 64)
        if 'SQ_INSTS_VALU' in res and res.get('duration_ns'):
            # against the measured integer-VALU issue peak (scripts/micro/valu_peak.hip)
            res['valu_insts_per_s'] = res['SQ_INSTS_VALU'] / (res['duration_ns'] * 1e-9)
            res['valu_frac_of_measured_peak'] = res['valu_insts_per_s'] / peak
        if 'SQ_INSTS_VALU' in res and 'SQ_WAVES' in res and res['SQ_WAVES']:
            res['valu_insts_per_wave'] = res['SQ_INSTS_VALU'] / res['SQ_WAVES']
        path = os.path.join(dest, '{}_{}_pmc.json'.format(tag, k))
        with open(path, 'w') as f:
            json.dump(res, f, indent=1, sort_keys=True)
        print(path, json.dumps({x: res.get(x) for x in ('duration_ns', 'hbm_bytes_per_launch',
                                                        'valu_issue_pct', 'valu_lane_util_pct')}))


if __name__ == '__main__':
    main()
