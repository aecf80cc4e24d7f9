"""Summarise rocprofv3 kernel-trace + PMC passes of the bench into per-kernel JSON.

usage: python scripts/pmc_summary.py <prof root (e.g. gpurun_out/r01)> <tag> [dest dir] [key=substr|substr,...]

Reads <root>/prof_trace or <root>/trace (--kernel-trace --stats) and every
other subdirectory's PMC pass (counter_collection.csv), groups dispatches by (kernel, grid size),
keeps each kernel's most frequent shape (the bench's timed launches) and
writes <dest>/<tag>_<kernel>_pmc.json with per-launch means:

* duration_ns     kernel-trace average over those dispatches
* write_bytes     WRITE_SIZE x 1024 (exact for 16-B-per-lane streaming stores)
* fetch_bytes     FETCH_SIZE x 1024 x 2: on gfx950 FETCH_SIZE reads 1/2 of a
                  wide coalesced read (MI355X_MICROARCH.md, HBM section)
* hbm_bytes_per_launch = write_bytes + fetch_bytes
* SQ_* / GRBM_* raw means; VALU busy = SQ_ACTIVE_INST_VALU * 4 / (4 SIMD x 256 CU)
  / (GRBM_GUI_ACTIVE / 8 XCDs); VALU issue share = SQ_INSTS_VALU x 4 cycles on
  the same denominator; lane utilisation = SQ_THREAD_CYCLES_VALU /
  (SQ_ACTIVE_INST_VALU x 64)
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
KERNELS = {'ramsey': ('straight_kernel',), 'active_reset': ('branch_kernel',), 'rb': ('macro_kernel',),
           'dds': ('dds_tile_kernel',), 'dds_index': ('dds_index_kernel',), 'hist_reduce': ('hist_reduce_kernel',)}


# wave64 integer-VALU instructions per second, whole chip: the best rate of
# scripts/micro/valu_peak.hip (independent add/shift/xor chains, 2-8 waves per
# SIMD) measured on MI355X (profiles/r01_valu_peak.jsonl)
VALU_PEAK_WAVE_INSTS = 7.7e11


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def which(name):
    for k, subs in KERNELS.items():
        if any(sub in name for sub in subs):
            return k
    return None


def main():
    root, tag = sys.argv[1], sys.argv[2]
    dest = sys.argv[3] if len(sys.argv) > 3 else root
    if len(sys.argv) > 4:          # kernel keys of this run: key=substr|substr,...
        KERNELS.clear()
        for item in sys.argv[4].split(','):
            k, subs = item.split('=')
            KERNELS[k] = tuple(subs.split('|'))
    os.makedirs(dest, exist_ok=True)
    # kernel trace: per (kernel, grid) durations
    dur = collections.defaultdict(list)
    names = {}
    tdir = 'prof_trace' if os.path.isdir(os.path.join(root, 'prof_trace')) else 'trace'
    for r in rows(os.path.join(root, tdir, '**', '*kernel_trace.csv')):
        k = which(r['Kernel_Name'])
        if k:
            grid = int(r['Grid_Size']) if r.get('Grid_Size') else \
                int(r['Grid_Size_X']) * int(r.get('Grid_Size_Y') or 1) * int(r.get('Grid_Size_Z') or 1)
            dur[(k, grid)].append(int(r['End_Timestamp']) - int(r['Start_Timestamp']))
            names[(k, grid)] = r['Kernel_Name']
    shape = {}
    for (k, grid), v in dur.items():
        if k not in shape or len(v) > len(dur[(k, shape[k])]):
            shape[k] = grid
    # counters: per (kernel, grid, dispatch, counter) sums
    ctr = collections.defaultdict(lambda: collections.defaultdict(float))
    for d in sorted(glob.glob(os.path.join(root, '*'))):
        if not os.path.isdir(d) or os.path.basename(d) == tdir:
            continue
        for r in rows(os.path.join(d, '**', '*counter_collection.csv')):
            k = which(r['Kernel_Name'])
            if not k:
                continue
            grid = int(r.get('Grid_Size') or 0)
            ctr[(k, grid, r['Counter_Name'])][(d, r['Dispatch_Id'])] += float(r['Counter_Value'])
    for k, grid in shape.items():
        res = {'kernel': names[(k, grid)], 'grid_size': grid, 'dispatches_traced': len(dur[(k, grid)]),
               'duration_ns': sum(dur[(k, grid)]) / len(dur[(k, grid)])}
        for (kk, g, name), per in ctr.items():
            if kk == k and g == grid:
                res[name] = sum(per.values()) / len(per)
        if 'WRITE_SIZE' in res:
            res['write_bytes'] = res['WRITE_SIZE'] * 1024
        if 'FETCH_SIZE' in res:
            res['fetch_bytes'] = res['FETCH_SIZE'] * 1024 * 2
        if 'write_bytes' in res and 'fetch_bytes' in res:
            res['hbm_bytes_per_launch'] = res['write_bytes'] + res['fetch_bytes']
            res['hbm_GBps_at_traced_duration'] = res['hbm_bytes_per_launch'] / res['duration_ns']
        if 'SQ_ACTIVE_INST_VALU' in res and 'GRBM_GUI_ACTIVE' in res and res['GRBM_GUI_ACTIVE']:
            # GRBM_GUI_ACTIVE is summed over the 8 XCDs; SQ_ACTIVE_INST_VALU counts quad-cycles
            res['valu_busy_pct'] = 100.0 * res['SQ_ACTIVE_INST_VALU'] * 4 / (4 * 256) / (res['GRBM_GUI_ACTIVE'] / 8)
        if 'SQ_INSTS_VALU' in res and 'GRBM_GUI_ACTIVE' in res and res['GRBM_GUI_ACTIVE']:
            # a wave64 VALU instruction holds a 16-lane SIMD for 4 cycles: issue-limited share
            res['valu_issue_pct'] = 100.0 * res['SQ_INSTS_VALU'] * 4 / (4 * 256) / (res['GRBM_GUI_ACTIVE'] / 8)
        if 'SQ_THREAD_CYCLES_VALU' in res and 'SQ_ACTIVE_INST_VALU' in res and res['SQ_ACTIVE_INST_VALU']:
            # active lanes per VALU instruction (divergence): thread-cycles / (quad-cycles * 64)
            res['valu_lane_util_pct'] = 100.0 * res['SQ_THREAD_CYCLES_VALU'] / (res['SQ_ACTIVE_INST_VALU'] * 64)
        if 'SQ_INSTS_VALU' in res and res.get('duration_ns'):
            # against the measured integer-VALU issue peak (scripts/micro/valu_peak.hip)
            res['valu_insts_per_s'] = res['SQ_INSTS_VALU'] / (res['duration_ns'] * 1e-9)
            res['valu_frac_of_measured_peak'] = res['valu_insts_per_s'] / VALU_PEAK_WAVE_INSTS
        if 'SQ_INSTS_VALU' in res and 'SQ_WAVES' in res and res['SQ_WAVES']:
            res['valu_insts_per_wave'] = res['SQ_INSTS_VALU'] / res['SQ_WAVES']
        path = os.path.join(dest, '{}_{}_pmc.json'.format(tag, k))
        with open(path, 'w') as f:
            json.dump(res, f, indent=1, sort_keys=True)
        print(path, json.dumps({x: res.get(x) for x in ('duration_ns', 'hbm_bytes_per_launch', 'valu_busy_pct',
                                                        'valu_issue_pct', 'valu_lane_util_pct')}))


if __name__ == '__main__':
    main()
