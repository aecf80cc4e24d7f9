"""Summarise the VALU-peak microbenchmark (scripts/micro/valu_peak.hip) from
rocprofv3: a --kernel-trace pass (durations) and ONE --pmc pass holding
SQ_INSTS_VALU, SQ_WAVES, SQ_ACTIVE_INST_VALU, SQ_BUSY_CYCLES and
GRBM_GUI_ACTIVE, so every ratio comes from counters of the same dispatches.

usage: python scripts/valu_peak_summary.py <root with trace/ and pmc/> <out.json>

Per variant (chains, waves per SIMD), averaged over its dispatches:
  valu_insts_per_s   SQ_INSTS_VALU / kernel-trace duration (whole chip)
  clock_ghz          GRBM_GUI_ACTIVE / 8 XCDs / duration (MI355X_MICROARCH.md
                     'DVFS give-back': the counter sums the 8 XCDs)
  cycles_per_inst    SIMD-cycles per wave64 VALU instruction:
                     (1024 SIMDs x GRBM_GUI_ACTIVE / 8) / SQ_INSTS_VALU
The peak record is the variant with the highest valu_insts_per_s; its
cycles_per_inst is the issue cost the interpreter legs' VALU fractions use
(scripts/pmc_summary.py, bench.py).
"""
import collections
import csv
import glob
import json
import os
import re
import sys

SIMDS = 256 * 4
XCDS = 8


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


# op_kernel<OP> of scripts/micro/valu_peak.hip: the opcode each one chains
OPS = ['v_xor_b32', 'v_add_u32', 'v_sub_u32', 'v_and_b32', 'v_lshrrev_b32', 'v_lshlrev_b32', 'v_min_u32',
       'v_mov_b32', 'v_cndmask_b32', 'v_bfe_i32', 'v_bitop3_b32', 'v_mad_u64_u32', 'v_lshl_add_u64',
       'v_cmp_eq_u32', 'v_readlane_b32', 'v_mul_lo_u32', 'v_mul_hi_u32', 'v_ashrrev_i64']


def variant(name):
    m = re.search(r'(valu|add|fma)_kernel<(\d+), (\d+)>', name)
    if m:
        return (m.group(1), int(m.group(2)), int(m.group(3)))
    m = re.search(r'op_kernel<(\d+)>', name)
    return ('op', int(m.group(1)), 8) if m else None


def main():
    root, dest = sys.argv[1], sys.argv[2]
    dur = collections.defaultdict(list)
    for r in rows(os.path.join(root, 'trace', '**', '*kernel_trace.csv')):
        v = variant(r['Kernel_Name'])
        if v:
            dur[v].append(int(r['End_Timestamp']) - int(r['Start_Timestamp']))
    ctr = collections.defaultdict(lambda: collections.defaultdict(float))   # (variant, dispatch) -> counter sums
    for r in rows(os.path.join(root, 'pmc', '**', '*counter_collection.csv')):
        v = variant(r['Kernel_Name'])
        if v:
            ctr[(v, r['Dispatch_Id'])][r['Counter_Name']] += float(r['Counter_Value'])
    res = []
    for v in sorted(dur):
        d_ns = sum(dur[v]) / len(dur[v])
        disp = [c for (vv, _), c in ctr.items() if vv == v]
        if not disp:
            continue
        mean = {k: sum(c.get(k, 0.0) for c in disp) / len(disp) for k in disp[0]}
        # per-dispatch ratios from the same pass, then averaged
        cpi = [SIMDS * (c['GRBM_GUI_ACTIVE'] / XCDS) / c['SQ_INSTS_VALU'] for c in disp
               if c.get('SQ_INSTS_VALU') and c.get('GRBM_GUI_ACTIVE')]
        if v[0] == 'op':
            kname, mix_ = 'op_kernel<{}>'.format(v[1]), OPS[v[1]] + ' only'
        else:
            kname = '{}_kernel<{}, {}>'.format(*v)
            mix_ = {'valu': 'add/shift/xor (int)', 'add': 'v_add_u32 only', 'fma': 'v_fma_f32 only'}[v[0]]
        rec = {'kernel': kname, 'mix': mix_,
               'chains': v[1], 'waves_per_simd': v[2],
               'dispatches_traced': len(dur[v]), 'dispatches_counted': len(disp), 'duration_ns': d_ns,
               'counters': mean,
               'valu_insts_per_s': mean['SQ_INSTS_VALU'] / (d_ns * 1e-9),
               'valu_insts_per_wave': mean['SQ_INSTS_VALU'] / mean['SQ_WAVES'] if mean.get('SQ_WAVES') else None,
               'clock_ghz': mean['GRBM_GUI_ACTIVE'] / XCDS / d_ns,
               'cycles_per_inst': sum(cpi) / len(cpi) if cpi else None}
        res.append(rec)
    best = max((r for r in res if r['mix'] != 'v_fma_f32 only' and not r['kernel'].startswith('op_')),
               key=lambda r: r['valu_insts_per_s'])
    # per opcode: cycles per wave64 instruction per SIMD of its chain kernel
    # (the loop's few other VALU -- the iteration counter, the chains' seeds --
    # are counted in with it, so an opcode's figure is a slight upper bound
    # on its own rate)
    opcode_cpi = {r['mix'].replace(' only', ''): r['cycles_per_inst'] for r in res if r['kernel'].startswith('op_')}
    out = {'what': 'wave64 integer-VALU issue peak of MI355X, measured: scripts/micro/valu_peak.hip under '
                   'rocprofv3 (kernel trace + one PMC pass: SQ_INSTS_VALU SQ_WAVES SQ_ACTIVE_INST_VALU '
                   'SQ_BUSY_CYCLES GRBM_GUI_ACTIVE); summarised by scripts/valu_peak_summary.py',
           'peak_valu_insts_per_s': best['valu_insts_per_s'], 'peak_variant': best['kernel'],
           'peak_note': 'best integer variant (the interpreter kernels are integer code); the fma variants '
                        'are reported beside it for the float issue rate',
           'peak_cycles_per_inst': best['cycles_per_inst'], 'peak_clock_ghz': best['clock_ghz'],
           'guide_issue_model': '2 cycles per wave64 VALU instruction per SIMD (MI355X_MICROARCH.md:54): '
                                '1024 SIMDs x 2.4 GHz / 2 = 1.229e12 /s',
           'opcode_cycles_per_inst': opcode_cpi,
           'variants': res}
    with open(dest, 'w') as f:
        json.dump(out, f, indent=1)
    for r in res:
        print('{kernel:22s} {valu_insts_per_s:.3e}/s clock {clock_ghz:.2f} GHz cpi {cycles_per_inst}'.format(**r))
    print('peak', best['kernel'], '{:.4e}'.format(best['valu_insts_per_s']), 'cpi', best['cycles_per_inst'])


if __name__ == '__main__':
    main()
