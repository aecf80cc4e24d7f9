"""A kernel's own VALU issue peak: its VALU opcode mix (scripts/valu_mix.py,
static text of the kernel) weighted by the measured issue cost of each
opcode (scripts/micro/valu_peak.hip op_kernel<OP>, cycles per wave64
instruction per SIMD in profiles/<tag>_valu_peak_pmc.json
'opcode_cycles_per_inst').

    python scripts/kernel_valu_peak.py <valu_peak json> <mix json> [<mix json> ...] --out <json>

An opcode without a chain of its own takes its class's measured cost: v_cmp_*
that of v_cmp_eq_u32, v_readfirstlane / v_writelane that of v_readlane_b32,
a 64-bit shift or add that of v_lshl_add_u64 / v_ashrrev_i64, 24-bit and
low / high multiplies those of v_mul_lo_u32 / v_mul_hi_u32, float
conversions, multiplies and reciprocals that of v_mul_lo_u32 (quarter rate
on CDNA, an upper bound), every other 32-bit op the median of the simple
32-bit chains.  The kernel's cycles per instruction is the share-weighted
mean; its peak = 1024 SIMDs x clock / that, at the clock of the kernel's own
PMC pass when given (--pmc key=profiles/<tag>_<leg>_pmc.json), else at the
microbenchmark's clock.
"""
import argparse
import json
import os
import re
import statistics

SIMPLE = ('v_xor_b32', 'v_add_u32', 'v_sub_u32', 'v_and_b32', 'v_lshrrev_b32', 'v_lshlrev_b32', 'v_min_u32',
          'v_mov_b32', 'v_cndmask_b32', 'v_bfe_i32', 'v_bitop3_b32')


def op_cost(op, cpi):
    if op in cpi:
        return cpi[op], op
    if op.startswith('v_cmp'):
        return cpi['v_cmp_eq_u32'], 'v_cmp_eq_u32'
    if op in ('v_readfirstlane_b32', 'v_writelane_b32'):
        return cpi['v_readlane_b32'], 'v_readlane_b32'
    if op.endswith(('_u64', '_i64', '_b64')) or op in ('v_lshl_add_u64',):
        if 'mad' in op:
            return cpi['v_mad_u64_u32'], 'v_mad_u64_u32'
        if 'shr' in op or ('shl' in op and 'add' not in op):
            return cpi['v_ashrrev_i64'], 'v_ashrrev_i64'
        return cpi['v_lshl_add_u64'], 'v_lshl_add_u64'
    if op.startswith('v_mul_hi'):
        return cpi['v_mul_hi_u32'], 'v_mul_hi_u32'
    if op.startswith(('v_mul_lo', 'v_mad_u32', 'v_mul_u32_u24', 'v_mad_u32_u24')):
        return cpi['v_mul_lo_u32'], 'v_mul_lo_u32'
    if op.startswith(('v_cvt', 'v_rcp', 'v_mul_f32', 'v_fma', 'v_trunc', 'v_rndne')):
        return cpi['v_mul_lo_u32'], 'v_mul_lo_u32 (float class, upper bound)'
    simple = [cpi[o] for o in SIMPLE if o in cpi]
    return statistics.median(simple), 'median of simple 32-bit'


def readable(mangled):
    """_ZN5dpemu13branch_kernelILi11ELi8EEEvNS_7KParamsE -> branch_kernel<11,8>
    (the form bench.py matches against rocprofv3's kernel names)"""
    m = re.match(r'_ZN5dpemu(\d+)', mangled)
    if not m:
        return mangled
    n = int(m.group(1))
    rest = mangled[m.end():]
    name, rest = rest[:n], rest[n:]
    args = []
    if rest.startswith('I'):
        for kind, val in re.findall(r'L([ib])(\d+)E', rest[:rest.index('EE') + 1] if 'EE' in rest else rest):
            args.append(('true' if val == '1' else 'false') if kind == 'b' else val)
    return name + ('<' + ','.join(args) + '>' if args else '')


def kernel_peak(mix, cpi, clock_ghz):
    n = sum(mix['valu'].values())
    w_cpi, covered, rows = 0.0, 0, []
    for op, c in mix['valu'].items():
        v, by = op_cost(op, cpi)
        w_cpi += c / n * v
        covered += c if by == op else 0
        rows.append({'op': op, 'share': c / n, 'cycles_per_inst': v, 'from': by})
    peak = 1024 * clock_ghz * 1e9 / w_cpi
    return {'kernel': mix['kernel'], 'name': readable(mix['kernel']), 'valu_static': n, 'share_measured_directly': covered / n,
            'cycles_per_inst': w_cpi, 'clock_ghz': clock_ghz, 'peak_valu_insts_per_s': peak,
            'opcodes': sorted(rows, key=lambda r: -r['share'])[:40]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('peak')
    ap.add_argument('mix', nargs='+')
    ap.add_argument('--pmc', action='append', default=[], help='kernel substring=pmc json (its clock and rate)')
    ap.add_argument('--validation', default=None,
                    help='scripts/valu_model_check.py output: recorded with the peaks (does the table model issue?)')
    ap.add_argument('--out', required=True)
    a = ap.parse_args()
    with open(a.peak) as f:
        pk = json.load(f)
    cpi = pk['opcode_cycles_per_inst']
    pmcs = {}
    for kv in a.pmc:
        k, v = kv.split('=', 1)
        if not os.path.exists(v):
            continue
        with open(v) as f:
            pmcs[k] = json.load(f)
    out = {'what': 'per-kernel VALU issue peak from its own opcode mix (scripts/kernel_valu_peak.py)',
           'peak_source': a.peak, 'kernels': []}
    if a.validation and os.path.exists(a.validation):
        with open(a.validation) as f:
            v = json.load(f)
        out['validation'] = {'source': a.validation, 'kernel': v['kernel'],
                             'predicted_cycles_per_inst': v['predicted_cycles_per_inst'],
                             'measured_cycles_per_inst': v['measured_cycles_per_inst'], 'miss': v['miss'],
                             'issue_model': v['issue_model'], 'conclusion': v['conclusion']}
        out['graded_on'] = ('these own-mix peaks' if v['issue_model'] else
                            'the measured mixed-integer peak (bench.VALU_PEAK); frac_of_own_peak is shown, not graded')
    for m in a.mix:
        with open(m) as f:
            mix = json.load(f)
        prof = next((v for k, v in pmcs.items() if k in mix['kernel']), None)
        clock = pk['peak_clock_ghz']
        if prof and prof.get('GRBM_GUI_ACTIVE') and prof.get('duration_ns'):
            clock = prof['GRBM_GUI_ACTIVE'] / 8 / prof['duration_ns']
        r = kernel_peak(mix, cpi, clock)
        if prof and prof.get('SQ_INSTS_VALU') and prof.get('duration_ns'):
            r['achieved_valu_insts_per_s'] = prof['SQ_INSTS_VALU'] / (prof['duration_ns'] * 1e-9)
            r['frac_of_own_peak'] = r['achieved_valu_insts_per_s'] / r['peak_valu_insts_per_s']
            r['pmc_source'] = prof.get('kernel')
        out['kernels'].append(r)
        print('{}: cpi {:.3f} peak {:.3e}/s frac {}'.format(r['kernel'][:60], r['cycles_per_inst'],
                                                          r['peak_valu_insts_per_s'], r.get('frac_of_own_peak')))
    with open(a.out, 'w') as f:
        json.dump(out, f, indent=1)


if __name__ == '__main__':
    main()
