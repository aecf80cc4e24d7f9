"""Static instruction classes of one kernel's gfx950 assembly (whole body and
its loops), for comparing source variants on the CPU before a GPU A/B.

    python scripts/asm_stats.py distributed_processor_amd/csrc/branch.hip branch_kernelILi11ELi8 [-D...]

Prints VGPR / SGPR / spill counts and, per natural loop (a block range closed
by a backward branch), the VALU / SALU / LDS / VMEM instruction counts.
Static counts: a loop's body is counted once whatever paths run in it.
"""
import collections
import glob
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def classify(op):
    if op.startswith('v_'):
        return 'valu'
    if op.startswith('s_'):
        return 'salu'
    if op.startswith('ds_'):
        return 'lds'
    if op.startswith(('global_', 'buffer_', 'flat_', 'scratch_')):
        return 'vmem'
    return 'other'


def main():
    src, pat = sys.argv[1], sys.argv[2]
    defs = sys.argv[3:]
    with tempfile.TemporaryDirectory() as d:
        r = subprocess.run(['/opt/rocm/bin/hipcc', '--offload-arch=gfx950', '-O3', '-std=c++17', '--save-temps',
                            '-Rpass-analysis=kernel-resource-usage', '-c', '-o', os.path.join(d, 'k.o'),
                            os.path.abspath(src)] + defs, cwd=d, capture_output=True, text=True)
        if r.returncode:
            sys.exit(r.stderr[-3000:])
        asm = open(glob.glob(os.path.join(d, '*gfx950*.s'))[0]).read()
    name = next(m.group(1) for m in re.finditer(r'^(_Z\S+):', asm, re.M) if pat in m.group(1))
    # resource remarks for that kernel
    lines = r.stderr.splitlines()
    for i, ln in enumerate(lines):
        if 'Function Name: ' + name in ln:
            for x in lines[i + 1:i + 12]:
                if any(k in x for k in ('VGPRs:', 'TotalSGPRs:', 'Spill', 'Occupancy', 'LDS Size')):
                    print(re.sub(r'.*remark:\s*', '', re.sub(r'\s*\[-R.*', '', x)))
            break
    st = asm.index(name + ':')
    body = asm[st:asm.index('s_endpgm', st)].splitlines()
    insts, labels = [], {}
    for ln in body:
        t = ln.strip()
        m = re.match(r'^(\.LBB\w+):', ln)
        if m:
            labels[m.group(1)] = len(insts)
        elif t and ln[0] in ' \t' and not t.startswith((';', '.')):
            insts.append(t.split()[0] + ' ' + ' '.join(t.split()[1:2]))
    tot = collections.Counter(classify(i.split()[0]) for i in insts)
    print('kernel', name, 'total', dict(tot))
    for j, ins in enumerate(insts):
        op, *arg = ins.split()
        if op.startswith('s_cbranch') or op == 's_branch':
            tgt = arg[0] if arg else ''
            if tgt in labels and labels[tgt] <= j:
                c = collections.Counter(classify(x.split()[0]) for x in insts[labels[tgt]:j + 1])
                print('loop {} [{}..{}] {} insts'.format(tgt, labels[tgt], j, j + 1 - labels[tgt]), dict(c))


if __name__ == '__main__':
    main()
