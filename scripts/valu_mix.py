"""Static VALU opcode mix of a kernel from its gfx950 assembly (hipcc
--save-temps), for grading an interpreter against the issue rate of its OWN
instructions (scripts/micro/valu_peak.hip single-opcode chains).

    python scripts/valu_mix.py <file.s> <kernel-name substring> [--top 0.9]

Counts every VALU mnemonic (v_*, operand encodings _e32 / _e64 / _sdwa / _dpp
folded) in the kernel's function body, and prints them by count with their
cumulative share; --json writes the histogram.  Static counts: each
instruction of the body once, so a loop body's mix stands for the dynamic one
only as far as the body dominates the executed instructions (the interpreter
loops do; prologue and epilogue are a few percent of a kernel's text).
"""
import argparse
import collections
import json
import re
import sys


def kernel_body(lines, name):
    """the lines of the first function whose label contains `name`"""
    start = None
    for i, ln in enumerate(lines):
        m = re.match(r'^([A-Za-z_.$][\w.$]*):', ln)
        if m and name in m.group(1) and not m.group(1).startswith('.'):
            start = i
            break
    if start is None:
        raise SystemExit('kernel {!r} not found'.format(name))
    body = []
    for ln in lines[start + 1:]:
        if re.match(r'^\s*\.Lfunc_end', ln) or re.match(r'^\s*s_endpgm', ln):
            body.append(ln)
            if 'Lfunc_end' in ln:
                break
            continue
        body.append(ln)
    return lines[start].split(':')[0], body


def mnemonic(ln):
    ln = ln.split(';')[0].strip()
    if not ln or ln.startswith('.') or ln.endswith(':'):
        return None
    op = ln.split()[0]
    return re.sub(r'_(e32|e64|sdwa|dpp)$', '', op)


def mix(path, name):
    with open(path) as f:
        lines = f.read().splitlines()
    label, body = kernel_body(lines, name)
    valu, salu, other = collections.Counter(), collections.Counter(), collections.Counter()
    for ln in body:
        op = mnemonic(ln)
        if not op:
            continue
        if op.startswith('v_'):
            valu[op] += 1
        elif op.startswith('s_'):
            salu[op] += 1
        else:
            other[op] += 1
    return label, valu, salu, other


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('asm')
    ap.add_argument('kernel')
    ap.add_argument('--top', type=float, default=0.9)
    ap.add_argument('--json')
    a = ap.parse_args()
    label, valu, salu, other = mix(a.asm, a.kernel)
    n = sum(valu.values())
    print('{}: {} VALU, {} SALU, {} other (static)'.format(label, n, sum(salu.values()), sum(other.values())))
    cum = 0
    top = []
    for op, c in valu.most_common():
        cum += c
        print('  {:28s} {:6d} {:6.1%} {:6.1%}'.format(op, c, c / n, cum / n))
        top.append(op)
        if cum / n >= a.top and len(top) >= 1 and c / n < 0.01:
            break
    if a.json:
        with open(a.json, 'w') as f:
            json.dump({'kernel': label, 'source': a.asm, 'valu_total': n, 'valu': dict(valu.most_common()),
                       'salu_total': sum(salu.values()), 'salu': dict(salu.most_common())}, f, indent=1)


if __name__ == '__main__':
    sys.exit(main())
