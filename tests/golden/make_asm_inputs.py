"""Copy the reference's assembler-level test programs into a JSON fixture.

Run in the build container (where /root/reference exists):

    python tests/golden/make_asm_inputs.py

Reads, as data, the compiler golden outputs ``python/test/test_outputs/*.txt``
(assembly-level statement lists per proc group, the inputs of
``make_golden.py``'s ``asm_programs.json``) and ``python/test/channel_config.json``,
and writes ``asm_inputs.json`` / ``channel_config.json`` next to this script.
No reference code is imported or executed.  Tuples (proc-group keys, fproc
func_id, register dtypes) are encoded as {"__tuple__": [...]}, numpy
``array([...])`` envelopes as {"__ndarray__": values or [re, im] pairs}.
"""

import ast
import json
import os
import shutil

HERE = os.path.dirname(os.path.abspath(__file__))
REF_TEST = '/root/reference/python/test'


def enc(v):
    if isinstance(v, tuple):
        return {'__tuple__': [enc(x) for x in v]}
    if isinstance(v, list):
        return [enc(x) for x in v]
    if isinstance(v, dict) and '__ndarray__' not in v:
        return {k: enc(x) for k, x in v.items()}
    return v


def literal(node):
    """ast.literal_eval plus ``array([...])`` (numpy reprs), as {"__ndarray__": ...}"""
    if isinstance(node, ast.Call) and isinstance(node.func, ast.Name) and node.func.id == 'array':
        vals = literal(node.args[0])
        cplx = any(isinstance(v, complex) for v in vals)
        return {'__ndarray__': [[v.real, v.imag] for v in vals] if cplx else vals, 'complex': cplx}
    if isinstance(node, ast.Dict):
        return {literal(k): literal(v) for k, v in zip(node.keys, node.values)}
    if isinstance(node, ast.List):
        return [literal(x) for x in node.elts]
    if isinstance(node, ast.Tuple):
        return tuple(literal(x) for x in node.elts)
    return ast.literal_eval(node)


def main():
    out = {}
    src = os.path.join(REF_TEST, 'test_outputs')
    for fname in sorted(os.listdir(src)):
        if not fname.endswith('.txt') or 'globalasm' in fname:
            continue
        with open(os.path.join(src, fname)) as f:
            prog = literal(ast.parse(f.read().strip(), mode='eval').body)
        out[fname[:-4]] = [{'group': list(k), 'statements': enc(v)} for k, v in prog.items()]
    with open(os.path.join(HERE, 'asm_inputs.json'), 'w') as f:
        json.dump({'source': 'python/test/test_outputs/*.txt (reference compiler outputs, data)',
                   'programs': out}, f, indent=0)
    shutil.copyfile(os.path.join(REF_TEST, 'channel_config.json'), os.path.join(HERE, 'channel_config.json'))


if __name__ == '__main__':
    main()
