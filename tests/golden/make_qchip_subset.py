"""Extract the Q0/Q1 part of the reference's gate table (python/test/qubitcfg.json,
the QChip input of the reference's compiler tests) as a data fixture for
tests/test_schedule.py.  Run in the container that holds /root/reference:

    python tests/golden/make_qchip_subset.py
"""
import json
import os

SRC = '/root/reference/python/test/qubitcfg.json'
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'qchip_q01.json')

with open(SRC) as f:
    cfg = json.load(f)
qubits = ('Q0', 'Q1')
sub = {'source': 'python/test/qubitcfg.json (Qubits and Gates of Q0, Q1)',
       'Qubits': {q: cfg['Qubits'][q] for q in qubits},
       'Gates': {k: v for k, v in cfg['Gates'].items()
                 if any(k.startswith(q) and not k[len(q)].isdigit() for q in qubits)}}
with open(OUT, 'w') as f:
    json.dump(sub, f, indent=1, sort_keys=True)
print(OUT, len(sub['Gates']), 'gates')
