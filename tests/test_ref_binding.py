"""The reference-side binding (tests/ref_binding.py = the proposed
python/distproc/emulate.py of INTEGRATION.md §3) as tested code.

CPU: INTEGRATION.md holds the module verbatim; its structs match the
library's own layouts (dpemu_struct_sizes) and this package's mirror; its
packing of an assembled dict gives the cmd_mem images ProgramSet gives.
GPU: a GlobalAssembler.get_assembled_program() dict (python/distproc/
assembler.py:623-641) goes through run_assembled -- ctypes straight onto the
C ABI, none of this package's Python -- and every output equals oracle_fast's
on the same arrays: the reference's golden cmd_buf (test_linear_compile_globalasm,
both cores), the config-1 program, and a restated-assembler golden with two
cores."""

import ctypes as C
import json
import os
import re

import numpy as np
import pytest

from distributed_processor_amd import _abi, _native, workloads
from distributed_processor_amd.emulator import ProgramSet
from tests import ref_binding

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def golden_assembled():
    with open(os.path.join(HERE, 'golden', 'cmd_buf_golden.json')) as f:
        gold = json.load(f)
    return {k: {'cmd_buf': bytes.fromhex(v['cmd_buf']), 'env_buffers': [], 'freq_buffers': []}
            for k, v in gold['cores'].items()}


def test_integration_doc_holds_the_module_verbatim():
    with open(os.path.join(REPO, 'INTEGRATION.md')) as f:
        doc = f.read()
    with open(os.path.join(HERE, 'ref_binding.py')) as f:
        src = f.read()
    blocks = re.findall(r'```python\n(.*?)```', doc, re.S)
    assert any(b == src for b in blocks), 'INTEGRATION.md §3 must hold tests/ref_binding.py verbatim'


def bind():
    """the binding on the in-tree library, loaded the way a distproc user
    would load it (ref_binding.load brings in torch's HIP runtime itself)"""
    return ref_binding.load(_native.LIB_PATH)


def test_binding_layouts_match_library_and_mirror():
    L = bind()
    sizes = (C.c_uint64 * 3)()
    L.dpemu_struct_sizes(sizes)
    assert sizes[0] == C.sizeof(ref_binding.DpemuConfig) == C.sizeof(_abi.Config)
    assert sizes[1] == C.sizeof(ref_binding.DpemuOutputs) == C.sizeof(_abi.Outputs)
    # field by field: same names, offsets and sizes as the package's mirror
    for (n, _), (m, _) in zip(ref_binding.DpemuConfig._fields_, _abi.Config._fields_):
        a, b = getattr(ref_binding.DpemuConfig, n), getattr(_abi.Config, m)
        assert (n, a.offset, a.size) == (m, b.offset, b.size)


@pytest.mark.parametrize('which', ['golden', 'config1', 'restated'])
def test_pack_assembled_matches_programset(which):
    asm = assembled_case(which)
    words, offsets, n_instr, table, C_ = ref_binding.pack_assembled(asm)
    ps = ProgramSet([asm])
    assert C_ == ps.cores_per_shot
    for c in range(C_):
        o, n = int(offsets[table[c]]), int(n_instr[table[c]])
        assert np.array_equal(words[o:o + n], ps.program(0, c)), c


def assembled_case(which):
    if which == 'golden':
        return golden_assembled()
    if which == 'config1':
        return workloads.config1_linear()
    from distributed_processor_amd import hwconfig
    from tests.test_assembler import assemble
    return assemble('test_hw_virtualz_out', hwconfig.DDSElementConfig)


def binding_config(C_, **kw):
    """a DpemuConfig filled the way a distproc user would (p1 etc. through
    this package's validated make_config, copied byte for byte)"""
    src = _abi.make_config(C_, **kw)
    cfg = ref_binding.DpemuConfig()
    C.memmove(C.addressof(cfg), C.addressof(src), C.sizeof(cfg))
    return cfg, src


@pytest.mark.gpu
@pytest.mark.parametrize('which', ['golden', 'config1', 'restated'])
def test_run_assembled_vs_oracle(which):
    import oracle
    bind()
    asm = assembled_case(which)
    words, offsets, n_instr, table, C_ = ref_binding.pack_assembled(asm)
    n_shots = 20000
    cfg, ocfg = binding_config(C_, max_cycles=20000, event_cap=16, meas_cap=4, meas_latency=64, p1=0.5,
                               seed=0x5EED + len(which))
    summary, ev, meas, hist = ref_binding.run_assembled(asm, n_shots, cfg, path=_native.LIB_PATH)
    f = oracle.fast_run(ocfg, words, offsets, n_instr, table, 0, n_shots,
                        want=('summary', 'events', 'meas', 'hist'))
    assert np.array_equal(summary, f['summary'])
    assert np.array_equal(ev, f['events'])
    assert np.array_equal(meas, f['meas'])
    assert np.array_equal(hist, np.asarray(f['hist']).reshape(-1))
    s = _abi.unpack_summary(summary)
    assert (s['n_events'] > 0).any()
    if which == 'golden':
        # the reference's golden core 0: pulse_reset at 0, cstrobes at 8 / 24 / 324
        # (test_gpu_parity.test_config1_golden_program; lane = core * n_shots + shot)
        assert [int(e[0]) for e in ev[:4, 0]] == [0, 8, 24, 324]


CHILD = r'''
import sys
sys.path.insert(0, {repo!r})
from tests import ref_binding
L = ref_binding.load({lib!r})                  # the binding first, as a distproc user would
import torch                                    # then PyTorch
assert torch.cuda.device_count() > 0, 'torch sees no GPU after the binding loaded'
runtimes = ref_binding.hip_runtimes()
assert len(runtimes) == 1, runtimes
x = torch.arange(1024, device='cuda', dtype=torch.int32)
assert int(x.sum().item()) == 1023 * 1024 // 2
import ctypes
cfg = ref_binding.DpemuConfig()                 # filled by the parent (make_config), byte for byte
raw = bytes.fromhex({cfg_hex!r})
ctypes.memmove(ctypes.addressof(cfg), raw, len(raw))
golden = {golden!r}
asm = {{k: {{'cmd_buf': bytes.fromhex(v), 'env_buffers': [], 'freq_buffers': []}} for k, v in golden.items()}}
summary, ev, meas, hist = ref_binding.run_assembled(asm, 1000, cfg, path={lib!r})
assert [int(e[0]) for e in ev[:4, 0]] == [0, 8, 24, 324], ev[:4, 0]
print('ok', torch.cuda.device_count(), runtimes[0])
'''


@pytest.mark.gpu
@pytest.mark.fresh_process
def test_binding_first_then_torch_in_a_fresh_process():
    """INTEGRATION.md §3 as a distproc user runs it: a fresh Python loads the
    binding BEFORE importing torch, then uses torch on the GPU and runs the
    reference's golden cmd_buf through the binding -- one HIP runtime, torch
    sees the device.  (Runs first in the session, before this process touches
    the GPU: tests/conftest.py orders fresh_process tests.)"""
    import subprocess
    import sys
    with open(os.path.join(HERE, 'golden', 'cmd_buf_golden.json')) as f:
        gold = {k: v['cmd_buf'] for k, v in json.load(f)['cores'].items()}
    cfg, _ = binding_config(2, max_cycles=4000, event_cap=8, meas_cap=2, meas_latency=64, p1=0.5)
    src = CHILD.format(repo=REPO, lib=_native.LIB_PATH, golden=gold, cfg_hex=bytes(cfg).hex())
    r = subprocess.run([sys.executable, '-c', src], capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert r.stdout.startswith('ok'), r.stdout
