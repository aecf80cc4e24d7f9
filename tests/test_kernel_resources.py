"""Resource guard of the product kernels, on the CPU: a
kernel whose state falls into scratch still produces the right bytes --
round 5's three-slot macro_kernel did, 10x slower (4.85 -> 44 ms on config
4), and only a manual sweep noticed.  These tests read the gfx950 code
objects embedded in the built libdpemu.so (llvm-objdump --offloading) and
assert, for every product kernel:

* scratch: private_segment_fixed_size 0 and no spilled VGPRs, except the
  recorded allowances below (a kernel whose budget is set by
  amdgpu_waves_per_eu and spills a few bytes on purpose, measured faster
  than the spill-free build);
* no scratch_* instruction beyond those allowances, and no flat_* memory
  instruction (a generic-pointer access where a global / LDS one belongs);
* occupancy: the waves per SIMD the register count allows is at least the
  kernel's recorded floor (the bench kernels: the budget each was measured at).

The round-5 pre-fix macro.hip (git a95f585^) builds a macro_kernel with 824
bytes of scratch per lane (hipcc -Rpass-analysis=kernel-resource-usage), which
test_no_scratch_beyond_allowances rejects; HEAD's has the recorded 20."""

import os
import re
import shutil
import subprocess

import pytest

from distributed_processor_amd import _native

LLVM = '/opt/rocm/lib/llvm/bin'
pytestmark = [pytest.mark.fresh_process,      # runs llvm tools: before any test touches the GPU
              pytest.mark.skipif(not os.path.exists(os.path.join(LLVM, 'llvm-objdump')),
                                 reason='ROCm llvm tools not available')]

# kernel-name substring -> allowed scratch bytes per lane (and scratch instructions)
SCRATCH_ALLOWED = {
    # amdgpu_waves_per_eu(6): 80 VGPRs, 20 B spilled; the 5-wave build has no
    # spill but measured 5.65 vs 5.07 ms on config 4 through this kernel
    # (scripts/ab.py --flags 0x40, profiles/r06_macro_ab.json)
    '12macro_kernelE': (20, 8),
}
# kernel-name substring -> minimum waves per SIMD (register-limited occupancy)
# (each the occupancy the kernel was measured at: a build that loses a wave
# fails here before it reaches the GPU)
OCCUPANCY_FLOOR = {
    'straight_kernelILi0ELi1E': 6,         # config 2 headline (rows fetch, fb1)
    'branch_kernelILi11ELi8E': 6,          # config 3
    'branch_kernelILi14ELi8E': 7,          # config 3 through the LUT
    'branch_kernelILi75ELi8E': 4,          # config 3 with the DEMOD readout model
    'macro_staged_kernelILi2ELb1ELi8E': 4, # config 4
    '12macro_kernelE': 6,                  # config 4, DPEMU_X_MACRO_DIRECT
    'dds_tile_kernel': 7,                  # config 5
    'dds_index_kernel': 8,
}


@pytest.fixture(scope='module')
def code_objects(tmp_path_factory):
    if not os.path.exists(_native.LIB_PATH):
        pytest.skip('libdpemu.so not built')
    d = tmp_path_factory.mktemp('co')
    lib = str(d / 'libdpemu.so')
    shutil.copy(_native.LIB_PATH, lib)
    subprocess.run([os.path.join(LLVM, 'llvm-objdump'), '--offloading', lib], cwd=str(d), check=True,
                   capture_output=True)
    cos = sorted(str(d / f) for f in os.listdir(str(d)) if 'amdgcn' in f and f.endswith('gfx950'))
    assert cos, 'no gfx950 code object in libdpemu.so'
    return cos


def kernel_meta(co):
    """{kernel symbol: {field: int}} from the code object's AMDGPU metadata note"""
    txt = subprocess.run([os.path.join(LLVM, 'llvm-readelf'), '--notes', co], check=True, capture_output=True,
                         text=True).stdout
    out, cur = {}, None
    for ln in txt.splitlines():
        m = re.match(r'\s+\.name:\s+(\S+)', ln)
        if m:
            cur = out.setdefault(m.group(1), {})
            continue
        m = re.match(r'\s+\.(vgpr_count|agpr_count|vgpr_spill_count|sgpr_spill_count|private_segment_fixed_size|'
                     r'group_segment_fixed_size):\s+(\d+)', ln)
        if m and cur is not None:
            cur[m.group(1)] = int(m.group(2))
    return {k: v for k, v in out.items() if 'vgpr_count' in v}


def memory_instrs(co):
    """{kernel symbol: (scratch_* count, flat_* count)} from the disassembly"""
    txt = subprocess.run([os.path.join(LLVM, 'llvm-objdump'), '-d', '--no-show-raw-insn', co], check=True,
                         capture_output=True, text=True).stdout
    out, cur = {}, None
    for ln in txt.splitlines():
        m = re.match(r'^[0-9a-f]+ <(\S+)>:$', ln)
        if m:
            cur = m.group(1)
            out.setdefault(cur, [0, 0])
            continue
        if cur is None:
            continue
        ins = ln.strip().split(' ')[0]
        if ins.startswith('scratch_'):
            out[cur][0] += 1
        elif ins.startswith('flat_'):
            out[cur][1] += 1
    return {k: tuple(v) for k, v in out.items()}


def waves_per_simd(vgprs, agprs=0):
    """register-limited occupancy on gfx950: 512 unified VGPRs per lane per SIMD,
    allocated in granules of 8, at most 8 waves"""
    n = max(vgprs + agprs, 1)
    return min(8, 512 // ((n + 7) // 8 * 8))


def product_kernels(code_objects):
    meta = {}
    for co in code_objects:
        meta.update(kernel_meta(co))
    return {k: v for k, v in meta.items() if k.startswith('_ZN5dpemu')}


def allowance(table, name, default):
    for k, v in table.items():
        if k in name:
            return v
    return default


def test_every_kernel_found(code_objects):
    ks = product_kernels(code_objects)
    for sub in OCCUPANCY_FLOOR:
        assert any(sub in k for k in ks), sub
    assert len(ks) > 100


def test_no_scratch_beyond_allowances(code_objects):
    bad = []
    for name, m in product_kernels(code_objects).items():
        lim = allowance(SCRATCH_ALLOWED, name, (0, 0))[0]
        if m.get('private_segment_fixed_size', 0) > lim:
            bad.append((name, 'scratch {} B > {}'.format(m['private_segment_fixed_size'], lim)))
        if lim == 0 and m.get('vgpr_spill_count', 0):
            bad.append((name, '{} VGPRs spilled'.format(m['vgpr_spill_count'])))
    assert not bad, bad


def test_no_scratch_or_flat_instructions(code_objects):
    bad = []
    for co in code_objects:
        for name, (n_scratch, n_flat) in memory_instrs(co).items():
            if not name.startswith('_ZN5dpemu'):
                continue
            lim = allowance(SCRATCH_ALLOWED, name, (0, 0))[1]
            if n_scratch > lim:
                bad.append((name, '{} scratch_* instructions > {}'.format(n_scratch, lim)))
            if n_flat:
                bad.append((name, '{} flat_* instructions'.format(n_flat)))
    assert not bad, bad


def test_occupancy_floors(code_objects):
    ks = product_kernels(code_objects)
    bad = []
    for name, m in ks.items():
        floor = allowance(OCCUPANCY_FLOOR, name, 1)
        w = waves_per_simd(m['vgpr_count'], m.get('agpr_count', 0))
        if w < floor:
            bad.append((name, 'VGPRs {} -> {} waves / SIMD < {}'.format(m['vgpr_count'], w, floor)))
    assert not bad, bad
