# python/distproc/emulate.py  (proposed; binds libdpemu.so from this repo)
#
# The ctypes module a distproc maintainer would add to the reference to run
# GlobalAssembler.get_assembled_program() output (python/distproc/assembler.py:623-641)
# on libdpemu.so instead of the cocotb/Verilator testbench (cocotb/proc/test_proc.py:29-38).
# It mirrors include/dpemu.h by itself -- it imports nothing from this repo's
# Python package -- so it is what the reference side would hold.
# INTEGRATION.md §3 includes this file verbatim (tests/test_ref_binding.py
# checks the two agree) and the -m gpu tests run it against oracle_fast.
import ctypes as C

import numpy as np

ABI_VERSION = 8                                    # DPEMU_ABI_VERSION, include/dpemu.h
_vp, _u32, _u64 = C.c_void_p, C.c_uint32, C.c_uint64


class DpemuConfig(C.Structure):                    # dpemu_config, include/dpemu.h (ABI 8)
    _fields_ = [(n, C.c_uint32) for n in ('cores_per_shot', 'n_groups', 'shots_per_group',
                'max_cycles', 'event_cap', 'trace_cap', 'meas_cap', 'fproc_mode', 'meas_elem',
                'meas_latency', 'sync_latency', 'exec_flags')] + [
               ('sync_mask', C.c_uint64), ('seed', C.c_uint64), ('lut_mask', C.c_uint32),
               ('meas_model', C.c_uint32), ('p1_threshold', C.c_uint32 * 64),
               ('lut_table', C.c_uint64 * 256), ('ro_sep', C.c_int32), ('ro_sigma', C.c_uint32),
               ('ro_thr', C.c_int32), ('ro_win', C.c_uint32), ('hist_assign', C.c_uint32),
               ('lane_order', C.c_uint32), ('ro_drv_elem', C.c_uint32), ('ro_cpw', C.c_uint32),
               ('ro_delay', C.c_uint32), ('ro_theta', C.c_uint32 * 2), ('ro_gain', C.c_uint32 * 2),
               ('ro_axis', C.c_uint32 * 64)]


class DpemuOutputs(C.Structure):                   # dpemu_outputs
    _fields_ = [(n, C.c_void_p) for n in ('summary', 'events', 'trace', 'meas', 'regs', 'hist', 'hist_next',
                                          'acc')]


_L = None


def hip_runtimes():
    """paths of the HIP runtimes (libamdhip64) mapped into this process"""
    try:
        with open('/proc/self/maps') as f:
            return sorted({ln.split()[-1] for ln in f if 'libamdhip64' in ln})
    except OSError:
        return []


def load(path='libdpemu.so'):
    """bind the library once: entry points, ABI version, struct layouts.
    One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64, and
    a torch imported AFTER libdpemu.so bound /opt/rocm's would start a second
    runtime that sees no GPU.  So when torch is installed it is imported
    first (libdpemu.so then binds torch's runtime), and two runtimes already
    mapped raise here instead of failing later."""
    global _L
    if _L is not None:
        return _L
    try:
        import torch  # noqa: F401  (its HIP runtime, before libdpemu.so's dependency resolves)
    except ImportError:
        pass
    L = C.CDLL(path)
    if len(hip_runtimes()) > 1:
        raise RuntimeError('two HIP runtimes in one process ({}): load torch before other HIP '
                           'libraries'.format(', '.join(hip_runtimes())))
    L.dpemu_abi_version.restype = C.c_int
    if L.dpemu_abi_version() != ABI_VERSION:
        raise RuntimeError('libdpemu ABI {} != {}'.format(L.dpemu_abi_version(), ABI_VERSION))
    L.dpemu_struct_sizes.argtypes = [_vp]
    sizes = (C.c_uint64 * 3)()                     # the library's own layouts
    L.dpemu_struct_sizes(sizes)
    if (sizes[0], sizes[1]) != (C.sizeof(DpemuConfig), C.sizeof(DpemuOutputs)):
        raise RuntimeError('dpemu_config / dpemu_outputs layout differs from the library')
    L.dpemu_create.argtypes = [C.c_int, C.POINTER(_vp)]
    L.dpemu_destroy.argtypes = [_vp]
    L.dpemu_last_error.argtypes = [_vp]
    L.dpemu_last_error.restype = C.c_char_p
    L.dpemu_load_programs.argtypes = [_vp, _vp, _u64, _vp, _vp, _u32, _vp, _u32, _u32]
    L.dpemu_run_host.argtypes = [_vp, _vp, _u64, _u64, _vp]
    _L = L
    return L


def _check(ctx, rc, what):
    if rc:
        msg = _L.dpemu_last_error(ctx) if ctx else b''
        raise RuntimeError('{}: {} ({})'.format(what, (msg or b'').decode(), rc))


def pack_assembled(assembled):
    """cmd_mem images of an assembled program, the dpemu_load_programs arrays:
    (words (n, 4) u32, offsets, n_instr, table, C).  Cores absent from the
    program get an empty image (cmd_mem reads 0 = DONE)."""
    progs = {int(k): np.frombuffer(bytes(v['cmd_buf']), '<u4').reshape(-1, 4) for k, v in assembled.items()}
    C_ = 1
    while C_ <= max(progs):
        C_ <<= 1
    images = [progs.get(c, np.zeros((0, 4), np.uint32)) for c in range(C_)]
    n_instr = np.array([len(p) for p in images], np.uint32)
    offsets = np.concatenate([[0], np.cumsum(n_instr)[:-1]]).astype(np.uint32)
    words = np.ascontiguousarray(np.concatenate(images) if n_instr.sum() else np.zeros((1, 4)), np.uint32)
    table = np.arange(C_, dtype=np.uint32)         # one group: core c runs image c
    return words, offsets, n_instr, table, C_


def run_assembled(assembled, n_shots, cfg: DpemuConfig, device=0, path='libdpemu.so'):
    """assembled: GlobalAssembler.get_assembled_program() output.  Runs shots
    [0, n_shots) of every core; returns (summary [lanes, 8], events
    [event_cap, lanes, 4], meas [meas_cap, lanes, 2], hist [2^C] or None) with lane =
    core * n_shots + shot (cfg.lane_order 0)."""
    L = load(path)
    words, offsets, n_instr, table, C_ = pack_assembled(assembled)
    ctx = _vp()
    _check(None, L.dpemu_create(device, C.byref(ctx)), 'dpemu_create')
    try:
        _check(ctx, L.dpemu_load_programs(ctx, words.ctypes.data, len(words), offsets.ctypes.data,
               n_instr.ctypes.data, len(n_instr), table.ctypes.data, 1, C_), 'dpemu_load_programs')
        cfg.cores_per_shot, cfg.n_groups, cfg.shots_per_group = C_, 1, 1
        n_lanes = n_shots * C_
        summary = np.zeros((n_lanes, 8), np.uint32)
        ev = np.zeros((cfg.event_cap, n_lanes, 4), np.uint32)
        meas = np.zeros((cfg.meas_cap, n_lanes, 2), np.uint32)
        hist = np.zeros(1 << C_, np.uint64) if C_ <= 12 else None     # 2^C bins (C <= 12)
        out = DpemuOutputs(summary.ctypes.data, ev.ctypes.data if cfg.event_cap else None, None,
                           meas.ctypes.data if cfg.meas_cap else None, None,
                           hist.ctypes.data if hist is not None else None, None)
        _check(ctx, L.dpemu_run_host(ctx, C.byref(cfg), 0, n_shots, C.byref(out)), 'dpemu_run_host')
        return summary, ev, meas, hist
    finally:
        L.dpemu_destroy(ctx)
