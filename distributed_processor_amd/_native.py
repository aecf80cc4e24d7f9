"""ctypes binding of libdpemu.so (include/dpemu.h).  No fallback: if the HIP
library is missing or a GPU call fails, this raises."""

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, 'libdpemu.so')

# every entry point declared in include/dpemu.h
EXPORTS = ('dpemu_abi_version', 'dpemu_struct_sizes', 'dpemu_create', 'dpemu_destroy', 'dpemu_last_error',
           'dpemu_load_programs', 'dpemu_load_readout_freqs', 'dpemu_run', 'dpemu_run_host', 'dpemu_dds', 'dpemu_dds_sin_lut',
           'dpemu_set_kernel_timing', 'dpemu_kernel_times', 'dpemu_last_kernel')

_libs = {}


class DpemuError(RuntimeError):
    pass


def load_library(path=LIB_PATH):
    """the ctypes handle of libdpemu.so (another build's path for A/B runs)"""
    if path in _libs:
        return _libs[path]
    if not os.path.exists(path):
        raise DpemuError('libdpemu.so not built ({}); run __graft_entry__.build() '
                         '(hipcc --offload-arch=gfx950)'.format(path))
    # One HIP runtime per process.  PyTorch-ROCm ships its own
    # libamdhip64.so (soname libamdhip64.so.7) and libhsa-runtime64; loaded
    # first, it satisfies libdpemu.so's libamdhip64.so.7 dependency, so both
    # share one runtime and device pointers / streams pass freely.  Loaded
    # after ours, torch would bring up a second runtime that finds no GPU.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(path)
    # an older build lacks later entry points: name them instead of letting
    # ctypes raise a bare AttributeError on the first argtypes assignment
    missing = [s for s in EXPORTS if not hasattr(L, s)]
    if missing:
        raise DpemuError('{} lacks {} (a build older than this binding); rebuild it with '
                         '__graft_entry__.build()'.format(path, ', '.join(missing)))
    vp, u32, u64 = C.c_void_p, C.c_uint32, C.c_uint64
    L.dpemu_abi_version.restype = C.c_int
    L.dpemu_struct_sizes.argtypes = [vp]
    L.dpemu_create.argtypes = [C.c_int, C.POINTER(vp)]
    L.dpemu_destroy.argtypes = [vp]
    L.dpemu_last_error.argtypes = [vp]
    L.dpemu_last_error.restype = C.c_char_p
    L.dpemu_load_programs.argtypes = [vp, vp, u64, vp, vp, u32, vp, u32, u32]
    L.dpemu_load_readout_freqs.argtypes = [vp, vp, u64, vp, vp, vp, vp]
    L.dpemu_run.argtypes = [vp, vp, u64, u64, vp, vp]
    L.dpemu_run_host.argtypes = [vp, vp, u64, u64, vp]
    L.dpemu_dds.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp]
    L.dpemu_dds_sin_lut.argtypes = [vp]
    L.dpemu_set_kernel_timing.argtypes = [vp, C.c_int]
    L.dpemu_kernel_times.argtypes = [vp, vp, C.c_int, vp]
    L.dpemu_last_kernel.argtypes = [vp]
    L.dpemu_last_kernel.restype = C.c_char_p
    from . import _abi
    if L.dpemu_abi_version() != _abi.ABI_VERSION:
        raise DpemuError('ABI version mismatch: library {} vs host {}'.format(
            L.dpemu_abi_version(), _abi.ABI_VERSION))
    # the struct layouts too: two builds of one ABI version from different
    # header states must not share a process with a mismatched ctypes mirror
    sizes = (C.c_uint64 * 3)()
    L.dpemu_struct_sizes(sizes)
    mine = (C.sizeof(_abi.Config), C.sizeof(_abi.Outputs), C.sizeof(_abi.DDSChannels))
    if tuple(sizes) != mine:
        raise DpemuError('struct layout mismatch: library {} vs host {} ({})'.format(tuple(sizes), mine, path))
    _libs[path] = L
    return L


def check(ctx_handle, rc, what, L=None):
    if rc != 0:
        L = L or load_library()
        msg = L.dpemu_last_error(ctx_handle)
        raise DpemuError('{} failed ({}): {}'.format(what, rc, msg.decode() if msg else ''))
