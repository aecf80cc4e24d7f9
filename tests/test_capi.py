"""The C-ABI library: builds, loads, exports every entry point of
include/dpemu.h, and fails loudly (no CPU fallback) when no GPU is present.
No compute call is made here."""

import ctypes as C
import os
import re

import pytest

from distributed_processor_amd import _abi, _native

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    with open(os.path.join(REPO, 'include', 'dpemu.h')) as f:
        txt = f.read()
    return sorted(set(re.findall(r'\b(dpemu_[a-z_0-9]+)\s*\(', txt)))


def test_header_symbols_exported():
    names = header_functions()
    assert set(names) == set(_native.EXPORTS)
    L = _native.load_library()
    for n in names:
        assert hasattr(L, n), n


def test_abi_version_and_struct_sizes():
    L = _native.load_library()
    assert L.dpemu_abi_version() == _abi.ABI_VERSION
    # dpemu_config: 12 u32 + 2 u64 + 2 u32 + 64 u32 + 256 u64 + the readout model's 4 x 32 bit
    # + hist_assign, lane_order + the DEMOD model's 3 + 2 + 2 + 64 u32 (ABI 8), padded to 8
    assert C.sizeof(_abi.Config) == (12 * 4 + 16 + 8 + 64 * 4 + 256 * 8 + 16 + 8 + 71 * 4 + 7) // 8 * 8
    assert C.sizeof(_abi.Outputs) == 8 * 8
    assert C.sizeof(_abi.DDSChannels) == 4 * 4 + 8 * 8
    sizes = (C.c_uint64 * 3)()
    assert L.dpemu_struct_sizes(sizes) == 0
    assert tuple(sizes) == (C.sizeof(_abi.Config), C.sizeof(_abi.Outputs), C.sizeof(_abi.DDSChannels))
    assert L.dpemu_struct_sizes(None) != 0


def test_output_struct_matches_header():
    """the ctypes mirror lists dpemu_outputs' fields in the header's order"""
    with open(os.path.join(REPO, 'include', 'dpemu.h')) as f:
        txt = f.read()
    body = re.search(r'typedef struct dpemu_outputs \{(.*?)\} dpemu_outputs;', txt, re.S).group(1)
    fields = re.findall(r'\*\s*(\w+);', body)
    assert fields == [n for n, _ in _abi.Outputs._fields_] == list(_abi.OUTPUT_NAMES)


def test_sin_lut_symmetry():
    L = _native.load_library()
    buf = (C.c_int16 * 4096)()
    assert L.dpemu_dds_sin_lut(buf) == 0
    v = list(buf)
    assert v[0] == 0 and v[1024] == 32767 and v[2048] == 0 and v[3072] == -32767
    for i in range(1, 1024):
        assert v[i] == v[2048 - i] == -v[2048 + i] == -v[4096 - i]


def test_create_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip('GPU present')
    from distributed_processor_amd.emulator import Emulator
    with pytest.raises(_native.DpemuError):
        Emulator(0)


def test_config_validation():
    with pytest.raises(ValueError):
        _abi.make_config(3)
    with pytest.raises(ValueError):
        _abi.make_config(4, max_cycles=2 ** 31)
    with pytest.raises(ValueError):
        _abi.make_config(4, lut_mask=0)
    with pytest.raises(ValueError):
        _abi.make_config(4, event_cap=2 ** 21)
    with pytest.raises(ValueError):
        _abi.make_config(4, readout=dict(sep=1, win=4096))
    with pytest.raises(ValueError):                  # the drive element must differ from the LO's
        _abi.make_config(4, meas_elem=2, demod=dict(drv_elem=2))
    with pytest.raises(ValueError):
        _abi.make_config(4, demod=dict(cpw=9))
    with pytest.raises(ValueError):
        _abi.make_config(4, demod=dict(sigma=256.0))
    with pytest.raises(ValueError):
        _abi.make_config(4, demod=dict(gain=(1.5, 1.0)))
    with pytest.raises(ValueError):
        _abi.make_config(4, readout=dict(sep=1), demod=dict())
    d = _abi.make_config(4, demod=dict(drv_elem=1, cpw=4, delay=300, theta=(0.0, 3.141592653589793),
                                       gain=(0.5, 1.0), axis=[0.0, 1.5707963267948966], sigma=2.0, thr=-7))
    assert d.meas_model == _abi.MEAS_DEMOD and d.ro_theta[1] == 2 ** 31 and d.ro_gain[0] == 32768
    assert d.ro_axis[0] == 32767 and d.ro_axis[1] == 32767 << 16 and d.ro_axis[2] == 32767
    assert d.ro_sigma == 2 << 16 and d.ro_thr == -7 and (d.ro_drv_elem, d.ro_cpw, d.ro_delay) == (1, 4, 300)
    cfg = _abi.make_config(8, p1=[0.0, 1.0, 0.5])
    assert cfg.p1_threshold[0] == 0 and cfg.p1_threshold[1] == 0xFFFFFFFF and cfg.p1_threshold[2] == 2 ** 31


def test_struct_layout_mismatch_refused(tmp_path, monkeypatch):
    """a library whose struct layouts differ from the binding's ctypes mirror
    is refused at load (dpemu_struct_sizes), whatever its version number"""
    import shutil
    lib = str(tmp_path / 'libdpemu_copy.so')
    shutil.copy(_native.LIB_PATH, lib)

    class Shorter(C.Structure):                 # a mirror missing dpemu_config's last field
        _fields_ = [('x', C.c_uint8 * (C.sizeof(_abi.Config) - 4))]
    monkeypatch.setattr(_abi, 'Config', Shorter)
    with pytest.raises(_native.DpemuError, match='struct layout mismatch'):
        _native.load_library(lib)


def test_exec_flags_mirror_header():
    """every DPEMU_X_* execution knob of include/dpemu.h has the same value in _abi"""
    with open(os.path.join(REPO, 'include', 'dpemu.h')) as f:
        txt = f.read()
    flags = dict(re.findall(r'#define DPEMU_(X_[A-Z_]+)\s+(0x[0-9a-fA-F]+)', txt))
    assert 'X_STREAM_EVENTS' in flags and len(flags) >= 7
    for name, val in flags.items():
        assert getattr(_abi, name) == int(val, 16), name
