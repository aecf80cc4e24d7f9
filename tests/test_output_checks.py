"""Host-side checks run_device applies to every caller buffer before the C
ABI sees a bare pointer (emulator._check_tensor): type, device, dtype width,
contiguity and element count.  CPU-only: a CPU tensor fails the device
check, so the later checks run on real tensors whose device queries report
a CUDA device (the checks read only is_cuda / get_device / device)."""
import pytest
import torch

from distributed_processor_amd import _abi
from distributed_processor_amd._native import DpemuError
from distributed_processor_amd.emulator import _check_tensor, device_output_specs


def _specs():
    cfg = _abi.make_config(8, n_groups=4, event_cap=8, meas_cap=2)
    return device_output_specs(cfg, 16)


class _OnDevice(torch.Tensor):
    """a CPU tensor that reports cuda:<_index> to the checks"""
    _index = 0
    is_cuda = property(lambda self: True)
    device = property(lambda self: torch.device('cuda', self._index))

    def get_device(self):
        return self._index


def _dev(t, index=0):
    x = t.as_subclass(_OnDevice)
    x._index = index
    return x


def test_rejects_non_tensor_and_cpu_tensor():
    spec = _specs()['summary']
    with pytest.raises(DpemuError, match='expected a torch tensor'):
        _check_tensor('summary', [0] * 8, spec, 0)
    with pytest.raises(DpemuError, match='emulator runs on cuda:0'):
        _check_tensor('summary', torch.zeros(spec[0], dtype=spec[1]), spec, 0)


def test_rejects_wrong_device_dtype_layout_size():
    spec = _specs()['events']
    shape, dtype = spec
    _check_tensor('events', _dev(torch.zeros(shape, dtype=dtype)), spec, 0)          # accepted
    with pytest.raises(DpemuError, match='emulator runs on cuda:0'):
        _check_tensor('events', _dev(torch.zeros(shape, dtype=dtype), index=1), spec, 0)
    with pytest.raises(DpemuError, match='dtype'):
        _check_tensor('events', _dev(torch.zeros(shape, dtype=torch.int16)), spec, 0)
    with pytest.raises(DpemuError, match='dtype'):
        _check_tensor('events', _dev(torch.zeros(shape, dtype=torch.float32)), spec, 0)
    with pytest.raises(DpemuError, match='contiguous'):
        _check_tensor('events', _dev(torch.zeros(shape[::-1], dtype=dtype).permute(2, 1, 0)), spec, 0)
    with pytest.raises(DpemuError, match='elements'):
        _check_tensor('events', _dev(torch.zeros((shape[0] - 1,) + tuple(shape[1:]), dtype=dtype)), spec, 0)
