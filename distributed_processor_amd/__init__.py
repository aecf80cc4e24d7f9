"""MI355X-native batched emulator of the QubiC distributed processor.

Host side of the emulator: ISA encoder/decoder (``isa``), hardware-config
plugins (``hwconfig``), and the ``Emulator`` front end that runs assembled
distproc programs on hand-written CDNA4 HIP kernels through the C ABI in
``include/dpemu.h``.
"""

from . import isa, hwconfig, lint  # noqa: F401

__all__ = ['isa', 'hwconfig', 'lint']
