"""MI355X-native batched emulator of the QubiC distributed processor.

Host side of the emulator: ISA encoder/decoder (``isa``), hardware-config
plugins (``hwconfig``), and the ``Emulator`` front end that runs assembled
distproc programs on hand-written CDNA4 HIP kernels through the C ABI in
``include/dpemu.h``; upstream of it, the restated compiler scheduling
stage (``schedule``) and the API-compatible assembler (``assembler``) that turn QubiC circuits
into that machine code.
"""

from . import isa, hwconfig, lint, schedule  # noqa: F401

__all__ = ['isa', 'hwconfig', 'lint', 'schedule']
