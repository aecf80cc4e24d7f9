"""Per-wave execution counts of branch_kernel's loop sections (diagnostic
build -DBRANCH_PROBE_COUNTS, scripts/ab_libs.sh) on a scripts/ab.py workload:
one launch, the counters per wave.  One JSON line.

    python scripts/branch_counts.py --lib ab_build/libdpemu_bcnt.so --workload ar_sm
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

NAMES = ['iterations', 'fproc_bound', 'pulse_write', 'emit', 'measure', 'alu_section', 'meas_lookup',
         'finish', 'flush_pending', 'flush_row', 'flush_row2', 'sync']


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--lib', required=True)
    ap.add_argument('--workload', default='ar_sm')
    a = ap.parse_args()
    import torch
    from ab import workload
    from distributed_processor_amd.emulator import Emulator, alloc_device_outputs
    ps, cfg, n = workload(a.workload)
    e = Emulator(0, lib_path=os.path.abspath(a.lib))
    e.load(ps)
    out = alloc_device_outputs(cfg, n, want=('summary', 'events', 'meas', 'hist'))
    f = e._L.dpemu_probe_branch_counts
    f.restype = C.c_int
    f.argtypes = [C.c_void_p, C.c_int]
    buf = np.zeros(16, np.uint64)
    e.run_device(cfg, n, 0, out)
    torch.cuda.synchronize()
    f(buf.ctypes.data, 1)                       # reset after the warm-up launch
    e.run_device(cfg, n, 0, out)
    torch.cuda.synchronize()
    f(buf.ctypes.data, 1)
    waves = (n * cfg.cores_per_shot + 63) // 64
    print(json.dumps({'workload': a.workload, 'kernel': e.last_kernel(), 'waves': waves,
                      'per_wave': {k: round(float(buf[i]) / waves, 3) for i, k in enumerate(NAMES)}}))


if __name__ == '__main__':
    main()
