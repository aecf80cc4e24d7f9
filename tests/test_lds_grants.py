"""The dynamic-LDS opt-in bookkeeping (csrc/lds_grants.h) on the CPU: per
(device, kernel), growing requests, failed opt-ins, many threads.  The
round-3 kernels kept one process-wide static per kernel, so a second device
(or a racing thread) skipped its own hipFuncSetAttribute."""

import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.fresh_process        # runs g++ and a binary: before any test touches the GPU (tests/conftest.py)
@pytest.mark.skipif(shutil.which('g++') is None, reason='g++ not available')
def test_lds_grants_bookkeeping(tmp_path):
    exe = str(tmp_path / 'lds_grants_test')
    subprocess.run(['g++', '-std=c++17', '-O1', '-pthread', '-Wall', '-o', exe,
                    os.path.join(HERE, 'lds_grants_test.cpp')], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().endswith('OK')
