"""bench.py on the CPU: the roofline / byte accounting helpers, the CPU
baseline's timing loop and thread count, and the committed bench line
(profiles/r02_bench.json) against the driver's JSON contract and its own
same-box rocprof evidence."""

import json
import os

import numpy as np
import pytest

import bench
from distributed_processor_amd import _abi

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_hbm_roofline_caps_at_the_step_and_prefers_the_leg_profile(tmp_path, monkeypatch):
    prof = {'duration_ns': 200000.0, 'hbm_bytes_per_launch': 1.1e9}
    r = bench.hbm_roofline(1e9, kernel_ms=0.30, ms_per_step=0.25, kernel='k', prof=prof, rocprof_key='k')
    assert r['kernel_ms'] == 0.25 and r['kernel_ms_events'] == 0.30          # capped at the step
    assert r['achieved'] == pytest.approx(1e9 / 0.25e-3 / 1e9)
    assert r['frac'] == pytest.approx(r['achieved'] / bench.HBM_PEAK_GBS)
    assert r['traffic'] == 1.1e9
    assert r['kernel_ms_rocprof'] == pytest.approx(0.2)
    assert r['frac_rocprof'] == pytest.approx(1e9 / 0.2e-3 / 1e9 / bench.HBM_PEAK_GBS)
    # no per-leg duration: the --stats row of the kernel
    (tmp_path / (bench.PROFILE_TAG + '_kernel_stats.csv')).write_text('"Name","Calls","AverageNs"\n"void dpemu::my_kernel(x)",3,"150000"\n')
    monkeypatch.setattr(bench, 'PROFILE_DIR', str(tmp_path))
    r = bench.hbm_roofline(1e9, 0.2, 1.0, 'k', {'hbm_bytes_per_launch': None}, 'my_kernel')
    assert r['kernel_ms_rocprof'] == pytest.approx(0.15)
    assert 'kernel_ms_rocprof' not in bench.hbm_roofline(1e9, 0.2, 1.0, 'k', None, 'my_kernel')


def test_bytes_per_lane_counts_written_records_only():
    cfg = _abi.make_config(8, event_cap=8, meas_cap=2)
    s = np.zeros((3, 8), np.uint32)
    s[:, 2] = [0, 5, 20]          # n_events (20 > event_cap: 8 written)
    s[:, 5] = [0, 1, 9]           # n_meas (9 > meas_cap: 2 written)
    np.testing.assert_array_equal(bench.bytes_per_lane(s, cfg), [32.0, 32 + 80 + 8, 32 + 128 + 16])


def test_host_cores_respects_the_job_share(monkeypatch):
    aff = len(os.sched_getaffinity(0))
    monkeypatch.setenv('OMP_NUM_THREADS', '1')
    use, info = bench.host_cores()
    assert use == 1 and info['nproc'] == aff and info['omp_num_threads'] == '1'
    monkeypatch.delenv('OMP_NUM_THREADS')
    assert bench.host_cores()[0] == aff


def test_median_rate_times_a_fixed_sample():
    calls = []
    rate, n, times = bench.median_rate(lambda k: calls.append(k), units_per_n=8, n0=10, target_s=0.001, reps=5)
    assert len(calls) == 6 and calls[0] == 10 and set(calls[1:]) == {n} and len(times) == 5
    assert rate == pytest.approx(n * 8 / float(np.median(times)))


def _bench_line():
    with open(os.path.join(REPO, 'profiles', 'r02_bench.json')) as f:
        lines = [json.loads(x) for x in f if x.startswith('{')]
    assert len(lines) == 1, 'one JSON line'
    return lines[0]


def test_committed_bench_line_keeps_the_contract():
    d = _bench_line()
    for k in ('metric', 'value', 'unit', 'n_gpus', 'steps', 'warmup', 'ms_per_step', 'higher_is_better', 'scaling',
              'vs_baseline', 'dtype', 'data', 'config', 'roofline', 'cpu_baseline'):
        assert k in d, k
    assert d['n_gpus'] == 1 and d['scaling'] == 'weak' and d['higher_is_better'] is True
    assert 'workload' in d['config']
    # value = emulated core-shots per second of the whole job
    assert d['value'] == pytest.approx(d['config']['shots_per_gpu'] * 8 / (d['ms_per_step'] * 1e-3), rel=1e-6)
    roof = d['roofline']
    for k in ('bound', 'achieved', 'peak', 'unit', 'frac', 'traffic'):
        assert k in roof, k
    assert roof['frac'] == pytest.approx(roof['achieved'] / roof['peak'])
    cb = d['cpu_baseline']
    for k in ('value', 'unit', 'cores', 'kind', 'sample'):
        assert k in cb, k
    assert cb['kind'] in ('port', 'reference')


@pytest.mark.parametrize('leg', [None, 'dds', 'active_reset', 'rb'])
def test_committed_bench_agrees_with_its_same_box_rocprof(leg):
    """the bench's kernel time (HIP events inside real steps) and the rocprofv3
    kernel-trace average of the same launch, profiled on the same box"""
    d = _bench_line()
    x = d if leg is None else d[leg]
    roof = x['roofline']
    roof = roof.get('hbm', roof)
    assert roof['kernel_ms'] <= x['ms_per_step'] + 1e-9
    assert roof['kernel_ms_rocprof'] == pytest.approx(roof['kernel_ms'], rel=0.05)


def test_valu_view_recomputes_from_the_measured_peak():
    """the interpreter legs' VALU fractions: SQ_INSTS_VALU over the kernel time
    against the committed microbenchmark peak (profiles/r03_valu_peak_pmc.json)"""
    peak, cpi, variant = bench._valu_peak()
    assert 3e11 < peak < 1.3e12 and 2.0 <= cpi < 8.0 and 'kernel' in variant
    prof = {'SQ_INSTS_VALU': 1e8, 'duration_ns': 250000.0, 'valu_issue_pct': 50.0}
    v = bench.valu_view(prof, 0.2)
    assert v['achieved'] == pytest.approx(1e8 / 0.2e-3)
    assert v['frac'] == pytest.approx(1e8 / 0.2e-3 / peak)
    assert v['frac_rocprof'] == pytest.approx(1e8 / 0.25e-3 / peak)
    assert bench.valu_view({'duration_ns': 1.0}) is None
