"""ctypes mirror of include/dpemu.h (structs, constants, output layout)."""

import ctypes as C

import numpy as np

ABI_VERSION = 7
MAX_CORES = 64
MEAS_LOOKUP = 16     # measurements per core visible to fproc reads

ST_DONE, ST_MAX_CYCLES, ST_HUNG_OPCODE, ST_DEADLOCK = 1, 2, 3, 4
F_LATE, F_EVENT_OVF, F_TRACE_OVF, F_MEAS_OVF, F_DOUBLE_STROBE, F_GUARD = 0x01, 0x02, 0x04, 0x08, 0x10, 0x20
FPROC_MEAS, FPROC_LUT = 0, 1
MEAS_STATE, MEAS_READOUT = 0, 1
LANES_CORE_MAJOR, LANES_SHOT_MAJOR = 0, 1
EV_STROBE, EV_PULSE_RESET = 0, 1
TRACE_QCLK_LOAD, TRACE_QCLK_RST = 16, 17
MAX_CYCLES_LIMIT = 2 ** 31 - 64
MAX_EVENT_CAP = 1 << 20
X_PROG_LDS = 0x1
X_HIST_DIRECT = 0x4
X_HIST_REPL = 0x8
X_PROG_MAJOR = 0x10
X_GENERAL = 0x20
X_MACRO_DIRECT = 0x40

STATUS_NAMES = {0: 'running', ST_DONE: 'done', ST_MAX_CYCLES: 'max_cycles',
                ST_HUNG_OPCODE: 'hung_opcode', ST_DEADLOCK: 'deadlock'}


class Config(C.Structure):
    _fields_ = [('cores_per_shot', C.c_uint32), ('n_groups', C.c_uint32),
                ('shots_per_group', C.c_uint32), ('max_cycles', C.c_uint32),
                ('event_cap', C.c_uint32), ('trace_cap', C.c_uint32), ('meas_cap', C.c_uint32),
                ('fproc_mode', C.c_uint32), ('meas_elem', C.c_uint32), ('meas_latency', C.c_uint32),
                ('sync_latency', C.c_uint32), ('exec_flags', C.c_uint32),
                ('sync_mask', C.c_uint64), ('seed', C.c_uint64),
                ('lut_mask', C.c_uint32), ('meas_model', C.c_uint32),
                ('p1_threshold', C.c_uint32 * MAX_CORES), ('lut_table', C.c_uint64 * 256),
                ('ro_sep', C.c_int32), ('ro_sigma', C.c_uint32), ('ro_thr', C.c_int32),
                ('ro_win', C.c_uint32), ('hist_assign', C.c_uint32), ('lane_order', C.c_uint32)]


class Outputs(C.Structure):
    _fields_ = [('summary', C.c_void_p), ('events', C.c_void_p),
                ('trace', C.c_void_p), ('meas', C.c_void_p), ('regs', C.c_void_p),
                ('hist', C.c_void_p), ('hist_next', C.c_void_p)]


class DDSChannels(C.Structure):
    _fields_ = [('n_channels', C.c_uint32), ('n_lanes', C.c_uint32), ('n_samples', C.c_uint32),
                ('event_cap', C.c_uint32)] + [(n, C.c_void_p) for n in (
                    'ch_lane', 'ch_elem', 'spc', 'interp', 'env_off', 'env_len', 'freq_off', 'freq_len')]


DEFAULT_LUT_TABLE = (0b00000, 0b00100, 0b10000, 0b01000)   # meas_lut.sv:17-20


def make_config(cores_per_shot, n_groups=1, shots_per_group=1, max_cycles=1 << 20,
                event_cap=64, trace_cap=0, meas_cap=8, fproc_mode=FPROC_MEAS, meas_elem=2,
                meas_latency=64, sync_latency=1, sync_mask=0, seed=0x5EED, p1=0.5,
                lut_mask=0b00011, lut_table=DEFAULT_LUT_TABLE, exec_flags=0, readout=None,
                hist_assign=False, lane_order=LANES_CORE_MAJOR):
    """Validated Config.  p1: float or per-core list of P(state = 1).
    readout: None (outcome = prepared state) or dict(sep=, sigma=, thr=) for the
    readout model of include/dpemu.h (sigma a float noise scale, stored Q16).
    hist_assign: a run writes its outcome histogram instead of adding to it.
    lane_order: LANES_CORE_MAJOR (lane = core * n_shots + shot) or
    LANES_SHOT_MAJOR (lane = shot * C + core)."""
    C_ = int(cores_per_shot)
    if C_ < 1 or C_ > MAX_CORES or (C_ & (C_ - 1)):
        raise ValueError('cores_per_shot must be a power of two in [1, 64]')
    if not (0 < max_cycles <= MAX_CYCLES_LIMIT):
        raise ValueError('max_cycles must be in (0, 2^31 - 64]')
    if meas_latency < 1 or sync_latency < 1:
        raise ValueError('meas_latency and sync_latency must be >= 1')
    if lut_mask == 0:
        raise ValueError('lut_mask must be nonzero')
    if meas_cap > 32:
        raise ValueError('meas_cap must be <= 32')
    if not (0 <= event_cap <= MAX_EVENT_CAP and 0 <= trace_cap <= MAX_EVENT_CAP):
        raise ValueError('event_cap and trace_cap must be <= 2^20')
    cfg = Config()
    cfg.cores_per_shot = C_
    cfg.n_groups = int(n_groups)
    cfg.shots_per_group = int(shots_per_group)
    cfg.max_cycles = int(max_cycles)
    cfg.event_cap = int(event_cap)
    cfg.trace_cap = int(trace_cap)
    cfg.meas_cap = int(meas_cap)
    cfg.fproc_mode = int(fproc_mode)
    cfg.meas_elem = int(meas_elem)
    cfg.meas_latency = int(meas_latency)
    cfg.sync_latency = int(sync_latency)
    cfg.sync_mask = int(sync_mask)
    cfg.seed = int(seed) & (2 ** 64 - 1)
    cfg.lut_mask = int(lut_mask)
    cfg.exec_flags = int(exec_flags)
    cfg.hist_assign = 1 if hist_assign else 0
    if lane_order not in (LANES_CORE_MAJOR, LANES_SHOT_MAJOR):
        raise ValueError('lane_order must be LANES_CORE_MAJOR or LANES_SHOT_MAJOR')
    cfg.lane_order = int(lane_order)
    ps = list(p1) if isinstance(p1, (list, tuple, np.ndarray)) else [p1] * C_
    for c, p in enumerate(ps):
        cfg.p1_threshold[c] = prob_to_threshold(p)
    for i, v in enumerate(lut_table):
        cfg.lut_table[i] = int(v)
    if readout is not None:
        sep, thr = int(readout.get('sep', 0)), int(readout.get('thr', 0))
        sigma = int(round(float(readout.get('sigma', 0.0)) * 65536))
        if not (-2 ** 31 <= sep < 2 ** 31 and -2 ** 31 <= thr < 2 ** 31 and 0 <= sigma < 2 ** 32):
            raise ValueError('readout sep / thr must fit int32 and sigma * 2^16 uint32')
        cfg.meas_model = MEAS_READOUT
        cfg.ro_sep, cfg.ro_sigma, cfg.ro_thr = sep, sigma, thr
        win = int(readout.get('win', 0))
        if not 0 <= win < 2 ** 12:
            raise ValueError('readout win must fit the 12-bit envelope-length field')
        cfg.ro_win = win
    return cfg


def prob_to_threshold(p):
    p = float(p)
    if p >= 1.0:
        return 0xFFFFFFFF
    if p <= 0.0:
        return 0
    return min(int(round(p * 2 ** 32)), 0xFFFFFFFE)


OUTPUT_NAMES = ('summary', 'events', 'trace', 'meas', 'regs', 'hist', 'hist_next')


def lane_index(shot_local, core, n_shots, cores_per_shot=None, lane_order=LANES_CORE_MAJOR):
    """output lane of (shot - shot_begin, core) in a run of n_shots shots
    (include/dpemu.h): core-major L = core * n_shots + shot_local, or
    shot-major L = shot_local * C + core"""
    if lane_order == LANES_SHOT_MAJOR:
        return np.asarray(shot_local) * int(cores_per_shot) + np.asarray(core)
    return np.asarray(core) * int(n_shots) + np.asarray(shot_local)


def by_shot(arr, cores_per_shot, axis=0, lane_order=LANES_CORE_MAJOR):
    """per-lane array with the lane axis split into (core, shot), whatever
    the lane order (a view for core-major lanes)"""
    a = np.asarray(arr)
    n = a.shape[axis] // cores_per_shot
    if lane_order == LANES_SHOT_MAJOR:
        shp = a.shape[:axis] + (n, cores_per_shot) + a.shape[axis + 1:]
        return np.swapaxes(a.reshape(shp), axis, axis + 1)
    shp = a.shape[:axis] + (cores_per_shot, n) + a.shape[axis + 1:]
    return a.reshape(shp)


def alloc_host_outputs(cfg, n_shots, want=OUTPUT_NAMES):
    """numpy arrays laid out as dpemu_outputs describes (host side)."""
    n_lanes = int(n_shots) * cfg.cores_per_shot
    out = {}
    if 'summary' in want:
        out['summary'] = np.zeros((n_lanes, 8), np.uint32)
    if 'events' in want and cfg.event_cap:
        out['events'] = np.zeros((cfg.event_cap, n_lanes, 4), np.uint32)
    if 'trace' in want and cfg.trace_cap:
        out['trace'] = np.zeros((cfg.trace_cap, n_lanes, 4), np.uint32)
    if 'meas' in want and cfg.meas_cap:
        out['meas'] = np.zeros((cfg.meas_cap, n_lanes, 2), np.uint32)
    if 'regs' in want:
        out['regs'] = np.zeros((16, n_lanes), np.uint32)
    if 'hist' in want and cfg.cores_per_shot <= 12:
        out['hist'] = np.zeros((cfg.n_groups, 1 << cfg.cores_per_shot), np.uint64)
    return out


def outputs_struct(arrays):
    o = Outputs()
    for name, _ in Outputs._fields_:
        a = arrays.get(name)
        setattr(o, name, a.ctypes.data if a is not None else None)
    return o


def unpack_summary(summary):
    s = np.asarray(summary)
    return {'t_end': s[:, 0], 'ip': s[:, 1] & 0xFFFF, 'status': (s[:, 1] >> 16) & 0xFF,
            'flags': s[:, 1] >> 24, 'n_events': s[:, 2], 'n_instr': s[:, 3], 'qclk_end': s[:, 4],
            'n_meas': s[:, 5], 'meas_bits': s[:, 6], 'n_trace': s[:, 7]}
