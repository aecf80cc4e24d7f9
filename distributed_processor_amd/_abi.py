"""ctypes mirror of include/dpemu.h (structs, constants, output layout)."""

import ctypes as C

import numpy as np

ABI_VERSION = 8
MAX_CORES = 64
MEAS_LOOKUP = 16     # measurements per core visible to fproc reads

ST_DONE, ST_MAX_CYCLES, ST_HUNG_OPCODE, ST_DEADLOCK = 1, 2, 3, 4
F_LATE, F_EVENT_OVF, F_TRACE_OVF, F_MEAS_OVF, F_DOUBLE_STROBE, F_GUARD = 0x01, 0x02, 0x04, 0x08, 0x10, 0x20
FPROC_MEAS, FPROC_LUT = 0, 1
MEAS_STATE, MEAS_READOUT, MEAS_DEMOD = 0, 1, 2
RO_CPW_MAX = 8
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
X_STREAM_EVENTS = 0x80

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
                ('ro_win', C.c_uint32), ('hist_assign', C.c_uint32), ('lane_order', C.c_uint32),
                ('ro_drv_elem', C.c_uint32), ('ro_cpw', C.c_uint32), ('ro_delay', C.c_uint32),
                ('ro_theta', C.c_uint32 * 2), ('ro_gain', C.c_uint32 * 2), ('ro_axis', C.c_uint32 * MAX_CORES)]


class Outputs(C.Structure):
    _fields_ = [('summary', C.c_void_p), ('events', C.c_void_p),
                ('trace', C.c_void_p), ('meas', C.c_void_p), ('regs', C.c_void_p),
                ('hist', C.c_void_p), ('hist_next', C.c_void_p), ('acc', C.c_void_p)]


class DDSChannels(C.Structure):
    _fields_ = [('n_channels', C.c_uint32), ('n_lanes', C.c_uint32), ('n_samples', C.c_uint32),
                ('event_cap', C.c_uint32)] + [(n, C.c_void_p) for n in (
                    'ch_lane', 'ch_elem', 'spc', 'interp', 'env_off', 'env_len', 'freq_off', 'freq_len')]


DEFAULT_LUT_TABLE = (0b00000, 0b00100, 0b10000, 0b01000)   # meas_lut.sv:17-20


def make_config(cores_per_shot, n_groups=1, shots_per_group=1, max_cycles=1 << 20,
                event_cap=64, trace_cap=0, meas_cap=8, fproc_mode=FPROC_MEAS, meas_elem=2,
                meas_latency=64, sync_latency=1, sync_mask=0, seed=0x5EED, p1=0.5,
                lut_mask=0b00011, lut_table=DEFAULT_LUT_TABLE, exec_flags=0, readout=None,
                hist_assign=False, lane_order=LANES_CORE_MAJOR, demod=None):
    """Validated Config.  p1: float or per-core list of P(state = 1).
    readout: None (outcome = prepared state) or dict(sep=, sigma=, thr=) for the
    readout model of include/dpemu.h (sigma a float noise scale, stored Q16).
    demod: None or dict for the demodulation model (meas_model DEMOD,
    include/dpemu.h; meas_elem is the LO element): drv_elem, cpw (clocks per
    env word, default 4), delay (clocks), theta=(state-0, state-1 return
    phase, radians), gain=(state-0, state-1 amplitude, <= 1.0), axis (radians,
    one or per core: the discriminator direction), sigma (noise scale of the
    accumulated value, float; stored Q16), thr (int).
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
    if demod is not None:
        if readout is not None:
            raise ValueError('readout and demod are exclusive measurement models')
        set_demod(cfg, **demod)
    return cfg


def phase_u32(rad):
    """a phase in radians as the model's 32-bit phase (2^32 = 2 pi)"""
    return int(round(float(rad) / (2 * np.pi) * 2 ** 32)) & 0xFFFFFFFF


def axis_word(rad):
    """discriminator axis word: Q15 cos | Q15 sin << 16 (include/dpemu.h ro_axis)"""
    i = max(-32768, min(32767, int(round(np.cos(rad) * 32767))))
    q = max(-32768, min(32767, int(round(np.sin(rad) * 32767))))
    return (i & 0xFFFF) | ((q & 0xFFFF) << 16)


def set_demod(cfg, drv_elem=1, cpw=4, delay=0, theta=(0.0, np.pi), gain=(1.0, 1.0), axis=0.0, sigma=0.0, thr=0):
    """switch cfg to meas_model DEMOD (see make_config)"""
    if not 0 <= int(drv_elem) <= 3 or int(drv_elem) == cfg.meas_elem:
        raise ValueError('demod drv_elem must be an element 0..3 other than meas_elem')
    if not 1 <= int(cpw) <= RO_CPW_MAX:
        raise ValueError('demod cpw must be in [1, {}]'.format(RO_CPW_MAX))
    if not 0 <= int(delay) < 2 ** 20:
        raise ValueError('demod delay must be in [0, 2^20)')
    sig = int(round(float(sigma) * 65536))
    if not 0 <= sig < 2 ** 24:
        raise ValueError('demod sigma * 2^16 must be < 2^24')
    if not -2 ** 31 <= int(thr) < 2 ** 31:
        raise ValueError('demod thr must fit int32')
    cfg.meas_model = MEAS_DEMOD
    cfg.ro_drv_elem, cfg.ro_cpw, cfg.ro_delay = int(drv_elem), int(cpw), int(delay)
    for s_ in (0, 1):
        g = int(round(float(gain[s_]) * 65536))
        if not 0 <= g <= 65536:
            raise ValueError('demod gain must be in [0, 1]')
        cfg.ro_gain[s_] = g
        cfg.ro_theta[s_] = phase_u32(theta[s_])
    axes = list(axis) if isinstance(axis, (list, tuple, np.ndarray)) else [axis] * MAX_CORES
    for c in range(MAX_CORES):
        cfg.ro_axis[c] = axis_word(axes[c] if c < len(axes) else 0.0)
    cfg.ro_sigma, cfg.ro_thr = sig, int(thr)
    return cfg


def prob_to_threshold(p):
    p = float(p)
    if p >= 1.0:
        return 0xFFFFFFFF
    if p <= 0.0:
        return 0
    return min(int(round(p * 2 ** 32)), 0xFFFFFFFE)


OUTPUT_NAMES = ('summary', 'events', 'trace', 'meas', 'regs', 'hist', 'hist_next', 'acc')


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
    if 'acc' in want and cfg.meas_cap and cfg.meas_model == MEAS_DEMOD:
        out['acc'] = np.zeros((cfg.meas_cap, n_lanes, 2), np.int32)
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
