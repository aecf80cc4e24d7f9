"""Host front end: run assembled distproc programs on the MI355X emulator.

Drop-in for the reference simulation path: where the reference loads one
``cmd_buf`` into a Verilator ``toplevel_sim`` and clocks it from cocotb
(cocotb/proc/test_proc.py:29-38, sim_modules/toplevel_sim.sv:13-33), here the
output of ``GlobalAssembler.get_assembled_program()`` (assembler.py:623-641)
-- ``{core_ind: {'cmd_buf': bytes, 'env_buffers': [...], 'freq_buffers': [...]}}``
-- or raw command words go to :class:`Emulator`, which runs n_shots x C
cores on the GPU through libdpemu.so and returns pulse events, register
traces, measurements and outcome histograms.
"""

from __future__ import annotations

import ctypes as C
import math
from typing import Dict, Iterable, List, Optional, Sequence, Union

import numpy as np

from . import _abi, isa
from ._native import DpemuError, check, load_library

ProgramLike = Union[bytes, Sequence[int], np.ndarray]


def _to_u32(prog: ProgramLike) -> np.ndarray:
    if isinstance(prog, (bytes, bytearray)):
        return isa.cmd_buf_to_u32(bytes(prog))
    if isinstance(prog, np.ndarray) and prog.dtype == np.uint32:
        return np.ascontiguousarray(prog.reshape(-1, 4))
    return isa.words_to_u32([int(w) for w in prog])


def _next_pow2(n: int) -> int:
    c = 1
    while c < n:
        c <<= 1
    return c


def _shot_programs(shot):
    """one shot's programs: assembler dict {core: {'cmd_buf': ..., 'env_buffers':
    [...], 'freq_buffers': [...]}}, dict {core: words}, or a list (index = core).
    Returns ({core: (n, 4) u32}, {core: (env_buffers, freq_buffers)})."""
    progs, bufs = {}, {}
    items = shot.items() if isinstance(shot, dict) else enumerate(shot)
    for k, v in items:
        if isinstance(v, dict):
            bufs[int(k)] = ([np.frombuffer(bytes(b), '<u4').astype(np.uint32) for b in v.get('env_buffers', [])],
                            [np.frombuffer(bytes(b), '<u4').astype(np.uint32) for b in v.get('freq_buffers', [])])
            v = v['cmd_buf']
        progs[int(k)] = _to_u32(v)
    return progs, bufs


class ProgramSet:
    """cmd_mem images for every (group, core), packed for the device.

    groups: list of shots' programs (see ``_shot_programs``); group g runs for
    shots with (shot // shots_per_group) % n_groups == g.  Identical programs
    are stored once.
    """

    def __init__(self, groups: Sequence, cores_per_shot: Optional[int] = None):
        if isinstance(groups, dict):
            groups = [groups]
        parsed = [_shot_programs(g) for g in groups]
        per_group = [p for p, _ in parsed]
        # env / freq buffers of (group, core), when the programs came from an assembler
        self.buffers = {(g, c): b for g, (_, bs) in enumerate(parsed) for c, b in bs.items()}
        if not per_group:
            raise ValueError('no programs')
        ncore = max((max(g) + 1 if g else 1) for g in per_group)
        C_ = cores_per_shot or _next_pow2(ncore)
        if C_ < ncore or C_ & (C_ - 1) or C_ > _abi.MAX_CORES:
            raise ValueError('cores_per_shot must be a power of two >= {}'.format(ncore))
        uniq: Dict[bytes, int] = {}
        blobs: List[np.ndarray] = []
        table = np.zeros(len(per_group) * C_, np.uint32)
        empty = np.zeros((0, 4), np.uint32)
        for g, progs in enumerate(per_group):
            for c in range(C_):
                p = progs.get(c, empty)
                key = p.tobytes()
                if key not in uniq:
                    uniq[key] = len(blobs)
                    blobs.append(p)
                table[g * C_ + c] = uniq[key]
        self.cores_per_shot = C_
        self.n_groups = len(per_group)
        self.n_instr = np.array([len(b) for b in blobs], np.uint32)
        self.offsets = np.concatenate([[0], np.cumsum(self.n_instr)[:-1]]).astype(np.uint32)
        self.words = (np.concatenate(blobs) if sum(self.n_instr) else np.zeros((1, 4), np.uint32)).astype(np.uint32)
        self.words = np.ascontiguousarray(self.words)
        self.table = table

    @classmethod
    def from_arrays(cls, words, offsets, n_instr, table, n_groups, cores_per_shot, buffers=None):
        """A ProgramSet from packed arrays (the dpemu_load_programs layout):
        words (n, 4) u32, program p = words[offsets[p]:offsets[p] + n_instr[p]],
        table[g * C + c] = program of core c in group g.  For program tables
        too large to pass through assembler dicts (config 4: 2 * 10^5
        programs, workloads.config4_rb_set)."""
        self = cls.__new__(cls)
        C_ = int(cores_per_shot)
        if C_ < 1 or C_ & (C_ - 1) or C_ > _abi.MAX_CORES:
            raise ValueError('cores_per_shot must be a power of two in [1, 64]')
        self.words = np.ascontiguousarray(np.asarray(words, np.uint32).reshape(-1, 4))
        self.offsets = np.ascontiguousarray(offsets, np.uint32)
        self.n_instr = np.ascontiguousarray(n_instr, np.uint32)
        self.table = np.ascontiguousarray(table, np.uint32).reshape(-1)
        if len(self.offsets) != len(self.n_instr) or len(self.table) != int(n_groups) * C_:
            raise ValueError('offsets / n_instr / table sizes disagree')
        if len(self.n_instr) and (self.offsets.astype(np.uint64) + self.n_instr).max() > len(self.words):
            raise ValueError('a program runs past the end of words')
        if len(self.table) and self.table.max() >= len(self.n_instr):
            raise ValueError('table names a program that does not exist')
        self.cores_per_shot = C_
        self.n_groups = int(n_groups)
        self.buffers = buffers if buffers is not None else {}
        return self

    def program(self, group: int, core: int) -> np.ndarray:
        """(n, 4) u32 machine code of core ``core`` in group ``group``"""
        p = int(self.table[group * self.cores_per_shot + core])
        o = int(self.offsets[p])
        return self.words[o:o + int(self.n_instr[p])]

    @property
    def n_programs(self):
        return len(self.n_instr)

    def readout_freqs(self, drv_elem: int, lo_elem: int):
        """The DEMOD readout model's frequency tables (dpemu_load_readout_freqs):
        per program, word 0 of every entry of the readout drive element's and
        the LO element's freq_buffer (f / f_clk * 2^32, asmparse.py:64-86), from
        the assembler buffers of a (group, core) that runs it.  Returns (words,
        drv_off, drv_len, lo_off, lo_len); a program without buffers gets empty
        tables (its frequency words read 0)."""
        owner = {}
        for i, pr in enumerate(self.table):
            owner.setdefault(int(pr), (i // self.cores_per_shot, i % self.cores_per_shot))
        words, cache = [], {}
        off = np.zeros((2, self.n_programs), np.uint32)
        ln = np.zeros((2, self.n_programs), np.uint32)
        n = 0
        for pr in range(self.n_programs):
            b = self.buffers.get(owner[pr]) if pr in owner else None
            for k, e in enumerate((drv_elem, lo_elem)):
                f = b[1][e] if b is not None and e < len(b[1]) else np.zeros(0, np.uint32)
                key = (id(f), k) if len(f) else None
                if key is not None and key in cache:
                    off[k, pr], ln[k, pr] = cache[key]
                    continue
                fw = np.asarray(f, np.uint32)[0::16]
                off[k, pr], ln[k, pr] = n, len(fw)
                if key is not None:
                    cache[key] = (n, len(fw))
                words.append(fw)
                n += len(fw)
        w = np.concatenate(words).astype(np.uint32) if n else np.zeros(0, np.uint32)
        return w, off[0], ln[0], off[1], ln[1]


class EmulationResult:
    """Host copies of a run's outputs (layouts as in include/dpemu.h)."""

    def __init__(self, cfg, n_shots, shot_begin, arrays):
        self.cfg = cfg
        self.n_shots = n_shots
        self.shot_begin = shot_begin
        self.arrays = arrays
        self.summary = _abi.unpack_summary(arrays['summary'])

    @property
    def n_lanes(self):
        return self.n_shots * self.cfg.cores_per_shot

    def lane(self, shot, core):
        """output lane of (absolute shot, core) in the run's lane order (include/dpemu.h)"""
        return int(_abi.lane_index(shot - self.shot_begin, core, self.n_shots, self.cfg.cores_per_shot,
                                   self.cfg.lane_order))

    def events(self, shot, core) -> np.ndarray:
        """structured events of one lane: t, env_word, cfg, kind, phase, freq, amp"""
        L = self.lane(shot, core)
        n = min(int(self.summary['n_events'][L]), self.cfg.event_cap)
        return decode_events(self.arrays['events'][:n, L])

    def status_counts(self):
        st, n = np.unique(self.summary['status'], return_counts=True)
        return {_abi.STATUS_NAMES.get(int(s), str(s)): int(c) for s, c in zip(st, n)}

    @property
    def histogram(self):
        return self.arrays.get('hist')


def decode_events(ev) -> np.ndarray:
    """structured view of event records (..., 4) u32: t, env_word, cfg, kind,
    phase, freq, amp (the pulse_iface fields, hdl/pulse_iface.sv:2-6)"""
    ev = np.asarray(ev).view(np.uint32)
    out = np.zeros(ev.shape[:-1], dtype=[('t', 'u4'), ('env_word', 'u4'), ('cfg', 'u1'), ('kind', 'u1'),
                                         ('phase', 'u4'), ('freq', 'u2'), ('amp', 'u2')])
    out['t'] = ev[..., 0]
    out['env_word'] = ev[..., 1] & 0xFFFFFF
    out['cfg'] = (ev[..., 1] >> 24) & 0xF
    out['kind'] = ev[..., 1] >> 28
    out['phase'] = ev[..., 2] & 0x1FFFF
    out['freq'] = ev[..., 2] >> 17
    out['amp'] = ev[..., 3] & 0xFFFF
    return out


class Emulator:
    """One context per GPU (one process per device)."""

    def __init__(self, device: int = 0, lib_path: Optional[str] = None):
        self._L = load_library(lib_path) if lib_path else load_library()
        h = C.c_void_p()
        rc = self._L.dpemu_create(int(device), C.byref(h))
        if rc != 0:
            raise DpemuError('dpemu_create(device={}) failed ({}): no usable HIP device'.format(device, rc))
        self._h = h
        self.device = device
        self.lib_path = lib_path          # None: the in-tree build
        self.programs: Optional[ProgramSet] = None
        self._ro_key = None               # (drv_elem, lo_elem) of the loaded DEMOD tables

    def close(self):
        if getattr(self, '_h', None):
            self._L.dpemu_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ---- measurement (dpemu_set_kernel_timing / dpemu_kernel_times) ----
    def kernel_timing(self, enable: bool = True):
        """record a HIP event pair around every main-kernel launch (interpreter, DDS)"""
        check(self._h, self._L.dpemu_set_kernel_timing(self._h, int(bool(enable))), 'dpemu_set_kernel_timing',
              self._L)

    def kernel_times(self, max_n: int = 4096):
        """elapsed ms of the launches recorded since the last call (waits for them)"""
        buf = np.zeros(max_n, np.float32)
        n = C.c_int(0)
        check(self._h, self._L.dpemu_kernel_times(self._h, buf.ctypes.data, int(max_n), C.byref(n)),
              'dpemu_kernel_times', self._L)
        return [float(x) for x in buf[:n.value]]

    def last_kernel(self) -> str:
        """the interpreter variant the last run launched"""
        return self._L.dpemu_last_kernel(self._h).decode()

    # -------------------------------------------------------------- programs
    def load(self, programs, cores_per_shot: Optional[int] = None) -> ProgramSet:
        ps = programs if isinstance(programs, ProgramSet) else ProgramSet(programs, cores_per_shot)
        rc = self._L.dpemu_load_programs(self._h, ps.words.ctypes.data, int(ps.words.shape[0]),
                                         ps.offsets.ctypes.data,
                                         ps.n_instr.ctypes.data, ps.n_programs, ps.table.ctypes.data,
                                         ps.n_groups, ps.cores_per_shot)
        check(self._h, rc, 'dpemu_load_programs', self._L)
        self.programs = ps
        self._ro_key = None                                 # load_programs clears the DEMOD tables
        return ps

    def load_readout_freqs(self, drv_elem: int, lo_elem: int, tables=None):
        """dpemu_load_readout_freqs: the DEMOD model's per-program frequency
        words -- ``tables`` = (words, drv_off, drv_len, lo_off, lo_len), default
        ProgramSet.readout_freqs(drv_elem, lo_elem) of the loaded programs"""
        if self.programs is None:
            raise DpemuError('load() programs first')
        t = tables if tables is not None else self.programs.readout_freqs(drv_elem, lo_elem)
        w = np.ascontiguousarray(t[0], np.uint32)
        arrs = [np.ascontiguousarray(a, np.uint32) for a in t[1:5]]
        if any(len(a) != self.programs.n_programs for a in arrs):
            raise DpemuError('readout tables need one entry per loaded program')
        rc = self._L.dpemu_load_readout_freqs(self._h, w.ctypes.data if len(w) else None, len(w),
                                              *[a.ctypes.data for a in arrs])
        check(self._h, rc, 'dpemu_load_readout_freqs', self._L)
        self._ro_key = (int(drv_elem), int(lo_elem)) if tables is None else ('caller', id(tables))

    def _demod_tables(self, cfg):
        """a DEMOD run reads the loaded programs' own frequency tables unless the
        caller loaded others"""
        if cfg.meas_model == _abi.MEAS_DEMOD and (self._ro_key is None or (
                self._ro_key[0] != 'caller' and self._ro_key != (cfg.ro_drv_elem, cfg.meas_elem))):
            self.load_readout_freqs(cfg.ro_drv_elem, cfg.meas_elem)

    def config(self, **kw) -> _abi.Config:
        if self.programs is None:
            raise DpemuError('load() programs first')
        kw.setdefault('n_groups', self.programs.n_groups)
        return _abi.make_config(self.programs.cores_per_shot, **kw)

    # -------------------------------------------------------------- running
    def run(self, n_shots: int, shot_begin: int = 0, cfg: Optional[_abi.Config] = None,
            outputs: Iterable[str] = ('summary', 'events', 'meas', 'hist'),
            **cfg_kw) -> EmulationResult:
        """Emulate shots [shot_begin, shot_begin + n_shots); results copied to host."""
        cfg = cfg or self.config(**cfg_kw)
        self._demod_tables(cfg)
        want = set(outputs) | {'summary'}
        arrays = _abi.alloc_host_outputs(cfg, n_shots, want)
        o = _abi.outputs_struct(arrays)
        rc = self._L.dpemu_run_host(self._h, C.addressof(cfg), int(shot_begin), int(n_shots), C.addressof(o))
        check(self._h, rc, 'dpemu_run_host', self._L)
        return EmulationResult(cfg, n_shots, shot_begin, arrays)

    def run_device(self, cfg: _abi.Config, n_shots: int, shot_begin: int, outputs: dict,
                   stream=None):
        """Asynchronous run into caller-owned device buffers: torch tensors
        {name: tensor} shaped as alloc_device_outputs makes them (checked: the
        C ABI takes bare pointers); stream: torch.cuda.Stream / raw handle / None."""
        unknown = set(outputs) - set(_abi.OUTPUT_NAMES)
        if unknown:
            raise DpemuError('unknown outputs {}'.format(sorted(unknown)))
        want = device_output_specs(cfg, n_shots)
        o = _abi.Outputs()
        for name, _ in _abi.Outputs._fields_:
            t = outputs.get(name)
            if t is not None:
                _check_tensor(name, t, want[name], self.device)
            setattr(o, name, None if t is None else t.data_ptr())
        self._demod_tables(cfg)
        s = getattr(stream, 'cuda_stream', stream)
        rc = self._L.dpemu_run(self._h, C.addressof(cfg), int(shot_begin), int(n_shots), C.addressof(o),
                               C.c_void_p(s) if s else None)
        check(self._h, rc, 'dpemu_run', self._L)

    def synthesize(self, plan, outputs: dict, n_samples: int, iq=None, stream=None):
        """DDS I/Q of every channel of ``plan`` (dds.ChannelPlan) from a device
        run's outputs (summary / ev_main / ev_amp tensors of run_device).
        Returns (or fills) an int32 device tensor [n_channels, n_samples]
        whose words hold I in the low and Q in the high 16 bits."""
        import torch
        for k in ('summary', 'events'):
            if k not in outputs:
                raise DpemuError('synthesize needs the run\'s {} output'.format(k))
        if tuple(outputs['events'].shape) != (plan.event_cap, plan.n_lanes, 4) or \
                tuple(outputs['summary'].shape) != (plan.n_lanes, 8):
            raise DpemuError('event / summary arrays do not match the plan (event_cap, n_lanes)')
        for k in ('summary', 'events'):
            if not outputs[k].is_contiguous() or outputs[k].device.type != 'cuda':
                raise DpemuError('{} must be a contiguous device tensor'.format(k))
        dev = outputs['summary'].device
        if iq is None:
            iq = torch.empty((plan.n_channels, int(n_samples)), dtype=torch.int32, device=dev)
        elif tuple(iq.shape) != (plan.n_channels, int(n_samples)) or iq.dtype != torch.int32:
            raise DpemuError('iq must be int32 [n_channels, n_samples]')
        env, freq = plan.device_tables(dev)
        ch = plan.struct(n_samples)
        s = getattr(stream, 'cuda_stream', stream)
        rc = self._L.dpemu_dds(self._h, C.addressof(ch), outputs['summary'].data_ptr(),
                               outputs['events'].data_ptr(), env.data_ptr(), freq.data_ptr(), iq.data_ptr(),
                               C.c_void_p(s) if s else None)
        check(self._h, rc, 'dpemu_dds', self._L)
        return iq


class RunPipeline:
    """Successive device runs with ``depth`` batches in flight.

    One context runs its calls in call order (dpemu.h), so batch k + 1's
    launch cannot start before batch k's kernel has drained.  A launch whose
    waves run programs of different lengths (config 4: each wave holds ~7
    RB sequences) has a long tail in which most of the GPU idles; the
    pipeline holds ``depth`` contexts with the same programs loaded, one
    stream and one output set each, and sends batch k to context k % depth,
    so batch k + 1's waves fill the CUs batch k's tail leaves idle (config 4:
    3.65 -> 2.86 ms per batch at depth 2, ``profiles/r03_pipe_probe.json``).

    ``streams``: the caller's streams (default: new ones from torch's pool).
    Streams beyond the process's hardware queues (GPU_MAX_HW_QUEUES, 4 by
    default) share queues, and kernels on one queue run in turn: a pipeline
    whose streams were created after many others measured no overlap at all
    in bench.py (3.60 ms per batch), the same on the first streams of the
    process 2.79 -- so the bench makes its pipeline streams first.

    ``launch(cfg, n_shots, shot_begin, hist=None)`` makes the slot's stream
    wait for the caller's current stream, runs the batch there (into
    ``hist`` instead of the slot's own histogram when given) and returns
    (outputs, stream); the outputs are valid on that stream and are
    overwritten by the launch ``depth`` batches later.  ``drain()`` waits
    for every batch.  Memory: ``depth`` output sets and program images.
    """

    def __init__(self, programs, cfg: _abi.Config, n_shots: int, want=('summary', 'events', 'meas', 'hist'),
                 depth: int = 2, device: int = 0, first: Optional['Emulator'] = None, streams=None,
                 lib_path: Optional[str] = None):
        import torch
        if depth < 1:
            raise ValueError('depth must be >= 1')
        if streams is not None and len(streams) < depth:
            raise ValueError('need {} streams, got {}'.format(depth, len(streams)))
        self.emus, self._own = [], []
        # every context on ONE library: the caller's, else first's (an A/B
        # build passed as first=Emulator(0, lib_path=...) stays alone)
        if lib_path is None and first is not None:
            lib_path = first.lib_path
        try:
            for j in range(depth):
                if j == 0 and first is not None:
                    e = first                                  # the caller's context, programs loaded
                else:
                    e = Emulator(device, lib_path=lib_path)
                    self._own.append(e)
                    e.load(programs)
                self.emus.append(e)
        except Exception:
            self.close()
            raise
        self.device = torch.device('cuda', device)
        # streams: the caller's (e.g. created once at start-up, each on its own
        # hardware queue: streams that share a queue run their kernels in turn)
        self.streams = list(streams[:depth]) if streams is not None else \
            [torch.cuda.Stream(device=self.device) for _ in range(depth)]
        self.outputs = [alloc_device_outputs(cfg, n_shots, want=want, device=self.device) for _ in range(depth)]
        self.k = 0

    def launch(self, cfg: _abi.Config, n_shots: int, shot_begin: int, hist=None):
        import torch
        j = self.k % len(self.emus)
        s = self.streams[j]
        s.wait_stream(torch.cuda.current_stream(self.device))
        out = self.outputs[j]
        if hist is not None:
            out = dict(out, hist=hist)
        self.emus[j].run_device(cfg, n_shots, shot_begin, out, s)
        self.k += 1
        return out, s

    def drain(self):
        for s in self.streams:
            s.synchronize()

    def close(self):
        for e in self._own:
            e.close()
        self._own, self.emus = [], []


def device_output_specs(cfg: _abi.Config, n_shots: int):
    """{name: (shape, torch dtype)} of the dpemu_outputs arrays of a run"""
    import torch
    n_lanes = int(n_shots) * cfg.cores_per_shot
    return {'summary': ((n_lanes, 8), torch.int32), 'events': ((cfg.event_cap, n_lanes, 4), torch.int32),
            'trace': ((cfg.trace_cap, n_lanes, 4), torch.int32),
            'meas': ((cfg.meas_cap, n_lanes, 2), torch.int32), 'regs': ((16, n_lanes), torch.int32),
            'hist': ((cfg.n_groups, 1 << cfg.cores_per_shot), torch.int64),
            'hist_next': ((cfg.n_groups, 1 << cfg.cores_per_shot), torch.int64),   # zeroed by the run
            'acc': ((cfg.meas_cap, n_lanes, 2), torch.int32)}                    # DEMOD runs only


def _check_tensor(name, t, spec, device):
    """a caller tensor must match what the kernel writes: size, dtype,
    contiguity and device (the C ABI has no size arguments)"""
    import torch
    shape, dtype = spec
    if not isinstance(t, torch.Tensor):
        raise DpemuError('{}: expected a torch tensor'.format(name))
    if name in ('hist', 'hist_next') and len(shape) == 2 and shape[1] > 4096:
        raise DpemuError('{} needs cores_per_shot <= 12'.format(name))
    # (cheap attribute calls only: this runs for every output of every launch,
    # and a bench step of config 1 is 27 us of GPU time)
    if not t.is_cuda or t.get_device() != device:
        raise DpemuError('{}: tensor on {} but the emulator runs on cuda:{}'.format(name, t.device, device))
    if t.element_size() != dtype.itemsize or t.is_floating_point():
        raise DpemuError('{}: dtype {} (want {})'.format(name, t.dtype, dtype))
    if not t.is_contiguous():
        raise DpemuError('{}: tensor must be contiguous'.format(name))
    if t.numel() != math.prod(shape):
        raise DpemuError('{}: {} elements, the run writes {} ({})'.format(name, t.numel(), int(np.prod(shape)),
                                                                        tuple(shape)))


def alloc_device_outputs(cfg: _abi.Config, n_shots: int, want=('summary', 'events', 'meas', 'hist'),
                         device='cuda'):
    """torch device tensors laid out as dpemu_outputs."""
    import torch
    shapes = device_output_specs(cfg, n_shots)
    out = {}
    for k in want:
        shp, dt = shapes[k]
        if k in ('hist', 'hist_next'):
            if cfg.cores_per_shot > 12:
                continue
            out[k] = torch.zeros(shp, dtype=dt, device=device)
        elif 0 not in shp:
            out[k] = torch.empty(shp, dtype=dt, device=device)
    return out
