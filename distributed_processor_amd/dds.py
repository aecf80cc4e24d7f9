"""DDS I/Q synthesis from emulated pulse events (hot-path row 4).

The reference stops at the pulse interface: each core drives
``pulse_iface`` {env_word, phase, freq, amp, cfg} plus ``cstrobe`` into the
external QubiC DSP (hdl/pulse_iface.sv:2-6, hdl/proc.sv:131-136), and the
assembler hands that DSP its per-element env / freq buffers
(assembler.py:472-476, asmparse.py:46-86).  This module plays the emulated
pulse timelines through a fixed-point DDS on the GPU (``dpemu_dds``,
csrc/dds.hip) so a caller gets sample-level I/Q per (shot, core, element)
channel.  The arithmetic is build-defined and pinned
bit-exactly by oracle/dds_ref.c.

Usage::

    plan = ChannelPlan(programs, cfg, shot_begin, n_shots,
                       [(shot, core, elem), ...], elem_params={0: (16, 1), 2: (4, 4)})
    iq = emu.synthesize(plan, device_outputs, n_samples)     # torch int32 [n_ch, n_samples]
"""

from __future__ import annotations

from typing import Dict, Iterable, Optional, Sequence, Tuple

import numpy as np

from . import _abi

DESC_FIELDS = ('ch_lane', 'ch_elem', 'spc', 'interp', 'env_off', 'env_len', 'freq_off', 'freq_len')


class ChannelPlan:
    """Channel descriptors and concatenated env / freq tables for one run.

    programs: the ProgramSet that was run (its ``buffers`` hold the
    assembler's env_buffers / freq_buffers of every (group, core));
    channels: (absolute shot, core, element) triples, all inside
    [shot_begin, shot_begin + n_shots); elem_params: element -> (samples per
    clock, interpolation ratio).  Tables shared by several channels are stored
    once.
    """

    def __init__(self, programs, cfg, shot_begin: int, n_shots: int,
                 channels: Iterable[Tuple[int, int, int]],
                 elem_params: Dict[int, Tuple[int, int]]):
        C_ = cfg.cores_per_shot
        spg, ng = max(int(cfg.shots_per_group), 1), max(int(cfg.n_groups), 1)
        envs, freqs = [], []
        env_at: Dict[bytes, Tuple[int, int]] = {}
        freq_at: Dict[bytes, Tuple[int, int]] = {}
        n_env = n_freq = 0

        def place(tab, store, at, n):
            key = tab.tobytes()
            if key not in at:
                at[key] = (n, len(tab))
                store.append(tab)
                n += len(tab)
            return at[key], n

        rows = []
        for shot, core, elem in channels:
            shot, core, elem = int(shot), int(core), int(elem)
            if not (shot_begin <= shot < shot_begin + n_shots) or not (0 <= core < C_):
                raise ValueError('channel ({}, {}, {}) outside the run'.format(shot, core, elem))
            if elem not in elem_params:
                raise ValueError('no (spc, interp) for element {}'.format(elem))
            g = (shot // spg) % ng
            env_l, freq_l = programs.buffers.get((g, core), ([], []))
            env = env_l[elem] if elem < len(env_l) else np.zeros(0, np.uint32)
            frq = freq_l[elem] if elem < len(freq_l) else np.zeros(0, np.uint32)
            (eo, el), n_env = place(np.ascontiguousarray(env, np.uint32), envs, env_at, n_env)
            (fo, fl), n_freq = place(np.ascontiguousarray(frq, np.uint32), freqs, freq_at, n_freq)
            spc, interp = elem_params[elem]
            lane = int(_abi.lane_index(shot - shot_begin, core, n_shots, C_, cfg.lane_order))
            rows.append((lane, elem, spc, interp, eo, el, fo, fl))
        self.desc = np.array(rows, np.uint32).reshape(-1, 8)
        self.env = np.concatenate(envs).astype(np.uint32) if n_env else np.zeros(1, np.uint32)
        self.freq = np.concatenate(freqs).astype(np.uint32) if n_freq else np.zeros(1, np.uint32)
        self.n_lanes = int(n_shots) * C_
        self.event_cap = int(cfg.event_cap)
        self._cols = {f: np.ascontiguousarray(self.desc[:, i]) for i, f in enumerate(DESC_FIELDS)}
        self._dev = None

    @property
    def n_channels(self):
        return self.desc.shape[0]

    def struct(self, n_samples: int) -> _abi.DDSChannels:
        s = _abi.DDSChannels(self.n_channels, self.n_lanes, int(n_samples), self.event_cap)
        for f in DESC_FIELDS:
            setattr(s, f, self._cols[f].ctypes.data)
        return s

    def device_tables(self, device='cuda'):
        """env / freq tables as device tensors (uploaded once per plan)."""
        if self._dev is None:
            import torch
            self._dev = (torch.from_numpy(self.env.view(np.int32)).to(device),
                         torch.from_numpy(self.freq.view(np.int32)).to(device))
        return self._dev


class SynthesisPipeline:
    """DDS synthesis of successive batches with ``depth`` batches in flight.

    One ``dpemu_dds`` call runs ``dds_index_kernel`` (the per-channel event
    index, latency-bound: ~15 us at config 5) and then ``dds_tile_kernel`` on
    one stream, so the index cannot overlap its own batch's tiles -- but it
    can overlap the previous batch's.  The pipeline holds ``depth`` library
    contexts (each owns its event index, so their calls are independent),
    one stream and one I/Q buffer per context, and sends batch k to context
    k % depth: batch k + 1's index kernel runs beside batch k's tile kernel.
    On the builder's box that measured 0.329 -> 0.317 ms per config-5 step
    (``profiles/r03_dds_pipe.json``), but the driver's round-4 record has the
    8-deep pipeline SLOWER than one context (0.3377 vs 0.3283 ms); ``bench.py``
    measures one context and depth 2 on the same line (``--dds-depth 2``) and
    reports the faster (round 5: 0.312 vs 0.327 ms, ``profiles/r05_dds_depth.json``).

    Streams beyond the process's hardware queues (``GPU_MAX_HW_QUEUES``, 4 by
    default) share them: at most 4 batches execute at once, the others wait
    on their queue behind one; depth 8 keeps every queue's
    next batch ready.

    ``synthesize`` makes its stream wait for the caller's current stream (the
    producer of ``outputs``) and returns (iq, stream): iq is valid on that
    stream, and is overwritten by the call ``depth`` batches later, so a
    consumer runs on ``stream`` (or waits for it) before then.  ``drain()``
    waits for every batch.
    """

    def __init__(self, device: int = 0, depth: int = 2, lib_path: Optional[str] = None, streams=None):
        import torch
        from .emulator import Emulator
        if depth < 1:
            raise ValueError('depth must be >= 1')
        if streams is not None and len(streams) < depth:
            raise ValueError('need {} streams, got {}'.format(depth, len(streams)))
        self.device = torch.device('cuda', device)
        self.emus = []
        try:
            for _ in range(depth):
                self.emus.append(Emulator(device, lib_path=lib_path))
        except Exception:
            self.close()
            raise
        # streams: the caller's (e.g. created once at start-up, each on its own
        # hardware queue: streams that share a queue run their kernels in turn)
        self.streams = list(streams[:depth]) if streams is not None else \
            [torch.cuda.Stream(device=self.device) for _ in range(depth)]
        self.iq = [None] * depth
        self.k = 0

    def synthesize(self, plan: ChannelPlan, outputs: dict, n_samples: int):
        import torch
        j = self.k % len(self.emus)
        shape = (plan.n_channels, int(n_samples))
        if self.iq[j] is None or tuple(self.iq[j].shape) != shape:
            self.streams[j].synchronize()           # the old buffer's last batch is done with it
            self.iq[j] = torch.empty(shape, dtype=torch.int32, device=self.device)
        s = self.streams[j]
        s.wait_stream(torch.cuda.current_stream(self.device))
        self.emus[j].synthesize(plan, outputs, n_samples, self.iq[j], s)
        self.k += 1
        return self.iq[j], s

    def drain(self):
        for s in self.streams:
            s.synchronize()

    def kernel_timing(self, on: bool):
        for e in self.emus:
            e.kernel_timing(on)

    def close(self):
        for e in self.emus:
            e.close()
        self.emus = []
        self.iq = [None] * len(self.iq) if hasattr(self, 'iq') else []


def split_iq(iq_u32: np.ndarray):
    """(I, Q) int16 arrays of dpemu_dds output words (I low half, Q high half)."""
    v = np.asarray(iq_u32).view(np.uint32)
    return (v & 0xFFFF).astype(np.uint16).view(np.int16), (v >> 16).astype(np.uint16).view(np.int16)
