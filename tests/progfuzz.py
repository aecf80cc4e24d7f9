"""Random distproc machine-code programs for differential testing.

Programs exercise every opcode class of hdl/ctrl.v: pulse write/trigger
(immediate and register-sourced fields), idle, pulse_reset, reg_alu (all 8
ALU ops, imm/reg forms), inc_qclk (all ALU ops via raw words), jump_i,
jump_cond (forward skips and bounded backward loops), alu_fproc/jump_fproc,
sync, done, hang opcodes, and late triggers.  A running qclk estimate keeps
most triggers in the future; the estimate only ever over-shoots, which is
safe (the core simply waits longer).
"""

import random

import numpy as np

import distributed_processor_amd.isa as isa

ALU = ['id0', 'add', 'sub', 'eq', 'le', 'ge', 'id1', 'zero']


def raw(op4, in0_reg=0, alu_op=0, imm=0, rs0=0, rs1=0, rd=0, target=0, fproc_id=0, cmd_time=0):
    w = (((op4 << 4) | (in0_reg << 3) | alu_op) << 120)
    if in0_reg:
        w |= rs0 << 116
    else:
        w |= (imm & 0xFFFFFFFF) << 88
    w |= (rs1 & 15) << 84
    w |= (rd & 15) << 80
    w |= (target & 0xFFFF) << 68 if op4 in (2, 3, 5) else 0
    w |= (fproc_id & 0xFF) << 52 if op4 in (4, 5) else 0
    w |= (cmd_time & 0xFFFFFFFF) << 5 if op4 in (9, 12) else 0
    return w


class Gen:
    def __init__(self, rng, ncores, mode='meas', allow_late=False, allow_hang=False, meas_latency=20,
                 straight=False, linear=False, regs=None):
        self.regs = list(regs) if regs else list(range(16))   # register indices the ALU / pulse fields name
        self.straight = straight          # pulse / idle / pulse_reset / done only
        self.linear = linear              # plus reg_alu / inc_qclk: no jump, fproc or sync
        self.shape = None                 # fixed opcode-kind sequence (shaped_case)
        self.rng = rng
        self.ncores = ncores
        self.mode = mode
        self.allow_late = allow_late
        self.allow_hang = allow_hang
        self.meas_latency = meas_latency

    def pulse_fields(self):
        r = self.rng
        f = dict(freq_word=r.randint(0, 511), phase_word=r.randint(0, 2 ** 17 - 1),
                 amp_word=r.randint(0, 2 ** 16 - 1), env_word=r.randint(0, 2 ** 24 - 1),
                 cfg_word=r.randint(0, 15))
        for k in list(f):
            if k != 'cfg_word' and r.random() < 0.25:
                del f[k]
        if r.random() < 0.2:
            k = r.choice(['freq', 'phase', 'amp', 'env'])
            f.pop(k + '_word', None)
            f[k + '_regaddr'] = r.randint(0, 15) if len(self.regs) == 16 else r.choice(self.regs)
        if r.random() < 0.1:
            f.pop('cfg_word', None)
        return f

    def block(self, words, q, n):
        """append ~n random instructions; returns the qclk estimate at the next decode"""
        r = self.rng
        i = 0
        while i < n:
            if self.shape is not None:
                kind = self.shape[i]
            else:
                kind = r.choices(['trig', 'pw', 'idle', 'prst', 'alu', 'incq', 'jc', 'ji', 'loop', 'fproc'],
                                 [10, 3, 2, 1, 0, 0, 0, 0, 0, 0] if self.straight else
                                 [10, 3, 2, 1, 6, 2, 0, 0, 0, 0] if self.linear else
                                 [10, 3, 2, 1, 6, 2, 2, 1, 1, 2])[0]
            if kind == 'trig':
                if self.allow_late and r.random() < 0.05:
                    t = (q - r.randint(1, 4)) & 0xFFFFFFFF
                else:
                    t = (q + r.randint(0, 12)) & 0xFFFFFFFF
                words.append(isa.pulse_cmd(cmd_time=t, **self.pulse_fields()))
                q = (t + 3) & 0xFFFFFFFF
            elif kind == 'pw':
                words.append(isa.pulse_cmd(**self.pulse_fields()))
                q += 3
            elif kind == 'idle':
                t = (q + r.randint(0, 30)) & 0xFFFFFFFF
                words.append(isa.idle(t))
                q = (t + 3) & 0xFFFFFFFF
            elif kind == 'prst':
                words.append(isa.pulse_reset())
                q += 3
            elif kind == 'alu':
                op = r.randrange(8)
                # (the default register set draws exactly as before: same random streams)
                reg = (lambda: r.randint(0, 15)) if len(self.regs) == 16 else (lambda: r.choice(self.regs))
                dst = (lambda: r.randint(0, 7)) if len(self.regs) == 16 else (lambda: r.choice(self.regs))
                if r.random() < 0.5:
                    words.append(raw(1, 0, op, imm=r.choice([r.randint(-40, 40), r.getrandbits(32)]),
                                     rs1=reg(), rd=dst()))
                else:
                    words.append(raw(1, 1, op, rs0=reg(), rs1=reg(), rd=dst()))
                q += 4
            elif kind == 'incq':
                ops = [1, 1, 1, 0, 6, 7] + ([2] if self.allow_late else [])
                op = r.choice(ops)
                v = r.randint(-3, 40)
                words.append(raw(6, 0, op, imm=v))
                res = {1: v + q, 0: v, 6: q, 7: 0, 2: v - q}[op]
                q = (res + 4) & 0xFFFFFFFF
            elif kind == 'jc':
                skip = r.randint(1, 3)
                op = r.randrange(8)
                words.append(('jc', skip, op, r.randint(-3, 3), r.randint(0, 15)))
                q += 6
            elif kind == 'ji':
                words.append(('ji', r.randint(1, 2)))
                q += 4
            elif kind == 'loop':
                reg = r.randint(8, 15)
                cnt = r.randint(1, 4)
                words.append(raw(1, 0, 0, imm=cnt, rd=reg))                    # reg = cnt
                start = len(words)
                words.append(raw(1, 0, 1, imm=-1, rs1=reg, rd=reg))            # reg = -1 + reg
                body = r.randint(0, 2)
                for _ in range(body):
                    words.append(isa.pulse_cmd(**self.pulse_fields()))
                words.append(raw(3, 0, 4, imm=0, rs1=reg, target=start))       # if 0 < reg goto start
                self.loops.append((start - 1, len(words) - 1))
                q += 4 + cnt * (4 + 3 * body + 6)
            elif kind == 'fproc':
                op = r.randrange(8)
                if self.mode == 'meas':
                    fid = r.randrange(max(self.ncores, 1)) if r.random() < 0.9 else r.randint(0, 255)
                else:
                    fid = 0 if r.random() < 0.6 else r.randint(1, 3)
                in0r = r.random() < 0.3
                if r.random() < 0.5:
                    words.append(raw(4, int(in0r), op, imm=r.randint(-2, 2), rs0=r.randint(0, 15),
                                     rd=r.randint(0, 7), fproc_id=fid))
                    q += 6
                else:
                    words.append(('jf', r.randint(1, 2), op, int(in0r), r.randint(-2, 2), r.randint(0, 15), fid))
                    q += 8
                if self.mode == 'lut':
                    q += self.meas_latency + 400
            i += 1
        return q

    def program(self, n_sync, body_len):
        self.loops = []
        words = []
        q = 0
        for s in range(n_sync + 1):
            q = self.block(words, q, body_len)
            if s < n_sync:
                words.append(isa.sync(self.rng.randint(0, 255)))
                q = 1
        if self.allow_hang and self.rng.random() < 0.1:
            words.append(raw(self.rng.choice([13, 14, 15])))
        else:
            words.append(isa.done_cmd() if self.rng.random() < 0.8 else 0)
        # resolve relative jumps (targets may point past the end: reads 0 = DONE)
        def fix(t):
            for a, b in self.loops:      # never jump into a loop's interior
                if a < t <= b:
                    return b + 1
            return t
        out = []
        for idx, w in enumerate(words):
            if isinstance(w, tuple):
                if w[0] == 'jc':
                    _, skip, op, imm, rs1 = w
                    out.append(raw(3, 0, op, imm=imm, rs1=rs1, target=fix(idx + 1 + skip)))
                elif w[0] == 'ji':
                    out.append(raw(2, target=fix(idx + 1 + w[1])))
                else:
                    _, skip, op, in0r, imm, rs0, fid = w
                    out.append(raw(5, in0r, op, imm=imm, rs0=rs0, target=fix(idx + 1 + skip), fproc_id=fid))
            else:
                out.append(w)
        return out


def pack_programs(progs):
    """list of word lists -> (words (n,4) u32, offsets, n_instr)"""
    offsets, n_instr, rows = [], [], []
    off = 0
    for p in progs:
        offsets.append(off)
        n_instr.append(len(p))
        rows.append(isa.words_to_u32(p))
        off += len(p)
    words = np.concatenate(rows) if rows else np.zeros((0, 4), np.uint32)
    return words, np.array(offsets, np.uint32), np.array(n_instr, np.uint32)


def random_case(seed, ncores=None, mode=None, allow_late=True, allow_hang=True, n_groups=None, straight=False,
                linear=False, regs=None):
    rng = random.Random(seed)
    ncores = ncores or rng.choice([1, 2, 4])
    mode = mode or rng.choice(['meas', 'meas', 'lut'])
    n_groups = n_groups or rng.choice([1, 2])
    n_sync = 0 if (straight or linear) else (rng.choice([0, 0, 1, 2]) if ncores > 1 else rng.choice([0, 1]))
    g = Gen(rng, ncores, mode, allow_late, allow_hang, straight=straight, linear=linear, regs=regs)
    body = rng.randint(3, 14)
    progs = [g.program(n_sync, body) for _ in range(n_groups * ncores)]
    table = np.arange(n_groups * ncores, dtype=np.uint32)
    return dict(ncores=ncores, mode=mode, n_groups=n_groups, progs=progs, table=table, rng=rng)


def shaped_case(seed, ncores, n_groups=4, allow_late=True, allow_hang=True, linear=False):
    """branch-free programs that share one opcode sequence with random
    parameters (cmd_times, pulse fields, ALU operands, late triggers) per
    (group, core), and a random final command: the batched-experiment shape
    whose lanes agree on the opcode at every step until their endings differ.
    linear: reg_alu / inc_qclk commands in the sequence too"""
    rng = random.Random(seed)
    g = Gen(rng, ncores, 'meas', allow_late, allow_hang, straight=not linear, linear=linear)
    kinds, weights = (['trig', 'pw', 'idle', 'prst', 'alu', 'incq'], [10, 3, 2, 1, 6, 2]) if linear else \
        (['trig', 'pw', 'idle', 'prst'], [10, 3, 2, 1])
    g.shape = rng.choices(kinds, weights, k=rng.randint(3, 16))
    progs = [g.program(0, len(g.shape)) for _ in range(n_groups * ncores)]
    table = np.arange(n_groups * ncores, dtype=np.uint32)
    return dict(ncores=ncores, mode='meas', n_groups=n_groups, progs=progs, table=table, rng=rng)
