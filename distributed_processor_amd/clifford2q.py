"""The two-qubit Clifford group for config 4's randomized benchmarking
(random Clifford sequences decomposed into X90 / Y90 /
virtual-Z / CNOT, each closed by its recovery Clifford).

Native operations, per qubit q of a (control, target) pair -- what the
machine code of ``workloads.config4_rb2q`` plays:

* ``('p', q, a)``: a pi/2 pulse about the axis at a quarter turns in the
  qubit's frame (a = 0: X90, 1: Y90, 2: X-90, 3: Y-90); logical unitary
  ``exp(-i pi/4 (cos(a pi/2) X + sin(a pi/2) Y))``.  Played as one reg_alu
  (TREG = PREG + a quarter turns) and one pulse whose phase comes from TREG.
* ``('z', q, k)``: a virtual Z, the frame register PREG += k quarter turns;
  logical unitary ``Rz(-k pi/2) = exp(+i k pi/4 Z)``.  One reg_alu.
* CNOT (control q0, target q1) = ZX90, then S-dagger on the control and
  X-90 on the target: ``CNOT ~ (Rz(-pi/2) (x) Rx(-pi/2)) exp(-i pi/4 Z (x) X)``.
  The ZX90 is a cross-resonance pulse on the control's drive at the target's
  frequency, its phase an immediate: the target's frame at that point, which
  the generator knows statically.

A pulse about logical axis a in a frame F plays the physical phase a + F
(``Rz(t) R_a Rz(-t) = R_(a + t)``), so the physical pulse sequence of a
whole RB sequence equals the logical identity up to a Z rotation per qubit:
its unitary is diagonal, and |00> returns to |00> (tests/test_rb2q.py
checks that on the generated machine code).

Single-qubit Cliffords (24): one of six pulse prefixes -- none, X90, X-90,
Y90, Y-90, X90 X90 -- that take Z to the six Pauli axes, then k quarter
turns of virtual Z.  Two-qubit Cliffords (11,520): every element is
``A_k CNOT ... A_1 CNOT A_0`` (time order A_0 first) with A_i in C1 (x) C1
and k <= 3 CNOTs; ``table()`` finds, breadth first, a decomposition of each
element with the fewest CNOTs and, among those, the fewest commands, and
checks that the group closes at 576 + 5184 + 5184 + 576 elements.
"""

from __future__ import annotations

import functools

import numpy as np

N_C1 = 24
N_C2 = 11520
C1_PRE = ((), (0,), (2,), (1,), (3,), (0, 0))      # axis quarter turns of the pi/2 pulses, in time order

_I2 = np.eye(2, dtype=np.complex128)
_X = np.array([[0, 1], [1, 0]], np.complex128)
_Y = np.array([[0, -1j], [1j, 0]], np.complex128)
_Z = np.array([[1, 0], [0, -1]], np.complex128)
_COS = (1.0, 0.0, -1.0, 0.0)
_SIN = (0.0, 1.0, 0.0, -1.0)


def pulse_u(a):
    """pi/2 rotation about the axis at a quarter turns (in the frame)"""
    a %= 4
    return (_I2 - 1j * (_COS[a] * _X + _SIN[a] * _Y)) / np.sqrt(2.0)


def vz_u(k):
    """the virtual Z of k quarter turns of the frame: Rz(-k pi/2)"""
    ph = np.exp(1j * np.pi / 4 * (k % 4))
    return np.diag([ph, np.conj(ph)])


def zx90_u(a=0):
    """exp(-i pi/4 Z (x) P_a), P_a the target axis at a quarter turns (qubit 0 = control, first factor)"""
    a %= 4
    return (np.eye(4, dtype=np.complex128) - 1j * np.kron(_Z, _COS[a] * _X + _SIN[a] * _Y)) / np.sqrt(2.0)


def c1_ops(i):
    """(pulse axes in time order, virtual-Z quarter turns after them) of single-qubit Clifford i"""
    return C1_PRE[i // 4], i % 4


def c1_u(i):
    pre, k = c1_ops(i)
    u = _I2
    for a in pre:
        u = pulse_u(a) @ u
    return vz_u(k) @ u


CNOT_U = np.kron(vz_u(1), pulse_u(2)) @ zx90_u(0)


def c1_cmds(i):
    """machine commands of single-qubit Clifford i: 2 per pulse (reg_alu + pulse), 1 for the Z"""
    pre, k = c1_ops(i)
    return 2 * len(pre) + (1 if k else 0)


# ---- canonical keys: a unitary up to global phase -> uint64.  The key reads
# U v for one fixed generic vector v: no element of a finite group other than
# the scalars has v as an eigenvector, so U v up to phase names U up to phase
# (Table checks that the 11,520 keys are distinct).
_V = np.random.default_rng(0xC11F).normal(size=(4, 2)) @ np.array([1.0, 1j])
_KEY_W = np.random.default_rng(0xC12F).integers(1, 2 ** 63, size=8, dtype=np.int64).astype(np.uint64)


def vec_keys(w):
    """w: (..., 4) = U v -> (...) uint64 keys, equal iff the U are equal up to global phase"""
    v = _phase_norm(w)
    q = np.concatenate([np.rint(v.real * 2.0 ** 14), np.rint(v.imag * 2.0 ** 14)], axis=1).astype(np.int64)
    with np.errstate(over='ignore'):
        h = (q.astype(np.uint64) * _KEY_W).sum(axis=1, dtype=np.uint64)
        h ^= h >> np.uint64(29)
    return h


def keys(u):
    """u: (..., 4, 4) unitaries -> (...) uint64 keys equal iff equal up to global phase"""
    return vec_keys(np.asarray(u).reshape(-1, 4, 4) @ _V)


class Table:
    """The 11,520 two-qubit Cliffords: element e -> decomposition, unitary, key.

    ``layers[e]``: the C1 (x) C1 pairs (i0, i1) A_0..A_k in time order, with a
    CNOT between consecutive ones; ``n_cnot[e]`` = k; ``u[e]`` its unitary;
    ``key[e]``; element 0 is the identity."""

    def __init__(self):
        c1 = np.stack([c1_u(i) for i in range(N_C1)])
        pairs = np.array([(i0, i1) for i0 in range(N_C1) for i1 in range(N_C1)], np.int64)
        a_u = np.einsum('aij,bkl->abikjl', c1, c1).reshape(N_C1 * N_C1, 4, 4)   # kron(c1[i0], c1[i1])
        a_cost = np.array([c1_cmds(i0) + c1_cmds(i1) for i0, i1 in pairs], np.int64)
        a_key = keys(a_u)
        if len(np.unique(a_key)) != N_C1 * N_C1:
            raise AssertionError('C1 x C1 is not 576 distinct elements')
        cnot_cost = 4                                   # CR + Z on the control, reg_alu + X-90 on the target
        seen = set(a_key.tolist())
        us, ks, costs, layers = [a_u], [a_key], [a_cost], [pairs[:, None, :]]
        prev = (a_u, a_key, a_cost, pairs[:, None, :])
        for level in (1, 2, 3):
            pu, _, pc, pl = prev
            m = np.matmul(CNOT_U, pu)                    # CNOT after the previous decomposition
            n = len(pu)
            mv = (m @ _V).T                               # [4, n]: (CNOT prev) v
            w = (a_u.reshape(-1, 4) @ mv).reshape(len(a_u), 4, n).transpose(0, 2, 1)
            ck = vec_keys(w)                             # candidate (a, previous) at a * n + previous
            cc = (a_cost[:, None] + pc[None, :] + cnot_cost).reshape(-1)
            cs = np.stack([np.tile(np.arange(n), len(a_u)), np.repeat(np.arange(len(a_u)), n)], axis=1)
            new = ~np.isin(ck, np.fromiter(seen, np.uint64, len(seen)))
            ck, cc, cs = ck[new], cc[new], cs[new]
            order = np.lexsort((np.arange(len(ck)), cc, ck))      # by key, then cost, then candidate order
            ck, cc, cs = ck[order], cc[order], cs[order]
            first = np.ones(len(ck), bool)
            first[1:] = ck[1:] != ck[:-1]
            ck, cc, cs = ck[first], cc[first], cs[first]
            nu = np.einsum('nij,njk->nik', a_u[cs[:, 1]], m[cs[:, 0]])
            nl = np.concatenate([pl[cs[:, 0]], pairs[cs[:, 1]][:, None, :]], axis=1)
            seen.update(ck.tolist())
            us.append(nu)
            ks.append(ck)
            costs.append(cc)
            layers.append(nl)
            prev = (nu, ck, cc, nl)
        sizes = [len(k) for k in ks]
        if sizes != [576, 5184, 5184, 576]:
            raise AssertionError(f'two-qubit Clifford classes {sizes}, expected [576, 5184, 5184, 576]')
        self.u = np.concatenate(us)
        self.key = np.concatenate(ks)
        self.cost = np.concatenate(costs)
        self.n_cnot = np.repeat(np.arange(4), sizes)
        self.layers = [l_ for lv in layers for l_ in lv]          # per element: (k + 1, 2) int64
        srt = np.argsort(self.key, kind='stable')
        self._sorted_keys = self.key[srt]
        self._sorted_idx = srt
        if len(np.unique(self.key)) != N_C2:
            raise AssertionError('duplicate two-qubit Clifford keys')

    def index(self, u):
        """element indices of unitaries u (..., 4, 4) (each must be a Clifford up
        to rounding): by key, and a nearest-neighbour search for the rare
        product whose rounding put a coordinate across a key cell boundary"""
        u = np.asarray(u).reshape(-1, 4, 4)
        k = keys(u)
        pos = np.minimum(np.searchsorted(self._sorted_keys, k), N_C2 - 1)
        idx = self._sorted_idx[pos]
        for j in np.flatnonzero(self._sorted_keys[pos] != k):
            w = _phase_norm(u[j] @ _V)
            ref = _phase_norm(self.u @ _V)
            d = np.abs(ref - w).max(axis=1)
            if d.min() > 1e-6:
                raise ValueError('not a two-qubit Clifford')
            idx[j] = int(np.argmin(d))
        return idx


def _phase_norm(w):
    w = np.asarray(w).reshape(-1, 4)
    return w * (np.conj(w[:, :1]) / np.abs(w[:, :1]))


@functools.lru_cache(maxsize=1)
def table() -> Table:
    return Table()
