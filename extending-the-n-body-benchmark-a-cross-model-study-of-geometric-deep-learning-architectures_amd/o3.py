"""Construction-time O(3) irreps bookkeeping (the subset of e3nn 0.5.1 that SEGNN's
module structure depends on: irreps strings, instruction enumeration of a
FullyConnectedTensorProduct, weight-block shapes).  No arithmetic happens here:
the tensor products themselves run in the HIP kernels (csrc/segnn.hip).

Reference call sites: models/segnn/o3_building_blocks.py:43-49 (FCTP),
models/segnn/segnn.py:37-51 (Irreps algebra), models/balanced_irreps.py:51-85.
"""
from __future__ import annotations

import math
import re
from typing import List, NamedTuple, Tuple

import torch

_PARITY = {"e": 1, "o": -1}


class Irrep(NamedTuple):
    l: int
    p: int

    @classmethod
    def of(cls, s: str) -> "Irrep":
        s = s.strip()
        return cls(int(s[:-1]), _PARITY[s[-1]] if s[-1] in _PARITY else (-1) ** int(s[:-1]))

    @property
    def dim(self) -> int:
        return 2 * self.l + 1

    def couples(self, a: "Irrep", b: "Irrep") -> bool:
        """self in a (x) b."""
        return self.p == a.p * b.p and abs(a.l - b.l) <= self.l <= a.l + b.l

    def __str__(self) -> str:
        return f"{self.l}{'e' if self.p == 1 else 'o'}"


class Irreps(tuple):
    """Tuple of (mul, Irrep); str form "96x0e+96x1o"."""

    def __new__(cls, spec=()):
        if isinstance(spec, str):
            items = []
            for tok in filter(None, (t.strip() for t in spec.split("+"))):
                m = re.fullmatch(r"(?:(\d+)x)?(\d+[eoy])", tok)
                if not m:
                    raise ValueError(f"bad irreps token {tok!r}")
                items.append((int(m.group(1) or 1), Irrep.of(m.group(2))))
            spec = items
        return super().__new__(cls, tuple((int(m), Irrep(*ir)) for m, ir in spec))

    @classmethod
    def spherical_harmonics(cls, lmax: int) -> "Irreps":
        return cls([(1, Irrep(l, (-1) ** l)) for l in range(lmax + 1)])

    @property
    def dim(self) -> int:
        return sum(m * ir.dim for m, ir in self)

    @property
    def num_irreps(self) -> int:
        return sum(m for m, _ in self)

    def simplify(self) -> "Irreps":
        out: List[Tuple[int, Irrep]] = []
        for m, ir in self:
            if out and out[-1][1] == ir:
                out[-1] = (out[-1][0] + m, ir)
            elif m:
                out.append((m, ir))
        return Irreps(out)

    def sorted(self) -> "Irreps":
        return Irreps(sorted(self, key=lambda mi: (mi[1].l, mi[1].p)))

    def __add__(self, other) -> "Irreps":
        return Irreps(tuple(self) + tuple(Irreps(other)))

    def __mul__(self, n: int) -> "Irreps":
        return Irreps(tuple(self) * n)

    def __str__(self) -> str:
        return "+".join(f"{m}x{ir}" for m, ir in self)

    __repr__ = __str__


class Instruction(NamedTuple):
    i_in1: int
    i_in2: int
    i_out: int
    shape: Tuple[int, int, int]   # (mul1, mul2, mul_out), "uvw"


def fctp_instructions(in1: Irreps, in2: Irreps, out: Irreps) -> List[Instruction]:
    """e3nn FullyConnectedTensorProduct instruction order."""
    return [Instruction(a, b, c, (m1, m2, mo))
            for a, (m1, ir1) in enumerate(in1)
            for b, (m2, ir2) in enumerate(in2)
            for c, (mo, iro) in enumerate(out) if iro.couples(ir1, ir2)]


def fctp_weight_numel(in1, in2, out) -> int:
    return sum(math.prod(i.shape) for i in fctp_instructions(Irreps(in1), Irreps(in2), Irreps(out)))


class FullyConnectedTensorProduct(torch.nn.Module):
    """Parameter container with e3nn's state_dict layout (``weight`` flat in
    instruction order, ``output_mask`` buffer).  Construction consumes the global
    torch RNG like e3nn does (``torch.randn(weight_numel)``) so that seeded model
    construction follows the reference's RNG stream (unpinned)."""

    def __init__(self, irreps_in1, irreps_in2, irreps_out):
        super().__init__()
        self.irreps_in1, self.irreps_in2, self.irreps_out = Irreps(irreps_in1), Irreps(irreps_in2), Irreps(irreps_out)
        self.instructions = fctp_instructions(self.irreps_in1, self.irreps_in2, self.irreps_out)
        self.weight_numel = sum(math.prod(i.shape) for i in self.instructions)
        self.weight = torch.nn.Parameter(torch.randn(self.weight_numel))
        mask = torch.zeros(self.irreps_out.dim)
        off = 0
        for io, (m, ir) in enumerate(self.irreps_out):
            if any(i.i_out == io for i in self.instructions):
                mask[off:off + m * ir.dim] = 1
            off += m * ir.dim
        self.register_buffer("output_mask", mask)

    def weight_views(self, weight=None):
        w = self.weight if weight is None else weight
        off = 0
        for ins in self.instructions:
            n = math.prod(ins.shape)
            yield w[off:off + n].view(ins.shape)
            off += n

    def forward(self, *a):  # pragma: no cover - arithmetic lives in the fused HIP kernels
        raise NotImplementedError("tensor products run fused inside the SEGNN HIP kernels")


def weight_balanced_irreps(hidden_features: int, irreps_in2: Irreps, lmax: int) -> Irreps:
    """models/balanced_irreps.py:51-85 with sh=True: smallest n such that the
    FCTP(n(0e+1o..), attrs -> same) weight count reaches hidden_features**2.
    Mirrors the reference's RNG consumption (each probe FCTP draws its randn)."""
    def probe(in1, in2, out):
        n = fctp_weight_numel(in1, in2, out)
        torch.randn(n)                      # e3nn FCTP internal-weight init
        return n

    n = 1
    ir1 = (Irreps.spherical_harmonics(lmax) * n).sorted().simplify()
    w1 = probe(ir1, irreps_in2, ir1)
    ws = probe(Irreps(f"{hidden_features}x0e"), "1x0e", Irreps(f"{hidden_features}x0e"))
    while w1 < ws:
        n += 1
        ir1 = (Irreps.spherical_harmonics(lmax) * n).sorted().simplify()
        w1 = probe(ir1, irreps_in2, ir1)
    return ir1
