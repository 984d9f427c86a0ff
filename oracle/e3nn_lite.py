"""numpy restatement of the e3nn 0.5.1 pieces SEGNN uses — TEST ORACLE ONLY.

e3nn is a third-party dependency of the reference (``requirements.txt:8`` pins
e3nn==0.5.1) that is not installed in this image.  The reference's call sites are

* ``FullyConnectedTensorProduct``   models/segnn/o3_building_blocks.py:43-49
* ``Gate``                           models/segnn/o3_building_blocks.py:187-193
* ``spherical_harmonics``            models/segnn/o3_building_blocks.py:243-255
* ``BatchNorm``                      models/segnn/segnn.py:4,233-235
* ``Irreps`` algebra                 models/segnn/segnn.py:37-51,209-210,
                                     models/balanced_irreps.py:51-85

This module restates the published e3nn 0.5.1 algorithm for these (irreps up
to l = 1, which is all SEGNN with lmax_h = lmax_attr = 1 touches).  Parity vs
e3nn itself is UNPINNED (no e3nn output exists anywhere in the reference); the
known-answer tests in tests/test_oracle_segnn.py guard it.
"""
from __future__ import annotations

import math
import re
from dataclasses import dataclass

import numpy as np

# --------------------------------------------------------------------------
# Irrep / Irreps algebra (e3nn.o3.Irrep / Irreps)
# --------------------------------------------------------------------------


@dataclass(frozen=True, order=False)
class Irrep:
    l: int
    p: int  # +1 even, -1 odd

    @staticmethod
    def parse(s: str) -> "Irrep":
        s = s.strip()
        l, par = int(s[:-1]), s[-1]
        return Irrep(l, {"e": 1, "o": -1, "y": (-1) ** l}[par])

    @property
    def dim(self) -> int:
        return 2 * self.l + 1

    def is_scalar(self) -> bool:
        return self.l == 0 and self.p == 1

    def key(self):
        # e3nn's Irrep is a tuple (l, p): ordering is lexicographic on (l, p)
        return (self.l, self.p)

    def __mul__(self, other: "Irrep"):
        p = self.p * other.p
        return [Irrep(l, p) for l in range(abs(self.l - other.l), self.l + other.l + 1)]

    def __str__(self) -> str:
        return f"{self.l}{'e' if self.p == 1 else 'o'}"


class Irreps(list):
    """List of (mul, Irrep)."""

    def __init__(self, spec=()):
        if isinstance(spec, str):
            items = []
            for part in spec.split("+"):
                part = part.strip()
                if not part:
                    continue
                m = re.fullmatch(r"(\d+)x(\d+[eoy])", part)
                if m:
                    items.append((int(m.group(1)), Irrep.parse(m.group(2))))
                else:
                    items.append((1, Irrep.parse(part)))
            super().__init__(items)
        else:
            super().__init__([(int(m), ir) for m, ir in spec])

    @staticmethod
    def spherical_harmonics(lmax: int, p: int = -1) -> "Irreps":
        return Irreps([(1, Irrep(l, p ** l)) for l in range(lmax + 1)])

    @property
    def dim(self) -> int:
        return sum(m * ir.dim for m, ir in self)

    @property
    def num_irreps(self) -> int:
        return sum(m for m, _ in self)

    @property
    def lmax(self) -> int:
        return max(ir.l for _, ir in self)

    def slices(self):
        out, i = [], 0
        for m, ir in self:
            out.append(slice(i, i + m * ir.dim))
            i += m * ir.dim
        return out

    def simplify(self) -> "Irreps":
        # merges ADJACENT equal irreps only (e3nn 0.5.1 Irreps.simplify)
        out = []
        for m, ir in self:
            if out and out[-1][1] == ir:
                out[-1] = (out[-1][0] + m, ir)
            elif m > 0:
                out.append((m, ir))
        return Irreps(out)

    def sort(self):
        """Stable sort by irrep; returns (irreps, p, inv) like e3nn."""
        order = sorted(range(len(self)), key=lambda i: (self[i][1].key(), i))
        inv = order
        p = [0] * len(order)
        for new, old in enumerate(order):
            p[old] = new
        return Irreps([self[i] for i in order]), p, inv

    def __add__(self, other):
        return Irreps(list(self) + list(Irreps(other)))

    def __mul__(self, n: int):
        return Irreps(list(self) * n)

    __rmul__ = __mul__

    def __str__(self):
        return "+".join(f"{m}x{ir}" for m, ir in self)


# --------------------------------------------------------------------------
# Wigner 3j (Frobenius-normalised, e3nn.o3.wigner_3j) for l <= 1
# --------------------------------------------------------------------------


def wigner_3j(l1: int, l2: int, l3: int) -> np.ndarray:
    """e3nn returns the real Clebsch-Gordan tensor normalised to ||C||_F = 1.
    Every path with an l=0 leg is a (scaled) identity, which is basis-order
    independent; (1,1,1) is the Levi-Civita tensor (unused by SEGNN at
    lmax=1: 1o x 1o -> 1e never reaches a 1o output)."""
    C = np.zeros((2 * l1 + 1, 2 * l2 + 1, 2 * l3 + 1))
    if (l1, l2, l3) == (0, 0, 0):
        C[0, 0, 0] = 1.0
    elif (l1, l2, l3) == (0, 1, 1):
        C[0] = np.eye(3)
    elif (l1, l2, l3) == (1, 0, 1):
        C[:, 0, :] = np.eye(3)
    elif (l1, l2, l3) == (1, 1, 0):
        C[:, :, 0] = np.eye(3)
    elif (l1, l2, l3) == (1, 1, 1):
        for i, j, k in [(0, 1, 2), (1, 2, 0), (2, 0, 1)]:
            C[i, j, k], C[j, i, k] = 1.0, -1.0
    else:
        raise NotImplementedError((l1, l2, l3))
    return C / np.linalg.norm(C)


# --------------------------------------------------------------------------
# FullyConnectedTensorProduct (e3nn.o3.FullyConnectedTensorProduct)
# --------------------------------------------------------------------------


class FullyConnectedTP:
    """Mode "uvw", irrep_normalization="component", path_normalization="element",
    shared weights.  Instructions are enumerated
    ``for i1 in in1, for i2 in in2, for io in out if ir_out in ir1*ir2``; the flat
    weight is the concatenation of per-instruction (mul1, mul2, mul_out) blocks.
    Path coefficient: sqrt(ir_out.dim / fan_in(io)), fan_in = sum mul1*mul2 over
    the instructions feeding the same output slot."""

    def __init__(self, irreps_in1, irreps_in2, irreps_out):
        self.irreps_in1 = Irreps(irreps_in1)
        self.irreps_in2 = Irreps(irreps_in2)
        self.irreps_out = Irreps(irreps_out)
        self.instructions = []
        for i1, (m1, ir1) in enumerate(self.irreps_in1):
            for i2, (m2, ir2) in enumerate(self.irreps_in2):
                for io, (mo, iro) in enumerate(self.irreps_out):
                    if iro in ir1 * ir2:
                        self.instructions.append((i1, i2, io, (m1, m2, mo)))
        fan_in = {}
        for i1, i2, io, (m1, m2, mo) in self.instructions:
            fan_in[io] = fan_in.get(io, 0) + m1 * m2
        self.fan_in = fan_in
        self.coeffs = [math.sqrt(self.irreps_out[io][1].dim / fan_in[io])
                       for (_, _, io, _) in self.instructions]
        self.weight_numel = sum(int(np.prod(s)) for *_, s in self.instructions)

    def weight_views(self, w: np.ndarray):
        off = 0
        for *_, shape in self.instructions:
            n = int(np.prod(shape))
            yield w[off:off + n].reshape(shape)
            off += n

    def __call__(self, x1: np.ndarray, x2: np.ndarray, w: np.ndarray) -> np.ndarray:
        Z = x1.shape[0]
        s1, s2, so = self.irreps_in1.slices(), self.irreps_in2.slices(), self.irreps_out.slices()
        out = np.zeros((Z, self.irreps_out.dim), dtype=np.result_type(x1, x2, w))
        for (i1, i2, io, (m1, m2, mo)), W, c in zip(self.instructions, self.weight_views(w), self.coeffs):
            d1, d2, do = self.irreps_in1[i1][1].dim, self.irreps_in2[i2][1].dim, self.irreps_out[io][1].dim
            C = wigner_3j(self.irreps_in1[i1][1].l, self.irreps_in2[i2][1].l, self.irreps_out[io][1].l)
            C = C.astype(out.dtype)      # fp32 runs stay in fp32 (the C2 fixture's fp32 reference)
            a = x1[:, s1[i1]].reshape(Z, m1, d1)
            b = x2[:, s2[i2]].reshape(Z, m2, d2)
            # t[z,u,v,k] = sum_ij a[z,u,i] b[z,v,j] C[i,j,k]
            ab = np.einsum("zui,zvj->zuvij", a, b).reshape(Z, m1, m2, d1 * d2)
            t = ab @ C.reshape(d1 * d2, do)                          # [Z,m1,m2,do]
            t = t.transpose(0, 3, 1, 2).reshape(Z * do, m1 * m2)     # [(Z,k), (u,v)]
            y = (t @ W.reshape(m1 * m2, mo)).reshape(Z, do, mo)      # [Z,k,w]
            out[:, so[io]] += c * y.transpose(0, 2, 1).reshape(Z, mo * do)
        return out


# --------------------------------------------------------------------------
# spherical_harmonics(lmax, x, normalize=True, normalization="integral")
# --------------------------------------------------------------------------

SH_C0 = 1.0 / math.sqrt(4.0 * math.pi)           # 0.28209479177387814
SH_C1 = math.sqrt(3.0 / (4.0 * math.pi))         # 0.4886025119029199


def spherical_harmonics_l1(x: np.ndarray) -> np.ndarray:
    """[Y0, Y1(x, y, z)] with torch.nn.functional.normalize semantics
    (x / max(||x||, 1e-12)) and "integral" normalisation."""
    n = np.sqrt((x * x).sum(-1, keepdims=True))
    xh = x / np.maximum(n, 1e-12)
    return np.concatenate([np.full(x.shape[:-1] + (1,), SH_C0, dtype=x.dtype), SH_C1 * xh], -1)


# --------------------------------------------------------------------------
# normalize2mom constants and Gate (e3nn.nn.Gate with SiLU / sigmoid)
# --------------------------------------------------------------------------

# c = E_{z~N(0,1)}[f(z)^2]^(-1/2), estimated by e3nn with
# torch.Generator("cpu").manual_seed(0) and randn(1_000_000, float64).
# Recomputed by tests/test_oracle_segnn.py::test_normalize2mom_constants.
C_SILU = 1.6791767923989418
C_SIGMOID = 1.8467055342154763


def normalize2mom_constant(f) -> float:
    import torch  # only to reproduce e3nn's RNG stream
    gen = torch.Generator(device="cpu").manual_seed(0)
    z = torch.randn(1_000_000, generator=gen, dtype=torch.float64)
    return f(z).pow(2).mean().pow(-0.5).item()


def silu(x):
    return x / (1.0 + np.exp(-x))


def sigmoid(x):
    return 1.0 / (1.0 + np.exp(-x))


def gate(x: np.ndarray, n_scalars: int, n_gates: int, irreps_gated: Irreps) -> np.ndarray:
    """Gate(irreps_scalars, [SiLU], irreps_gates, [sigmoid], irreps_gated)
    on input laid out [scalars | gates | gated] (e3nn _Sortcut of the simplified
    input keeps this order for 0e scalars/gates followed by 1o gated)."""
    s = C_SILU * silu(x[:, :n_scalars])
    g = C_SIGMOID * sigmoid(x[:, n_scalars:n_scalars + n_gates])
    gated = x[:, n_scalars + n_gates:]
    out, i, gi = [], 0, 0
    for m, ir in irreps_gated:
        seg = gated[:, i:i + m * ir.dim].reshape(-1, m, ir.dim)
        out.append((seg * g[:, gi:gi + m, None]).reshape(-1, m * ir.dim))
        i += m * ir.dim
        gi += m
    return np.concatenate([s] + out, axis=1)


# --------------------------------------------------------------------------
# BatchNorm (e3nn.nn.BatchNorm, reduce="mean", normalization="component")
# --------------------------------------------------------------------------


def batch_norm(x, irreps: Irreps, weight, bias, running_mean, running_var,
               training: bool, eps: float = 1e-5, momentum: float = 0.1):
    """Returns (y, new_running_mean, new_running_var).  Train mode: scalar (0e)
    fields are centred by the batch mean, every field is scaled by
    (mean over rows of mean over components of x^2 + eps)^-1/2 * weight,
    0e fields get + bias; running stats r <- (1-m) r + m * batch_stat."""
    ix = irm = irv = iw = ib = 0
    fields = []
    new_rm, new_rv = [], []
    Z = x.shape[0]
    for m, ir in irreps:
        d = ir.dim
        f = x[:, ix:ix + m * d].reshape(Z, m, d)
        ix += m * d
        if ir.is_scalar():
            if training:
                mu = f.mean(axis=(0, 2)) if d > 1 else f[:, :, 0].mean(0)
                new_rm.append((1 - momentum) * running_mean[irm:irm + m] + momentum * mu)
            else:
                mu = running_mean[irm:irm + m]
            irm += m
            f = f - mu[None, :, None]
        if training:
            n = (f ** 2).mean(2).mean(0)
            new_rv.append((1 - momentum) * running_var[irv:irv + m] + momentum * n)
        else:
            n = running_var[irv:irv + m]
        irv += m
        scale = (n + eps) ** -0.5 * weight[iw:iw + m]
        iw += m
        f = f * scale[None, :, None]
        if ir.is_scalar():
            f = f + bias[ib:ib + m][None, :, None]
            ib += m
        fields.append(f.reshape(Z, m * d))
    y = np.concatenate(fields, axis=1)
    rm = np.concatenate(new_rm) if (training and new_rm) else running_mean
    rv = np.concatenate(new_rv) if (training and new_rv) else running_var
    return y, rm, rv
