"""3-layer MLP fraud scorer 30 -> 128 -> 64 -> 1 (BASELINE.json config 2/3).

Replaces the reference's ``nakfour/modelfull`` Seldon model (deploy/model/modelfull.json:24),
which returns ``proba_1`` for a transaction's features (README.md:549-550).

Weight packing for the fused HIP kernel (csrc/kernels/score_mlp.hip)
--------------------------------------------------------------------
The kernel computes the *transposed* activations so that each MFMA accumulator is
directly the next MFMA's B operand (no LDS round trip, no lane shuffles):

  layer 1:  H1^T[128,16] = W1[128,32] . Xn^T[32,16]        (8 x mfma_f32_16x16x32_bf16)
  layer 2:  H2^T[ 64,16] = W2[ 64,128] . relu(H1^T)        (16 MFMAs, 4 M-tiles x 4 K-steps)
  layer 3:  z[16] = w3 . relu(H2^T) + b3                    (VALU + 2 cross-lane adds)

16x16x32 bf16 operand maps (gfx950): lane l holds A[l&15][8(l>>4)+j] and
B[8(l>>4)+j][l&15] (j=0..7); C/D: lane l holds D[4(l>>4)+r][l&15] (r=0..3).
Layer-1 output tile t therefore sits in lane group g=l>>4 as features 16t+4g+r.  Layer 2's
K-step s takes tiles 2s and 2s+1 as its B fragment, i.e. element j of group g is feature
  pi(s,g,j) = 32s + 4g + (j&3) + 16(j>>2)
and W2 is packed with the same k-permutation, so the sum is unchanged.

W64 wire blobs (``pack(wire=True)``, header flag FLAG_WIRE): the row's 16-B lane chunk IS
the layer-1 B fragment -- the bf16 V-columns go into the MFMA as raw bits, their
normalisation folded into W1 (columns x 1/sigma) and b1 (minus W1'.mu); b1 rides in
K-columns 30/31 as a bf16 hi/lo pair against constant-1 inputs; only Time and Amount are
normalised in the kernel (lane group 3).  Layer 3 is two more MFMAs on bf16 relu(H2^T) against
W3pad (w3 in rows 0/4/8/12: z lands in every lane group, no cross-lane reduction), appended
as ``[25920, 27968)`` (``WIRE_BLOB_BYTES``).  ``wire_logits`` is the numerics oracle of that path.

Blob layout (bytes, all 16-B aligned), ``BLOB_BYTES`` = 25920:
  [0,64)        header: 'MLP1', flags(u32), b3(f32)
  [64,192)      mu[32]   f32   (lane group g reads mu[8g..8g+7])
  [192,320)     isg[32]  f32
  [320,8512)    W1f [8 t][64 lane][8 j]           bf16   W1[16t+(l&15)][8(l>>4)+j]
  [8512,24896)  W2f [4 u][4 s][64 lane][8 j]      bf16   W2[16u+(l&15)][pi(s,l>>4,j)]
  [24896,25408) b1f [8 t][4 g][4 r]  f32   b1[16t+4g+r]        (zero in wire blobs)
  [25408,25664) b2f [4 u][4 g][4 r]  f32   b2[16u+4g+r]
  [25664,25920) w3f [4 u][4 g][4 r]  f32   w3[16u+4g+r]
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np

from ..contracts.transaction import AMOUNT_COL, N_FEATURES, TIME_COL, WIRE_PERM, decode_wire, encode_wire
from .common import (FLAG_WIRE, HEADER_BYTES, KPAD, Normalizer, bf16_bits, bf16_round, header, sigmoid)

H1, H2 = 128, 64
OFF_NORM = HEADER_BYTES
OFF_W1 = OFF_NORM + 256
OFF_W2 = OFF_W1 + 8 * 64 * 8 * 2
OFF_B1 = OFF_W2 + 4 * 4 * 64 * 8 * 2
OFF_B2 = OFF_B1 + 8 * 4 * 4 * 4
OFF_W3 = OFF_B2 + 4 * 4 * 4 * 4
BLOB_BYTES = OFF_W3 + 4 * 4 * 4 * 4
assert BLOB_BYTES == 25920 and BLOB_BYTES % 16 == 0

WIRE_N_BF16 = 28     # wire positions [0, 28) are bf16 V1..V28 (raw MFMA operands)
# wire blobs append layer 3 as MFMA A-fragments: W3pad [16 x 64] bf16 with w3 in rows 0, 4, 8,
# 12 (so every lane group's accumulator register 0 receives z), 2 K-steps x 64 lanes x 8
OFF_W3F = BLOB_BYTES
WIRE_BLOB_BYTES = OFF_W3F + 2 * 64 * 8 * 2


def _pi(s: int, g: int, j: int) -> int:
    return 32 * s + 4 * g + (j & 3) + 16 * (j >> 2)


@dataclass
class MLPModel:
    W1: np.ndarray   # [128, 30]
    b1: np.ndarray   # [128]
    W2: np.ndarray   # [64, 128]
    b2: np.ndarray   # [64]
    w3: np.ndarray   # [64]
    b3: float
    norm: Normalizer
    kind: str = "mlp"

    @property
    def n_params(self) -> int:
        return self.W1.size + self.b1.size + self.W2.size + self.b2.size + self.w3.size + 1

    @classmethod
    def random_init(cls, seed: int = 0, norm: Optional[Normalizer] = None) -> "MLPModel":
        """He-uniform init (what ``torch.nn.Linear`` would give, up to the constant)."""
        rng = np.random.default_rng(seed)

        def lin(fan_out, fan_in):
            bound = 1.0 / np.sqrt(fan_in)
            return (rng.uniform(-bound, bound, (fan_out, fan_in)).astype(np.float32),
                    rng.uniform(-bound, bound, fan_out).astype(np.float32))
        W1, b1 = lin(H1, N_FEATURES)
        W2, b2 = lin(H2, H1)
        w3, b3 = lin(1, H2)
        return cls(W1, b1, W2, b2, w3[0], float(b3[0]), norm or Normalizer.identity())

    # ---------------------------------------------------------------- oracles
    def logits(self, X: np.ndarray, emulate_bf16: bool = False) -> np.ndarray:
        """fp32 reference (or bf16-operand emulation of the kernel's numerics)."""
        Xn = self.norm(X).astype(np.float32)
        W1, W2 = self.W1, self.W2
        if emulate_bf16:
            Xn, W1, W2 = bf16_round(Xn), bf16_round(W1), bf16_round(W2)
        h1 = np.maximum(Xn.astype(np.float64) @ W1.T.astype(np.float64) + self.b1, 0.0)
        if emulate_bf16:
            h1 = bf16_round(h1.astype(np.float32)).astype(np.float64)
        h2 = np.maximum(h1 @ W2.T.astype(np.float64) + self.b2, 0.0)
        return (h2 @ self.w3.astype(np.float64) + self.b3).astype(np.float32)

    def predict_proba(self, X: np.ndarray, emulate_bf16: bool = False) -> np.ndarray:
        return sigmoid(self.logits(X, emulate_bf16))

    def calibrate_bias(self, X: np.ndarray, target_rate: float, threshold: float = 0.5) -> None:
        """Shift b3 so that a fraction ``target_rate`` of X scores >= threshold.

        Used with random-init weights so that routing volume resembles the dataset's
        fraud prior instead of ~50 % (documented in bench.py's ``data`` field)."""
        z = self.logits(X)
        zt = np.log(threshold / (1.0 - threshold))
        q = np.quantile(z, 1.0 - target_rate)
        self.b3 += float(zt - q)

    # ---------------------------------------------------------------- packing
    def _wire_w1(self):
        """Layer-1 matrix of a wire blob [128, 32] (wire K order; V-normalisation and the
        bias hi/lo pair folded in), as float32 before bf16 rounding."""
        W1p = np.zeros((H1, KPAD), np.float32)
        W1w = self.W1[:, WIRE_PERM].astype(np.float64)
        mu = self.norm.mu[WIRE_PERM].astype(np.float64)
        isg = self.norm.inv_sigma[WIRE_PERM].astype(np.float64)
        v = np.arange(N_FEATURES) < WIRE_N_BF16
        W1w[:, v] *= isg[v]
        b1w = self.b1.astype(np.float64) - W1w[:, v] @ mu[v]
        W1p[:, :N_FEATURES] = W1w
        hi = bf16_round(b1w.astype(np.float32))
        W1p[:, N_FEATURES] = hi
        W1p[:, N_FEATURES + 1] = bf16_round((b1w - hi).astype(np.float32))
        return W1p

    def wire_inputs(self, X: np.ndarray) -> np.ndarray:
        """The layer-1 B operand of the wire kernel, [n, 32] float32 (bf16-exact): raw bf16
        V-columns, bf16 of the normalised Time / Amount, then the two constant-1 bias inputs."""
        Xd = decode_wire(encode_wire(np.asarray(X, np.float32)))
        xin = np.ones((Xd.shape[0], KPAD), np.float32)
        xin[:, :WIRE_N_BF16] = Xd[:, WIRE_PERM[:WIRE_N_BF16]]
        t = Xd[:, TIME_COL].astype(np.float32)
        a = Xd[:, AMOUNT_COL].astype(np.float32)
        if self.norm.log_amount:
            a = np.log1p(np.maximum(a, 0.0)).astype(np.float32)
        mu, isg = self.norm.mu, self.norm.inv_sigma
        xin[:, WIRE_N_BF16] = (t - mu[TIME_COL]) * isg[TIME_COL]
        xin[:, WIRE_N_BF16 + 1] = (a - mu[AMOUNT_COL]) * isg[AMOUNT_COL]
        return bf16_round(xin)

    def wire_logits(self, X: np.ndarray) -> np.ndarray:
        """Numerics oracle of the W64 wire kernel (bf16 operands, fp32/fp64 accumulation)."""
        xin = self.wire_inputs(X).astype(np.float64)
        W1p = bf16_round(self._wire_w1()).astype(np.float64)
        h1 = bf16_round(np.maximum(xin @ W1p.T, 0.0).astype(np.float32)).astype(np.float64)
        h2 = np.maximum(h1 @ bf16_round(self.W2).T.astype(np.float64) + self.b2, 0.0)
        h2 = bf16_round(h2.astype(np.float32)).astype(np.float64)
        return (h2 @ bf16_round(self.w3).astype(np.float64) + self.b3).astype(np.float32)

    def wire_proba(self, X: np.ndarray) -> np.ndarray:
        return sigmoid(self.wire_logits(X))

    def pack(self, wire: bool = False) -> bytes:
        """``wire=True``: the W64 wire blob (module docstring) with the normaliser in W64
        row order and header flag FLAG_WIRE -- the blob for engines whose logs hold W64 rows."""
        if wire:
            W1p = self._wire_w1()
            b1 = np.zeros_like(self.b1)          # folded into W1p columns 30/31
        else:
            W1p = np.zeros((H1, KPAD), np.float32)
            W1p[:, :N_FEATURES] = self.W1
            b1 = self.b1
        lanes = np.arange(64)
        c, g = lanes & 15, lanes >> 4
        j = np.arange(8)
        # W1f[t][l][j] = W1[16t + (l&15)][8(l>>4)+j]
        w1f = W1p[(16 * np.arange(8)[:, None, None] + c[None, :, None]),
                  (8 * g[None, :, None] + j[None, None, :])]
        # W2f[u][s][l][j] = W2[16u + (l&15)][pi(s, l>>4, j)]
        kidx = np.array([[[_pi(s, gg, jj) for jj in range(8)] for gg in g] for s in range(4)])  # [4 s][64][8]
        rows = 16 * np.arange(4)[:, None, None, None] + c[None, None, :, None]                  # [4 u][1][64][1]
        w2f = self.W2[rows, kidx[None, :, :, :]]
        gi, ri = np.meshgrid(np.arange(4), np.arange(4), indexing="ij")
        b1f = np.stack([b1[16 * t + 4 * gi + ri] for t in range(8)])
        b2f = np.stack([self.b2[16 * u + 4 * gi + ri] for u in range(4)])
        w3f = np.stack([self.w3[16 * u + 4 * gi + ri] for u in range(4)])
        blob = (header(b"MLP1", self.norm.flags | (FLAG_WIRE if wire else 0), float(self.b3))
                + self.norm.packed(wire)
                + bf16_bits(w1f).tobytes() + bf16_bits(w2f).tobytes()
                + b1f.astype(np.float32).tobytes() + b2f.astype(np.float32).tobytes()
                + w3f.astype(np.float32).tobytes())
        assert len(blob) == BLOB_BYTES, len(blob)
        if wire:
            # W3f[s][l][j] = w3[pi(s, l>>4, j)] in rows (l&15) in {0,4,8,12}, else 0
            w3f = np.zeros((2, 64, 8), np.float32)
            for s_ in range(2):
                for ln in range(64):
                    if (ln & 15) % 4 == 0:
                        w3f[s_, ln] = [self.w3[_pi(s_, ln >> 4, jj)] for jj in range(8)]
            blob += bf16_bits(w3f).tobytes()
            assert len(blob) == WIRE_BLOB_BYTES
        return blob

    # ---------------------------------------------------------------- state io
    def state_dict(self) -> dict:
        st = {"mlp.W1": self.W1, "mlp.b1": self.b1, "mlp.W2": self.W2, "mlp.b2": self.b2,
              "mlp.w3": self.w3, "mlp.b3": np.array([self.b3], np.float32)}
        st.update(self.norm.state())
        return st

    @classmethod
    def from_state_dict(cls, st: dict) -> "MLPModel":
        return cls(np.asarray(st["mlp.W1"], np.float32), np.asarray(st["mlp.b1"], np.float32),
                   np.asarray(st["mlp.W2"], np.float32), np.asarray(st["mlp.b2"], np.float32),
                   np.asarray(st["mlp.w3"], np.float32), float(np.asarray(st["mlp.b3"]).reshape(-1)[0]),
                   Normalizer.from_state(st))


def emulate_packed_kernel(blob: bytes, X: np.ndarray) -> np.ndarray:
    """Pure-NumPy emulation of score_mlp.hip consuming the packed blob lane by lane.

    It walks the same fragment maps as the kernel (per 16-row tile, per lane) so a
    packing or operand-order bug shows up on CPU, before any GPU run.  Wire blobs take the
    wire kernel's operand path (raw bf16 V bits, Time/Amount normalised, constant-1 bias
    inputs)."""
    b = memoryview(blob)
    flags = int(np.frombuffer(b, np.uint32, 1, 4)[0])
    b3 = float(np.frombuffer(b, np.float32, 1, 8)[0])
    mu = np.frombuffer(b, np.float32, 32, OFF_NORM)
    isg = np.frombuffer(b, np.float32, 32, OFF_NORM + 128)
    wire = bool(flags & FLAG_WIRE)

    def bf(off, n):
        u = np.frombuffer(b, np.uint16, n, off).astype(np.uint32) << 16
        return u.view(np.float32)
    W1f = bf(OFF_W1, 8 * 64 * 8).reshape(8, 64, 8)
    W2f = bf(OFF_W2, 4 * 4 * 64 * 8).reshape(4, 4, 64, 8)
    b1f = np.frombuffer(b, np.float32, 128, OFF_B1).reshape(8, 4, 4)
    b2f = np.frombuffer(b, np.float32, 64, OFF_B2).reshape(4, 4, 4)
    w3f = np.frombuffer(b, np.float32, 64, OFF_W3).reshape(4, 4, 4)

    X = np.asarray(X, np.float32)
    if wire:
        # the kernel sees W64 rows: bf16 V-columns, permuted to wire order
        X = decode_wire(encode_wire(X))[:, WIRE_PERM]
    n = X.shape[0]
    out = np.empty(n, np.float32)
    lanes = np.arange(64)
    c, g = lanes & 15, lanes >> 4

    def mfma(A, B, C):
        # A: [64 lanes][8] fragment of A (16x32), B: [64][8] fragment of B (32x16), C: [64][4]
        Am = np.zeros((16, 32)); Bm = np.zeros((32, 16))
        for l in range(64):
            Am[l & 15, 8 * (l >> 4): 8 * (l >> 4) + 8] = A[l]
            Bm[8 * (l >> 4): 8 * (l >> 4) + 8, l & 15] = B[l]
        D = Am @ Bm
        res = C.astype(np.float64).copy()
        for l in range(64):
            for r in range(4):
                res[l, r] += D[4 * (l >> 4) + r, l & 15]
        return res

    for t0 in range(0, n, 16):
        rows = t0 + c
        valid = rows < n
        xin = np.zeros((64, 8), np.float32)
        for l in range(64):
            if valid[l]:
                for jj in range(8):
                    k = 8 * g[l] + jj
                    if wire and k >= N_FEATURES:
                        xin[l, jj] = 1.0                      # constant-1 bias inputs
                    elif wire and k < WIRE_N_BF16:
                        xin[l, jj] = X[rows[l], k]            # raw bf16 bits
                    elif k < N_FEATURES:
                        v = X[rows[l], k]
                        if (flags & 1) and k == N_FEATURES - 1:
                            v = np.log1p(max(v, 0.0))
                        xin[l, jj] = (v - mu[k]) * isg[k]
        xb = bf16_round(xin)
        acc1 = [mfma(W1f[t], xb, b1f[t][g]) for t in range(8)]
        acc2 = []
        for u in range(4):
            acc = b2f[u][g].astype(np.float64)
            for s in range(4):
                Bf = np.concatenate([np.maximum(acc1[2 * s], 0), np.maximum(acc1[2 * s + 1], 0)], axis=1)
                acc = mfma(W2f[u, s], bf16_round(Bf.astype(np.float32)), acc)
            acc2.append(acc)
        if wire:
            W3f = bf(OFF_W3F, 2 * 64 * 8).reshape(2, 64, 8)
            acc3 = np.zeros((64, 4))
            for s_ in range(2):
                Bf = np.concatenate([np.maximum(acc2[2 * s_], 0), np.maximum(acc2[2 * s_ + 1], 0)], axis=1)
                acc3 = mfma(W3f[s_], bf16_round(Bf.astype(np.float32)), acc3)
            zt = acc3[:16, 0] + b3                      # lane group 0, register 0: row 0 of D
        else:
            z = np.zeros(64)
            for u in range(4):
                z += (np.maximum(acc2[u], 0) * w3f[u][g]).sum(1)
            zt = np.array([z[cc] + z[cc + 16] + z[cc + 32] + z[cc + 48] for cc in range(16)]) + b3
        for cc in range(16):
            if t0 + cc < n:
                out[t0 + cc] = 1.0 / (1.0 + np.exp(-zt[cc]))
    return out
