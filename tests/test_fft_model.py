"""CPU model of the RS(32,32) additive-FFT encode kernel (cess_amd/csrc/fft.hip, k_fft3232):
the Lin-Chung-Han IFFT over the subspace {0..31} and FFT over the coset 32 ^ {0..31}, on
bit-sliced planes, with the kernel's lane-pair split (position t on lane t & 1) and its
cross-lane butterfly formulas, checked byte-exact against the Python oracle's matrix encode.
This pins the algorithm the kernel restates; tests/test_gpu_parity.py pins the kernel itself."""
from functools import reduce

import numpy as np
import pytest

from oracle import rs_oracle as o

EXP = [0] * 512
LOG = [0] * 256
_x = 1
for _i in range(255):
    EXP[_i] = _x
    LOG[_x] = _i
    _x <<= 1
    if _x & 0x100:
        _x ^= 0x11D
for _i in range(255, 512):
    EXP[_i] = EXP[_i - 255]


def mul(a, b):
    return 0 if a == 0 or b == 0 else EXP[LOG[a] + LOG[b]]


def inv(a):
    return EXP[255 - LOG[a]]


def W(i, x):
    return reduce(mul, [x ^ a for a in range(1 << i)], 1)


def What(i, x):
    return mul(W(i, x), inv(W(i, 1 << i)))


def skews(beta, K=5):
    return {(i, b): What(i, (b << (i + 1)) ^ beta) for i in range(K) for b in range(1 << (K - 1 - i))}


SI, SF = skews(0), skews(32)
M32 = 0xFFFFFFFF


def mulplanes(s, z):
    rows = [[p for p in range(8) if (mul(s, 1 << p) >> q) & 1] for q in range(8)]
    return [reduce(lambda a, b: a ^ b, [z[p] for p in r], 0) for r in rows]


def swapmove(a, b, s, m):
    return (m & a) | (~m & ((b << s) & M32)) & M32, ((m & (a >> s)) | (~m & b)) & M32


def tr8(w):
    w = list(w)
    for s, m in ((4, 0x0F0F0F0F), (2, 0x33333333), (1, 0x55555555)):
        for d in range(8):
            if not d & s:
                w[d], w[d + s] = swapmove(w[d], w[d + s], s, m)
    return w


def kernel_model(data):
    """data: 32 shards x 32 bytes -> 32 parity shards, as one lane pair of k_fft3232 does."""
    X = [[tr8([int.from_bytes(bytes(data[2 * j + ln][4 * d:4 * d + 4]), "little")
               for d in range(8)]) for j in range(16)] for ln in range(2)]
    em = [M32, 0]
    for j in range(16):  # IFFT layer 0, across the pair
        s, new = SI[(0, j)], []
        for ln in range(2):
            x, y = X[ln][j], X[1 - ln][j]
            z = [x[q] ^ y[q] for q in range(8)]
            w = [x[q] ^ z[q] for q in range(8)]
            if s:
                w = [a ^ b for a, b in zip(w, mulplanes(s, z))]
            new.append([z[q] ^ (em[ln] & w[q]) for q in range(8)])
        X[0][j], X[1][j] = new
    for i in range(1, 5):  # IFFT layers, in-lane
        hj = 1 << (i - 1)
        for ln in range(2):
            for j in range(16):
                if j & hj:
                    continue
                s = SI[(i, j >> i)]
                X[ln][j + hj] = [b ^ a for a, b in zip(X[ln][j], X[ln][j + hj])]
                if s:
                    X[ln][j] = [a ^ b for a, b in zip(X[ln][j], mulplanes(s, X[ln][j + hj]))]
    for i in range(4, 0, -1):  # FFT layers, in-lane
        hj = 1 << (i - 1)
        for ln in range(2):
            for j in range(16):
                if j & hj:
                    continue
                s = SF[(i, j >> i)]
                if s:
                    X[ln][j] = [a ^ b for a, b in zip(X[ln][j], mulplanes(s, X[ln][j + hj]))]
                X[ln][j + hj] = [b ^ a for a, b in zip(X[ln][j], X[ln][j + hj])]
    for j in range(16):  # FFT layer 0, across the pair
        s, new = SF[(0, j)], []
        for ln in range(2):
            x, y = X[ln][j], X[1 - ln][j]
            p = [y[q] if em[ln] else x[q] for q in range(8)]
            t = [x[q] ^ ((~em[ln] & M32) & y[q]) for q in range(8)]
            new.append([a ^ b for a, b in zip(t, mulplanes(s, p))] if s else t)
        X[0][j], X[1][j] = new
    return [b"".join(v.to_bytes(4, "little") for v in tr8(X[t & 1][t >> 1])) for t in range(32)]


def test_transpose_is_bit_slicing_and_involution():
    rng = np.random.default_rng(0)
    w = [int(v) for v in rng.integers(0, 2**32, 8, dtype=np.uint64)]
    p = tr8(w)
    assert all(((p[b] >> (8 * j + d)) & 1) == ((w[d] >> (8 * j + b)) & 1)
               for b in range(8) for j in range(4) for d in range(8))
    assert tr8(p) == w


def test_skew_zeros_and_fft_nonzero():
    # the kernel specialises zero skews of the IFFT (block 0 of every layer) and needs none in
    # the FFT over the coset
    assert [b for (i, b), s in SI.items() if s == 0] == [0] * 5
    assert all(SF.values())


@pytest.mark.parametrize("seed", range(4))
def test_kernel_model_matches_matrix_encode(seed):
    rng = np.random.default_rng(seed)
    data = [rng.integers(0, 256, 32, dtype=np.uint8) for _ in range(32)]
    if seed == 3:
        data = [np.full(32, 255, np.uint8) for _ in range(32)]
    want = o.ReedSolomon(32, 32).encode(data)
    got = kernel_model(data)
    assert got == [w.tobytes() for w in want]
