"""CPU oracle for the CESS segment -> fragment Reed-Solomon path (numpy restatement).

TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
may import this module, and only as the checker. The product path (cess_amd/) never imports it.

What is restated, and from where
--------------------------------
The reference (/root/reference, the CESS chain) holds no codec: it fixes the
geometry and records the codec's outputs.
  * SEGMENT_SIZE = 16 MiB, FRAGMENT_SIZE = 8 MiB      primitives/common/src/lib.rs:60-61
  * FRAGMENT_COUNT = 3 fragments per segment          runtime/src/lib.rs:1027
    -> k = 2 data fragments, m = 1 parity fragment
  * space per segment = SEGMENT_SIZE * 15 / 10        c-pallets/file-bank/src/lib.rs:440
  * Hash([u8; 64]) per segment and per fragment       primitives/common/src/lib.rs:16
  * SegmentList { hash, fragment_list }               c-pallets/file-bank/src/types.rs:13-16
  * check_file_spec: len(fragment_list) == 3          c-pallets/file-bank/src/functions.rs:4-14
The arithmetic lives in the off-chain codec the CESS tools call, klauspost/reedsolomon (Go),
which is NOT vendored in the reference and whose version no reference file pins (Cargo.lock has
no erasure crate). Its published algorithm, restated here:
  * galois.go: GF(2^8), polynomial 0x11D (x^8+x^4+x^3+x^2+1), generator 2; galMultiply via
    log/exp; galExp(a, n) = a^n with 0^0 = 1.
  * matrix.go: Gauss-Jordan inverse with row swap on a zero pivot.
  * reedsolomon.go buildMatrix: vandermonde(k+m, k)[r][c] = galExp(r, c); E = V * inv(V[:k]).
  * Encode: parity_i = XOR_j E[k+i][j] * data_j, bytewise.
  * Reconstruct: rows of E for the first k present shards (index order) form a k x k submatrix;
    its inverse rebuilds missing data shards; missing parity is then re-encoded from the data.
  * Split: perShard = ceil(len / k); shard i = data[i*perShard:(i+1)*perShard], zero padded.
Hash convention [ecosystem, unpinned by the reference]: fragment / segment Hash = the 64 ASCII
characters of lowercase hex SHA-256 (FIPS 180-4) of the bytes; file hash [build convention] =
SHA-256 hex over the concatenated segment hashes.

PARITY STATUS: RS arithmetic is *parity unpinned by the reference* (it holds no codec, no RS
test and no RS fixture); SHA-256 is pinned by the reference's own NIST SHAVS files.
Pinning: public known answers (Backblaze / klauspost TestOneEncode RS(5,5), galois and matrix
unit-test values) and NIST SHAVS vectors from the reference's own tree
(utils/ring/third_party/NIST/SHAVS/SHA256{Short,Long}Msg.rsp). See tests/test_oracle.py.
"""
from __future__ import annotations

import hashlib
from typing import List, Optional, Sequence

import numpy as np

POLY = 0x11D

# ---------------------------------------------------------------------------------------------
# Field
# ---------------------------------------------------------------------------------------------


def _build_tables():
    exp = np.zeros(512, dtype=np.uint8)
    log = np.zeros(256, dtype=np.int32)
    x = 1
    for i in range(255):
        exp[i] = x
        log[x] = i
        x <<= 1
        if x & 0x100:
            x ^= POLY
    exp[255:510] = exp[0:255]
    mul = np.zeros((256, 256), dtype=np.uint8)
    for a in range(1, 256):
        mul[a, 1:] = exp[(log[a] + log[1:]) % 255]
    return exp, log, mul


EXP, LOG, MUL = _build_tables()


def gal_mul(a: int, b: int) -> int:
    return int(MUL[a, b])


def gal_div(a: int, b: int) -> int:
    if b == 0:
        raise ZeroDivisionError("GF(2^8) division by zero")
    if a == 0:
        return 0
    return int(EXP[(LOG[a] - LOG[b]) % 255])


def gal_exp(a: int, n: int) -> int:
    """a^n, with 0^0 = 1 (klauspost galExp)."""
    if n == 0:
        return 1
    if a == 0:
        return 0
    return int(EXP[(LOG[a] * n) % 255])


# ---------------------------------------------------------------------------------------------
# Matrices (lists of lists of ints; tiny, so plain Python)
# ---------------------------------------------------------------------------------------------


def mat_mul(a, b):
    rows, inner, cols = len(a), len(b), len(b[0])
    out = [[0] * cols for _ in range(rows)]
    for r in range(rows):
        for c in range(cols):
            acc = 0
            for t in range(inner):
                acc ^= gal_mul(a[r][t], b[t][c])
            out[r][c] = acc
    return out


def mat_invert(a):
    n = len(a)
    work = [list(a[r]) + [1 if c == r else 0 for c in range(n)] for r in range(n)]
    for col in range(n):
        if work[col][col] == 0:
            for r in range(col + 1, n):
                if work[r][col] != 0:
                    work[col], work[r] = work[r], work[col]
                    break
            else:
                raise ValueError("matrix is singular")
        scale = gal_div(1, work[col][col])
        work[col] = [gal_mul(v, scale) for v in work[col]]
        for r in range(n):
            if r != col and work[r][col] != 0:
                f = work[r][col]
                work[r] = [v ^ gal_mul(f, w) for v, w in zip(work[r], work[col])]
    return [row[n:] for row in work]


def vandermonde(rows: int, cols: int):
    return [[gal_exp(r, c) for c in range(cols)] for r in range(rows)]


def build_matrix(k: int, n: int):
    """(k+m) x k systematic encode matrix E = V * inv(V[:k])."""
    vm = vandermonde(n, k)
    return mat_mul(vm, mat_invert(vm[:k]))


# ---------------------------------------------------------------------------------------------
# Codec
# ---------------------------------------------------------------------------------------------


def mul_row_acc(out: np.ndarray, coef: int, src: np.ndarray) -> None:
    if coef == 0:
        return
    if coef == 1:
        np.bitwise_xor(out, src, out=out)
    else:
        np.bitwise_xor(out, MUL[coef][src], out=out)


def code_rows(rows, inputs: Sequence[np.ndarray]) -> List[np.ndarray]:
    n = len(inputs[0])
    outs = []
    for row in rows:
        acc = np.zeros(n, dtype=np.uint8)
        for c, src in zip(row, inputs):
            mul_row_acc(acc, c, src)
        outs.append(acc)
    return outs


class ReedSolomon:
    """klauspost-shaped oracle codec over numpy uint8 shards."""

    def __init__(self, k: int, m: int):
        if k < 1 or m < 1 or k + m > 256:
            raise ValueError("invalid shard counts")
        self.k, self.m, self.n = k, m, k + m
        self.matrix = build_matrix(k, self.n)
        self.parity = self.matrix[k:]

    def encode(self, data: Sequence[np.ndarray]) -> List[np.ndarray]:
        assert len(data) == self.k
        return code_rows(self.parity, [np.asarray(d, dtype=np.uint8) for d in data])

    def decode_plan(self, present: Sequence[bool], data_only: bool = False):
        """(survivor indices, output indices, coefficient rows) for an erasure pattern."""
        survivors = [i for i in range(self.n) if present[i]][: self.k]
        if len(survivors) < self.k:
            raise ValueError("too few shards")
        inv = mat_invert([self.matrix[i] for i in survivors])
        outs, rows = [], []
        for i in range(self.n):
            if present[i] or (data_only and i >= self.k):
                continue
            outs.append(i)
            rows.append(inv[i] if i < self.k else mat_mul([self.matrix[i]], inv)[0])
        return survivors, outs, rows

    def reconstruct(self, shards: List[Optional[np.ndarray]], data_only: bool = False):
        """Two-pass klauspost Reconstruct: missing data from inv(sub), then parity re-encoded."""
        present = [s is not None and len(s) > 0 for s in shards]
        if all(present):
            return list(shards)
        survivors = [i for i in range(self.n) if present[i]][: self.k]
        if len(survivors) < self.k:
            raise ValueError("too few shards")
        inv = mat_invert([self.matrix[i] for i in survivors])
        sub = [np.asarray(shards[i], dtype=np.uint8) for i in survivors]
        out = list(shards)
        missing_data = [i for i in range(self.k) if not present[i]]
        for i, v in zip(missing_data, code_rows([inv[i] for i in missing_data], sub)):
            out[i] = v
        if not data_only:
            missing_par = [i for i in range(self.k, self.n) if not present[i]]
            data = [np.asarray(out[i], dtype=np.uint8) for i in range(self.k)]
            rows = [self.matrix[i] for i in missing_par]
            for i, v in zip(missing_par, code_rows(rows, data)):
                out[i] = v
        return out

    def verify(self, shards: Sequence[np.ndarray]) -> bool:
        par = self.encode(shards[: self.k])
        return all(np.array_equal(p, np.asarray(s, dtype=np.uint8))
                   for p, s in zip(par, shards[self.k:]))

    def split(self, data: bytes) -> List[np.ndarray]:
        if len(data) == 0:
            raise ValueError("short data")
        per = (len(data) + self.k - 1) // self.k
        buf = np.zeros(per * self.n, dtype=np.uint8)
        buf[: len(data)] = np.frombuffer(bytes(data), dtype=np.uint8)
        return [buf[i * per:(i + 1) * per].copy() for i in range(self.n)]


# ---------------------------------------------------------------------------------------------
# Hashes, segments, synthetic data
# ---------------------------------------------------------------------------------------------


def sha256_hex(buf) -> bytes:
    """64-byte Hash value: lowercase hex SHA-256 (primitives/common/src/lib.rs:16 width)."""
    return hashlib.sha256(bytes(np.asarray(buf, dtype=np.uint8))).hexdigest().encode()


SEGMENT_SIZE = 16 * 1024 * 1024   # primitives/common/src/lib.rs:60
FRAGMENT_SIZE = 8 * 1024 * 1024   # primitives/common/src/lib.rs:61
FRAGMENT_COUNT = 3                # runtime/src/lib.rs:1027


def segment_list(file_bytes: bytes, k: int = 2, m: int = 1, segment_size: int = SEGMENT_SIZE):
    """[(segment hash, [fragment hashes])] for a file: 16 MiB segments (last zero padded),
    each split into k fragments + m parity, every piece hashed (types.rs:13-16 record)."""
    if len(file_bytes) == 0:
        raise ValueError("short data")
    rs = ReedSolomon(k, m)
    out = []
    nseg = (len(file_bytes) + segment_size - 1) // segment_size
    for s in range(nseg):
        seg = np.zeros(segment_size, dtype=np.uint8)
        chunk = np.frombuffer(file_bytes[s * segment_size:(s + 1) * segment_size], dtype=np.uint8)
        seg[: len(chunk)] = chunk
        shards = rs.split(seg.tobytes())
        shards[k:] = rs.encode(shards[:k])
        out.append((sha256_hex(seg), [sha256_hex(x) for x in shards]))
    return out


def file_hash(segments) -> bytes:
    """[build convention, unpinned] SHA-256 hex over the concatenated hex segment hashes."""
    h = hashlib.sha256()
    for seg_hash, _ in segments:
        h.update(seg_hash)
    return h.hexdigest().encode()


_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x.astype(np.uint64) + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def synthetic_segment(seed: int, seg: int, nbytes: int) -> np.ndarray:
    """Word w (little-endian u64) = splitmix64(seed ^ (seg << 32) ^ w)."""
    assert nbytes % 8 == 0
    w = np.arange(nbytes // 8, dtype=np.uint64)
    words = splitmix64(np.uint64(seed) ^ (np.uint64(seg) << np.uint64(32)) ^ w)
    return words.astype("<u8").view(np.uint8)


# ---- storage audit (c-pallets/audit) -----------------------------------------------------------
def challenge_indices(randoms, chunk_count=1024, need=1024 * 46 // 1000):
    """generation_challenge's chunk selection (c-pallets/audit/src/lib.rs:955-964): for seed =
    1, 2, ..., random_index = random_number(seed) % CHUNK_COUNT, kept if new, until `need`
    indices. `randoms[i]` = random_number(i + 1). Returns (indices, randoms consumed)."""
    out = []
    used = 0
    for r in randoms:
        if len(out) >= need:
            break
        used += 1
        idx = int(r) % chunk_count
        if idx not in out:
            out.append(idx)
    if len(out) < need:
        raise ValueError("random stream exhausted")
    return out, used


def chunk(fragment, index, chunk_count=1024):
    """Chunk `index` of a fragment: CHUNK_COUNT equal chunks (primitives/common/src/lib.rs:62)."""
    n = len(fragment) // chunk_count
    return fragment[index * n:(index + 1) * n]
