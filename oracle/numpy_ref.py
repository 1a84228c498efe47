"""numpy restatement of the reference codec -- TEST INFRASTRUCTURE ONLY.

The twin of oracle/rs_oracle.c, written independently so the two check each
other.  Used to generate the golden fixtures (tests/golden/make_golden.py) and
by the CPU tests.  Never imported by the product package.

Follows (paths under /root/reference/src/main/java/edu/cmu/):
  reedsolomon/Galois.java:258-305   log/exp/multiplication tables, poly 29
  reedsolomon/Galois.java:198-253   multiply / divide / exp
  reedsolomon/Matrix.java:191-344   times / invert (Gauss-Jordan, same pivot rule)
  reedsolomon/ReedSolomon.java:312-343  buildMatrix / vandermonde
  reedsolomon/ReedSolomon.java:90-104   encodeParity
  reedsolomon/ReedSolomon.java:175-272  decodeMissing (first-k-present survivors)
  reedsolomon/InputOutputByteTableCodingLoop.java:12-44  the coding loop
  reedsolomonfs/client/ReedSolomonEncoder.java:56-85, ReedSolomonDecoder.java:62-103 layout
"""
from __future__ import annotations

import numpy as np

FIELD_SIZE = 256
GENERATING_POLYNOMIAL = 29  # Galois.java:42


def generate_log_table(polynomial: int = GENERATING_POLYNOMIAL) -> np.ndarray:
    """Galois.java:258-275."""
    result = np.full(FIELD_SIZE, -1, dtype=np.int16)
    b = 1
    for log in range(FIELD_SIZE - 1):
        if result[b] != -1:
            raise RuntimeError("BUG: duplicate logarithm (bad polynomial?)")
        result[b] = log
        b <<= 1
        if b >= FIELD_SIZE:
            b = (b - FIELD_SIZE) ^ polynomial
    return result


def generate_exp_table(log_table: np.ndarray) -> np.ndarray:
    """Galois.java:280-288: 510 entries, two copies of the 255-cycle."""
    result = np.zeros(FIELD_SIZE * 2 - 2, dtype=np.uint8)
    for i in range(1, FIELD_SIZE):
        log = int(log_table[i])
        result[log] = i
        result[log + FIELD_SIZE - 1] = i
    return result


LOG_TABLE = generate_log_table()
EXP_TABLE = generate_exp_table(LOG_TABLE)


def gal_multiply(a: int, b: int) -> int:
    """Galois.java:198-208."""
    if a == 0 or b == 0:
        return 0
    return int(EXP_TABLE[int(LOG_TABLE[a]) + int(LOG_TABLE[b])])


def gal_divide(a: int, b: int) -> int:
    """Galois.java:213-227."""
    if a == 0:
        return 0
    if b == 0:
        raise ValueError("Argument 'divisor' is 0")
    r = int(LOG_TABLE[a]) - int(LOG_TABLE[b])
    if r < 0:
        r += 255
    return int(EXP_TABLE[r])


def gal_exp(a: int, n: int) -> int:
    """Galois.java:238-253."""
    if n == 0:
        return 1
    if a == 0:
        return 0
    r = int(LOG_TABLE[a]) * n
    while r >= 255:
        r -= 255
    return int(EXP_TABLE[r])


def generate_multiplication_table() -> np.ndarray:
    """Galois.java:297-305: MUL[a][b]."""
    t = np.zeros((FIELD_SIZE, FIELD_SIZE), dtype=np.uint8)
    for a in range(FIELD_SIZE):
        for b in range(FIELD_SIZE):
            t[a, b] = gal_multiply(a, b)
    return t


MUL_TABLE = generate_multiplication_table()


def matrix_times(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """Matrix.java:191-208."""
    rows, n = a.shape
    n2, cols = b.shape
    if n != n2:
        raise ValueError(f"Columns on left ({n}) is different than rows on right ({n2})")
    out = np.zeros((rows, cols), dtype=np.uint8)
    for r in range(rows):
        for c in range(cols):
            v = 0
            for i in range(n):
                v ^= int(MUL_TABLE[a[r, i], b[i, c]])
            out[r, c] = v
    return out


def matrix_invert(m: np.ndarray) -> np.ndarray:
    """Matrix.java:271-344 (augment with I, gaussianElimination, right half)."""
    n = m.shape[0]
    if m.shape[1] != n:
        raise ValueError("Only square matrices can be inverted")
    w = np.concatenate([m.astype(np.uint8), np.eye(n, dtype=np.uint8)], axis=1)
    cols = 2 * n
    for r in range(n):
        if w[r, r] == 0:
            for below in range(r + 1, n):
                if w[below, r] != 0:
                    w[[r, below]] = w[[below, r]]
                    break
        if w[r, r] == 0:
            raise ValueError("Matrix is singular")
        if w[r, r] != 1:
            scale = gal_divide(1, int(w[r, r]))
            w[r] = MUL_TABLE[w[r], scale]
        for below in range(r + 1, n):
            if w[below, r] != 0:
                scale = int(w[below, r])
                w[below] ^= MUL_TABLE[scale, w[r]]
    for d in range(n):
        for above in range(d):
            if w[above, d] != 0:
                scale = int(w[above, d])
                w[above] ^= MUL_TABLE[scale, w[d]]
    assert cols == w.shape[1]
    return w[:, n:].copy()


def vandermonde(rows: int, cols: int) -> np.ndarray:
    """ReedSolomon.java:335-343: V[r][c] = exp(r, c)."""
    v = np.zeros((rows, cols), dtype=np.uint8)
    for r in range(rows):
        for c in range(cols):
            v[r, c] = gal_exp(r & 0xFF, c)
    return v


def build_matrix(k: int, total: int) -> np.ndarray:
    """ReedSolomon.java:312-324."""
    v = vandermonde(total, k)
    return matrix_times(v, matrix_invert(v[:k, :k]))


def code_some_shards(rows: np.ndarray, inputs: list, outputs: list, offset: int, byte_count: int) -> None:
    """InputOutputByteTableCodingLoop.java:12-44 (vectorised over the byte loop).

    rows: (n_out, n_in) uint8; inputs/outputs: lists of 1-D uint8 arrays (written in place).
    """
    n_out, n_in = rows.shape
    sl = slice(offset, offset + byte_count)
    for o in range(n_out):
        outputs[o][sl] = MUL_TABLE[rows[o, 0]][inputs[0][sl]]
    for i in range(1, n_in):
        for o in range(n_out):
            outputs[o][sl] ^= MUL_TABLE[rows[o, i]][inputs[i][sl]]


class ReedSolomonRef:
    """ReedSolomon.java:13-344 restated (default coding loop only)."""

    def __init__(self, k: int, m: int):
        if 256 < k + m:
            raise ValueError("too many shards - max is 256")
        self.k, self.m, self.total = k, m, k + m
        self.matrix = build_matrix(k, self.total)
        self.parity_rows = self.matrix[k:]

    def _check(self, shards, offset, byte_count):
        """ReedSolomon.java:277-302."""
        if len(shards) != self.total:
            raise ValueError(f"wrong number of shards: {len(shards)}")
        n = len(shards[0])
        if any(len(s) != n for s in shards[1:]):
            raise ValueError("Shards are different sizes")
        if offset < 0:
            raise ValueError(f"offset is negative: {offset}")
        if byte_count < 0:
            raise ValueError(f"byteCount is negative: {byte_count}")
        if n < offset + byte_count:
            raise ValueError(f"buffers to small: {byte_count}{offset}")

    def encode_parity(self, shards, offset, byte_count):
        """ReedSolomon.java:90-104."""
        self._check(shards, offset, byte_count)
        code_some_shards(self.parity_rows, shards[: self.k], shards[self.k:], offset, byte_count)

    def is_parity_correct(self, shards, offset, byte_count) -> bool:
        """ReedSolomon.java:115-130 (CodingLoopBase.java:17-41 semantics)."""
        self._check(shards, offset, byte_count)
        tmp = [np.zeros(len(shards[0]), dtype=np.uint8) for _ in range(self.m)]
        code_some_shards(self.parity_rows, shards[: self.k], tmp, offset, byte_count)
        sl = slice(offset, offset + byte_count)
        return all(np.array_equal(tmp[p][sl], shards[self.k + p][sl]) for p in range(self.m))

    def survivors(self, present):
        return [i for i in range(self.total) if present[i]][: self.k]

    def decode_missing(self, shards, present, offset, byte_count):
        """ReedSolomon.java:175-272: two codeSomeShards passes."""
        self._check(shards, offset, byte_count)
        n_present = sum(1 for i in range(self.total) if present[i])
        if n_present == self.total:
            return
        if n_present < self.k:
            raise ValueError("Not enough shards present")
        surv = self.survivors(present)
        sub = self.matrix[surv]
        dec = matrix_invert(sub)
        miss_d = [i for i in range(self.k) if not present[i]]
        if miss_d:
            code_some_shards(dec[miss_d], [shards[s] for s in surv], [shards[i] for i in miss_d],
                             offset, byte_count)
        miss_p = [i for i in range(self.k, self.total) if not present[i]]
        if miss_p:
            code_some_shards(self.parity_rows[[i - self.k for i in miss_p]], shards[: self.k],
                             [shards[i] for i in miss_p], offset, byte_count)

    def decode_rows(self, present):
        """The single matrix that maps survivors to each missing shard (ascending)."""
        surv = self.survivors(present)
        dec = matrix_invert(self.matrix[surv])
        rows, missing = [], []
        for j in range(self.total):
            if present[j]:
                continue
            rows.append(dec[j] if j < self.k else matrix_times(self.parity_rows[j - self.k][None, :], dec)[0])
            missing.append(j)
        return surv, missing, np.array(rows, dtype=np.uint8).reshape(len(missing), self.k)


# ---------------- client layout (ReedSolomonEncoder/Decoder) ----------------

def padded_size(file_len: int, k: int = 4, block: int = 1000) -> int:
    """ReedSolomonEncoder.java:76-85."""
    mult = k * block
    return file_len if file_len % mult == 0 else file_len // mult * mult + mult


def split_file(data: bytes, k: int, m: int, block: int = 1000) -> np.ndarray:
    """ReedSolomonEncoder.java:62-74 after pad(): returns (k+m, S) with parity zero."""
    padded = padded_size(len(data), k, block)
    buf = np.zeros(padded, dtype=np.uint8)
    buf[: len(data)] = np.frombuffer(bytes(data), dtype=np.uint8)
    S = padded // k
    shards = np.zeros((k + m, S), dtype=np.uint8)
    # block b -> shard b % k, offset (b // k) * block
    blocks = buf.reshape(-1, block) if padded else buf.reshape(0, block)
    for b in range(blocks.shape[0]):
        shards[b % k, (b // k) * block:(b // k + 1) * block] = blocks[b]
    return shards


def merge_file(shards: np.ndarray, k: int, file_size: int, block: int = 1000) -> bytes:
    """ReedSolomonDecoder.java:92-103 + trimPadding :62-66."""
    S = shards.shape[1]
    out = np.zeros(S * k, dtype=np.uint8)
    for b in range(S * k // block):
        out[b * block:(b + 1) * block] = shards[b % k, (b // k) * block:(b // k + 1) * block]
    return out[:file_size].tobytes()


# ---------------- synthetic data (same definition as the device fill) ----------------

_GAMMA = np.uint64(0x9E3779B97F4A7C15)


def splitmix64_words(seed: int, first: int, count: int) -> np.ndarray:
    """Outputs first..first+count-1 (1-based) of splitmix64 seeded with `seed`."""
    n = np.arange(first, first + count, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + n * _GAMMA
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def synthetic_stripe(seed: int, stripe: int, k: int, S: int) -> np.ndarray:
    """The k data shards of one synthetic stripe, shape (k, S); S % 8 == 0."""
    assert S % 8 == 0
    words = splitmix64_words(seed ^ stripe, 1, k * S // 8)
    return words.view(np.uint8).reshape(k, S).copy()
