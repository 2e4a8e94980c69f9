"""Independent pure-Python restatement of the reference codec, for SMALL
inputs only.  Written separately from oracle/dietgpu_oracle.c (different
structure, Python ints, struct packing) so the two can pin each other.

Citations relative to /root/reference/dietgpu.
"""
import struct

import numpy as np

BLOCK = 4096


def round_up(a, b):
    return (a + b - 1) // b * b


def quantize(count, total, W):
    # ans/GpuANSStatistics.cuh:212-218 in IEEE float32
    r = np.float32(count) / np.float32(total)
    f = np.float32(W) * r
    return int(f)


def normalize(hist, total, pb):
    """normalizeProbabilitiesFromHistogram (ans/GpuANSStatistics.cuh:178-366)"""
    if total == 0:
        return [0] * 256
    W = 1 << pb
    q = []
    for s in range(256):
        v = quantize(hist[s], total, W)
        if hist[s] > 0 and v == 0:
            v = 1
        q.append(v)
    order = sorted(range(256), key=lambda s: (q[s] << 16) | s, reverse=True)
    diff = W - sum(q)
    while diff > 0:
        step = min(diff, 256)
        for s in range(step):
            q[s] += 1
        diff -= step
    d = -diff
    while d > 0:
        g = sum(1 for v in q if v > 1)
        k = min(d, g)
        for r in range(g - k, g):
            q[order[r]] -= 1
        d -= k
    return q


def ans_encode(data, pb=10, checksum=False):
    data = bytes(bytearray(np.asarray(data, dtype=np.uint8)))
    n = len(data)
    hist = [0] * 256
    for b in data:
        hist[b] += 1
    pdf = normalize(hist, n, pb)
    cdf = [0] * 256
    for s in range(1, 256):
        cdf[s] = cdf[s - 1] + pdf[s - 1]
    nb = (n + BLOCK - 1) // BLOCK
    blocks = []
    for b in range(nb):
        chunk = data[b * BLOCK:(b + 1) * BLOCK]
        states = [1 << 15] * 32
        words = []
        for t in range((len(chunk) + 31) // 32):
            for lane in range(32):
                i = 32 * t + lane
                if i >= len(chunk):
                    continue
                s = chunk[i]
                x = states[lane]
                if x >= pdf[s] << (31 - pb):
                    words.append(x & 0xFFFF)
                    x >>= 16
                states[lane] = (x // pdf[s]) * (1 << pb) + x % pdf[s] + cdf[s]
        blocks.append((len(chunk), states, words))
    pre = []
    run = 0
    for (_, _, w) in blocks:
        pre.append(run)
        run += round_up(len(w), 8)
    total = run
    ck = 0
    if checksum:
        for b in data:
            ck ^= b
    out = bytearray()
    out += struct.pack("<8I", 0xD00D0001, nb, n, total, pb | (16 if checksum else 0), ck, 0, 0)
    out += struct.pack("<256H", *pdf)
    for (_, st, _) in blocks:
        out += struct.pack("<32I", *st)
    for b, (uw, _, w) in enumerate(blocks):
        out += struct.pack("<2I", (uw << 16) | len(w), pre[b])
    if nb % 2:
        out += bytes(8)
    for (_, _, w) in blocks:
        out += struct.pack(f"<{len(w)}H", *w) + bytes(2 * (round_up(len(w), 8) - len(w)))
    return np.frombuffer(bytes(out), dtype=np.uint8)


def ans_decode(arch, pb=10):
    a = bytes(np.asarray(arch, dtype=np.uint8))
    magic, nb, n, total, opts, ck, _, _ = struct.unpack_from("<8I", a, 0)
    assert magic == 0xD00D0001 and opts & 0xF == pb
    pdf = struct.unpack_from("<256H", a, 32)
    cdf = [0] * 256
    for s in range(1, 256):
        cdf[s] = cdf[s - 1] + pdf[s - 1]
    lut = []
    for s in range(256):
        lut += [(s, pdf[s], cdf[s])] * pdf[s]
    off_states = 544
    off_bw = off_states + 128 * nb
    off_data = off_bw + 8 * round_up(nb, 2)
    out = bytearray(n)
    for b in range(nb):
        states = list(struct.unpack_from("<32I", a, off_states + 128 * b))
        x0, start = struct.unpack_from("<2I", a, off_bw + 8 * b)
        uw, cw = x0 >> 16, x0 & 0xFFFF
        words = struct.unpack_from(f"<{cw}H", a, off_data + 2 * start)
        ptr = cw
        for t in reversed(range((uw + 31) // 32)):
            for lane in reversed(range(32)):
                i = 32 * t + lane
                if i >= uw:
                    continue
                x = states[lane]
                s, p, c = lut[x & ((1 << pb) - 1)]
                out[b * BLOCK + i] = s
                x = p * (x >> pb) + (x & ((1 << pb) - 1)) - c
                if x < (1 << 15):
                    ptr -= 1
                    x = (x << 16) + words[ptr]
                states[lane] = x
    return np.frombuffer(bytes(out), dtype=np.uint8)


def _rotl(v, s, bits):
    m = (1 << bits) - 1
    return ((v << s) | (v >> (bits - s))) & m


def float_split(ft, words):
    """(comp0 bytes, comp1 bytes, raw section bytes) per float/GpuFloatUtils.cuh."""
    n = len(words)
    c0 = bytearray(n)
    c1 = bytearray(n)
    if ft in (1, 2):
        raw = bytearray(round_up(n, 16))
        for i, w in enumerate(int(v) for v in words):
            if ft == 1:
                c0[i], raw[i] = w >> 8, w & 0xFF
            else:
                v = _rotl((w << 16) | w, 1, 32)
                c0[i], raw[i] = v >> 24, v & 0xFF
    elif ft == 3:
        lo = bytearray(2 * round_up(n, 8))
        hi = bytearray(round_up(n, 16))
        for i, w in enumerate(int(v) for v in words):
            v = _rotl(w, 1, 32)
            c0[i] = v >> 24
            struct.pack_into("<H", lo, 2 * i, v & 0xFFFF)
            hi[i] = (v >> 16) & 0xFF
        raw = lo + hi
    else:
        lo = bytearray(4 * round_up(n, 4))
        hi = bytearray(2 * round_up(n, 8))
        for i, w in enumerate(int(v) for v in words):
            v = _rotl(w, 1, 64)
            c0[i] = v >> 56
            c1[i] = (v >> 48) & 0xFF
            struct.pack_into("<I", lo, 4 * i, v & 0xFFFFFFFF)
            struct.pack_into("<H", hi, 2 * i, (v >> 32) & 0xFFFF)
        raw = lo + hi
    return bytes(c0), bytes(c1), bytes(raw)


def float_compress(ft, words, pb=10, checksum=False, word_bytes=None):
    c0, c1, raw = float_split(ft, words)
    n = len(words)
    a1 = ans_encode(np.frombuffer(c0, np.uint8), pb).tobytes()
    ck = 0
    if checksum:
        for b in word_bytes[:n]:
            ck ^= b
    out = struct.pack("<4I", 0xF00F0001, n, ft | (16 if checksum else 0), ck)
    out += struct.pack("<4I", round_up(len(a1), 16), 0, 0, 0)
    out += raw + a1
    if ft == 4:
        out += bytes(round_up(len(a1), 16) - len(a1))
        out += ans_encode(np.frombuffer(c1, np.uint8), pb).tobytes()
    return np.frombuffer(out, dtype=np.uint8)
