"""Minimal FLAC *encoder* used only by the tests to make fixture files for the native reader
(robust-audio-deepfake-evolution_amd/csrc/flac.cpp). Test infrastructure, never shipped.

soundfile/libsndfile and the `flac` tool are absent from this image and the reference ships no
.flac files, so the reader is pinned by round trips through an independent, spec-driven encoder
that can emit every subframe type the reader handles: CONSTANT, VERBATIM, FIXED 0..4, LPC (with
quantised coefficients), wasted bits, Rice / Rice2 with partitions and escaped partitions, and
independent / left-side / right-side / mid-side stereo.
"""
import numpy as np


class BitWriter:
    def __init__(self):
        self.buf = bytearray()
        self.acc = 0
        self.nacc = 0

    def write(self, value, nbits):
        if nbits == 0:
            return
        self.acc = (self.acc << nbits) | (int(value) & ((1 << nbits) - 1))
        self.nacc += nbits
        while self.nacc >= 8:
            self.nacc -= 8
            self.buf.append((self.acc >> self.nacc) & 0xFF)
        self.acc &= (1 << self.nacc) - 1

    def write_signed(self, value, nbits):
        self.write(int(value) & ((1 << nbits) - 1), nbits)

    def unary(self, q):
        while q >= 32:
            self.write(0, 32)
            q -= 32
        self.write(1, q + 1)

    def align(self):
        if self.nacc:
            self.write(0, 8 - self.nacc)

    def bytes(self):
        assert self.nacc == 0
        return bytes(self.buf)


def crc8(data):
    c = 0
    for b in data:
        c ^= b
        for _ in range(8):
            c = ((c << 1) ^ 0x07) & 0xFF if c & 0x80 else (c << 1) & 0xFF
    return c


def crc16(data):
    c = 0
    for b in data:
        c ^= b << 8
        for _ in range(8):
            c = ((c << 1) ^ 0x8005) & 0xFFFF if c & 0x8000 else (c << 1) & 0xFFFF
    return c


def utf8_num(n):
    if n < 0x80:
        return bytes([n])
    out = []
    nbytes = 2
    while n >= (1 << (5 * nbytes + 1)):
        nbytes += 1
    for _ in range(nbytes - 1):
        out.append(0x80 | (n & 0x3F))
        n >>= 6
    lead = ((0xFF << (8 - nbytes)) & 0xFF) | n
    return bytes([lead] + out[::-1])


FIXED = {0: [], 1: [1], 2: [2, -1], 3: [3, -3, 1], 4: [4, -6, 4, -1]}


def _rice(bw, res, order, bs, porder, method=0, escape_bits=None):
    bw.write(method, 2)
    bw.write(porder, 4)
    parts = 1 << porder
    esc = 15 if method == 0 else 31
    pbits = 4 if method == 0 else 5
    i = 0
    for p in range(parts):
        cnt = (bs >> porder) - (order if p == 0 else 0)
        seg = res[i:i + cnt]
        i += cnt
        if escape_bits is not None:
            bw.write(esc, pbits)
            bw.write(escape_bits, 5)
            for v in seg:
                bw.write_signed(v, escape_bits)
            continue
        u = [(2 * v) if v >= 0 else (-2 * v - 1) for v in seg]
        mean = (sum(u) / max(1, len(u)))
        k = max(0, min(esc - 1, int(np.floor(np.log2(mean + 1))) if mean > 0 else 0))
        bw.write(k, pbits)
        for x in u:
            bw.unary(x >> k)
            bw.write(x & ((1 << k) - 1), k)


def _subframe(bw, x, bps, kind, bs, porder=0, method=0, wasted=0, lpc=None, escape_bits=None):
    x = [int(v) for v in x]
    if wasted:
        assert all(v % (1 << wasted) == 0 for v in x)
        x = [v >> wasted for v in x]
    sbps = bps - wasted
    bw.write(0, 1)
    if kind == "constant":
        bw.write(0, 6)
    elif kind == "verbatim":
        bw.write(1, 6)
    elif kind.startswith("fixed"):
        bw.write(8 + int(kind[5:]), 6)
    elif kind == "lpc":
        bw.write(32 + len(lpc[0]) - 1, 6)
    if wasted:
        bw.write(1, 1)
        bw.unary(wasted - 1)
    else:
        bw.write(0, 1)
    if kind == "constant":
        bw.write_signed(x[0], sbps)
        return
    if kind == "verbatim":
        for v in x:
            bw.write_signed(v, sbps)
        return
    if kind.startswith("fixed"):
        order = int(kind[5:])
        co = FIXED[order]
        for v in x[:order]:
            bw.write_signed(v, sbps)
        res = [x[i] - sum(c * x[i - 1 - j] for j, c in enumerate(co)) for i in range(order, bs)]
        _rice(bw, res, order, bs, porder, method, escape_bits)
        return
    coefs, prec, shift = lpc
    order = len(coefs)
    for v in x[:order]:
        bw.write_signed(v, sbps)
    bw.write(prec - 1, 4)
    bw.write_signed(shift, 5)
    for c in coefs:
        bw.write_signed(c, prec)
    res = [x[i] - (sum(c * x[i - 1 - j] for j, c in enumerate(coefs)) >> shift) for i in range(order, bs)]
    _rice(bw, res, order, bs, porder, method, escape_bits)


def lpc_coefs(x, order, prec=12):
    """Least-squares predictor, quantised to `prec` bits with a shift (any coefficients are legal)."""
    x = np.asarray(x, dtype=np.float64)
    if len(x) <= order + 1:
        return [0] * order, prec, 0
    A = np.stack([x[order - 1 - j:len(x) - 1 - j] for j in range(order)], axis=1)
    a, *_ = np.linalg.lstsq(A, x[order:], rcond=None)
    cmax = max(1e-9, float(np.abs(a).max()))
    shift = max(0, min(15, prec - 1 - int(np.ceil(np.log2(cmax + 1e-12))) - 1))
    q = np.clip(np.round(a * (1 << shift)), -(1 << (prec - 1)), (1 << (prec - 1)) - 1).astype(int)
    return [int(c) for c in q], prec, shift


def encode(samples, sample_rate=16000, bps=16, blocksize=4096, plan=None, stereo_mode="independent"):
    """samples: int array [n] (mono) or [n, 2]. plan(frame_idx, ch, block) -> dict of subframe
    options (kind, porder, method, wasted, lpc_order, escape_bits). Returns the .flac bytes."""
    s = np.asarray(samples, dtype=np.int64)
    if s.ndim == 1:
        s = s[:, None]
    n, nch = s.shape
    out = bytearray(b"fLaC")
    si = BitWriter()
    si.write(blocksize, 16)
    si.write(blocksize, 16)
    si.write(0, 24)
    si.write(0, 24)
    si.write(sample_rate, 20)
    si.write(nch - 1, 3)
    si.write(bps - 1, 5)
    si.write(n, 36)
    si.write(0, 128)
    body = si.bytes()
    out += bytes([0x80 | 0]) + len(body).to_bytes(3, "big") + body
    for fi, start in enumerate(range(0, n, blocksize)):
        blk = s[start:start + blocksize]
        bs = blk.shape[0]
        fw = BitWriter()
        fw.write(0xFFF8 >> 1, 15)
        fw.write(0, 1)
        if bs == 4096:
            fw.write(12, 4)
            tail_bs = None
        elif bs <= 256:
            fw.write(6, 4)
            tail_bs = (bs - 1, 8)
        else:
            fw.write(7, 4)
            tail_bs = (bs - 1, 16)
        fw.write(5 if sample_rate == 16000 else 0, 4)
        chans = [blk[:, c] for c in range(nch)]
        extra = [0] * nch
        if nch == 2 and stereo_mode != "independent":
            L, R = chans
            if stereo_mode == "left_side":
                code, chans, extra = 8, [L, L - R], [0, 1]
            elif stereo_mode == "right_side":
                code, chans, extra = 9, [L - R, R], [1, 0]
            else:
                code, chans, extra = 10, [(L + R) >> 1, L - R], [0, 1]
        else:
            code = nch - 1
        fw.write(code, 4)
        fw.write({8: 1, 12: 2, 16: 4, 20: 5, 24: 6}[bps], 3)
        fw.write(0, 1)
        for b in utf8_num(fi):
            fw.write(b, 8)
        if tail_bs:
            fw.write(*tail_bs)
        head = fw.bytes()
        fw.write(crc8(head), 8)
        for c, x in enumerate(chans):
            opt = dict(plan(fi, c, x) if plan else {"kind": "fixed2"})
            kind = opt.pop("kind")
            lpc = None
            if kind == "lpc":
                lpc = lpc_coefs(x, opt.pop("lpc_order", 8), opt.pop("prec", 12))
            _subframe(fw, x, bps + extra[c], kind, bs, lpc=lpc, **opt)
        fw.align()
        frame = fw.bytes()
        out += frame + crc16(frame).to_bytes(2, "big")
    return bytes(out)
