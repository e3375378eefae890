"""Hand-built zlib streams whose dynamic Huffman block is invalid in ways
zlib's inflate_table / inflate reject before any data is decoded:
over-subscribed or incomplete code-length sets and a literal/length set with
no end-of-block code.  Used by tests/test_inflate_gpu.py (the GPU inflate
must reject each) and tests/test_deflate.py (zlib itself rejects each, with
the message named here)."""


class _Bits:
    """RFC 1951 bit packing: fields LSB first, Huffman codes MSB first."""

    def __init__(self):
        self.acc, self.n, self.out = 0, 0, bytearray()

    def put(self, v, n):
        self.acc |= v << self.n
        self.n += n
        while self.n >= 8:
            self.out.append(self.acc & 255)
            self.acc >>= 8
            self.n -= 8

    def code(self, c, n):   # a Huffman code, its first bit first
        for i in range(n - 1, -1, -1):
            self.put((c >> i) & 1, 1)

    def bytes(self):
        return bytes(self.out) + (bytes([self.acc & 255]) if self.n else b"")


_CLEN_ORDER = (16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15)


def _canonical(lengths):
    """symbol -> (code, length) for a canonical code (RFC 1951 3.2.2)."""
    mx = max(lengths.values())
    bl = [0] * (mx + 1)
    for L in lengths.values():
        bl[L] += 1
    code, nxt = 0, [0] * (mx + 2)
    for b in range(1, mx + 1):
        code = (code + bl[b - 1]) << 1 if b > 1 else 0
        nxt[b] = code
    out = {}
    for s in sorted(lengths):
        L = lengths[s]
        out[s] = (nxt[L], L)
        nxt[L] += 1
    return out


def dynamic_stream(clen, litlen, dist, tail=64):
    """A zlib stream with one final dynamic block: code-length code lengths
    `clen` {symbol: length}, literal/length lengths `litlen` (257 entries) and
    distance lengths `dist`, run-length coded with symbols 0..15 and 18, then
    `tail` zero bytes (so a decoder that accepts the trees does not overrun)."""
    b = _Bits()
    b.put(0x78, 8)
    b.put(0x9C, 8)
    b.put(1, 1)      # BFINAL
    b.put(2, 2)      # BTYPE dynamic
    b.put(len(litlen) - 257, 5)
    b.put(len(dist) - 1, 5)
    b.put(19 - 4, 4)  # all 19 code-length code lengths
    for s in _CLEN_ORDER:
        b.put(clen.get(s, 0), 3)
    codes = _canonical({s: L for s, L in clen.items() if L})
    seq = list(litlen) + list(dist)
    i = 0
    while i < len(seq):
        v = seq[i]
        run = 1
        while i + run < len(seq) and seq[i + run] == v:
            run += 1
        if v == 0 and run >= 11 and 18 in codes:
            r = min(run, 138)
            b.code(*codes[18])
            b.put(r - 11, 7)
            i += r
            continue
        b.code(*codes[v])
        i += 1
    return b.bytes() + bytes(tail)


def _lens(ones):
    a = [0] * 257
    for s, L in ones.items():
        a[s] = L
    return a


# (name, stream, zlib's message, the GPU inflate's status code)
CASES = [
    ("clen_oversubscribed", dynamic_stream({18: 1, 0: 1, 1: 1}, _lens({0: 1, 256: 1}), [1]),
     "invalid code lengths set", -8),
    ("clen_incomplete", dynamic_stream({18: 1}, [0] * 257, [0]), "invalid code lengths set", -8),
    ("litlen_oversubscribed", dynamic_stream({18: 1, 0: 2, 1: 2}, _lens({0: 1, 1: 1, 256: 1}), [1]),
     "invalid literal/lengths set", -8),
    ("litlen_incomplete", dynamic_stream({18: 1, 1: 2, 2: 2}, _lens({0: 2, 256: 2}), [1]),
     "invalid literal/lengths set", -8),
    ("missing_eob", dynamic_stream({18: 1, 0: 2, 1: 2}, _lens({0: 1, 1: 1}), [1]),
     "invalid code -- missing end-of-block", -9),
]
