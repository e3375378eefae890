"""Diagnostic: a zlib stream (RFC 1950/1951) as its LZ77 tokens, to locate the
first parse decision where two encoders of the same input differ.
tokens(stream) -> list of (position, length, distance) with length 0 for a
literal (distance = the byte), and the block boundaries (positions)."""
from __future__ import annotations

_LBASE = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195,
          227, 258]
_LEXT = [0] * 8 + [1] * 4 + [2] * 4 + [3] * 4 + [4] * 4 + [5] * 4 + [0]
_DBASE = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073,
          4097, 6145, 8193, 12289, 16385, 24577]
_DEXT = [0, 0, 0, 0] + [i // 2 for i in range(2, 28)]
_ORDER = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]


class _Bits:
    def __init__(self, data: bytes):
        self.d, self.pos = data, 0

    def get(self, n: int) -> int:
        v = 0
        for i in range(n):
            byte = self.d[self.pos >> 3]
            v |= ((byte >> (self.pos & 7)) & 1) << i
            self.pos += 1
        return v


def _decoder(lengths):
    codes, code = {}, 0
    bl = [0] * 16
    for l in lengths:
        if l:
            bl[l] += 1
    nxt, code = [0] * 16, 0
    for b in range(1, 16):
        code = (code + bl[b - 1]) << 1
        nxt[b] = code
    for s, l in enumerate(lengths):
        if l:
            codes[(l, nxt[l])] = s
            nxt[l] += 1
    return codes


def _sym(bits: _Bits, dec) -> int:
    code = 0
    for l in range(1, 16):
        code = (code << 1) | bits.get(1)
        s = dec.get((l, code))
        if s is not None:
            return s
    raise ValueError("bad code")


def tokens(stream: bytes):
    bits = _Bits(stream[2:])
    out, toks, blocks = bytearray(), [], []
    while True:
        final = bits.get(1)
        kind = bits.get(2)
        blocks.append((len(out), kind))
        if kind == 0:
            bits.pos = (bits.pos + 7) & ~7
            n = bits.get(16)
            bits.get(16)
            for _ in range(n):
                b = bits.get(8)
                toks.append((len(out), 0, b))
                out.append(b)
        else:
            if kind == 1:
                ll = [8] * 144 + [9] * 112 + [7] * 24 + [8] * 8
                dl = [5] * 30
            else:
                hlit, hdist, hclen = bits.get(5) + 257, bits.get(5) + 1, bits.get(4) + 4
                cl = [0] * 19
                for i in range(hclen):
                    cl[_ORDER[i]] = bits.get(3)
                cdec = _decoder(cl)
                lens = []
                while len(lens) < hlit + hdist:
                    s = _sym(bits, cdec)
                    if s < 16:
                        lens.append(s)
                    elif s == 16:
                        lens += [lens[-1]] * (3 + bits.get(2))
                    elif s == 17:
                        lens += [0] * (3 + bits.get(3))
                    else:
                        lens += [0] * (11 + bits.get(7))
                ll, dl = lens[:hlit], lens[hlit:]
            ldec, ddec = _decoder(ll), _decoder(dl)
            while True:
                s = _sym(bits, ldec)
                if s < 256:
                    toks.append((len(out), 0, s))
                    out.append(s)
                elif s == 256:
                    break
                else:
                    i = s - 257
                    ln = _LBASE[i] + bits.get(_LEXT[i])
                    ds = _sym(bits, ddec)
                    dist = _DBASE[ds] + bits.get(_DEXT[ds])
                    toks.append((len(out), ln, dist))
                    for _ in range(ln):
                        out.append(out[-dist])
        if final:
            break
    return toks, blocks, bytes(out)


def first_divergence(a: bytes, b: bytes):
    """(index, token of a, token of b, context) of the first differing token."""
    ta, ba, oa = tokens(a)
    tb, bb, ob = tokens(b)
    for i, (x, y) in enumerate(zip(ta, tb)):
        if x != y:
            return {"token": i, "a": x, "b": y, "prev": ta[max(0, i - 3):i], "blocks_a": ba[:6], "blocks_b": bb[:6],
                    "a_inflates_to_b": oa == ob}
    return {"token": None, "len_a": len(ta), "len_b": len(tb), "blocks_a": ba, "blocks_b": bb,
            "a_inflates_to_b": oa == ob}
