"""Shared deflate test inputs (CPU harness and GPU kernel tests)."""
import numpy as np


def slide_nil_strip(n: int = 65400, seed: int = 3) -> bytes:
    """A strip where zlib's slide_hash NIL mapping decides the output.

    zlib 1.2.11 slides the window once, at the first deflate_slow step with
    strstart >= wsize + MAX_DIST = 65274, and slide_hash turns a head entry
    equal to wsize (input position 32768) into NIL.  Here the same 8 bytes
    sit at 32768 and 65274, no position in between shares their hash, and
    unique bytes before 65274 make the parse reach it as a fresh position:
    zlib emits a literal there (and matches from 65275 on), a matcher that
    treats 32768 as a live head emits a match of 8 at distance MAX_DIST.
    The background is a 16-symbol alphabet so the blocks are Huffman coded
    (a stored block would hide the difference)."""
    rng = np.random.default_rng(seed)
    a = rng.integers(0, 16, n, dtype=np.uint8)
    a[65266:65274] = np.arange(240, 248)
    a[32760:32768] = np.arange(224, 232)
    pat = np.array([101, 99, 120, 105, 110, 103, 117, 107], np.uint8)
    a[32768:32776] = pat
    a[65274:65282] = pat

    def hashes(x):
        b = x.astype(np.int64)
        return (((b[:-2] & 31) << 10) ^ (b[1:-1] << 5) ^ b[2:]) & 0x7fff

    for _ in range(100):
        h = hashes(a)
        bad = [q for q in np.nonzero(h == h[32768])[0] if 32768 < q < 65274]
        if not bad:
            break
        for q in bad:
            a[q + 2 if q + 2 < 65266 and not (32768 <= q + 2 < 32776) else q - 1] ^= 0x5
    else:
        raise AssertionError("could not isolate the planted hash")
    return a.tobytes()
