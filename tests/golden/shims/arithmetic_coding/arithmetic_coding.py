"""A8: the un-vendored arithmetic_coding package's coder, as SURVEY.md's
assumption A8 states it and vcf_amd/csrc/vcf_cbaac.cpp implements it: a
32-bit Witten-Neal-Cleary integer coder with pending (underflow) bits, bits
appended MSB-first to a bitarray(endian='big'), flush = one more pending bit
and a disambiguating bit; the decoder reads zeros past the end.  Interface
as CBAAC.py:115-150 calls it: Arithmetic_Encoding().encode_symbol(symbol,
model, output) / .flush(output); Arithmetic_Decoding().start(bits) /
.decode_symbol(model), with model.get_range(s) -> (low, high, total) and
model.get_symbol_from_scaled_value(v) -> (s, low, high)."""

HALF, Q1, Q3, MASK = 0x80000000, 0x40000000, 0xC0000000, 0xFFFFFFFF


class Arithmetic_Coding:
    MAX = MASK


class Arithmetic_Encoding(Arithmetic_Coding):
    def __init__(self):
        self.low, self.high, self.pending = 0, MASK, 0

    def _emit(self, bit, output):
        output.append(bit)
        for _ in range(self.pending):
            output.append(1 - bit)
        self.pending = 0

    def encode_symbol(self, symbol, model, output):
        lo, hi, tot = model.get_range(symbol)
        rng = self.high - self.low + 1
        self.high = self.low + (rng * hi) // tot - 1
        self.low = self.low + (rng * lo) // tot
        while True:
            if self.high < HALF:
                self._emit(0, output)
            elif self.low >= HALF:
                self._emit(1, output)
                self.low -= HALF
                self.high -= HALF
            elif self.low >= Q1 and self.high < Q3:
                self.pending += 1
                self.low -= Q1
                self.high -= Q1
            else:
                break
            self.low = (self.low << 1) & MASK
            self.high = ((self.high << 1) | 1) & MASK

    def flush(self, output):
        self.pending += 1
        self._emit(0 if self.low < Q1 else 1, output)


class Arithmetic_Decoding(Arithmetic_Coding):
    def start(self, bits):
        self.bits, self.pos = bits, 0
        self.low, self.high, self.value = 0, MASK, 0
        for _ in range(32):
            self.value = (self.value << 1) | self._bit()

    def _bit(self):
        b = int(self.bits[self.pos]) if self.pos < len(self.bits) else 0
        self.pos += 1
        return b

    def decode_symbol(self, model):
        rng = self.high - self.low + 1
        tot = model.total
        scaled = ((self.value - self.low + 1) * tot - 1) // rng
        s, lo, hi = model.get_symbol_from_scaled_value(scaled)
        self.high = self.low + (rng * hi) // tot - 1
        self.low = self.low + (rng * lo) // tot
        while True:
            if self.high < HALF:
                pass
            elif self.low >= HALF:
                self.low -= HALF
                self.high -= HALF
                self.value -= HALF
            elif self.low >= Q1 and self.high < Q3:
                self.low -= Q1
                self.high -= Q1
                self.value -= Q1
            else:
                break
            self.low = (self.low << 1) & MASK
            self.high = ((self.high << 1) | 1) & MASK
            self.value = ((self.value << 1) | self._bit()) & MASK
        return s
