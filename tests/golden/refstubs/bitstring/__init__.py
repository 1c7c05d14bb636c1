"""Minimal stand-in for the third-party ``bitstring`` package (unpinned in the
reference: run_savio.sh:38 ``pip-3.2 install bitstring``), written from its
published semantics so that the reference game modules
(toot_and_otto_bitstring.py, othello_bit_new.py) import in THIS container to
generate golden fixtures.  Test infrastructure only; never shipped, never run
on the GPU box.

Semantics relied on by the reference (SURVEY.md §8c row "Third-party"):
  * MSB-first bit order; ``.bytes`` get/set packs bit 0 into the MSB of byte 0.
  * ``.int`` is signed two's complement over the bitstring's length.
  * ``s[a:b] = <int>`` stores the int as uint (>=0) or int (<0) of width b-a.
  * ``s[a:b] = <BitArray>`` splices (here always equal width).
"""


class BitArray:
    __slots__ = ("_v", "_n")  # value as python int (bit 0 = MSB), length

    def __init__(self, auto=None):
        self._v = 0
        self._n = 0
        if auto is None:
            return
        if isinstance(auto, BitArray):
            self._v, self._n = auto._v, auto._n
        elif isinstance(auto, str):
            if not auto.startswith("0b"):
                raise ValueError("only '0b...' literals are supported")
            bits = auto[2:]
            self._n = len(bits)
            self._v = int(bits, 2) if bits else 0
        else:
            raise TypeError("unsupported BitArray initialiser %r" % (auto,))

    @classmethod
    def _make(cls, v, n):
        b = cls.__new__(cls)
        b._v = v & ((1 << n) - 1) if n else 0
        b._n = n
        return b

    # -- sizes / repetition / concatenation ---------------------------------
    def __len__(self):
        return self._n

    def __mul__(self, k):
        v, n = 0, 0
        for _ in range(int(k)):
            v = (v << self._n) | self._v
            n += self._n
        return BitArray._make(v, n)

    __rmul__ = __mul__

    def append(self, other):
        o = other if isinstance(other, BitArray) else BitArray(other)
        self._v = (self._v << o._n) | o._v
        self._n += o._n

    # -- bit access ----------------------------------------------------------
    def _norm(self, i):
        i = int(i)
        if i < 0:
            i += self._n
        if not 0 <= i < self._n:
            raise IndexError(i)
        return i

    def __getitem__(self, key):
        if isinstance(key, slice):
            start, stop, step = key.indices(self._n)
            if step != 1:
                raise NotImplementedError
            width = max(0, stop - start)
            return BitArray._make(self._v >> (self._n - start - width), width)
        i = self._norm(key)
        return bool((self._v >> (self._n - 1 - i)) & 1)

    def __setitem__(self, key, value):
        if isinstance(key, slice):
            start, stop, step = key.indices(self._n)
            if step != 1:
                raise NotImplementedError
            width = max(0, stop - start)
            if isinstance(value, bool) or not isinstance(value, int):
                val = value if isinstance(value, BitArray) else BitArray(value)
                if val._n != width:
                    # general splice (unused by the reference)
                    head = self[0:start]
                    tail = self[stop:self._n]
                    head.append(val)
                    head.append(tail)
                    self._v, self._n = head._v, head._n
                    return
                bits = val._v
            else:
                if value >= 0:
                    if value >= (1 << width):
                        raise ValueError("uint out of range")
                    bits = value
                else:
                    if value < -(1 << (width - 1)):
                        raise ValueError("int out of range")
                    bits = value & ((1 << width) - 1)
            shift = self._n - start - width
            mask = ((1 << width) - 1) << shift
            self._v = (self._v & ~mask) | (bits << shift)
            return
        i = self._norm(key)
        shift = self._n - 1 - i
        if value:
            self._v |= 1 << shift
        else:
            self._v &= ~(1 << shift)

    # -- interpretations -----------------------------------------------------
    @property
    def int(self):
        if self._n == 0:
            raise ValueError("empty bitstring")
        if self._v >> (self._n - 1):
            return self._v - (1 << self._n)
        return self._v

    @int.setter
    def int(self, value):
        n = self._n
        if not -(1 << (n - 1)) <= value < (1 << (n - 1)):
            raise ValueError("int out of range")
        self._v = value & ((1 << n) - 1)

    @property
    def uint(self):
        return self._v

    @property
    def bytes(self):
        if self._n % 8:
            raise ValueError("not a whole number of bytes")
        return self._v.to_bytes(self._n // 8, "big")

    @bytes.setter
    def bytes(self, data):
        self._n = 8 * len(data)
        self._v = int.from_bytes(data, "big")

    @property
    def bin(self):
        return format(self._v, "0%db" % self._n) if self._n else ""

    # -- operators -----------------------------------------------------------
    def __or__(self, other):
        if other._n != self._n:
            raise ValueError("length mismatch")
        return BitArray._make(self._v | other._v, self._n)

    def __and__(self, other):
        if other._n != self._n:
            raise ValueError("length mismatch")
        return BitArray._make(self._v & other._v, self._n)

    def __eq__(self, other):
        if not isinstance(other, BitArray):
            try:
                other = BitArray(other)
            except Exception:
                return NotImplemented
        return self._n == other._n and self._v == other._v

    def __ne__(self, other):
        r = self.__eq__(other)
        return r if r is NotImplemented else not r

    __hash__ = None

    def __repr__(self):
        return "BitArray('0b%s')" % self.bin


Bits = BitArray
