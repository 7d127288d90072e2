"""java.util.Random (48-bit LCG, JDK spec) so the reference tests' random data is reproduced exactly."""
MASK = (1 << 48) - 1
MULT = 0x5DEECE66D


def _i32(x):
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x & 0x80000000 else x


class JavaRandom:
    def __init__(self, seed):
        self.seed = (seed ^ MULT) & MASK

    def next(self, bits):
        self.seed = (self.seed * MULT + 0xB) & MASK
        return _i32(self.seed >> (48 - bits))

    def nextInt(self, bound=None):
        if bound is None:
            return self.next(32)
        if bound <= 0:
            raise ValueError("bound must be positive")
        if (bound & -bound) == bound:
            return _i32((bound * self.next(31)) >> 31)
        while True:
            bits = self.next(31)
            val = bits % bound
            if _i32(bits - val + (bound - 1)) >= 0:
                return val

    def nextLong(self):
        v = (self.next(32) << 32) + self.next(32)
        v &= (1 << 64) - 1
        return v - (1 << 64) if v >> 63 else v

    def nextFloat(self):
        """next(24) / (float)(1 << 24) (JDK 8+)."""
        import numpy as np
        return np.float32(self.next(24)) / np.float32(1 << 24)
