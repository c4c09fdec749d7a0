"""Input buffer of the reference CityHash KAT.

Restates setup() of cityhash/test/city.cc:46-58 (a=9, b=777, k0 multiplier,
1 MiB, byte = b >> 37).  Pure data generator for tests/golden/cityhash64_kat.json.
"""
import functools

import numpy as np

K0 = 0xc3a5c85c97cb3127
M = (1 << 64) - 1


@functools.lru_cache(maxsize=1)
def kat_data() -> bytes:
    a, b = 9, 777
    out = bytearray(1 << 20)
    for i in range(1 << 20):
        a = (a + b) & M
        b = (b + a) & M
        a = ((a ^ (a >> 41)) * K0) & M
        b = (((b ^ (b >> 41)) * K0) + i) & M
        out[i] = (b >> 37) & 0xff
    return bytes(out)


def kat_array() -> np.ndarray:
    return np.frombuffer(kat_data(), dtype=np.uint8)
