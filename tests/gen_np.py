"""Independent numpy restatement of the synthetic generators (DESIGN.md "Inputs"),
used to cross-check oracle/chunker_oracle.c and the device generator."""
import numpy as np

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)
VM_SEED_PAGE = 0x7A65726F50414745
VM_SEED_WORD = 0x52414E44574F5244
VM_SEED_EXT = 0x4558544E54000000


def splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = (x + np.uint64(0x9E3779B97F4A7C15))
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _bytes_of_words(words: np.ndarray, offset: int, length: int) -> np.ndarray:
    b = words.astype("<u8").view(np.uint8)
    start = offset & 7
    return b[start:start + length].copy()


def gen_counter(length: int, offset: int = 0) -> np.ndarray:
    x = np.arange(offset, offset + length, dtype=np.uint64)
    i = (x >> np.uint64(2)).astype(np.uint32)
    return ((i >> ((x & np.uint64(3)) * np.uint64(8)).astype(np.uint32)) & np.uint32(0xFF)).astype(np.uint8)


def gen_random(length: int, seed: int, offset: int = 0) -> np.ndarray:
    w0, w1 = offset >> 3, (offset + length + 7) >> 3
    w = np.arange(w0, w1, dtype=np.uint64)
    return _bytes_of_words(splitmix64(np.uint64(seed) ^ w), offset, length)


def gen_vmimage(length: int, seed: int, offset: int = 0) -> np.ndarray:
    w0, w1 = offset >> 3, (offset + length + 7) >> 3
    w = np.arange(w0, w1, dtype=np.uint64)
    x = w << np.uint64(3)
    g = x >> np.uint64(30)
    ext = (splitmix64(np.uint64(seed ^ VM_SEED_EXT) ^ g) & np.uint64(15)) << np.uint64(26)
    in_g = x & np.uint64((1 << 30) - 1)
    zero_ext = (in_g >= ext) & (in_g < ext + np.uint64(1 << 26))
    zero_page = (splitmix64(np.uint64(seed ^ VM_SEED_PAGE) ^ (x >> np.uint64(12))) % np.uint64(100)) < np.uint64(40)
    v = splitmix64(np.uint64(seed ^ VM_SEED_WORD) ^ w)
    v[zero_ext | zero_page] = 0
    return _bytes_of_words(v, offset, length)
