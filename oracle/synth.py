"""TEST INFRASTRUCTURE ONLY -- the synthetic-genome PRNG of SURVEY.md section 8(d).

base[i] = "ACGT"[(splitmix64(seed_g + (i >> 5)) >> (2 * (i & 31))) & 3],
seed_g = splitmix64(0x6B6D65724D4C0000 + g).  (SURVEY.md 8(d) used seed_g = base + g,
which makes genome g+1 a 32-base shift of genome g; hashing the genome id keeps the
streams unrelated.)  The device generator (kmh_synth_dev) must produce the same bytes;
tests check that.
"""
import numpy as np

SEED_BASE = 0x6B6D65724D4C0000
ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)

# S. cerevisiae R64 chromosome lengths (17 records, 12,157,105 bases): the
# config-1 stand-in when the real GCF_000146045.2 file is not supplied.
YEAST_LENGTHS = [230218, 813184, 316620, 1531933, 576874, 270161, 1090940, 562643,
                 439888, 745751, 666816, 1078177, 924431, 784333, 1091291, 948066,
                 85779]


def splitmix64(x):
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def genome_seed(g):
    return int(splitmix64(np.uint64(SEED_BASE + int(g))))


def synth_bases(length, seed, start=0):
    """uint8 array of ASCII bases [start, start + length) of the genome with ``seed``."""
    idx = np.arange(start, start + length, dtype=np.uint64)
    with np.errstate(over="ignore"):
        words = splitmix64(np.uint64(seed) + (idx >> np.uint64(5)))
    sel = (words >> (np.uint64(2) * (idx & np.uint64(31)))) & np.uint64(3)
    return ACGT[sel.astype(np.intp)]


def write_fasta(path, records, width=80):
    """records: list of (id, bytes-like ASCII sequence)."""
    with open(path, "wb") as f:
        for rid, seq in records:
            seq = bytes(seq)
            f.write(b">" + rid.encode() + b"\n")
            for i in range(0, len(seq), width):
                f.write(seq[i:i + width] + b"\n")


def yeast_standin_records(seed=genome_seed(0)):
    """17 records with the yeast chromosome lengths, bases from consecutive PRNG ranges."""
    out, pos = [], 0
    for i, n in enumerate(YEAST_LENGTHS):
        out.append((f"SYN_chr{i + 1:02d}", synth_bases(n, seed, pos).tobytes()))
        pos += n
    return out
