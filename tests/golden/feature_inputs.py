"""Input genomes of the features2/ fixtures (shared by make_features.py and the tests)."""
from oracle.synth import synth_bases


def genome_c():
    """6 kbp synthetic genome with an N run, a lowercase run and a '-'."""
    b = bytearray(synth_bases(6000, 0xC0FFEE).tobytes())
    b[1000:1013] = b"N" * 13
    b[2500:2530] = bytes(x | 0x20 for x in b[2500:2530])
    b[4000:4001] = b"-"
    return bytes(b)


def genome_d():
    """Low-complexity genome: poly-A, CpG and AT repeats, random, TTTTGGGG repeats."""
    return (b"A" * 700 + b"CG" * 400 + b"AT" * 300 + bytes(synth_bases(700, 0xD15EA5E).tobytes())
            + b"TTTTGGGG" * 50)


CASES = (("orgC", genome_c, [3, 12, 20, 21]), ("orgD", genome_d, [1, 5, 12]))
