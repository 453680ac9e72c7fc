"""Test-only ``Bio.SeqIO.parse(path, "fasta")`` for running the reference's generate.py
(/root/reference/kmerml/kmers/generate.py:4,39) when biopython 1.85 is absent.

Records carry ``.id`` and ``.seq`` (a str: the reference only calls ``str(record.seq)``).
The parsing algorithm is the restatement in oracle/fasta.py (Biopython SimpleFastaParser /
FastaIterator semantics), so parser edge cases are "parity unpinned" (DESIGN.md)."""
from oracle.fasta import record_id, simple_fasta_parser


class _Record:
    __slots__ = ("id", "description", "seq")

    def __init__(self, title, seq):
        self.id = record_id(title)
        self.description = title
        self.seq = seq


def parse(source, fmt):
    if fmt != "fasta":
        raise ValueError(f"bio_shim only supports 'fasta', got {fmt!r}")
    with open(source, "r") as handle:
        for title, seq in simple_fasta_parser(handle):
            yield _Record(title, seq)
