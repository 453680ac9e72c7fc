"""TEST INFRASTRUCTURE ONLY -- faithful Python restatement of the reference hot path.

Restates /root/reference/kmerml/kmers/generate.py:

* :36      ``all_kmers = {k: defaultdict(int) for k in k_values}`` (duplicate k values
           collapse to one dict, first-occurrence order of k);
* :39-46   per record: ``sequence = str(record.seq).upper()``; a record shorter than
           ``max(k_values)`` is skipped for EVERY k, with a "Skipping" line;
* :49-58   for each k in ``k_values`` (duplicates included, so they double-count),
           slide a window, skip windows with a non-ACGT character, count;
* :60      "Processed chromosome/contig" line per kept record;
* :68-91   text lines ``digits\\tcount`` with A=0 T=1 C=2 G=3, in dict (first
           occurrence) order.

It is deliberately the same pure-Python per-window loop as the reference, so that
bench.py can time it as the reference CPU path ("kind": "port").

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may import this.
"""
from collections import defaultdict

DIGIT = {"A": "0", "T": "1", "C": "2", "G": "3"}


def count_records(records, k_values, messages=None):
    """records: iterable of (id, sequence).  Returns {k: dict(kmer -> count)}."""
    all_kmers = {k: defaultdict(int) for k in k_values}
    for rid, seq in records:
        sequence = seq.upper()
        if len(sequence) < max(k_values):
            if messages is not None:
                messages.append(f"Skipping {rid}: too short for k-mer extraction")
            continue
        for k in k_values:
            table = all_kmers[k]
            for i in range(len(sequence) - k + 1):
                kmer = sequence[i:i + k]
                if not all(base in "ACGT" for base in kmer):
                    continue
                table[kmer] += 1
        if messages is not None:
            messages.append(f"Processed chromosome/contig: {rid}")
    return all_kmers


def count_sequence(sequence, k):
    """Count one uppercase-able sequence for one k (the :49-58 loop)."""
    table = defaultdict(int)
    sequence = sequence.upper()
    for i in range(len(sequence) - k + 1):
        kmer = sequence[i:i + k]
        if not all(base in "ACGT" for base in kmer):
            continue
        table[kmer] += 1
    return table


def kmer_text(kmers):
    """The exact text _save_kmers_to_file writes (generate.py:86-91), uncompressed."""
    out = []
    for kmer, count in kmers.items():
        out.append("".join(DIGIT.get(b, "X") for b in kmer) + "\t" + str(count) + "\n")
    return "".join(out)


def save_kmers(kmers, path):
    """_save_kmers_to_file's write loop (generate.py:84-91) for compress=False (the CLI default,
    scripts/extract_kmers.py:19-20): text mode, one f.write per k-mer, digits built by the same
    per-base generator expression.  bench.py times it as the reference's save phase."""
    encoding = {'A': 0, 'T': 1, 'C': 2, 'G': 3}
    with open(path, "w") as f:
        for kmer, count in kmers.items():
            numeric_kmer = ''.join(str(encoding.get(base, 'X')) for base in kmer)
            f.write(f"{numeric_kmer}\t{count}\n")


_CODE = {"A": 0, "C": 1, "G": 2, "T": 3}


def kmer_code(kmer):
    """2-bit code, A0 C1 G2 T3, first base most significant."""
    c = 0
    for b in kmer:
        c = (c << 2) | _CODE[b]
    return c


def code_kmer(code, k):
    return "".join("ACGT"[(code >> (2 * (k - 1 - i))) & 3] for i in range(k))
