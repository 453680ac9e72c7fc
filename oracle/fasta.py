"""TEST INFRASTRUCTURE ONLY -- CPU restatement of the reference's FASTA record iteration.

The reference reads genomes with ``SeqIO.parse(fasta_file, "fasta")``
(/root/reference/kmerml/kmers/generate.py:39) from Biopython 1.85
(/root/reference/requirements.txt:1).  Biopython is a third-party dependency that
is NOT vendored in /root/reference and not installed here, so this module restates
its published ``SimpleFastaParser`` / ``FastaIterator`` algorithm (Bio/SeqIO/FastaIO.py,
biopython 1.85):

* the file is opened in text mode (universal newlines: \\r\\n, \\r and \\n all end a
  line);
* lines before the first line starting with ``>`` are skipped;
* ``title = line[1:].rstrip()``; the record id is the first whitespace-separated
  token of the title ("" for an empty title);
* sequence lines are ``rstrip()``-ed, joined, and every " " and "\\r" is removed.

Parser-edge behaviour no reference test pins (text before the first ``>``,
non-UTF-8 bytes, non-ASCII whitespace) is "parity unpinned" (DESIGN.md).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may import this.
"""


def simple_fasta_parser(handle):
    """Yield (title, sequence) string tuples -- Biopython SimpleFastaParser semantics."""
    for line in handle:
        if line[0] == ">":
            title = line[1:].rstrip()
            break
    else:
        return
    lines = []
    for line in handle:
        if line[0] == ">":
            yield title, "".join(lines).replace(" ", "").replace("\r", "")
            lines = []
            title = line[1:].rstrip()
            continue
        lines.append(line.rstrip())
    yield title, "".join(lines).replace(" ", "").replace("\r", "")


def record_id(title):
    """FastaIterator's id: first word of the title, "" if the title is empty."""
    parts = title.split(None, 1)
    return parts[0] if parts else ""


def parse_fasta(path):
    """List of (id, title, sequence) for every record of ``path`` (text mode)."""
    with open(path, "r") as handle:
        return [(record_id(t), t, s) for t, s in simple_fasta_parser(handle)]
