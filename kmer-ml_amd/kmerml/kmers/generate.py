"""GPU k-mer extraction behind the reference's ``KmerExtractor`` API.

Mirror of /root/reference/kmerml/kmers/generate.py (class at :7).  Same constructor,
method names, arguments, return values, stdout lines, on-disk layout and error
behaviour; the per-window Python loop (:36-58) is replaced by libkmerhip.so on a HIP
device (MI355X / gfx950) and the text writer loop (:86-91) by a native formatter.

Behaviour kept from the reference (each is tested against fixtures produced by running
the reference itself, tests/golden/):

* records come from the FASTA parser of generate.py:39 (Biopython semantics), are
  upper-cased (:41), and a record shorter than ``max(k_values)`` is skipped for every k
  with ``Skipping <id>: too short for k-mer extraction`` (:44-46);
* windows with a character outside ACGT are not counted (:55-56);
* a k listed twice counts twice (the dict at :36 collapses it, the loop at :49 does not);
* ``Processed chromosome/contig: <id>`` per kept record (:60);
* ``<output_dir>/<organism_id>/k{k}.txt[.gz]``, one ``digits<TAB>count`` line per
  distinct k-mer, digits A=0 T=1 C=2 G=3, lines in first-occurrence order (:68-91); an
  empty result still creates the file.

Differences: 1 <= k <= 1024 is supported (k > 1024 raises NotImplementedError,
k <= 0 raises ValueError; k >= 33 is counted by sorting ceil(k / 32) code words per window
and its lines are written from the sequence); counting never falls back to the CPU --
without the HIP library or a device it raises.  Size limits per organism (its kept records
joined): below 2^32 - 1 bytes for every k, and fewer than 2^31 windows for k >= 13 (a
3.1 Gbp human genome fits the first and not the second: it raises NotImplementedError for
k >= 13, which extract_from_genome_list reports as "Error processing <id>" like any other
failure).  The reference's dict has no such limit but needs tens of bytes per distinct
k-mer of host memory.
"""
import os
from pathlib import Path

import numpy as np

from kmerml import _native
from kmerml.utils.path_utils import ensure_directory_exists

_DIGITS = {"A": "0", "T": "1", "C": "2", "G": "3"}


def _device():
    return int(os.environ.get("KMERML_DEVICE", "0"))


class KmerExtractor:
    """Extract k-mers from genomic sequences for multiple k values (on the GPU)."""

    def __init__(self, output_dir="kmer_data", compress=True):
        self.output_dir = ensure_directory_exists(Path(output_dir))
        self.compress = compress

    # generate.py:21-66
    def extract_kmers_from_fasta(self, fasta_file, k_values, organism_id=None):
        if organism_id is None:
            organism_id = Path(fasta_file).stem
        k_order = list(dict.fromkeys(k_values))       # the dict of generate.py:36
        multiplicity = {k: 0 for k in k_order}
        for k in k_values:                            # the loop of generate.py:49
            multiplicity[k] += 1
        fasta = _native.FastaFile(fasta_file)
        results = {}
        packed = np.zeros(0, np.uint8)
        if len(fasta):
            longest = max(k_values)
            for k in k_order:
                if not isinstance(k, (int, np.integer)) or isinstance(k, bool):
                    raise TypeError(f"k values must be integers, got {k!r}")
                if k < 1:
                    raise ValueError(f"k must be >= 1 (got {k})")
            packed, kept = fasta.pack(longest)
            ctx = _native.context(_device())
            for k in k_order:
                if kept.any():
                    results[k] = ctx.count(packed, k)
            for rid, keep in zip(fasta.ids, kept):
                if keep:
                    print(f"Processed chromosome/contig: {rid}")
                else:
                    print(f"Skipping {rid}: too short for k-mer extraction")
        fasta.close()
        for k in k_order:
            codes, counts, first = results.get(k, (np.empty(0, np.uint64), np.empty(0, np.uint32),
                                                   np.empty(0, np.uint64)))
            counts = np.multiply(counts, np.uint64(multiplicity[k]), dtype=np.uint64)
            if k > 32:   # a code holds 32 bases: the line digits come from the sequence
                self._write_bytes(self._kmer_path(organism_id, k),
                                  _native.format_lines_seq(k, packed, first, counts))
            else:
                self._write_kmer_file(organism_id, k, codes, counts)
        return organism_id

    def _kmer_path(self, organism_id, k):
        organism_dir = ensure_directory_exists(self.output_dir / organism_id)
        return organism_dir / (f"k{k}.txt.gz" if self.compress else f"k{k}.txt")

    def _write_bytes(self, path, data):
        # gzip.open's default level 9 (generate.py:82-85), deflated on several host threads
        _native.write_file(path, data, gzip_level=9 if self.compress else -1)

    def _write_kmer_file(self, organism_id, k, codes, counts):
        self._write_bytes(self._kmer_path(organism_id, k), _native.format_lines_array(k, codes, counts))

    # generate.py:68-91 -- kept for callers that hand in a {kmer: count} dict.
    def _save_kmers_to_file(self, kmers, organism_id, k):
        text = "".join("".join(_DIGITS.get(b, "X") for b in kmer) + f"\t{count}\n"
                       for kmer, count in kmers.items())
        self._write_bytes(self._kmer_path(organism_id, k), text.encode())

    # generate.py:93-129
    def extract_from_genome_list(self, genome_paths, k_values, organism_ids=None):
        if organism_ids is None:
            organism_ids = [Path(path).stem for path in genome_paths]
        if len(organism_ids) != len(genome_paths):
            raise ValueError("Number of organism IDs must match number of genome paths")
        processed_ids = []
        total = len(genome_paths)
        for i, (fasta_path, org_id) in enumerate(zip(genome_paths, organism_ids)):
            print(f"Processing genome {org_id} ({i + 1}/{total})")
            try:
                self.extract_kmers_from_fasta(fasta_path, k_values, org_id)
                processed_ids.append(org_id)
                print(f"Completed {org_id}")
            except Exception as e:
                print(f"Error processing {org_id}: {str(e)}")
        print(f"Completed processing {len(processed_ids)} out of {total} genomes")
        return processed_ids
