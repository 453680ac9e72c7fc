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

* k <= 0 and bool k behave as in the reference's loop (tests/golden: k = 0 counts the empty
  k-mer len + 1 times per record and writes ``"\t{count}"``; a negative k counts the slices
  ``seq[i:i + k]``; True / False are k = 1 / 0 under the key True / False, file
  ``kTrue.txt``); these degenerate k are counted on the host (they are no hot path).  A
  non-integer k raises the reference's TypeError from ``range()`` at the first kept record,
  after the "Skipping" lines of the records before it, and leaves no file; with no kept
  record it writes an empty ``k{k}.txt`` as the reference does.

Differences: k <= 1024 is supported (k > 1024 raises NotImplementedError;
k >= 33 is counted by sorting ceil(k / 32) code words per window
and its lines are written from the sequence); counting never falls back to the CPU --
without the HIP library or a device it raises.  Size limit per organism (its kept records
joined): below 2^32 - 1 bytes for every k (u32 positions and counts; a 3.1 Gbp human genome
fits, 2^31 windows and more are counted at every k).  Larger organisms raise
NotImplementedError, which extract_from_genome_list reports as "Error processing <id>" like
any other failure.  The reference's dict has no such limit but needs tens of bytes per
distinct k-mer of host memory.

Device memory: the organism crosses PCIe once for all its k (kmh_stage_host, then one
kmh_count_staged per k), and after each organism the context's cached workspace is released
if it holds more than KMERML_WORKSPACE_MB (default 4096 MiB; kmh_ctx_trim), so a long
extract_from_genome_list loop (generate.py:116-126) does not keep the tens of GB a large
organism needed.
"""
import contextlib
import operator
import os
import time
from pathlib import Path

import numpy as np

from kmerml import _native
from kmerml.utils.path_utils import ensure_directory_exists

_DIGITS = {"A": "0", "T": "1", "C": "2", "G": "3"}

# Stage clocks of the drop-in (bench.py's "e2e" object): set to a dict and every
# extract_kmers_from_fasta call adds its wall seconds per stage to it.
PROFILE = None


@contextlib.contextmanager
def _stage(name):
    if PROFILE is None:
        yield
        return
    t0 = time.perf_counter()
    try:
        yield
    finally:
        PROFILE[name] = PROFILE.get(name, 0.0) + time.perf_counter() - t0


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
        with _stage("parse"):
            fasta = _native.FastaFile(fasta_file)
        results = {}
        packed = np.zeros(0, np.uint8)
        if len(fasta):
            longest = max(k_values)                   # generate.py:44 (same error for odd k)
            if not all(_is_index(k) for k in k_values):
                _raise_like_reference(fasta, k_values, longest)
                longest = float("inf")                # no record is kept: nothing to count
            with _stage("pack"):
                packed, kept = fasta.pack(_min_len(longest))
            results = _count_all(packed, kept, k_order)
            for rid, keep in zip(fasta.ids, kept):
                if keep:
                    print(f"Processed chromosome/contig: {rid}")
                else:
                    print(f"Skipping {rid}: too short for k-mer extraction")
        fasta.close()
        for k in k_order:
            path = self._kmer_path(organism_id, k)
            res = results.get(k)
            if isinstance(res, dict):                 # k <= 0
                self._write_bytes(path, _degenerate_text(res, multiplicity[k]))
                continue
            if res is None or not _is_index(k) or operator.index(k) < 1:
                self._write_bytes(path, b"")          # no kept record: an empty file (:87-91)
                continue
            codes, counts, first = res
            kv = operator.index(k)
            counts = np.multiply(counts, np.uint64(multiplicity[k]), dtype=np.uint64)
            with _stage("format"):
                if kv > 32:   # a code holds 32 bases: the line digits come from the sequence
                    text = _native.format_lines_seq(kv, packed, first, counts)
                else:
                    text = _native.format_lines_array(kv, codes, counts)
            with _stage("write"):
                self._write_bytes(path, text)
        return organism_id

    def _kmer_path(self, organism_id, k):
        organism_dir = ensure_directory_exists(self.output_dir / organism_id)
        return organism_dir / (f"k{k}.txt.gz" if self.compress else f"k{k}.txt")

    def _write_bytes(self, path, data):
        # gzip.open's default level 9 (generate.py:82-85), deflated on several host threads
        _native.write_file(path, data, gzip_level=9 if self.compress else -1)

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


def _count_all(packed, kept, k_order):
    """{k: result} for the kept records joined in ``packed``: the GPU counts every k >= 1 from one
    device copy of the organism; k <= 0 is counted on the host."""
    results = {}
    if not kept.any():
        return results
    ctx = None
    try:
        for k in k_order:
            kv = operator.index(k)                # True / False count as k = 1 / 0
            if kv >= 1:
                if ctx is None:                   # one host-to-device copy for every k
                    ctx = _native.context(_device())
                    ctx.lock.acquire()
                    with _stage("h2d"):
                        ctx.stage(packed)
                with _stage("count"):             # kernels, first-occurrence order, D2H
                    results[k] = ctx.count_staged(kv)
            else:
                bodies = bytes(packed).split(b"\n")[:int(kept.sum())]
                results[k] = _count_degenerate(bodies, kv)
    finally:
        if ctx is not None:
            try:
                with _stage("trim"):
                    ctx.trim(_workspace_limit())
            finally:
                ctx.lock.release()
    return results


def _workspace_limit():
    """Bytes of device workspace a context may keep between organisms (KMERML_WORKSPACE_MB)."""
    return int(os.environ.get("KMERML_WORKSPACE_MB", "4096")) << 20


def _is_index(k):
    """True for the k values range() accepts (int, bool, numpy integers)."""
    try:
        operator.index(k)
        return True
    except TypeError:
        return False


def _min_len(longest):
    """The record filter of generate.py:44 as a minimum character length."""
    if longest == float("inf"):
        return 1 << 62
    return max(0, -(-longest // 1)) if not _is_index(longest) else max(0, operator.index(longest))


def _raise_like_reference(fasta, k_values, longest):
    """A k that is no integer: the reference prints its "Skipping" lines up to the first record
    that passes the length rule and raises from ``range(len(sequence) - k + 1)`` there
    (generate.py:44-51).  Returns only if no record passes the rule."""
    skipped = []
    for i, rid in enumerate(fasta.ids):
        n = _upper_len(fasta, i)
        if n < longest:                     # may itself raise (e.g. a str k), as :44 does
            skipped.append(f"Skipping {rid}: too short for k-mer extraction")
            continue
        for line in skipped:
            print(line)
        for k in k_values:
            range(n - k + 1)                # the reference's TypeError
        return


def _upper_len(fasta, i):
    if fasta.char_lens[i] == fasta.seq_lens[i]:
        return fasta.char_lens[i]
    return len(fasta.sequence(i).decode("utf-8", errors="surrogateescape").upper())


def _count_degenerate(bodies, k):
    """generate.py:49-58 for k <= 0 over the kept records (upper-cased bytes, one per record).
    Windows i >= -k are empty slices (the empty k-mer, which passes the ACGT test of :55); the
    first -k windows are ``seq[i:i + k]``, counted when every character is a base.  Returns the
    dict in the reference's insertion order."""
    table = {}
    m = -k
    for body in bodies:
        s = body.upper()
        n = len(s) - k + 1                  # range(len(sequence) - k + 1)
        for i in range(min(m, n)):
            t = s[i:i + k]
            if not t.translate(None, b"ACGT"):
                table[t] = table.get(t, 0) + 1
        if n > m:
            table[b""] = table.get(b"", 0) + (n - m)
    return table


_DIGIT_TABLE = bytes.maketrans(b"ACGT", b"0231")


def _degenerate_text(table, mult):
    """_save_kmers_to_file's lines (generate.py:86-91) for the dict of _count_degenerate."""
    return b"".join(t.translate(_DIGIT_TABLE) + b"\t" + str(c * mult).encode() + b"\n"
                    for t, c in table.items())
