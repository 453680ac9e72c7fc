"""Shared by the drop-in tests: run the drop-in KmerExtractor the way the reference's
callers do (generate.py:21-66) and collect its return value, stdout lines and files."""
import contextlib
import gzip
import io

import pytest

from kmerml.kmers.generate import KmerExtractor


def run_extractor(tmp_path, fasta, ks, compress=False, org="org", expect_error=None):
    """expect_error: the golden case's {"type", "message"} when the reference raised."""
    buf = io.StringIO()
    ret = None
    with contextlib.redirect_stdout(buf):
        ext = KmerExtractor(output_dir=str(tmp_path), compress=compress)
        if expect_error:
            with pytest.raises(Exception) as e:
                ext.extract_kmers_from_fasta(fasta, ks, organism_id=org)
            assert type(e.value).__name__ == expect_error["type"]
            assert str(e.value) == expect_error["message"]
        else:
            ret = ext.extract_kmers_from_fasta(fasta, ks, organism_id=org)
    odir = tmp_path / org
    files = {}
    if odir.is_dir():
        for p in sorted(odir.iterdir()):
            data = p.read_bytes()
            if p.suffix == ".gz":
                data = gzip.decompress(data)
            files[p.name.replace(".gz", "")] = data.decode()
    return ret, buf.getvalue().splitlines(), files
