"""Test-only stand-in for the third-party ``Bio`` package (biopython 1.85), used ONLY by
tests/golden/make_golden.py to run the reference's own generate.py here.  Not product code."""
