"""File helpers used by the k-mer CLI path.

Same behaviour as /root/reference/kmerml/utils/path_utils.py:
``find_files`` (:4-33) returns the SORTED union of the glob matches of every pattern
(``**/`` prefixed when recursive) -- the sort fixes the genome order of
scripts/extract_kmers.py and therefore the row order of the feature matrix;
``ensure_directory_exists`` (:35-48) creates a directory tree and returns its Path;
``is_valid_file`` (:50-61) tests for a readable regular file.
"""
import os
from pathlib import Path


def find_files(directory, patterns=None, recursive=False):
    root = Path(directory)
    prefix = "**/" if recursive else ""
    found = []
    for pattern in (patterns if patterns is not None else ["*"]):
        found += root.glob(prefix + pattern)
    found.sort()
    return found


def ensure_directory_exists(directory_path):
    path = Path(directory_path)
    if not path.exists():
        path.mkdir(parents=True, exist_ok=True)
    return path


def is_valid_file(file_path):
    p = Path(file_path)
    return p.is_file() and os.access(p, os.R_OK)
