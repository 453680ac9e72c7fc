"""Console progress line with a remaining-time estimate.

Same output as the reference's helper (/root/reference/kmerml/utils/progress.py:3-41),
which statistics.py prints while it works: an optional title line at the first and last
step, then "\\r|ooo---| i/n - Expected completion in: MM:SS" and a newline at the end.
"""
import time


def progress_bar(current, total, start_time=None, bar_length=30, title=None):
    """Print the progress line for step `current` of `total`; returns the start time."""
    if title is not None and current in (1, total):
        print(f"\n{title}")
    start_time = time.time() if start_time is None else start_time
    done = int(current / total * bar_length)
    remaining = (time.time() - start_time) / current * (total - current) if current > 0 else 0
    mm, ss = divmod(int(remaining), 60)
    bar = "|" + "o" * done + "-" * (bar_length - done) + "|"
    print(f"\r{bar} {current}/{total} - Expected completion in: {mm:02d}:{ss:02d}", end="", flush=True)
    if current == total:
        print()
    return start_time
