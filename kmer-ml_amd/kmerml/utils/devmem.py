"""Device-memory reports for multi-process runs: a rank whose allocation fails says so itself.

A rank of a torch.distributed job that runs out of device memory used to die with a traceback
that torchrun's SIGTERM of the other ranks could push out of the captured log; ``run_guarded``
prints the rank, the failing allocation and hipMemGetInfo (torch.cuda.mem_get_info) on stderr
before the exception propagates.
"""
import os
import sys


def _is_oom(exc):
    import torch
    if isinstance(exc, (MemoryError, torch.OutOfMemoryError)):
        return True
    msg = str(exc).lower()
    return "out of memory" in msg or "hiperroroutofmemory" in msg or "kmh_err_nomem" in msg


def memory_line():
    """'free X GiB / total Y GiB on cuda:i (torch reserved Z GiB)' for the current device."""
    import torch
    try:
        i = torch.cuda.current_device()
        free, total = torch.cuda.mem_get_info(i)
        res = torch.cuda.memory_reserved(i)
        return (f"hipMemGetInfo on cuda:{i}: free {free / 2**30:.1f} GiB of {total / 2**30:.1f} GiB "
                f"(this process's torch cache {res / 2**30:.1f} GiB)")
    except Exception as e:   # the report must never hide the original error
        return f"hipMemGetInfo unavailable ({type(e).__name__}: {e})"


def run_guarded(main):
    """main() with allocation failures reported by the failing rank itself."""
    try:
        return main()
    except BaseException as e:
        if not isinstance(e, (KeyboardInterrupt, SystemExit)) and _is_oom(e):
            rank = os.environ.get("RANK", "0")
            print(f"[rank {rank}] device allocation failed: {type(e).__name__}: {e}\n"
                  f"[rank {rank}] {memory_line()}", file=sys.stderr, flush=True)
        raise
