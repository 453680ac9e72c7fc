"""Which torch-init state makes dlopen(libkmerhip.so) hang?  argv[1] selects the variant."""
import ctypes
import faulthandler
import os
import sys
import time

faulthandler.dump_traceback_later(25, exit=True)
HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(os.path.dirname(os.path.dirname(HERE)), "kmer-ml_amd", "kmerml", "_lib", "libkmerhip.so")
v = sys.argv[1]
t0 = time.time()
import torch  # noqa: E402
if v == "avail":
    torch.cuda.is_available()
elif v == "init":
    torch.cuda.init()
elif v == "tensor":
    torch.zeros(1, device="cuda")
elif v == "count":
    torch.cuda.device_count()
elif v == "global":
    torch.cuda.is_available()
    ctypes.CDLL(LIB, mode=os.RTLD_NOW | os.RTLD_GLOBAL)
    print(v, "loaded", round(time.time() - t0, 2), flush=True)
    sys.exit(0)
ctypes.CDLL(LIB)
print(v, "loaded", round(time.time() - t0, 2), flush=True)
