"""GPU-box diagnostic: load libsa_hip stepwise (with/without torch first)."""
import faulthandler, sys, os, ctypes
faulthandler.enable()
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mode = sys.argv[1] if len(sys.argv) > 1 else "torch_first"
if mode == "torch_first":
    import torch
    print("torch", torch.__version__, torch.cuda.is_available(), flush=True)
from hpc_suffix_array_amd import _native as N
L = N.lib()
print("loaded", L.sa_version(), flush=True)
print("devices", L.sa_device_count(), flush=True)
import numpy as np
t = np.frombuffer(b"banana", np.uint8)
out = np.zeros(6, np.uint32)
rc = L.sa_build_ex(t.ctypes.data, 6, out.ctypes.data, 4, None, None)
print("rc", rc, L.sa_last_error(), out, flush=True)
