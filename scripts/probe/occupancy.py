"""Diagnostic: the resident-workgroup counts libkcc sizes its grids by (the occupancy API's
answer per CU x CUs), read through the library's internal C++ symbols on cuda:0."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

torch.cuda.init()
from kubernetesclustercapacity_amd import _lib  # noqa: E402

L = _lib.load()
h = C.c_void_p()
assert L.kcc_create(C.byref(h), 0, 1) == 0
rr = getattr(L, "_ZN3kcc12reduce_rangeElbl")
rr.restype = C.c_int32
rr.argtypes = [C.c_int64, C.c_bool, C.c_int64]
for n in (39_602_467, 4_950_000, 1_210_000_000):
    r = rr(n, False, 0)
    print(f"reduce_range({n}) = {r}: waves {(n + r - 1) // r}")
# slots: the smallest range is one tile; find the slot count from a size that is an exact
# multiple: range = ceil(n / (slots * 512)) * 512 -> with n = slots * 512 * k
for k in (1, 3):
    for slots in (2048, 3072, 4096, 5120, 6144, 8192):
        n = slots * 512 * k
        print(f"  n={n}: range {rr(n, False, 0)}")
fr = getattr(L, "_ZN3kcc19fit_resident_blocksEv")
fr.restype = C.c_int64
print("fit_resident_blocks", fr())
props = torch.cuda.get_device_properties(0)
print("CUs", props.multi_processor_count, "name", props.name, getattr(props, "gcnArchName", ""))
