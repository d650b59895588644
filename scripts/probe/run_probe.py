"""Diagnostic: streaming-read rate of the reduce's load patterns (scripts/probe/hbm_probe.hip)."""
import ctypes as C
import json
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
L = C.CDLL(os.path.join(HERE, "libprobe.so"))
L.probe_launch.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_int64, C.c_int64,
                           C.c_void_p, C.c_void_p]
n = 39_602_467 // 2 * 2
a = torch.randint(0, 1 << 40, (n,), dtype=torch.int64, device="cuda")
b = torch.randint(0, 1 << 40, (n,), dtype=torch.int64, device="cuda")
out = torch.zeros(1 << 20, dtype=torch.int64, device="cuda")
flush = torch.ones(1 << 27, dtype=torch.int64, device="cuda")  # 1 GiB, read-only flush
sink = torch.zeros(1, dtype=torch.int64, device="cuda")
s = torch.cuda.current_stream()
for fl in (True, False):
  for mode in (0, 1):
    for unroll in (1, 4):
        for per_wave in (2048, 4096, 8192):
            ts = []
            for r in range(6):
                if fl:
                    torch.sum(flush, dim=(0,), out=sink[0])  # reads only: nothing dirty left behind
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                rc = L.probe_launch(mode, unroll, a.data_ptr(), b.data_ptr(), n, per_wave,
                                    out.data_ptr(), C.c_void_p(s.cuda_stream))
                e1.record()
                torch.cuda.synchronize()
                assert rc == 0
                if r:
                    ts.append(e0.elapsed_time(e1))
            ms = sorted(ts)[len(ts) // 2]
            print(json.dumps({"flush": fl, "mode": ["contig", "strided32"][mode], "unroll": unroll,
                              "per_wave": per_wave, "ms": ms, "TBps": 16 * n / ms / 1e9}))
