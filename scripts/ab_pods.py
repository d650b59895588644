"""A/B timing of pod_requests_kernel variants in ONE process, interleaved.

  python scripts/ab_pods.py NAME=PATH ...   (GPU; PATH a libkcc build, e.g. variants/libkcc_X.so)

Same device inputs as bench.py's `pods` leg (C4 containers cut into ~2-container pods,
an init container on every third pod, overhead on every fifth); checks every variant's
outputs are identical; prints one JSON line per variant (median ms over the rounds).
"""
import ctypes as C

import numpy as np
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(specs):
    import torch

    from kubernetesclustercapacity_amd import _lib, synth

    dev = torch.device("cuda", 0)
    torch.zeros(1, device=dev)
    cl = synth.config_cluster("C4")
    ptr = torch.from_numpy(cl.node_ptr).to(dev)
    cpu = torch.from_numpy(cl.cpu_req.view(np.int64)).to(dev)
    mem = torch.from_numpy(cl.mem_req).to(dev)
    Cn = cpu.numel()
    g = torch.Generator(device=dev)
    g.manual_seed(20261017)
    start = torch.rand(Cn, device=dev, generator=g) < 0.5
    start[ptr[:-1][torch.diff(ptr) > 0]] = True
    pod_ptr = torch.cat([torch.nonzero(start).flatten(), torch.tensor([Cn], device=dev)])
    P = pod_ptr.numel() - 1
    has_init = (torch.arange(P, device=dev) % 3) == 0
    init_ptr = torch.cat([torch.zeros(1, device=dev, dtype=torch.int64),
                          torch.cumsum(has_init.to(torch.int64), 0)])
    I = int(init_ptr[-1].item())
    icpu = torch.randint(0, 40, (I,), device=dev, generator=g, dtype=torch.int64) * 50
    imem = torch.randint(0, 256, (I,), device=dev, generator=g, dtype=torch.int64) << 26
    rst = (torch.rand(I, device=dev, generator=g) < 0.3).to(torch.uint8)
    sel = (torch.arange(P, device=dev) % 5) == 0
    ocpu = torch.where(sel, 100, 0).to(torch.int64)
    omem = torch.where(sel, 1 << 27, 0).to(torch.int64)
    libs = {}
    for s in specs:
        name, _, path = s.partition("=")
        L = _lib.load(os.path.join(ROOT, path))
        h = C.c_void_p()
        assert L.kcc_create(C.byref(h), 0, 1) == 0
        libs[name] = (L, h, torch.empty(P, dtype=torch.int64, device=dev),
                      torch.empty(P, dtype=torch.int64, device=dev))
    dp = lambda t: C.c_void_p(t.data_ptr())
    stream = torch.cuda.current_stream().cuda_stream

    def run(name):
        L, h, pc, pm = libs[name]
        rc = L.kcc_pod_requests_async(h, P, Cn, I, dp(pod_ptr), dp(cpu), dp(mem), dp(init_ptr),
                                      dp(icpu), dp(imem), dp(rst), dp(ocpu), dp(omem), dp(pc),
                                      dp(pm), C.c_void_p(stream))
        assert rc == 0, L.kcc_last_error(h)

    times = {n: [] for n in libs}
    for _ in range(7):
        for n in libs:
            for _ in range(3):
                run(n)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                run(n)
            e1.record()
            torch.cuda.synchronize()
            times[n].append(e0.elapsed_time(e1) / 10)
    ref = None
    for n, (L, h, pc, pm) in libs.items():
        same = True
        if ref is None:
            ref = (pc, pm)
        else:
            same = bool(torch.equal(pc, ref[0]) and torch.equal(pm, ref[1]))
        t = sorted(times[n])[len(times[n]) // 2]
        alg = P * 16 + Cn * 16 + I * 17 + P * 16 + P * 16
        print(json.dumps({"variant": n, "ms": t, "tbps": alg / t / 1e9, "same_as_first": same}))
        L.kcc_destroy(h)


if __name__ == "__main__":
    import numpy as np
    main(sys.argv[1:])
