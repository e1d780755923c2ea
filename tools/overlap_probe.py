#!/usr/bin/env python3
"""Can two independent maps overlap on one MI355X?  Two copies of libasp_hip.so are loaded
(separate workspaces, no cross-call ordering between them) and consecutive maps of the
bench workload alternate between them on two HIP streams; the throughput is compared
with one library on one stream.  A feasibility probe for pipelining maps inside the
library: nothing here is a product path.

    python tools/overlap_probe.py [--n 1e8] [--grid 4096] [--maps 20]
"""
import argparse
import ctypes as C
import json
import os
import shutil
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "astro-sph-tools_amd"))


def load(path):
    from asp_amd import _lib
    L = C.CDLL(path)
    L.asp_project2d.argtypes = [_lib._f] * 5 + [C.c_int64] + [C.c_double] * 4 + \
        [C.c_int32] * 5 + [_lib._f, _lib._f, C.c_int32, C.c_void_p]
    L.asp_last_error.restype = C.c_char_p
    return L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=float, default=1e8)
    ap.add_argument("--grid", type=int, default=4096)
    ap.add_argument("--maps", type=int, default=20)
    ap.add_argument("--out")
    a = ap.parse_args()
    import torch
    from asp_amd import _lib
    from asp_amd.plummer import plummer_torch
    dev = torch.device("cuda:0")
    src = _lib.LIB_PATH
    dst = "/tmp/asp_overlap_copy/libasp_hip.so"
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    shutil.copyfile(src, dst)
    libs = [load(src), load(dst)]
    G = a.grid
    d = plummer_torch(int(a.n), seed=0, h_law="pixel", extent=4.0, grid=G, device=dev)
    u, v, h, m = d["x"], d["y"], d["h"], d["m"]
    a0 = (m * d["T"]).contiguous()
    outs = [torch.empty((2, G, G), dtype=torch.float32, device=dev) for _ in range(2)]
    streams = [torch.cuda.Stream(device=dev) for _ in range(2)]
    P = _lib.ptr
    flags = _lib.ASP_F_DEVICE_PTRS | _lib.ASP_F_RATIO

    def one(k, L, s):
        rc = L.asp_project2d(P(u), P(v), P(h), P(a0), P(m), u.shape[0], -4.0, 4.0, -4.0, 4.0,
                             G, G, 64, 1, flags, P(outs[k][0]), P(outs[k][1]), 0,
                             s.cuda_stream)
        if rc:
            raise RuntimeError(L.asp_last_error())

    res = {}
    for mode in ("serial", "two_streams", "serial", "two_streams"):
        for k in range(4):  # warm-up (placement trials run on each library's first call)
            one(k % 2, libs[k % 2] if mode == "two_streams" else libs[0],
                streams[k % 2] if mode == "two_streams" else streams[0])
        torch.cuda.synchronize()
        t = time.perf_counter()
        for k in range(a.maps):
            if mode == "two_streams":
                one(k % 2, libs[k % 2], streams[k % 2])
            else:
                one(k % 2, libs[0], streams[0])
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) / a.maps * 1e3
        res.setdefault(mode, []).append(round(ms, 4))
        print(mode, round(ms, 4), "ms per map", flush=True)
    r0 = outs[0].clone()
    one(0, libs[0], streams[0])
    torch.cuda.synchronize()
    res["same_map"] = bool(torch.allclose(r0, outs[0], rtol=1e-6, atol=0))
    print(json.dumps(res))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f)


if __name__ == "__main__":
    main()
