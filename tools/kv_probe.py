"""Timing-only probe of the decode attention's K / V cache reads (tools/kv_probe.hip), alone.

    python tools/kv_probe.py [--rows 16] [--pos 3200] [--layers 26]

Builds tools/kv_probe.hip into zonos_vibes_amd/var/libkvprobe.so when missing (hipcc, gfx950). Each launch reads
another layer's random caches (HBM, not the Infinity Cache). Prints one JSON line per (mode, workgroups per CU):
us per launch and GB/s of K / V bytes.
"""
import argparse
import ctypes
import json
import os
import subprocess

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SO = os.path.join(ROOT, "zonos_vibes_amd", "var", "libkvprobe.so")
HD, HKV = 128, 4


def build():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-std=c++17", "-fPIC", "-shared",
                           os.path.join(HERE, "kv_probe.hip"), "-o", SO])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=16)
    ap.add_argument("--pos", type=int, default=3200)
    ap.add_argument("--layers", type=int, default=26)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--build-only", action="store_true")
    ap.add_argument("--modes", default="0,1,2")
    ap.add_argument("--occ", default="2,3,4,6,8")
    args = ap.parse_args()
    if args.build_only or not os.path.exists(SO):
        build()
        if args.build_only:
            return
    lib = ctypes.CDLL(SO)
    lib.kv_probe.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                             ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    dev = "cuda"
    rows, p = args.rows, args.pos
    smax = p + 72
    smax += (-smax) % 128  # whole 128-position tiles for mode 6
    units = rows * HKV
    kc = [torch.randn(units, smax, HD, device=dev).to(torch.bfloat16) for _ in range(args.layers)]
    vt = [torch.randn(units, HD, smax, device=dev).to(torch.bfloat16) for _ in range(args.layers)]
    nch = p // 128 + 1
    out = torch.zeros(max(units * nch, 256 * 16) * 256 * 4, dtype=torch.int32, device=dev)  # mode 7 reads beyond
    s = torch.cuda.current_stream().cuda_stream
    nbytes = units * (p + 1) * HD * 2 * 2
    names = ["attn", "linear", "stream", "konly", "vonly", "vlin", "vtile", "vfinish"]
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def run(mode, occ):
        lds = 65536 if occ == 2 else 163840 // occ - 1024
        grid = 256 * occ

        def launch(i):
            rc = lib.kv_probe(mode, kc[i].data_ptr(), vt[i].data_ptr(), out.data_ptr(), units, smax, p, grid, lds, s)
            assert rc == 0, rc

        for i in range(args.layers):
            launch(i)
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            st.record()
            for i in range(args.layers):
                launch(i)
            en.record()
            en.synchronize()
            ts.append(st.elapsed_time(en) * 1000.0 / args.layers)
        us = min(ts)
        nb = nbytes // 2 if mode >= 3 else nbytes
        print(json.dumps(dict(mode=names[mode], wg_per_cu=occ, rows=rows, pos=p, us=round(us, 2),
                              kv_bytes=nb, GBps=round(nb / us / 1e3, 1))), flush=True)

    for mode in [int(m) for m in args.modes.split(",")]:
        for occ in [int(o) for o in args.occ.split(",")]:
            run(mode, occ)


if __name__ == "__main__":
    main()
