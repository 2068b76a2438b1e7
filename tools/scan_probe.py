"""Mamba2 prefill scan timing at the Zonos-v0.1-hybrid dims (d_ssm 4096, 64 heads), two sequences of seq_len
rows: the single-workgroup zmi_mamba2_scan and the parallel zmi_mamba2_scan_ws (HIP events, 10 launches each).

    python tools/scan_probe.py [seq_len ...]"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zonos_vibes_amd import _lib  # noqa: E402
from zonos_vibes_amd.config import zonos_v01_hybrid  # noqa: E402


def stamps(lib):
    """Per-tile phases of the scan_ws launch from the diagnostic build (-DZMI_SCAN_STAMPS): median cycles of
    (operands into LDS, positions) per tile over workgroups, and the launch's workgroup start spread."""
    import numpy as np
    lib.zmi_scan_stamps_read.restype = ctypes.c_int
    lib.zmi_scan_stamps_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    st = np.zeros((1024, 32), dtype=np.uint64)
    assert lib.zmi_scan_stamps_read(st.ctypes.data, st.nbytes) == 0
    st = st[st[:, 0] > 0].astype(np.int64)
    out = {"workgroups": len(st), "start_spread_cyc": int(st[:, 0].max() - st[:, 0].min())}
    prev = st[:, 0]
    tiles = []
    for k in range(12):
        if not (st[:, 2 + 2 * k] > 0).all():
            break
        tiles.append([int(np.median(st[:, 1 + 2 * k] - prev)), int(np.median(st[:, 2 + 2 * k] - st[:, 1 + 2 * k]))])
        prev = st[:, 2 + 2 * k]
    out["tiles_stage_positions_cyc"] = tiles
    return out


def main():
    dev = torch.device("cuda", 0)
    lib = _lib.lib()
    md = zonos_v01_hybrid().backbone.mamba2_dims()
    for S in [int(x) for x in sys.argv[1:]] or [1, 32, 64, 161, 322]:
        m = 2 * S
        bf = lambda *sh: (torch.randn(*sh, device=dev) * 0.5).to(torch.bfloat16)  # noqa: E731
        zx, cw, cb = bf(m, md["d_in_proj"]), bf(md["conv_dim"], 4), bf(md["conv_dim"])
        dtb = torch.full((md["nheads"],), -2.0, device=dev)
        A, D = -torch.ones(md["nheads"], device=dev), torch.ones(md["nheads"], device=dev)
        ring = torch.zeros(2, 4, md["conv_dim"], dtype=torch.bfloat16, device=dev)
        ssm = torch.zeros(2, md["nheads"], 64, 128, dtype=torch.bfloat16, device=dev)
        y = torch.zeros(m, md["d_ssm"], dtype=torch.bfloat16, device=dev)
        rp = torch.arange(S, dtype=torch.int32, device=dev).repeat(2)
        a = _lib.Mamba2Args()
        a.zxbcdt, a.ld_zx, a.M = zx.data_ptr(), md["d_in_proj"], m
        a.d_ssm, a.nheads, a.headdim, a.d_state, a.d_conv, a.ngroups = md["d_ssm"], md["nheads"], 64, 128, 4, 1
        a.conv_w, a.conv_b, a.dt_bias, a.A, a.D = cw.data_ptr(), cb.data_ptr(), dtb.data_ptr(), A.data_ptr(), D.data_ptr()
        a.conv_ring, a.ssm, a.y, a.ldy, a.row_pos = ring.data_ptr(), ssm.data_ptr(), y.data_ptr(), md["d_ssm"], rp.data_ptr()
        nb = int(lib.zmi_mamba2_scan_ws_bytes(m, md["d_ssm"], md["nheads"]))
        ws = torch.zeros(nb, dtype=torch.uint8, device=dev)
        s = torch.cuda.current_stream().cuda_stream
        out = {"seq_len": S}
        arms = [("scan", lambda: lib.zmi_mamba2_scan(ctypes.byref(a), S, s))]
        for pq in (1, 2, 4):
            arms.append((f"scan_ws_pq{pq}", lambda pq=pq: (lib.zmi_set_option(_lib.OPT_SCAN_PQ, pq),
                                                           lib.zmi_mamba2_scan_ws(ctypes.byref(a), S, ws.data_ptr(),
                                                                                  nb, s))[1]))
        for name, fn in arms:
            _lib.check(fn(), name)
            torch.cuda.synchronize()
            st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            st.record()
            for _ in range(10):
                fn()
            en.record()
            en.synchronize()
            out[name + "_us"] = round(st.elapsed_time(en) * 100, 2)
        lib.zmi_set_option(_lib.OPT_SCAN_PQ, 4)
        if os.environ.get("ZMI_LIB_PATH", "").endswith("scanst.so"):
            _lib.check(lib.zmi_mamba2_scan_ws(ctypes.byref(a), S, ws.data_ptr(), nb, s), "scan_ws")
            torch.cuda.synchronize()
            out["stamps"] = stamps(lib)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
