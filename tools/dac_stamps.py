"""Timeline of one DAC conv_stage_kernel launch from the diagnostic build's in-kernel stamps.

    tools/build_variant.sh dacst -DZMI_DAC_STAMPS=192 && mv zonos_vibes_amd/var/libdacst.so zonos_vibes_amd/ab/
    ZMI_LIB_PATH=zonos_vibes_amd/ab/libdacst.so python tools/dac_stamps.py [frames]
Stamps (s_memrealtime, 10 ns) per workgroup of the launches with c_out == ZMI_DAC_STAMPS and tap_step 1 (the
first k7 conv of the block with that width; the last such launch of the decode wins), thread 0 (wave 0): start;
per stage: loads landed (barrier passed), next stage's loads issued, MFMAs issued; all MFMAs done, epilogue done.
Prints per-workgroup medians (us) and the launch's start-time spread."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zonos_vibes_amd import _lib  # noqa: E402
from zonos_vibes_amd.autoencoder import DACAutoencoder  # noqa: E402


def med(x):
    return round(float(np.median(x)) / 100, 3)


def main():
    frames = int(sys.argv[1]) if len(sys.argv) > 1 else 861
    ae = DACAutoencoder("cuda")
    codes = torch.randint(0, 1024, (1, 9, frames), generator=torch.Generator().manual_seed(0)).cuda()
    lib = _lib.lib()
    lib.zmi_dac_stamps_read.restype = ctypes.c_int
    lib.zmi_dac_stamps_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    for _ in range(2):
        ae.decode(codes)
    torch.cuda.synchronize()
    st = np.zeros((8192, 32), dtype=np.uint64)
    assert lib.zmi_dac_stamps_read(st.ctypes.data, st.nbytes) == 0
    st = st[st[:, 0] > 0].astype(np.int64)
    t0 = st[:, 0].min()
    ns = int(max(s for s in range(8) if (st[:, 1 + 3 * s] > 0).any())) + 1
    stages = []
    prev = st[:, 0]
    for s in range(ns):
        land, iss, mf = st[:, 1 + 3 * s], st[:, 2 + 3 * s], st[:, 3 + 3 * s]
        stages.append(dict(wait=med(land - prev), issue=med(iss - land), mfma=med(mf - iss)))
        prev = mf
    out = dict(workgroups=len(st), stages=ns, launch_us=round(float((st[:, 31] - t0).max()) / 100, 2),
               start_quantiles_us=[round(float(x) / 100, 2) for x in np.quantile(st[:, 0] - t0, [0, 0.25, 0.5, 0.75, 1])],
               per_stage=stages, tail_to_mfma_done=med(st[:, 30] - prev), epilogue=med(st[:, 31] - st[:, 30]),
               wg_total=med(st[:, 31] - st[:, 0]))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
