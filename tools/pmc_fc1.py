"""Small driver for the HBM-traffic PMC pass (rocprofv3 --pmc FETCH_SIZE): builds the synthetic
Zonos-v0.1-transformer engine and runs only the fc1 GEMV of each of the 26 layers once, so the
counter pass (which serialises every dispatch) stays short. Run under:

    rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc -o pmc -- \
        python tools/pmc_fc1.py

FETCH_SIZE (KB) of the fc1 dispatches x 2 (gfx950 wide-read correction, MI355X_MICROARCH.md
§HBM) is the HBM traffic per launch reported as bench.py's roofline.traffic.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import time_dominant_kernel  # noqa: E402
from zonos_vibes_amd.config import zonos_v01_transformer  # noqa: E402
from zonos_vibes_amd.model import Zonos  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    model = Zonos.synthetic(zonos_v01_transformer(), dev, seed=0, zero_eos=True, max_seqlen=64, max_prefill=16)
    torch.cuda.synchronize()
    us, bl = time_dominant_kernel(model, reps=1)
    print(f"fc1 {us:.2f} us/launch under the counter pass, {bl} algorithmic bytes", flush=True)
