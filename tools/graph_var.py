"""Spread of the C2 step time over repeated graph captures in one process: plan rebuilt + recaptured, and
recaptured with the plan kept (one JSON line per capture)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from zonos_vibes_amd import _lib  # noqa: E402
from zonos_vibes_amd.config import zonos_v01_transformer  # noqa: E402
from zonos_vibes_amd.model import Zonos  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    tag = sys.argv[1] if len(sys.argv) > 1 else ""
    m = Zonos.synthetic(zonos_v01_transformer(), dev, seed=0, zero_eos=True, max_seqlen=bench.LC + bench.N_NEW + 9,
                        max_prefill=bench.LC + 1)
    e = m.engine
    cond = bench.cond_tensor(0, e.d, dev)
    for how in ("rebuild", "recapture", "keep"):
        for i in range(5):
            if how == "rebuild":
                e._build_plan()
            elif how == "recapture":
                for g in e._graphs.values():
                    _lib.check(e.lib.zmi_graph_destroy(g))
                e._graphs.clear()
            us, pos = bench.time_decode_step(m, cond, steps=128)
            print(json.dumps(dict(env=tag, how=how, i=i, us=round(us, 1))), flush=True)


if __name__ == "__main__":
    main()
