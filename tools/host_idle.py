"""Diagnostic: host enqueue cost of ONE C2 training step issued onto an idle
device (queue empty, so no back-pressure from a full hardware queue), against
the steady-state wall time, for each micro-batch count given on the command line.

    python tools/host_idle.py 1 2
"""
import os
import sys
import time

import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "super-resolution-climate_amd"))
sys.path.insert(0, ROOT)
from bench import synthetic_hr  # noqa: E402
from srmi.engine import NetSpec  # noqa: E402
from srmi.trainer import FusedTrainer  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    spec = NetSpec(arch="rcan", nchannels_in=2, nchannels_out=2, nfeatures=64, nlayers=10, nblocks=20,
                   cbottleneck=2, scale=4)
    hr = torch.tensor(synthetic_hr(64, 2, 192, 1234)).to(dev)
    for m in [int(a) for a in sys.argv[1:]] or [2]:
        tr = FusedTrainer(spec, 64, (48, 48), lr=1e-4, device=dev, seed=0, micro=m)
        for _ in range(3):
            tr.step(hr)
        torch.cuda.synchronize()
        idle = []
        for _ in range(5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            tr.step(hr)
            idle.append(time.perf_counter() - t0)
            torch.cuda.synchronize()
        K = 20
        t0 = time.perf_counter()
        for _ in range(K):
            tr.step(hr)
        th = time.perf_counter() - t0
        torch.cuda.synchronize()
        tw = time.perf_counter() - t0
        idle.sort()
        print(f"micro={m}: idle-queue enqueue of one step {1e3 * idle[len(idle) // 2]:.2f} ms (min "
              f"{1e3 * idle[0]:.2f}); back-to-back enqueue {1e3 * th / K:.2f} ms/step, wall {1e3 * tw / K:.2f} "
              f"ms/step = {64 * K / tw:.1f} tiles/s", flush=True)
        del tr
        torch.cuda.synchronize()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
