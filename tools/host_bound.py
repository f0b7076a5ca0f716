"""Diagnostic: is the C2 training step host-launch bound?  Times the host-side
enqueue of K steps against the GPU wall time, then tries to capture one step in
a HIP graph and times its replay (the Adam step count is frozen in the capture,
so replayed numerics are not a training run -- timing only)."""
import os
import sys
import time
import faulthandler

faulthandler.enable()

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "super-resolution-climate_amd"))
from srmi.engine import NetSpec  # noqa: E402
from srmi.trainer import FusedTrainer  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    B, C, K = 64, 2, 10
    spec = NetSpec(arch="rcan", nchannels_in=C, nchannels_out=C, nfeatures=64, nlayers=10, nblocks=20,
                   cbottleneck=2, scale=4)
    tr = FusedTrainer(spec, B, (48, 48), lr=1e-4, device=dev, seed=0)
    hr = torch.randn(B, C, 192, 192, generator=torch.Generator().manual_seed(1)).to(dev)
    for _ in range(3):
        tr.step(hr)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        tr.step(hr)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"eager: enqueue {1e3 * (t1 - t0) / K:.2f} ms/step, wall {1e3 * (t2 - t0) / K:.2f} ms/step", flush=True)

    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        tr.step(hr)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    print("capturing", flush=True)
    with torch.cuda.graph(g, stream=s):
        tr.step(hr)
    print("captured", flush=True)
    torch.cuda.synchronize()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        g.replay()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"graph: enqueue {1e3 * (t1 - t0) / K:.2f} ms/step, wall {1e3 * (t2 - t0) / K:.2f} ms/step "
          f"({B * K / (t2 - t0):.1f} tiles/s)", flush=True)
    print("loss", float(tr.loss4[3]))


if __name__ == "__main__":
    main()
