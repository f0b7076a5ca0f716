"""Diagnostic: GPU time of the micro-batch engines' forward+backward, eager vs
per-engine HIP graphs replayed on the engines' own streams (timing only)."""
import faulthandler
import os
import sys
import time

faulthandler.enable()
import torch  # noqa: E402

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
    for _ in range(2):
        tr.step(hr)
    torch.cuda.synchronize()
    mb = tr.mb
    sl = [slice(k * mb, (k + 1) * mb) for k in range(2)]

    def fb(k, eng):
        eng.forward(tr.params, tr.lrbuf[sl[k]], out=tr.sr[sl[k]])
        eng.backward(tr.params, tr.lrbuf[sl[k]], tr.mgrads[k], sr=tr.sr[sl[k]], hr=hr[sl[k]], loss4=tr.loss4)

    main_s = torch.cuda.current_stream()

    def eager():
        tr.streams[1].wait_stream(main_s)
        for k, eng in enumerate(tr.engines):
            with tr._ctx(k):
                fb(k, eng)
        main_s.wait_stream(tr.streams[1])

    def timeit(fn, label):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            fn()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"{label}: enqueue {1e3 * (t1 - t0) / K:.2f} ms, wall {1e3 * (t2 - t0) / K:.2f} ms", flush=True)

    timeit(eager, "eager fwd+bwd x2 engines")
    gs = []
    for k, eng in enumerate(tr.engines):
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(main_s)
        with torch.cuda.graph(g, stream=s):
            fb(k, eng)
        torch.cuda.synchronize()
        gs.append(g)
    print("captured", flush=True)

    def graphs():
        tr.streams[1].wait_stream(main_s)
        gs[0].replay()
        with torch.cuda.stream(tr.streams[1]):
            gs[1].replay()
        main_s.wait_stream(tr.streams[1])

    timeit(graphs, "graphs fwd+bwd x2 engines")

    def g0():
        gs[0].replay()

    def e0():
        fb(0, tr.engines[0])
    timeit(e0, "eager engine0 alone")
    timeit(g0, "graph engine0 alone")


if __name__ == "__main__":
    main()
