"""Diagnostic: which part of the training step can be captured in a HIP graph.
Captures, one graph each and in this order: engine 0 forward, its backward,
the Adam step, the filter repack; prints after each capture."""
import faulthandler
import os
import sys

faulthandler.enable()
import torch  # noqa: E402

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "super-resolution-climate_amd"))
from srmi.engine import NetSpec, adam_step  # noqa: E402
from srmi.trainer import FusedTrainer  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    B, C = 64, 2
    spec = NetSpec(arch="rcan", nchannels_in=C, nchannels_out=C, nfeatures=64, nlayers=10, nblocks=20,
                   cbottleneck=2, scale=4)
    tr = FusedTrainer(spec, B, (48, 48), lr=1e-4, device=dev, seed=0)
    hr = torch.randn(B, C, 192, 192, generator=torch.Generator().manual_seed(1)).to(dev)
    for _ in range(2):
        tr.step(hr)
    torch.cuda.synchronize()
    e, mb = tr.engines[0], tr.mb
    parts = {
        "forward": lambda: e.forward(tr.params, tr.lrbuf[:mb], out=tr.sr[:mb]),
        "backward": lambda: e.backward(tr.params, tr.lrbuf[:mb], tr.mgrads[0], sr=tr.sr[:mb], hr=hr[:mb],
                                       loss4=tr.loss4, events=None),
        "adam": lambda: adam_step(tr.params, tr.grads, tr.m, tr.v, 5, tr.lr),
        "pack": lambda: e.pack(tr.params),
        "step": lambda: tr.step(hr),
        "bwd2": lambda: two(lambda k, eng: eng.backward(tr.params, tr.lrbuf[k * mb:(k + 1) * mb], tr.mgrads[k],
                                                        sr=tr.sr[k * mb:(k + 1) * mb], hr=hr[k * mb:(k + 1) * mb],
                                                        loss4=tr.loss4, events=None)),
        "fwd2": lambda: two(lambda k, eng: eng.forward(tr.params, tr.lrbuf[k * mb:(k + 1) * mb],
                                                       out=tr.sr[k * mb:(k + 1) * mb])),
    }

    def two(fn):
        main = torch.cuda.current_stream()
        tr.streams[1].wait_stream(main)
        for k, eng in enumerate(tr.engines):
            with tr._ctx(k):
                fn(k, eng)
        main.wait_stream(tr.streams[1])
    which = sys.argv[1:] or list(parts)
    gs = []
    for k in which:
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream())
        print("capture", k, flush=True)
        with torch.cuda.graph(g, stream=s):
            parts[k]()
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        print("ok", k, flush=True)
        gs.append(g)


if __name__ == "__main__":
    main()
