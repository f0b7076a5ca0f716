"""Run the bench's training step and the in-step roofline probes (for rocprofv3
--pmc passes and kernel-trace agreement checks).

    python tools/roofline_driver.py [--batch 64] [--micro 2] [--steps 2] [--reps 10]

(--reps 0: the steps only -- tools/pmc_step_total.sh sums a whole step's PMC bytes)

The FusedTrainer of bench.py (rcan-10-20-64, 2-var, B tiles of 48x48, micro-batch
engines) runs `steps` steps, then every engine re-issues its fused backward
launches (srmi_engine_probe: conv1's dgrad + filter gradient, then conv2's) `reps`
times on its own stream, concurrently as in the step.  Every dispatch of the
dominant kernel in this run has the in-step launch configuration.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "super-resolution-climate_amd"), ROOT]

import torch  # noqa: E402

from srmi._lib import call  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--micro", type=int, default=2)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    from bench import synthetic_hr
    from srmi.engine import NetSpec
    from srmi.trainer import FusedTrainer
    d = torch.device("cuda", 0)
    spec = NetSpec(arch="rcan", nchannels_in=2, nchannels_out=2, nlayers=10, nblocks=20, cbottleneck=2, scale=4)
    tr = FusedTrainer(spec, a.batch, (48, 48), device=d, micro=a.micro)
    hr = torch.tensor(synthetic_hr(a.batch, 2, 192, 1234)).to(d)
    for _ in range(a.steps):
        tr.step(hr)
    torch.cuda.synchronize()
    main_st = torch.cuda.current_stream()
    for which in ((1, 2) if a.reps > 0 else ()):
        for k, eng in enumerate(tr.engines):
            st = tr.streams[k] or main_st
            st.wait_stream(main_st)
            call("srmi_engine_probe", eng._h, which, a.reps, st.cuda_stream)
        for st in tr.streams[1:]:
            main_st.wait_stream(st)
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
