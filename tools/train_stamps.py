"""Phase timing of the training forward convs (conv1 EPI_RELU_POOL = 8, conv2
EPI_CA_RESID_U = 10) inside the C2 step, from s_memtime stamps (diagnostic build:
make stamps -> libsrmi_stamps.so).

The bench's trainer (rcan-10-20-64, B = 64, two micro-batch engines) runs a few steps,
then one step with the stamps on for ONE epilogue (SRMI_STAMP_EPI); the buffer keeps
the last such launch of the step.  Per workgroup: prologue (incl. conv2's CA scale,
whose own sub-phases follow the body's stamps), the run's strips.
    python tools/train_stamps.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "super-resolution-climate_amd"), ROOT]
os.environ.setdefault("SRMI_LIB", os.path.join(ROOT, "super-resolution-climate_amd", "srmi", "libsrmi_stamps.so"))

import torch  # noqa: E402

import bench  # noqa: E402
from srmi._lib import call, ptr  # noqa: E402
from srmi.dist import DistInfo  # noqa: E402
from srmi.engine import NetSpec  # noqa: E402
from srmi.trainer import FusedTrainer  # noqa: E402


def main():
    d = torch.device("cuda", 0)
    spec = NetSpec(arch="rcan", nchannels_in=2, nchannels_out=2, nfeatures=64, nlayers=10, nblocks=20,
                   cbottleneck=2, scale=4, flags=int(os.environ.get("STAMPS_FLAGS", "0")))  # (16: SRMI_FLAG_DU_PASS)
    tr = FusedTrainer(spec, 64, (48, 48), lr=1e-4, info=DistInfo(), device=d, seed=0, micro=2)
    hr = torch.tensor(bench.synthetic_hr(64, 2, 192, 1234)).to(d)
    for _ in range(3):
        tr.step(hr)
    torch.cuda.synchronize()
    for epi, name in ((8, "conv1 RELU_POOL"), (10, "conv2 CA_RESID_U"), (11, "F1 dgrad runs (DG_ACC_CA16)"),
                      (4, "F2 dgrad runs (DG_RELUMASK, deferred)")):
        buf = torch.zeros(2 * 4096 * 64, dtype=torch.int64, device=d)
        os.environ["SRMI_STAMP_EPI"] = str(epi)
        call("srmi_debug_conv_stamps", ptr(buf))
        tr.step(hr)
        torch.cuda.synchronize()
        call("srmi_debug_conv_stamps", None)
        flat = buf.view(-1, 64).cpu().numpy().astype(np.int64)
        if epi in (4, 7, 11):  # fused launch: the dgrad runs' blocks among the filter-gradient ones
            # [grid][64] dgrad rows, then [grid][64] filter-gradient rows (the launch's last
            # block is a filter-gradient one, so its row ends the second region)
            grid = (int(np.nonzero(flat[:8192, 0])[0][-1]) + 1) // 2
            wg = flat[grid:2 * grid]
            wg = wg[(wg[:, 0] != 0) & (wg[:, 63] != 0)]
            if len(wg):  # the filter-gradient bodies (wgrad48 WSTAMP 0 .. 63)
                print(f"  ({name[:2]} filter-gradient chunks: {len(wg)}, span median {np.median(wg[:, 63] - wg[:, 0]):.0f}, "
                      f"p90 {np.percentile(wg[:, 63] - wg[:, 0], 90):.0f}; their start after the launch's first "
                      f"stamp: median {np.median(wg[:, 0] - flat[:grid, 0][flat[:grid, 0] != 0].min()):.0f})")
                print(f"    filter-gradient prologue median {np.median(wg[:, 1] - wg[:, 0]):.0f}, main loop median "
                      f"{np.median(wg[:, 62 if np.all(wg[:, 62]) else 1] - wg[:, 1]):.0f}")
            body = flat[:grid][flat[:grid, 0] != 0]
            nst = np.array([sum(1 for j in range(11) if r[2 + 5 * j + 4] != 0) for r in body])
            if epi in (7, 11) and (nst == 1).any() and (nst > 1).any():
                t = body[nst == 1]
                print(f"  (F1 tail strips run by the filter-gradient workgroups: {len(t)}, span median "
                      f"{np.median(t[:, 61] - t[:, 0]):.0f}, prologue {np.median(t[:, 1] - t[:, 0]):.0f})")
                body = body[nst == nst.max()]
            cs = body
        else:
            # the scale's stamps follow the body's [grid][64] (grid: the last row with a
            # run-end stamp, the scale's rows hold stamps 0..6 only)
            nwg = int(np.nonzero(flat[:, 61])[0][-1]) + 1
            body, cs = flat[:nwg], flat[nwg:2 * nwg]
            if os.environ.get("TS_DEBUG"):
                nz = np.nonzero(flat[:, 0])[0]
                print("  (nonzero stamp rows:", nz[:4], "...", nz[-4:], len(nz), "of", len(flat), ")")
        ok = (body[:, 0] != 0) & (body[:, 61] != 0)
        body, cs = body[ok], cs[ok]
        tot = body[:, 61] - body[:, 0]
        print(f"{name}: {ok.sum()} workgroups, span median {np.median(tot):.0f} cycles")

        def row(nm, v):
            print(f"  {nm:30s} median {np.median(v):8.0f}  p90 {np.percentile(v, 90):8.0f}  "
                  f"share {np.median(v) / np.median(tot):6.3f}")
        row("prologue", body[:, 1] - body[:, 0])
        if epi == 4 and np.all(body[:, 34]):  # (du from g: the CA backward MLP and the first du groups)
            row("  start -> DMA landed", body[:, 32] - body[:, 0])
            row("  CA backward MLP", body[:, 33] - body[:, 32])
            row("  du of the first two groups", body[:, 34] - body[:, 33])
        if epi == 10:
            for i, nm in enumerate(("  scale: T + border lines", "  scale: barrier 1", "  scale: S_tap + matvec",
                                    "  scale: barrier 2", "  scale: z1 + s", "  scale: barrier 3")):
                row(nm, cs[:, i + 1] - cs[:, i])
            row("  body start -> scale start", cs[:, 0] - body[:, 0])
            if np.all(cs[:, 9]):  # (diagnostic build SRMI_TLAT: the t operands' latency alone)
                row("  t loads: barrier + issue", cs[:, 8] - body[:, 1])
                row("  t loads: latency", cs[:, 9] - cs[:, 8])
        if epi == 8 and np.all(body[:, 60]):  # conv1's run end: its share of the CA mean (SRMI_CA_MPART)
            last = max(j for j in range(11) if np.all(body[:, 2 + 5 * j + 4]))
            row("run end: colsums + wait (DMA, stores)", body[:, 57] - body[:, 2 + 5 * last + 4])
            row("run end: barrier", body[:, 58] - body[:, 57])
            row("run end: column reduce + barrier", body[:, 59] - body[:, 58])
            row("run end: matvec + store", body[:, 60] - body[:, 59])
        for j in range(6):
            base = 2 + 5 * j
            if not np.all(body[:, base + 4]):
                break
            prev = body[:, base - 1] if j else body[:, 1]
            parts = []
            for i, nm in enumerate(("issue", "mfma", "gstore", "epi", "barrier")):
                cur = body[:, base + i]
                parts.append(f"{nm} {np.median(cur - prev):6.0f}")
                prev = cur
            print(f"  strip {j}: " + "  ".join(parts))
    os.environ.pop("SRMI_STAMP_EPI", None)


if __name__ == "__main__":
    main()
