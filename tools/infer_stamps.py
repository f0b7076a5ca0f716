"""Phase timing of the one-launch inference RCAB (rcab_infer_kernel) from s_memtime
stamps (diagnostic build: make stamps -> libsrmi_stamps.so).

One inference engine at the C5 launch shape (N images of 48x48, default 221), one
forward, then one launch of its RCAB (0, 2) with the stamps on: per workgroup
conv1's body stamps, conv2's body stamps and the launch's phase stamps
(rcab_infer.hip ISTAMP).  Prints median / p90 cycles per phase.
    python tools/infer_stamps.py [N]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "super-resolution-climate_amd"), ROOT]
os.environ.setdefault("SRMI_LIB", os.path.join(ROOT, "super-resolution-climate_amd", "srmi", "libsrmi_stamps.so"))

import torch  # noqa: E402

from srmi._lib import call, ptr  # noqa: E402
from srmi.engine import Engine, NetSpec, param_table  # noqa: E402
from srmi.trainer import default_init_  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 221
    d = torch.device("cuda", 0)
    spec = NetSpec(arch="rcan", nchannels_in=1, nchannels_out=1, nfeatures=64, nlayers=10, nblocks=20,
                   cbottleneck=2, scale=4)
    table = param_table(spec)
    params = torch.empty(sum(t[2] for t in table), dtype=torch.float32, device=d)
    default_init_(params, table, 0)
    eng = Engine(spec, N, (48, 48), train=False, device=d)
    eng.pack(params)
    lr = torch.randn(N, 1, 48, 48, device=d)
    out = eng.forward(params, lr)
    torch.cuda.synchronize()
    buf = torch.zeros(4 * N * 64, dtype=torch.int64, device=d)
    call("srmi_debug_conv_stamps", ptr(buf))
    # one launch of the RCAB (0, 2) of the last forward alone (srmi_engine_probe 3): no
    # other conv launch writes the stamps buffer after it
    call("srmi_engine_probe", eng._h, 3, 1, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    call("srmi_debug_conv_stamps", None)
    st = buf.view(4, N, 64).cpu().numpy().astype(np.int64)
    c1, c2, k, cs = st[0], st[1], st[2], st[3]
    ok = (k[:, 0] != 0) & (k[:, 3] != 0)
    c1, c2, k, cs = c1[ok], c2[ok], k[ok], cs[ok]
    print(f"workgroups with stamps: {ok.sum()} of {N}")
    rt = c1[:, 62:64].astype(np.float64)
    clk = np.median((c1[:, 61] - c1[:, 0]) / np.maximum(rt[:, 1] - rt[:, 0], 1)) * 100.0
    print(f"shader clock ~{clk:.0f} MHz (s_memtime vs s_memrealtime over conv1)")
    tot = k[:, 3] - k[:, 0]
    print(f"launch span per workgroup: median {np.median(tot):.0f} cycles ({np.median(tot) / clk:.2f} us)")

    def row(name, v):
        print(f"  {name:34s} median {np.median(v):8.0f}  p90 {np.percentile(v, 90):8.0f}  "
              f"share {np.median(v) / np.median(tot):6.3f}")
    row("conv1 body", k[:, 1] - k[:, 0])
    row("  conv1 prologue", c1[:, 1] - c1[:, 0])
    row("  conv1 strips", c1[:, 61] - c1[:, 1])
    row("own_stores_visible", k[:, 2] - k[:, 1])
    row("conv2 body (the scale inside)", k[:, 3] - k[:, 2])
    row("  conv2 prologue", c2[:, 1] - c2[:, 0])
    row("  conv2 strips", c2[:, 61] - c2[:, 1])
    row("  ca_scale_finish (after strip 0's MFMAs)", cs[:, 7] - cs[:, 0])
    for i, nm in enumerate(("T partials + border lines", "barrier 1", "S_tap + matvec (LDS filters)", "barrier 2",
                            "z1", "barrier 3 + s", "barrier 4")):
        row("    " + nm, cs[:, i + 1] - cs[:, i])
    # conv2's per-strip phases (non-deferred body: issue, mfma, gstore, epi, barrier)
    names = ("issue", "mfma", "gstore", "epi", "barrier")
    for j in (0, 5, 10):
        base = 2 + 5 * j
        prev = c2[:, base - 1] if j else c2[:, 1]
        parts = []
        for i, nm in enumerate(names):
            cur = c2[:, base + i]
            parts.append(f"{nm} {np.median(cur - prev):6.0f}")
            prev = cur
        print(f"  conv2 strip {j:2d}: " + "  ".join(parts))
    # start skew over the launch
    rel0 = (c1[:, 62] - c1[:, 62].min()) / 100.0
    print(f"workgroup start spread (us): median {np.median(rel0):.2f} max {rel0.max():.2f}")


if __name__ == "__main__":
    main()
