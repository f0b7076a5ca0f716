"""Per-kernel microbenchmark at the BASELINE config-2 shapes (B=64, 48x48, 64 ch).

    python tools/kbench.py [--batch 64] [--iters 30]

Times each hot kernel alone with HIP events on its launch stream and prints
avg us and achieved TFLOP/s (algorithmic) / GB/s.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "super-resolution-climate_amd"), ROOT]
if os.environ.get("KBENCH_STAMPS"):  # phase stamps live only in the diagnostic build (make stamps)
    os.environ.setdefault("SRMI_LIB", os.path.join(ROOT, "super-resolution-climate_amd", "srmi", "libsrmi_stamps.so"))

import torch  # noqa: E402

from srmi._lib import call, ptr  # noqa: E402


def timeit(fn, iters):
    st = torch.cuda.current_stream()
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(iters):
        fn()
    e1.record(st)
    e1.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / iters  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--iters", type=int, default=30)
    args = ap.parse_args()
    d = torch.device("cuda", 0)
    N, H, W = args.batch, 48, 48
    S = lambda: torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.randn(N, H, W, 64, generator=g).to(d).to(torch.bfloat16)
    dy = torch.randn(N, H, W, 64, generator=g).to(d).to(torch.bfloat16)
    t = torch.randn(N, H, W, 64, generator=g).clamp_min(0).to(d).to(torch.bfloat16)
    r1 = torch.randn(N, H, W, 64, generator=g).to(d)
    yf = torch.empty_like(r1)
    yb = torch.empty_like(x)
    w = (torch.randn(64, 64, 3, 3, generator=g) * 0.05).to(d)
    b = torch.zeros(64, device=d)
    fp = torch.empty(64 * 64 * 9, dtype=torch.bfloat16, device=d)
    dp = torch.empty_like(fp)
    pb = torch.empty(64, device=d)
    call("srmi_pack_conv", ptr(w), ptr(b), 64, 64, 0, ptr(fp), ptr(dp), ptr(pb), 0, S())
    ns = call("srmi_conv3x3_nstrips", H, W)
    part = torch.zeros(N, ns, 128, device=d)
    flop = 2.0 * N * H * W * 64 * 576
    res = {}

    def conv(epi, xin, wp, **kw):
        def f():
            call("srmi_conv3x3", ptr(xin), ptr(wp), ptr(kw.get("bias")), N, H, W, 64, 64, 0, epi, ptr(kw.get("yb")),
                 ptr(kw.get("yf")), ptr(kw.get("r1")), None, None, ptr(kw.get("aux")), ptr(kw.get("part")), 1.0, 0, S())
        return f

    cases = {
        "fwd_relu": conv(0, x, fp, bias=pb, yb=yb),
        "fwd_pool": conv(1, x, fp, bias=pb, yb=yb, part=part),
        "fwd_resid": conv(2, x, fp, bias=pb, yb=yb, yf=yf, r1=r1),
        "dgrad_relumask": conv(4, dy, dp, yb=yb, aux=t),
        "dgrad_acc": conv(5, dy, dp, yb=None, yf=yf, r1=yf, aux=t, part=part),
        "dgrad_acc_ca": conv(7, dy, dp, yb=None, yf=yf, r1=yf, aux=t, part=part),
    }
    for k, f in cases.items():
        us = timeit(f, args.iters)
        res[k] = {"us": round(us, 2), "tflops": round(flop / us / 1e6, 1)}
    slab = torch.empty(64 << 20, dtype=torch.float32, device=d)
    gw = torch.empty(64, 64, 3, 3, device=d)
    gb = torch.empty(64, device=d)

    def wg():
        call("srmi_wgrad3x3", ptr(x), ptr(dy), N, H, W, 64, 0, 0, ptr(slab), slab.numel() * 4, 0, 1.0, ptr(gw),
             ptr(gb), 0, S())
    us = timeit(wg, args.iters)
    res["wgrad+reduce"] = {"us": round(us, 2), "tflops": round(flop / us / 1e6, 1)}

    def wg_only():
        call("srmi_wgrad3x3", ptr(x), ptr(dy), N, H, W, 64, 0, 0, ptr(slab), slab.numel() * 4, 0, 1.0, None, None, 0, S())
    us = timeit(wg_only, args.iters)
    res["wgrad"] = {"us": round(us, 2), "tflops": round(flop / us / 1e6, 1)}
    # channel attention elementwise kernels
    R = 2
    w1 = torch.randn(32, 64, device=d) * 0.1
    b1 = torch.zeros(32, device=d)
    w2 = torch.randn(64, 32, device=d) * 0.1
    b2 = torch.zeros(64, device=d)
    rec = torch.zeros(N, 160, device=d)
    brec = torch.zeros(N * 224, device=d)
    pool = torch.zeros(N, ns, 64, device=d)

    def caf():
        call("srmi_ca_forward", ptr(yb), ptr(pool), ns, ptr(w1), ptr(b1), ptr(w2), ptr(b2), N, H * W, 64, R, ptr(r1),
             ptr(yf), ptr(x), ptr(rec), 0, S())

    def cab():
        call("srmi_ca_backward", ptr(r1), ptr(part), ns, ptr(rec), ptr(w1), ptr(w2), N, H * W, 64, R, ptr(yb),
             ptr(brec), 0, S())
    for k, f, byt in (("ca_fwd", caf, N * H * W * 64 * 12), ("ca_bwd_du", cab, N * H * W * 64 * 6)):
        us = timeit(f, args.iters)
        res[k] = {"us": round(us, 2), "GBps": round(byt / us / 1e3, 1)}
    # batch preparation (lnorm + xyflip + downsample) of the C2 HR batch: 1 read + 1.06 writes
    Cb, T = 2, 4 * H
    raw = torch.randn(N, Cb, T, T, device=d) + 280.0
    hrb, lrb = torch.empty_like(raw), torch.empty(N, Cb, H, W, device=d)
    mb, sb = torch.empty(N, Cb, device=d), torch.empty(N, Cb, device=d)

    def prep():
        call("srmi_batch_prep", ptr(raw), N, Cb, T, 5, 4, ptr(hrb), ptr(lrb), ptr(mb), ptr(sb), S())
    us = timeit(prep, args.iters)
    res["batch_prep"] = {"us": round(us, 2), "GBps": round(raw.numel() * 4 * (2 + 1 / 16) / us / 1e3, 1)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()


def stamps():
    """Phase timing of the Cin=64 conv kernel from s_memtime stamps (KBENCH_EPI: epilogues)."""
    import numpy as np
    d = torch.device("cuda", 0)
    N, H, W = 64, 48, 48
    S = torch.cuda.current_stream().cuda_stream
    x = torch.randn(N, H, W, 64, device=d).to(torch.bfloat16)
    t = torch.randn(N, H, W, 64, device=d).clamp_min(0).to(torch.bfloat16)
    r1 = torch.randn(N, H, W, 64, device=d)
    w = torch.randn(64, 64, 3, 3, device=d) * 0.05
    b = torch.zeros(64, device=d)
    fp = torch.empty(64 * 64 * 9, dtype=torch.bfloat16, device=d)
    dp = torch.empty_like(fp)
    pb = torch.empty(64, device=d)
    call("srmi_pack_conv", ptr(w), ptr(b), 64, 64, 0, ptr(fp), ptr(dp), ptr(pb), 0, S)
    yb = torch.empty_like(x)
    ns = call("srmi_conv3x3_nstrips", H, W)
    part = torch.zeros(N, ns, 128, device=d)
    buf = torch.zeros(4096 * 64, dtype=torch.int64, device=d)
    for epi in [int(v) for v in os.environ.get("KBENCH_EPI", "0").split(",")]:
        if epi == 5:
            args = (ptr(x), ptr(dp), None, N, H, W, 64, 64, 0, 5, None, ptr(r1), ptr(r1), None, None, ptr(t), ptr(part))
        elif epi == 7:
            args = (ptr(x), ptr(dp), None, N, H, W, 64, 64, 0, 7, None, ptr(r1), ptr(r1), None, None, ptr(t), ptr(part))
        elif epi == 1:
            args = (ptr(x), ptr(fp), ptr(pb), N, H, W, 64, 64, 0, 1, ptr(yb), None, None, None, None, None, ptr(part))
        elif epi == 4:
            args = (ptr(x), ptr(dp), None, N, H, W, 64, 64, 0, 4, ptr(yb), None, None, None, None, ptr(t), None)
        elif epi == 2:
            args = (ptr(x), ptr(fp), ptr(pb), N, H, W, 64, 64, 0, 2, ptr(yb), ptr(r1), ptr(r1), None, None, None, None)
        else:
            args = (ptr(x), ptr(fp), ptr(pb), N, H, W, 64, 64, 0, epi, ptr(yb), None, None, None, None, None, None)
        for _ in range(3):
            call("srmi_conv3x3", *args, 1.0, 0, S)
        buf.zero_()
        call("srmi_debug_conv_stamps", ptr(buf))
        call("srmi_conv3x3", *args, 1.0, 0, S)
        call("srmi_debug_conv_stamps", None)
        torch.cuda.synchronize()
        st = buf.view(4096, 64).cpu().numpy()
        st = st[st[:, 0] != 0]
        rel = st - st[:, 0:1]
        rt = st[:, 62:64].astype(np.float64)  # s_memrealtime (100 MHz) at start / end
        clk = np.median((st[:, 61] - st[:, 0]) / np.maximum(rt[:, 1] - rt[:, 0], 1)) * 100.0
        span_us = (rt[:, 1] - rt[:, 0]) / 100.0
        print(f"conv epi={epi} workgroups {len(st)} clock {clk:.0f} MHz  WG span median {np.median(span_us):.2f} us "
              f"max {span_us.max():.2f} us; WG start spread {(rt[:, 0].max() - rt[:, 0].min()) / 100.0:.2f} us, "
              f"first start -> last end {(rt[:, 1].max() - rt[:, 0].min()) / 100.0:.2f} us")
        if os.environ.get("KBENCH_WAVES"):  # per-wave barrier arrival (deferred body diagnostic)
            for j in range(3):
                arr = st[:, 40 + 8 * j:48 + 8 * j].astype(np.int64)
                if not np.all(arr):
                    break
                rel_w = arr - arr[:, :1]
                print(f"strip {j} barrier arrival vs wave 0, median per wave: "
                      + " ".join(f"{int(np.median(rel_w[:, w])):6d}" for w in range(8)))
        names = ["prologue"] + [f"s{j}:{k}" for j in range(3) for k in ("issue", "mfma", "gstore", "epi", "barrier")]
        prev = np.zeros(len(st))
        for i, nm in enumerate(names, start=1):
            if i >= 64 or not np.all(st[:, i]):
                break
            cur = rel[:, i]
            print(f"{nm:12s} median dt {np.median(cur - prev):8.0f}  max {np.max(cur - prev):8.0f}")
            prev = cur


def wstamps():
    """Phase timing of the wgrad kernel from s_memtime stamps."""
    import numpy as np
    d = torch.device("cuda", 0)
    N, H, W = 64, 48, 48
    S = torch.cuda.current_stream().cuda_stream
    x = torch.randn(N, H, W, 64, device=d).to(torch.bfloat16)
    dy = torch.randn(N, H, W, 64, device=d).to(torch.bfloat16)
    slab = torch.empty(64 << 20, dtype=torch.float32, device=d)
    gw = torch.empty(64, 64, 3, 3, device=d)
    gb = torch.empty(64, device=d)
    buf = torch.zeros(4096 * 64, dtype=torch.int64, device=d)

    for rs in [int(v) for v in os.environ.get("KBENCH_RS", "0").split(",")]:
        def run():
            call("srmi_wgrad3x3", ptr(x), ptr(dy), N, H, W, 64, 0, rs, ptr(slab), slab.numel() * 4, 0, 1.0,
                 ptr(gw), ptr(gb), 0, S)
        us = timeit(run, 20)
        buf.zero_()
        call("srmi_debug_wgrad_stamps", ptr(buf))
        run()
        call("srmi_debug_wgrad_stamps", None)
        torch.cuda.synchronize()
        st = buf.view(4096, 64).cpu().numpy()
        st = st[st[:, 0] != 0]
        rel = st - st[:, 0:1]
        print(f"wgrad rs={rs} workgroups {len(st)} us {us:.2f} (wgrad+reduce)")
        cols = [i for i in range(1, 64) if np.all(st[:, i] != 0)]
        prev = np.zeros(len(st))
        for i in cols:
            print(f"stamp {i:2d} median dt {np.median(rel[:, i] - prev):8.0f}  max {np.max(rel[:, i] - prev):8.0f}")
            prev = rel[:, i]


if __name__ == "__main__" and os.environ.get("KBENCH_STAMPS"):
    stamps()
    wstamps()
